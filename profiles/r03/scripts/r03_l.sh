#!/usr/bin/env bash
# Round 3: the driver's exact sequence (GPU test suite, then a fresh
# `bench.py --gpus 1 --steps 20 --warmup 5`) once per span-kernel candidate
# (spans_pipe:blocks_per_cu:lab); the CPU baseline is skipped (it runs after
# the timed region and does not change it).  lab (round-3 knob) bit 0: the
# lean kernel computes its mask table; bit 1: 1024-thread blocks.
set -u
TAG=${TAG:-r03l}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
step() { local name=$1 secs=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  echo "   rc=$rc"; grep -v "^[EW]20\|amdgpu.ids" "$OUT/$name.log" | tail -n 1 | cut -c1-200
  case $rc in 0) ;; *) echo FATAL; exit $rc;; esac; }
for c in ${AB_CONFIGS:-2 5}; do
  step ab_c$c 300 python3 tools/ab.py --config $c --rounds 8 --variants spans_pipe=1 lab=1 lab=2 lab=3 blocks_per_cu=512 lab=1,blocks_per_cu=512 lab=2,blocks_per_cu=512 lab=3,blocks_per_cu=512 spans_pipe=0 spans_pipe=2
done
step ab_c2s 300 python3 tools/ab.py --config 2s --rounds 8 --variants spans_pipe=1 spans_pipe=0 blocks_per_cu=64 spans_geo=65 spans_pipe=0,blocks_per_cu=64
step ab_c2s_strided 300 python3 tools/ab.py --config 2s --api strided --rounds 8 --variants spans_pipe=1 spans_pipe=0 blocks_per_cu=64 spans_pipe=0,blocks_per_cu=64
for cand in ${CANDS:-1:0:0 1:512:0 1:0:2 1:512:2 1:0:1 0:0:0}; do
  IFS=: read -r p b l <<< "$cand"; tag=p${p}_b${b}_l${l}
  step pytest_$tag 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
  step bench_$tag 300 env UINET_CKSUM_SPANS_PIPE=$p UINET_CKSUM_BLOCKS_PER_CU=$b UINET_CKSUM_LAB=$l python3 bench.py --gpus 1 --steps 20 --warmup 5 --cpu-baseline off
  python3 - "$OUT/bench_$tag.log" <<'PY'
import json, sys
for line in open(sys.argv[1]):
    if line.startswith('{"metric"'):
        d = json.loads(line); r = d["roofline"]
        print("   %s value %.1f GiB/s ms/step %.4f frac %.4f kernel_ms_mean %.5f" % (
            sys.argv[1].split("/")[-1], d["value"], d["ms_per_step"], r["frac"], r["kernel_ms_mean"]))
PY
done
echo "== done"
