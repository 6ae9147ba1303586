#!/usr/bin/env bash
# Round 3 (with tools/ab.py's knob reset): small-packet grid sweep (k_spans
# vs k_spans_quad, span and strided APIs), then the driver's sequence twice
# per headline candidate (spans_pipe:blocks_per_cu:lab).
set -u
TAG=${TAG:-r03m}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
step() { local name=$1 secs=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  echo "   rc=$rc"; grep -v "^[EW]20\|amdgpu.ids" "$OUT/$name.log" | tail -n 1 | cut -c1-200
  case $rc in 0) ;; *) echo FATAL; exit $rc;; esac; }
step ab_c2s 300 python3 tools/ab.py --config 2s --rounds 6 --variants spans_pipe=0 spans_pipe=0,blocks_per_cu=32 spans_pipe=0,blocks_per_cu=64 spans_pipe=0,blocks_per_cu=128 spans_pipe=1 blocks_per_cu=64 blocks_per_cu=128 spans_geo=65 spans_geo=65,blocks_per_cu=64 spans_geo=65,blocks_per_cu=128
step ab_c2s_strided 300 python3 tools/ab.py --config 2s --api strided --rounds 6 --variants spans_pipe=0 spans_pipe=0,blocks_per_cu=64 spans_pipe=0,blocks_per_cu=1024 spans_pipe=1 blocks_per_cu=64 blocks_per_cu=128
for rep in 1 2; do
for cand in ${CANDS:-1:0:0 1:512:0 1:512:1}; do
  IFS=: read -r p b l <<< "$cand"; tag=p${p}_b${b}_l${l}_$rep
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
done
echo "== done"
