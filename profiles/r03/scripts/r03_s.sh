#!/usr/bin/env bash
# Round 3: k_spans_lean with the split 34-entry mask table (lab=1) against the
# 17 x 17 table: parity, interleaved A/B at 512 and 128 blocks per CU, and the
# driver's sequence twice each (alternating).
set -u
TAG=${TAG:-r03s}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
step() { local name=$1 secs=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  echo "   rc=$rc"; grep -v "^[EW]20\|amdgpu.ids" "$OUT/$name.log" | tail -n 1 | cut -c1-200
  case $rc in 0) ;; *) echo FATAL; exit $rc;; esac; }
step pytest_split 900 env UINET_CKSUM_LAB=1 python -u -m pytest tests/test_gpu_parity.py -x -q -k "spans or strided" --timeout 300 --timeout-method thread -p no:cacheprovider
for c in 2 5 4; do
  step ab_c$c 300 python3 tools/ab.py --config $c --rounds 8 --variants lab=0 lab=1 blocks_per_cu=128 lab=1,blocks_per_cu=128
done
for rep in 1 2; do
for l in 1 0; do
  tag=l${l}_$rep
  step pytest_$tag 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
  step bench_$tag 300 env UINET_CKSUM_LAB=$l python3 bench.py --gpus 1 --steps 20 --warmup 5 --cpu-baseline off
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
step cold_l1 300 env UINET_CKSUM_LAB=1 python3 tools/cold_start.py --launches 300 --idle-s 1.5
step cold_l0 300 env UINET_CKSUM_LAB=0 python3 tools/cold_start.py --launches 300 --idle-s 1.5
echo "== done"
