#!/usr/bin/env bash
# Round 3: split-table k_spans_lean at 256 vs 512 blocks per CU: the driver's
# sequence twice each (alternating), then the per-launch cold series.
set -u
TAG=${TAG:-r03t}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
step() { local name=$1 secs=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  echo "   rc=$rc"; grep -v "^[EW]20\|amdgpu.ids" "$OUT/$name.log" | tail -n 1 | cut -c1-200
  case $rc in 0) ;; *) echo FATAL; exit $rc;; esac; }
step ab_c2 300 python3 tools/ab.py --config 2 --rounds 8 --variants lab=1 lab=1,blocks_per_cu=256 lab=1,blocks_per_cu=128
for rep in 1 2; do
for b in 256 512; do
  tag=b${b}_$rep
  step pytest_$tag 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
  step bench_$tag 300 env UINET_CKSUM_LAB=1 UINET_CKSUM_BLOCKS_PER_CU=$b python3 bench.py --gpus 1 --steps 20 --warmup 5 --cpu-baseline off
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
for b in 256 128 512; do
  step cold_b$b 300 env UINET_CKSUM_LAB=1 UINET_CKSUM_BLOCKS_PER_CU=$b python3 tools/cold_start.py --launches 300 --idle-s 1.5
done
echo "== done"
