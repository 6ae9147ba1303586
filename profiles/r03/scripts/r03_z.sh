#!/usr/bin/env bash
# Round 3: k_spans_lean's grid sized for two steps per wave (default) against
# fixed widths, configs 2 / 4 / 5; the driver's sequence on config 2 and
# config 4 (the multi-GPU bench's per-GPU shape).
set -u
TAG=${TAG:-r03z}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
step() { local name=$1 secs=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  echo "   rc=$rc"; grep -v "^[EW]20\|amdgpu.ids" "$OUT/$name.log" | tail -n 1 | cut -c1-200
  case $rc in 0) ;; *) echo FATAL; exit $rc;; esac; }
step pytest_spans 900 python -u -m pytest tests/test_gpu_parity.py -x -q -k "spans or strided" --timeout 300 --timeout-method thread -p no:cacheprovider
for c in 2 4 5; do
  step ab_c$c 300 python3 tools/ab.py --config $c --rounds 8 --variants blocks_per_cu=0 blocks_per_cu=256 blocks_per_cu=512 blocks_per_cu=64 spans_pipe=0
done
for c in 4 2; do
  step pytest_c$c 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
  step bench_c$c 300 python3 bench.py --config $c --gpus 1 --steps 20 --warmup 5 --cpu-baseline off
  python3 - "$OUT/bench_c$c.log" <<'PY'
import json, sys
for line in open(sys.argv[1]):
    if line.startswith('{"metric"'):
        d = json.loads(line); r = d["roofline"]
        print("   %s frac %.4f kernel_ms_mean %.5f" % (sys.argv[1].split("/")[-1], r["frac"], r["kernel_ms_mean"]))
PY
done
step cold_c4 300 python3 tools/cold_start.py --config 4 --launches 200 --idle-s 1.5
echo "== done"
