#!/usr/bin/env bash
# Round 5: the bench line's host_resident_cpu field (N = 1): bench GPU tests,
# the driver's command, the default bench and config 3.
set -u
OUT=gpurun_out/${TAG:-r05j}; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  echo "   rc=$rc"; grep -v "^[EW]20\|amdgpu.ids" "$OUT/$name.log" | tail -n 2 | cut -c1-300
  case $rc in 0) ;; *) echo FATAL; exit $rc;; esac; }
step pytest_bench 600 python -u -m pytest tests/test_bench_gpu.py -m gpu -x -v --timeout 500 --timeout-method thread -p no:cacheprovider
step driver_bench 300 python3 bench.py --gpus 1 --steps 20 --warmup 5
step bench_c3 300 python3 bench.py --config 3
step bench_c5 300 python3 bench.py --config 5
echo "== done"
