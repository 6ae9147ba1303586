#!/usr/bin/env bash
# Round 4: the driver's sequence on the final tree -- every GPU test, smoke(),
# then the driver's exact bench command and its rocprofv3 kernel trace.
set -u
TAG=${TAG:-r04v}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
step() { local name=$1 secs=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  echo "   rc=$rc"; grep -v "^[EW]20\|amdgpu.ids" "$OUT/$name.log" | tail -n 2 | cut -c1-300
  case $rc in 0) ;; *) echo FATAL; exit $rc;; esac; }
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
step smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()"
step driver_bench 300 python3 bench.py --gpus 1 --steps 20 --warmup 5
step driver_trace 300 rocprofv3 --kernel-trace --stats -d "$OUT/driver_trace" -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5
python3 tools/pmc_summary.py "$OUT/driver_trace" --last 20 > "$OUT/driver_trace.summary.json"
echo "== done"
