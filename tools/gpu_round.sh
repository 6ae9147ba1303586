#!/usr/bin/env bash
# Full round check: GPU tests, default bench + its kernel trace, every config's
# bench + trace + FETCH_SIZE pass (prof_all.sh), HBM read microbench.
set -u
TAG=${TAG:-r01j}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  echo "   rc=$rc"; grep -v "^[EW]20" "$OUT/$name.log" | tail -n 2
  case $rc in 0) ;; *) echo FATAL; exit $rc;; esac; }
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
step bench_default 600 python3 bench.py
step trace_default 600 rocprofv3 --kernel-trace --stats -d "$OUT/trace_default" -o run --output-format csv -- python3 bench.py --cpu-baseline off
python3 tools/pmc_summary.py "$OUT/trace_default" > "$OUT/trace_default.summary.json"
TAG=$TAG CONFIGS="${CONFIGS:-2 2rx 2s 3 3tx 5 5tso 2@strided 2s@strided}" bash tools/prof_all.sh || exit $?
step hbm_read 300 tools/hbm_read
echo "== done"
