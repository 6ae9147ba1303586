#!/usr/bin/env bash
# One GPU-box session: parity tests, bench, rocprofv3 kernel trace + PMC pass.
# Each GPU step has its own time limit; a fault/abort/timeout ends the script.
# Usage: tools/gpu_session.sh <tag> [tests|bench|prof|host|variants|tests+host|tests+variants|all]
set -u
TAG=${1:-r01}
WHAT=${2:-all}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
fatal() { # exit codes that mean the GPU step crashed or hung
  case "$1" in 124|134|137|139) return 0;; *) return 1;; esac
}
run() { # name, seconds, command...
  local name=$1 secs=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "   rc=$rc"; tail -n 5 "$OUT/$name.log"
  if fatal $rc; then echo "FATAL step $name rc=$rc -- stopping"; exit $rc; fi
  return 0
}
if [[ $WHAT == all || $WHAT == tests || $WHAT == tests+host || $WHAT == tests+variants ]]; then
  run pytest_gpu 1200 python -m pytest tests -m gpu -q -x -p no:cacheprovider
fi
if [[ $WHAT == all || $WHAT == bench ]]; then
  run bench 600 python bench.py --steps 50 --warmup 10
  run bench_strided 300 python bench.py --steps 50 --warmup 10 --api strided --cpu-baseline off
fi
if [[ $WHAT == all || $WHAT == prof ]]; then
  run prof_trace 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof_trace" -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --cpu-baseline off
  run prof_pmc 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace --stats -d "$OUT/prof_pmc" -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --cpu-baseline off
fi
if [[ $WHAT == all || $WHAT == variants || $WHAT == tests+variants ]]; then
  run bench_c3tx 600 python bench.py --steps 30 --warmup 5 --config 3tx
  run bench_c5tso 600 python bench.py --steps 30 --warmup 5 --config 5tso
  run prof_variants 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof_variants" -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --config 3tx --cpu-baseline off
  run prof_variants_tso 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof_variants_tso" -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --config 5tso --cpu-baseline off
fi
if [[ $WHAT == all || $WHAT == host || $WHAT == tests+host ]]; then
  run echo_replay 600 python tests/perf/echo_replay.py
  run host_path 600 python tests/perf/host_path.py
  run offload_rate 600 python tests/perf/offload_rate.py
fi
echo "== done"
