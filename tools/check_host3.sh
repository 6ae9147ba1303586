#!/usr/bin/env bash
# Full GPU test suite, then every host-resident rate tool (tests/perf/).
set -u
OUT=gpurun_out/${TAG:-r01h3}; mkdir -p $OUT
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  echo "   rc=$rc"; tail -n ${TAILN:-3} "$OUT/$name.log"
  case $rc in 0) ;; *) echo FATAL; exit $rc;; esac; }
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
step host_path 600 python tests/perf/host_path.py
step echo_replay 600 python tests/perf/echo_replay.py
step offload_rate 600 python tests/perf/offload_rate.py
step percall 300 python tests/perf/percall_latency.py
echo "== done"
