#!/usr/bin/env bash
# GPU test pass: the named test files first (fast feedback), then the whole
# -m gpu suite, then the per-call / host-batch latency tool.
set -u
TAG=${TAG:-r02b}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  echo "   rc=$rc"; grep -v "^[EW]20" "$OUT/$name.log" | tail -n 4 | cut -c1-400
  case $rc in 0) ;; *) echo FATAL; exit $rc;; esac; }
if [ -n "${FIRST:-}" ]; then
  step pytest_first 900 python -u -m pytest $FIRST -m gpu -x -v --timeout 600 --timeout-method thread -p no:cacheprovider
fi
step pytest_gpu 1100 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -p no:cacheprovider
[ -n "${PERCALL:-}" ] && step percall 300 python -u tests/perf/percall_latency.py
echo "== done"
