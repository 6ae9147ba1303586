#!/usr/bin/env bash
# Round 3: the pcap replay harness through the GPU RX hook (tests/test_replay.py).
set -u
TAG=${TAG:-r03s2k}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
step() { local name=$1 secs=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  echo "   rc=$rc"; grep -v "^[EW]20\|amdgpu.ids" "$OUT/$name.log" | tail -n 1 | cut -c1-300
  case $rc in 0) ;; *) echo FATAL; exit $rc;; esac; }
step pytest_replay 300 python -u -m pytest tests/test_replay.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider
echo "== done"
