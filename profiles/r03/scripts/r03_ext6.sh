#!/usr/bin/env bash
# Round 3: IPv6 extension headers in the offload hooks (walked to the
# transport on RX and TX); the offload, IPv6 and pcap GPU tests against the
# oracle.
set -u
TAG=${TAG:-r03s2e}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
step() { local name=$1 secs=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  echo "   rc=$rc"; grep -v "^[EW]20\|amdgpu.ids" "$OUT/$name.log" | tail -n 1 | cut -c1-300
  case $rc in 0) ;; *) echo FATAL; exit $rc;; esac; }
step pytest_offload 600 python -u -m pytest tests/test_offload.py tests/test_in6.py tests/test_echo.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider
echo "== done"
