#!/usr/bin/env bash
# Round 4 host-resident rates on the final library (after the hooks' fused
# parse, r04hk): host-mbuf batches against the reference (16 and 1 threads),
# the driver offload hooks, config 1's echo call sequence.
set -u
TAG=${TAG:-r04h2}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
step() { local name=$1 secs=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  echo "   rc=$rc"; grep -v "^[EW]20\|amdgpu.ids" "$OUT/$name.log" | tail -n 1 | cut -c1-600
  case $rc in 0) ;; *) echo FATAL; exit $rc;; esac; }
step host_path 400 python3 -u tests/perf/host_path.py
step offload_rate 300 python3 -u tests/perf/offload_rate.py
step echo_replay 300 python3 -u tests/perf/echo_replay.py
echo "== done"
