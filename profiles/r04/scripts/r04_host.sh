#!/usr/bin/env bash
# Round 4 host-resident set on the final library:
# the zero-copy descriptor A/B (profiles/r04/scripts/r04_hostdesc.sh), then the host-mbuf
# batch rates against the reference (16 and 1 threads), the driver offload
# hooks, and config 1's echo call sequence.
set -u
TAG=${TAG:-r04h}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
TAG=$TAG bash profiles/r04/scripts/r04_hostdesc.sh || exit $?
step() { local name=$1 secs=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  echo "   rc=$rc"; grep -v "^[EW]20\|amdgpu.ids" "$OUT/$name.log" | tail -n 1 | cut -c1-400
  case $rc in 0) ;; *) echo FATAL; exit $rc;; esac; }
step host_path 400 python3 -u tests/perf/host_path.py
step offload_rate 300 python3 -u tests/perf/offload_rate.py
step echo_replay 300 python3 -u tests/perf/echo_replay.py
echo "== done"
