#!/usr/bin/env bash
# rocprofv3 kernel trace of the default bench command (50 steps, 10 warmup),
# so the committed per-kernel average is the bench line's own launches; plus
# per-launch drift with and without the profiler attached.
set -u
TAG=${TAG:-r01f}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  echo "   rc=$rc"; grep -v "^[EW]20" "$OUT/$name.log" | tail -n 2
  case $rc in 0) ;; *) echo FATAL; exit $rc;; esac; }
step bench_default 600 python3 bench.py --cpu-baseline off
step trace_default 600 rocprofv3 --kernel-trace --stats -d "$OUT/trace_default" -o run --output-format csv -- python3 bench.py --cpu-baseline off
python3 tools/pmc_summary.py "$OUT/trace_default" > "$OUT/trace_default.summary.json"
step drift_plain 600 python3 tools/drift.py --config 2 --launches 300
step drift_traced 600 rocprofv3 --kernel-trace -d "$OUT/drift_traced" -o run --output-format csv -- python3 tools/drift.py --config 2 --launches 300
echo "== done"
