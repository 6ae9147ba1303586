#!/usr/bin/env bash
# Round 5, first GPU pass: device-walk tests, the full GPU suite, smoke, the
# host CPU-time table (tests/perf/host_cpu.py), the single-GPU config-4 shard
# rate (scaling_ref) and the driver's default bench line (all-core baseline).
# SKIP_TESTS=1 skips the two pytest steps.
set -u
OUT=gpurun_out/${TAG:-r05a}; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  echo "   rc=$rc"; grep -v "^[EW]20\|amdgpu.ids" "$OUT/$name.log" | tail -n 3 | cut -c1-400
  case $rc in 0) ;; *) echo FATAL; exit $rc;; esac; }
if [ -z "${SKIP_TESTS:-}" ]; then
step pytest_walk 300 python -u -m pytest tests/test_device_walk.py tests/test_in6.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider
step pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
fi
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
step bench_c4_1gpu 300 python3 bench.py --gpus 1 --config 4 --steps 20 --warmup 20
step bench_default 300 python3 bench.py
step host_cpu 900 python -u tests/perf/host_cpu.py
echo "== done"
