#!/usr/bin/env bash
# Round 5 measurement set on the final device-walk tree: GPU suite, smoke, the
# driver's bench command and its kernel trace, the default bench, the N = 2
# rehearsal (gloo, one GPU) with the per-rank fields, and the host CPU-time
# table (tests/perf/host_cpu.py, three processes).
set -u
OUT=gpurun_out/${TAG:-r05f}; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  echo "   rc=$rc"; grep -v "^[EW]20\|amdgpu.ids" "$OUT/$name.log" | tail -n 1 | cut -c1-300
  case $rc in 0) ;; *) echo FATAL; exit $rc;; esac; }
# PART=1: tests, smoke and the benches; PART=2: the host CPU table (and the
# hook trace); unset: both (r05z ran them as two calls)
if [ "${PART:-1}" = 1 ] || [ -z "${PART:-}" ]; then
step pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
step driver_bench 300 python3 bench.py --gpus 1 --steps 20 --warmup 5
step driver_trace 300 rocprofv3 --kernel-trace --stats -d "$OUT/driver_trace" -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --cpu-baseline off
python3 tools/pmc_summary.py "$OUT/driver_trace" > "$OUT/driver_trace.summary.json"
step bench_default 300 python3 bench.py
step bench_gpus2_gloo 600 env UINET_BENCH_BACKEND=gloo python3 bench.py --gpus 2 --steps 20 --warmup 5
fi
if [ "${PART:-2}" = 2 ] || [ -z "${PART:-}" ]; then
for r in 1 2 3; do
  step host_cpu_$r 600 python -u tests/perf/host_cpu.py
done
echo "== done"
# (round 5, r05i and later) where a device hook batch's time goes
if [ -n "${HOOK_TRACE:-}" ]; then
step hook_trace 300 rocprofv3 --kernel-trace --stats -d "$OUT/hook_trace" -o run --output-format csv -- python3 tests/perf/host_cpu.py --work hooks --paths dev_walk --threads 1 --reps 3
echo "== done (hook trace)"
fi
fi
