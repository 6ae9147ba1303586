#!/usr/bin/env bash
# Round 6 final set: GPU suite, smoke, the driver's bench command and its
# kernel trace, the N = 2 rehearsal (gloo, one GPU); PART=2: the host CPU-time
# table (tests/perf/host_cpu.py, every workload and path, 1 and 16 threads).
set -u
OUT=gpurun_out/${TAG:-r06final}; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  echo "   rc=$rc"; grep -v "^[EW]20\|amdgpu.ids" "$OUT/$name.log" | tail -n 1 | cut -c1-300
  case $rc in 0) ;; *) echo FATAL; exit $rc;; esac; }
if [ "${PART:-1}" = 1 ]; then
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
step driver_bench 400 python3 bench.py --gpus 1 --steps 20 --warmup 5
step driver_trace 300 rocprofv3 --kernel-trace --stats -d "$OUT/driver_trace" -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --cpu-baseline off
python3 tools/pmc_summary.py "$OUT/driver_trace" > "$OUT/driver_trace.summary.json"
step bench_gpus2_gloo 600 env UINET_BENCH_BACKEND=gloo python3 bench.py --gpus 2 --steps 20 --warmup 5
fi
if [ "${PART:-1}" = 2 ]; then
step host_cpu 900 python -u tests/perf/host_cpu.py --paths staged,zero_copy,span,dev_walk,dev_walk2
step batch_latency 300 python -u tests/perf/batch_latency.py
fi
echo "== done"
