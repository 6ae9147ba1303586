#!/usr/bin/env bash
# Full round check (round 2): GPU tests; the driver's exact bench command and its
# rocprofv3 kernel trace; every config's bench + trace + FETCH_SIZE pass
# (prof_all.sh, folded into profiles/pmc_traffic.json); the pure-read ceiling.
# PART=host instead runs the host-resident tools and the N>1 rehearsals.
set -u
TAG=${TAG:-r02z}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  echo "   rc=$rc"; grep -v "^[EW]20\|amdgpu.ids" "$OUT/$name.log" | tail -n 2 | cut -c1-300
  case $rc in 0) ;; *) echo FATAL; exit $rc;; esac; }
if [ "${PART:-gpu}" = host ]; then
  step host_path 600 python3 -u tests/perf/host_path.py
  step offload_rate 600 python3 -u tests/perf/offload_rate.py
  step echo_replay 600 python3 -u tests/perf/echo_replay.py
  step percall 300 python3 -u tests/perf/percall_latency.py
  step bench_gpus2_gloo 600 env UINET_BENCH_BACKEND=gloo python3 bench.py --gpus 2 --steps 20 --warmup 5
  step bench_nccl_world1 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr=127.0.0.1 --master-port=29533 bench.py --gpus 1 --steps 20 --warmup 5 --cpu-baseline off
  echo "== done"; exit 0
fi
if [ -z "${SKIP_BASE:-}" ]; then
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -p no:cacheprovider
step driver_bench 300 python3 bench.py --gpus 1 --steps 20 --warmup 5
step driver_trace 300 rocprofv3 --kernel-trace --stats -d "$OUT/driver_trace" -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --cpu-baseline off
python3 tools/pmc_summary.py "$OUT/driver_trace" > "$OUT/driver_trace.summary.json"
step bench_default 600 python3 bench.py
step trace_default 600 rocprofv3 --kernel-trace --stats -d "$OUT/trace_default" -o run --output-format csv -- python3 bench.py --cpu-baseline off
python3 tools/pmc_summary.py "$OUT/trace_default" > "$OUT/trace_default.summary.json"
fi
TAG=$TAG CONFIGS="${CONFIGS:-2 2rx 2s 3 3tx 4 5 5tso 2@strided 2s@strided}" bash tools/prof_all.sh || exit $?
step hbm_read 300 tools/hbm_read
echo "== done"
