#!/usr/bin/env bash
# Round 3 measurement set.  PART=a: GPU tests; the driver's exact bench command
# (untraced, then under a per-dispatch rocprofv3 trace with amd-smi sampled);
# bench + trace + FETCH_SIZE for the span configs.  PART=b: small packets,
# chains, the pure-read ceiling.
set -u
TAG=${TAG:-r03q}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
step() { local name=$1 secs=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  echo "   rc=$rc"; grep -v "^[EW]20\|amdgpu.ids" "$OUT/$name.log" | tail -n 1 | cut -c1-300
  case $rc in 0) ;; *) echo FATAL; exit $rc;; esac; }
if [ "${PART:-a}" = a ]; then
  step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -p no:cacheprovider
  step driver_bench 300 python3 bench.py --gpus 1 --steps 20 --warmup 5
  step pytest_gpu2 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -p no:cacheprovider
  python3 tools/smi_sample.py "$OUT/smi_driver.json" --period-s 0.005 --max-s 240 & SMI=$!
  step driver_trace 300 rocprofv3 --kernel-trace --stats -d "$OUT/driver_trace" -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --cpu-baseline off
  kill $SMI; wait $SMI
  python3 tools/pmc_summary.py "$OUT/driver_trace" > "$OUT/driver_trace.summary.json"
  TAG=$TAG CONFIGS="${CONFIGS:-2 2@strided 2rx 4 5}" bash tools/prof_all.sh || exit $?
else
  TAG=$TAG CONFIGS="${CONFIGS:-2s 2s@strided 2su 3 3tx 5tso}" bash tools/prof_all.sh || exit $?
  step hbm_read 300 tools/hbm_read
fi
echo "== done"
