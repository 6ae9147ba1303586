#!/usr/bin/env bash
# The round-end driver's sequence, reproduced per span kernel: the full GPU
# test suite, then the driver's exact bench command under a per-dispatch
# rocprofv3 kernel trace, with amdsmi clocks / power sampled during it.
#   KERNELS="1 0" TAG=r03d bash tools/r03_driver_seq.sh   (spans_pipe values)
set -u
TAG=${TAG:-r03d}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
step() { local name=$1 secs=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  echo "   rc=$rc"; grep -v "^[EW]20\|amdgpu.ids" "$OUT/$name.log" | tail -n 2 | cut -c1-300
  case $rc in 0) ;; *) echo FATAL; exit $rc;; esac; }
for k in ${KERNELS:-1}; do
  step pytest_gpu_p$k 900 env UINET_CKSUM_SPANS_PIPE=$k python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -p no:cacheprovider
  python3 tools/smi_sample.py "$OUT/smi_p$k.json" --period-s 0.005 --max-s 240 & SMI=$!
  step driver_trace_p$k 300 env UINET_CKSUM_SPANS_PIPE=$k rocprofv3 --kernel-trace --stats -d "$OUT/driver_trace_p$k" -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5
  kill $SMI; wait $SMI
  python3 tools/pmc_summary.py "$OUT/driver_trace_p$k" > "$OUT/driver_trace_p$k.summary.json"
done
echo "== done"
