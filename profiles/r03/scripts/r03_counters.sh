#!/usr/bin/env bash
# Round 3: instruction counters of the final kernels (config 2: k_spans_lean,
# 2s: k_spans_quad, 3: k_chains_pipe), one rocprofv3 --pmc pass each; then
# the GPU suite, smoke() and the driver's command once more on this code.
set -u
TAG=${TAG:-r03c2}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
step() { local name=$1 secs=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  echo "   rc=$rc"; grep -v "^[EW]20\|amdgpu.ids" "$OUT/$name.log" | tail -n 1 | cut -c1-200
  case $rc in 0) ;; *) echo FATAL; exit $rc;; esac; }
for c in 2 2s 3; do
  step pmc_insts_c$c 180 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVES SQ_INSTS_LDS -d "$OUT/pmc_insts_c$c" -o run --output-format csv -- python3 bench.py --config $c --gpus 1 --steps 3 --warmup 1 --cpu-baseline off
done
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -p no:cacheprovider
step smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()"
step driver_bench 300 python3 bench.py --gpus 1 --steps 20 --warmup 5
echo "== done"
