#!/usr/bin/env bash
# Round 3, first look at k_spans_lean (spans_pipe=3): parity with it forced,
# interleaved A/B against k_spans_pp, the driver's command per variant (fresh
# processes), one kernel trace of the driver command, VALU counters per KiB.
set -u
TAG=${TAG:-r03a}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  echo "   rc=$rc"; grep -v "^[EW]20\|amdgpu.ids" "$OUT/$name.log" | tail -n 3 | cut -c1-400
  case $rc in 0) ;; *) echo FATAL; exit $rc;; esac; }
step pytest_lean 900 env UINET_CKSUM_SPANS_PIPE=3 python -u -m pytest tests/test_gpu_parity.py -x -q -k "spans or strided" --timeout 300 --timeout-method thread -p no:cacheprovider
V=${V:-"spans_pipe=1 spans_pipe=3 spans_pipe=3,blocks_per_cu=64 spans_pipe=3,blocks_per_cu=32 spans_pipe=3,blocks_per_cu=256"}
for c in 2 2rx 4 5; do step ab_c$c 300 python3 tools/ab.py --config $c --rounds 6 --variants $V; done
step ab_c2_strided 300 python3 tools/ab.py --config 2 --api strided --rounds 6 --variants $V
step drv_ab 900 env VARIANTS="pipe lean" bash tools/drv_ab.sh $TAG/drv 3
step trace_lean 300 env UINET_CKSUM_SPANS_PIPE=3 rocprofv3 --kernel-trace --stats -d "$OUT/trace_lean" -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --cpu-baseline off
for v in 1 3; do
  step pmc_valu_p$v 120 env UINET_CKSUM_SPANS_PIPE=$v rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVES SQ_INSTS_LDS -d "$OUT/pmc_valu_p$v" -o run --output-format csv -- python3 bench.py --gpus 1 --steps 3 --warmup 1 --cpu-baseline off
done
step pytest_bench_gpu 700 python -u -m pytest tests/test_bench_gpu.py -x -v --timeout 600 --timeout-method thread -p no:cacheprovider
echo "== done"
