#!/usr/bin/env bash
# Round 3: the dense strided kernel for small packets laid back to back:
# parity (its own tests and the strided / small-packet ones), then 2s / 2su
# on the strided API against the previous kernels (spans_pipe 0 keeps k_spans;
# the quad / k_spans path of spans_pipe 1 before this kernel is base.so).
set -u
TAG=${TAG:-r03s2m}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
step() { local name=$1 secs=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  echo "   rc=$rc"; grep -v "^[EW]20\|amdgpu.ids" "$OUT/$name.log" | tail -n 1 | cut -c1-300
  case $rc in 0) ;; *) echo FATAL; exit $rc;; esac; }
step pytest_dense 600 python -u -m pytest tests/test_strided_dense.py tests/test_gpu_parity.py -k "dense or strided or small_packets or every_kernel" -m gpu -x -q --timeout 500 --timeout-method thread -p no:cacheprovider
TAG=$TAG VARIANTS="base new" CONFIGS="2s 2su" ARGS="--api strided" ROUNDS=3 bash tools/ab_lib_multi.sh
echo "== done"
