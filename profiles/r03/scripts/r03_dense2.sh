#!/usr/bin/env bash
# Round 3: the dense strided kernel dispatched for small packets off 16-B
# alignment only: parity, then the 2su strided line (bench, trace, FETCH_SIZE).
set -u
TAG=${TAG:-r03s2n}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
step() { local name=$1 secs=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  echo "   rc=$rc"; grep -v "^[EW]20\|amdgpu.ids" "$OUT/$name.log" | tail -n 1 | cut -c1-300
  case $rc in 0) ;; *) echo FATAL; exit $rc;; esac; }
step pytest_dense 600 python -u -m pytest tests/test_strided_dense.py tests/test_gpu_parity.py -k "dense or strided or small_packets or every_kernel" -m gpu -x -q --timeout 500 --timeout-method thread -p no:cacheprovider
TAG=$TAG CONFIGS="2su@strided" bash tools/prof_all.sh || exit $?
echo "== done"
