#!/usr/bin/env bash
# Round 3: a chain-kernel change (base.so vs new.so in tools/ab_so/):
# chain parity tests on the new build, then base vs new in alternating
# bench processes (tools/ab_lib_swap.sh) on configs 3, 3tx, 5tso.
set -u
TAG=${TAG:-r03s2c}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
step() { local name=$1 secs=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  echo "   rc=$rc"; grep -v "^[EW]20\|amdgpu.ids" "$OUT/$name.log" | tail -n 1 | cut -c1-300
  case $rc in 0) ;; *) echo FATAL; exit $rc;; esac; }
step pytest_chains 900 python -u -m pytest tests/test_gpu_parity.py tests/test_chains32.py tests/test_variants.py tests/test_offload.py tests/test_in6.py -m gpu -x -q --timeout 600 --timeout-method thread -p no:cacheprovider
TAG=$TAG CONFIGS="3 3tx 5tso" bash tools/ab_lib_swap.sh
echo "== done"
