#!/usr/bin/env bash
# Round 3: the chain kernel's long-segment stream without masks on its whole
# steps (every chunk neither the segment's first nor last; wave-uniform).
# Chain parity on the new build, then base vs new in alternating processes on
# 5tso (the config with long segments), 3 and 3tx.
set -u
TAG=${TAG:-r03s3a}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_chains32.py tests/test_variants.py tests/test_offload.py tests/test_in6.py -m gpu -x -q --timeout 600 --timeout-method thread -p no:cacheprovider > $OUT/pytest_chains.log 2>&1
rc=$?; tail -n 2 $OUT/pytest_chains.log; [ $rc -eq 0 ] || { echo FATAL $rc; exit $rc; }
TAG=$TAG VARIANTS="base new" CONFIGS="5tso 3 3tx" ROUNDS=3 bash tools/ab_lib_multi.sh
echo "== done"
