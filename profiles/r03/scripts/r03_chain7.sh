#!/usr/bin/env bash
# Round 3: the chain kernel at 7 waves per SIMD with 2 long-segment chunks in
# flight per lane (shipped): chain / offload / IPv6 GPU parity, then the chain
# configs' measurement set (bench line, kernel trace, FETCH_SIZE).
set -u
TAG=${TAG:-r03s2v}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_chains32.py tests/test_variants.py tests/test_offload.py tests/test_in6.py tests/test_replay.py -m gpu -x -q --timeout 600 --timeout-method thread -p no:cacheprovider > $OUT/pytest_chains.log 2>&1
rc=$?; tail -n 2 $OUT/pytest_chains.log; [ $rc -eq 0 ] || { echo FATAL $rc; exit $rc; }
TAG=$TAG CONFIGS="3 3tx 5tso 3+packed" bash tools/prof_all.sh || exit $?
echo "== done"
