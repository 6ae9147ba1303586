#!/usr/bin/env bash
# Round 3 (lab): the chain kernel at 7 / 8 waves per SIMD with fewer chunks in
# flight on a long segment (UINET_CHAINS_LONGU 2 / 1), which removes the
# round-level spills r03s2d/ found at 7 waves (the long-segment loads were the
# pressure point). Builds in tools/ab_so/: base (6 waves, LONGU 4), w6u2, w7u2,
# w7u1, w8u1 (8 waves still spills 16-20 B). Chain parity on w7u2 first, then
# alternating bench processes on configs 3, 3tx, 5tso.
set -u
TAG=${TAG:-r03s2u}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
LIB=libuinet_amd/libuinet_cksum.so
cp $LIB tools/ab_so/keep.so
cp tools/ab_so/w7u2.so $LIB
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_chains32.py -m gpu -x -q -k chain --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest_w7u2.log 2>&1
rc=$?; tail -n 2 $OUT/pytest_w7u2.log; cp tools/ab_so/keep.so $LIB
[ $rc -eq 0 ] || { echo FATAL $rc; exit $rc; }
TAG=$TAG VARIANTS="base w6u2 w7u2 w7u1 w8u1" CONFIGS="3 3tx 5tso" ROUNDS=2 bash tools/ab_lib_multi.sh
echo "== done"
