#!/usr/bin/env bash
# Round 4: span-kernel A/Bs at 64 lanes (config 5's 9000-B frames) against
# the previous build: GPU tests on the new library (TESTS, default the whole
# GPU suite), then CONFIGS (default config 5, and config 2 as a control: its
# kernel's ISA is unchanged) alternating processes, 3 rounds.
# tools/ab_so/{base,new}.so are built beforehand.
set -u
TAG=${TAG:-r04c5}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
cp tools/ab_so/new.so libuinet_amd/libuinet_cksum.so
timeout -k 10 900 python3 -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
CONFIGS="${CONFIGS:-5 2}" TAG=$TAG bash tools/ab_lib_swap.sh
