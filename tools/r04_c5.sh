#!/usr/bin/env bash
# Round 4: the G = 64 span kernel's rounds 1-2 issued together (config 5's
# 9000-B frames), against the previous build: GPU suite on the new library,
# then config 5 (and config 2 as a control: its kernel's ISA is unchanged)
# alternating processes, 3 rounds.  tools/ab_so/{base,new}.so built beforehand.
set -u
TAG=${TAG:-r04c5}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
cp tools/ab_so/new.so libuinet_amd/libuinet_cksum.so
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
CONFIGS="5 2" TAG=$TAG bash tools/ab_lib_swap.sh
