#!/usr/bin/env bash
# Round 4, after the 64-lane span changes: the echo tests at full size, then
# every span config's bench line, trace and FETCH_SIZE pass (the span sources
# changed, so their pmc_traffic.json entries are re-measured), and config 2
# with packed descriptors for comparison.
set -u
TAG=${TAG:-r04s3}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
timeout -k 10 300 python3 -u -m pytest tests/test_echo.py -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_echo.log 2>&1 || { tail -30 $OUT/pytest_echo.log; exit 1; }
tail -2 $OUT/pytest_echo.log
HBM=1 TAG=$TAG CONFIGS="2 2@strided 2rx 4 5 2+packed 2s 2s+packed 2su 2su+packed 2su@strided" bash profiles/r04/scripts/r04_set.sh
