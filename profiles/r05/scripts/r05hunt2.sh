#!/bin/bash
# A long differential fuzz hunt on seeds not run before (UINET_FUZZ_BASE), malformed
# frames in a quarter of the offload trials.
set -o pipefail
out=gpurun_out/r05hunt2
mkdir -p $out
UINET_FUZZ_TRIALS=120000 UINET_FUZZ_BASE=700000 timeout -k 10 1100 python -u -m pytest -x -v -s \
  --timeout 1050 --timeout-method thread tests/test_gpu_fuzz.py > $out/fuzz.log 2>&1
rc=$?
tail -8 $out/fuzz.log
exit $rc
