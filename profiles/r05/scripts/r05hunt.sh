#!/bin/bash
# A long differential fuzz hunt on seeds not run before (UINET_FUZZ_BASE), malformed
# frames in a quarter of the offload trials.
set -o pipefail
out=gpurun_out/r05hunt
mkdir -p $out
UINET_FUZZ_TRIALS=60000 UINET_FUZZ_BASE=300000 timeout -k 10 1000 python -u -m pytest -x -v -s \
  --timeout 950 --timeout-method thread tests/test_gpu_fuzz.py > $out/fuzz.log 2>&1
rc=$?
tail -8 $out/fuzz.log
exit $rc
