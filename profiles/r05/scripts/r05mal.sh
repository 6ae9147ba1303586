#!/bin/bash
# Malformed-frame hook tests (frames.mangle_headers) on the GPU box, then the
# differential fuzz on seeds not run before (UINET_FUZZ_BASE), malformed
# frames in a quarter of the offload trials.
set -o pipefail
out=gpurun_out/r05mal
mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  tests/test_device_walk.py tests/test_offload.py > $out/tests.log 2>&1 &&
UINET_FUZZ_TRIALS=6000 UINET_FUZZ_BASE=200000 timeout -k 10 700 python -u -m pytest -x -v -s \
  --timeout 650 --timeout-method thread tests/test_gpu_fuzz.py > $out/fuzz.log 2>&1
rc=$?
tail -3 $out/tests.log; tail -8 $out/fuzz.log
exit $rc
