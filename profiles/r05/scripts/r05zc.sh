#!/usr/bin/env bash
# Round 5: long randomized differential run on the final tree -- host batches
# (staged / zero-copy / device walk) and the hooks (host / device, a third of
# the trials with headers cut across mbufs) against the oracle.
set -u
OUT=gpurun_out/${TAG:-r05zc}; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
echo "== fuzz"
timeout -k 10 1000 env UINET_FUZZ_TRIALS=8000 python -u -m pytest tests/test_gpu_fuzz.py -m gpu -x -v -s --timeout 980 --timeout-method thread -p no:cacheprovider > "$OUT/fuzz.log" 2>&1
rc=$?; echo "   rc=$rc"; tail -n 8 "$OUT/fuzz.log" | cut -c1-200; exit $rc
