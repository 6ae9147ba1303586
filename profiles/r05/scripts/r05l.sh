#!/usr/bin/env bash
# Round 5: small batches staged over registered memory (kStageBelowJobs,
# kHookDeviceMin): device-walk tests, GPU suite, hook fuzz with device-size
# batches, and the small-batch latency table again.
set -u
OUT=gpurun_out/${TAG:-r05l}; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  echo "   rc=$rc"; grep -v "^[EW]20\|amdgpu.ids" "$OUT/$name.log" | tail -n 2 | cut -c1-300
  case $rc in 0) ;; *) echo FATAL; exit $rc;; esac; }
step pytest_walk 300 python -u -m pytest tests/test_device_walk.py tests/test_in6.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider
step pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
step fuzz_hooks 900 env UINET_FUZZ_TRIALS=3000 python -u -m pytest tests/test_gpu_fuzz.py -m gpu -x -v -s -k offload_hooks --timeout 880 --timeout-method thread -p no:cacheprovider
step batch_latency 500 python -u tests/perf/batch_latency.py
echo "== done"
