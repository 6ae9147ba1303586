#!/usr/bin/env bash
# Round 5: long randomised differential run of the host-batch and hook fuzz
# (mbufs registered in a random half of the zero-copy trials: the device walk)
# against the oracle.
set -u
OUT=gpurun_out/${TAG:-r05g}; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  echo "   rc=$rc"; grep -v "^[EW]20\|amdgpu.ids" "$OUT/$name.log" | tail -n 3 | cut -c1-300
  case $rc in 0) ;; *) echo FATAL; exit $rc;; esac; }
step fuzz_host 900 env UINET_FUZZ_TRIALS=4500 python -u -m pytest tests/test_gpu_fuzz.py -m gpu -x -v -s -k "host_batches or offload_hooks" --timeout 880 --timeout-method thread -p no:cacheprovider
echo "== done"
