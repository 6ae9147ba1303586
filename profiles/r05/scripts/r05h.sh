#!/usr/bin/env bash
# Round 5: the driver hooks on the device (cksum_hookdev.hip) -- device-walk
# and hook tests, the GPU suite, a long hook fuzz, then the hooks' host CPU
# and wall time (tests/perf/host_cpu.py, hooks only, three processes).
set -u
OUT=gpurun_out/${TAG:-r05h}; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  echo "   rc=$rc"; grep -v "^[EW]20\|amdgpu.ids" "$OUT/$name.log" | tail -n 3 | cut -c1-300
  case $rc in 0) ;; *) echo FATAL; exit $rc;; esac; }
step pytest_walk 300 python -u -m pytest tests/test_device_walk.py tests/test_offload.py tests/test_in6.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider
step pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
step fuzz_hooks 600 env UINET_FUZZ_TRIALS=6000 python -u -m pytest tests/test_gpu_fuzz.py -m gpu -x -v -s -k offload_hooks --timeout 580 --timeout-method thread -p no:cacheprovider
for r in 1 2 3; do
  step host_cpu_$r 300 python -u tests/perf/host_cpu.py --work hooks,echo
done
echo "== done"
