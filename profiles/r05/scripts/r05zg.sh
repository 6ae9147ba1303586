#!/usr/bin/env bash
# Round 5: the device hooks write each walk group's verdicts as soon as its
# fold is done (hook_group.so = the tree; a group the device cannot take is
# redone by the host hook) against one apply after every group (hook_prev.so).
# Hook / device-walk / offload tests and the hook fuzz on the tree first; then
# 3 alternating rounds of the device hooks; hook trace under the tree.
set -u
OUT=gpurun_out/${TAG:-r05zg}; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
LIB=libuinet_amd/libuinet_cksum.so
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  echo "   rc=$rc"; grep -v "^[EW]20\|amdgpu.ids" "$OUT/$name.log" | tail -n 1 | cut -c1-200
  case $rc in 0) ;; *) echo FATAL; cp profiles/r05/ab/hook_group.so $LIB; exit $rc;; esac; }
step pytest 500 python -u -m pytest tests/test_device_walk.py tests/test_offload.py tests/test_in6.py tests/test_replay.py tests/test_echo.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
step fuzz 500 env UINET_FUZZ_TRIALS=3000 python -u -m pytest tests/test_gpu_fuzz.py -m gpu -x -q -s -k offload --timeout 480 --timeout-method thread -p no:cacheprovider
for r in 1 2 3; do for v in hook_group hook_prev; do
  cp profiles/r05/ab/$v.so $LIB
  step host_cpu_${v}_$r 300 python -u tests/perf/host_cpu.py --work hooks --paths dev_walk --threads 1 --reps 5
done; done
cp profiles/r05/ab/hook_group.so $LIB
step trace 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 tests/perf/host_cpu.py --work hooks --paths dev_walk --threads 1 --reps 3
echo "== done"
