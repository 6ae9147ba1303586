#!/usr/bin/env bash
# Round 5: the hook parse with four lanes per frame loading the header and
# window together (quad.so = the tree) against one lane per frame (g8.so, the
# r05m tree), alternating processes; hook tests and fuzz first; hook trace.
set -u
OUT=gpurun_out/${TAG:-r05n}; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
LIB=libuinet_amd/libuinet_cksum.so
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  echo "   rc=$rc"; grep -v "^[EW]20\|amdgpu.ids" "$OUT/$name.log" | tail -n 2 | cut -c1-300
  case $rc in 0) ;; *) echo FATAL; cp profiles/r05/ab/quad.so $LIB; exit $rc;; esac; }
step pytest_walk 300 python -u -m pytest tests/test_device_walk.py tests/test_offload.py -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider
step fuzz_hooks 600 env UINET_FUZZ_TRIALS=3000 python -u -m pytest tests/test_gpu_fuzz.py -m gpu -x -v -s -k offload_hooks --timeout 580 --timeout-method thread -p no:cacheprovider
for r in 1 2 3; do for v in quad g8; do
  cp profiles/r05/ab/$v.so $LIB
  step host_cpu_${v}_$r 300 python -u tests/perf/host_cpu.py --work hooks --paths dev_walk --threads 1
done; done
cp profiles/r05/ab/quad.so $LIB
step hook_trace 300 rocprofv3 --kernel-trace --stats -d "$OUT/hook_trace" -o run --output-format csv -- python3 tests/perf/host_cpu.py --work hooks --paths dev_walk --threads 1 --reps 3
echo "== done"
