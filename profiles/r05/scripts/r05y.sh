#!/usr/bin/env bash
# Round 5: the hook apply with fewer host writes (apply.so = the tree: a 2-B
# store for a 2-aligned th_sum / ip_sum, RX csum_flags + csum_data in one 8-B
# store) against trim.so; hook tests + fuzz first; 3 alternating rounds; trace.
set -u
OUT=gpurun_out/${TAG:-r05y}; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
LIB=libuinet_amd/libuinet_cksum.so
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  echo "   rc=$rc"; grep -v "^[EW]20\|amdgpu.ids" "$OUT/$name.log" | tail -n 1 | cut -c1-200
  case $rc in 0) ;; *) echo FATAL; cp profiles/r05/ab/apply.so $LIB; exit $rc;; esac; }
step pytest 500 python -u -m pytest tests/test_device_walk.py tests/test_offload.py tests/test_in6.py tests/test_replay.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
step fuzz 600 env UINET_FUZZ_TRIALS=3000 python -u -m pytest tests/test_gpu_fuzz.py -m gpu -x -q -s -k offload --timeout 580 --timeout-method thread -p no:cacheprovider
for r in 1 2 3; do for v in apply trim; do
  cp profiles/r05/ab/$v.so $LIB
  step host_cpu_${v}_$r 300 python -u tests/perf/host_cpu.py --work hooks --paths dev_walk --threads 1 --reps 5
done; done
cp profiles/r05/ab/apply.so $LIB
step trace 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 tests/perf/host_cpu.py --work hooks --paths dev_walk --threads 1 --reps 3
echo "== done"
