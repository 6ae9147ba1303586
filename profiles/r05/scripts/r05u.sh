#!/usr/bin/env bash
# Round 5: the zero-copy setup (packet bytes registered, mbufs not) no longer
# launches the device walk / device hook only to have it hand the batch back:
# precheck.so (the tree) against base.so, 3 alternating rounds of the zero-copy
# path at 1 and 16 threads; device-walk / offload / parity tests + fuzz first.
set -u
OUT=gpurun_out/${TAG:-r05u}; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
LIB=libuinet_amd/libuinet_cksum.so
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  echo "   rc=$rc"; grep -v "^[EW]20\|amdgpu.ids" "$OUT/$name.log" | tail -n 1 | cut -c1-200
  case $rc in 0) ;; *) echo FATAL; cp profiles/r05/ab/precheck.so $LIB; exit $rc;; esac; }
step pytest 500 python -u -m pytest tests/test_device_walk.py tests/test_offload.py tests/test_gpu_parity.py tests/test_in6.py tests/test_echo.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
step fuzz 500 env UINET_FUZZ_TRIALS=600 python -u -m pytest tests/test_gpu_fuzz.py -m gpu -x -q -s --timeout 480 --timeout-method thread -p no:cacheprovider
for r in 1 2 3; do for v in precheck base; do
  cp profiles/r05/ab/$v.so $LIB
  step host_cpu_${v}_$r 300 python -u tests/perf/host_cpu.py --work c2,c3,hooks,echo --paths zero_copy --threads 1,16 --reps 3
done; done
cp profiles/r05/ab/precheck.so $LIB
echo "== done"
