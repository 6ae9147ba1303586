#!/usr/bin/env bash
# Round 5: staged host batches packed with non-temporal stores (nt_copy.so =
# the tree) against plain memcpy (plain_copy.so), 3 alternating rounds of the
# staged path at 1 and 16 host threads; host-batch tests + fuzz on the tree first.
set -u
OUT=gpurun_out/${TAG:-r05t}; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
LIB=libuinet_amd/libuinet_cksum.so
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  echo "   rc=$rc"; grep -v "^[EW]20\|amdgpu.ids" "$OUT/$name.log" | tail -n 1 | cut -c1-200
  case $rc in 0) ;; *) echo FATAL; cp profiles/r05/ab/nt_copy.so $LIB; exit $rc;; esac; }
step pytest_host 400 python -u -m pytest tests/test_gpu_parity.py tests/test_offload.py tests/test_echo.py tests/test_in6.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
step fuzz 400 env UINET_FUZZ_TRIALS=600 python -u -m pytest tests/test_gpu_fuzz.py -m gpu -x -q -s --timeout 380 --timeout-method thread -p no:cacheprovider
for r in 1 2 3; do for v in nt_copy plain_copy; do
  cp profiles/r05/ab/$v.so $LIB
  step host_cpu_${v}_$r 300 python -u tests/perf/host_cpu.py --work c2,c3,hooks,echo --paths staged --threads 1,16 --reps 3
done; done
cp profiles/r05/ab/nt_copy.so $LIB
echo "== done"
