#!/usr/bin/env bash
# Round 5: the hook parse reads only the bytes it uses (trim.so = the tree:
# the IPv4 header length first, no L4 bytes on TX) against the previous build
# (precheck.so), which asked for 68 bytes from every IPv4 header and so, on
# TX frames whose header mbuf ends sooner, walked into the payload mbuf.
# Hook / parity tests + hook fuzz first; 3 alternating rounds of the hooks on
# the device; EA reads of the parse under trim.
set -u
OUT=gpurun_out/${TAG:-r05x}; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
LIB=libuinet_amd/libuinet_cksum.so
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  echo "   rc=$rc"; grep -v "^[EW]20\|amdgpu.ids" "$OUT/$name.log" | tail -n 1 | cut -c1-200
  case $rc in 0) ;; *) echo FATAL; cp profiles/r05/ab/trim.so $LIB; exit $rc;; esac; }
step pytest 500 python -u -m pytest tests/test_device_walk.py tests/test_offload.py tests/test_in6.py tests/test_echo.py tests/test_replay.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
step fuzz 600 env UINET_FUZZ_TRIALS=1500 python -u -m pytest tests/test_gpu_fuzz.py -m gpu -x -q -s -k offload --timeout 580 --timeout-method thread -p no:cacheprovider
for r in 1 2 3; do for v in trim precheck; do
  cp profiles/r05/ab/$v.so $LIB
  step host_cpu_${v}_$r 300 python -u tests/perf/host_cpu.py --work hooks --paths staged,dev_walk --threads 1 --reps 5
done; done
cp profiles/r05/ab/trim.so $LIB
step sizes 120 rocprofv3 --pmc TCC_EA0_RDREQ_IO_32B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_sum -d "$OUT/sizes" -o run --output-format csv -- python3 tests/perf/host_cpu.py --work hooks --paths dev_walk --threads 1 --reps 1
echo "== done"
