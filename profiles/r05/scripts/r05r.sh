#!/usr/bin/env bash
# Round 5: the walk's mbuf-header load marked nontemporal (nt.so) against the
# plain load (base.so), 3 alternating rounds of the device paths; then the IO
# counters under nt (does the TCC fetch less than a 128-B line per hop?).
set -u
OUT=gpurun_out/${TAG:-r05r}; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
LIB=libuinet_amd/libuinet_cksum.so
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  echo "   rc=$rc"; grep -v "^[EW]20\|amdgpu.ids" "$OUT/$name.log" | tail -n 1 | cut -c1-200
  case $rc in 0) ;; *) echo FATAL; cp profiles/r05/ab/base.so $LIB; exit $rc;; esac; }
for r in 1 2 3; do for v in nt base; do
  cp profiles/r05/ab/$v.so $LIB
  step host_cpu_${v}_$r 240 python -u tests/perf/host_cpu.py --work c2,c3,hooks --paths dev_walk --threads 1 --reps 3
done; done
cp profiles/r05/ab/nt.so $LIB
step io_nt 120 rocprofv3 --pmc TCC_EA0_RDREQ_IO_32B_sum TCC_EA0_RDREQ_IO_CREDIT_STALL_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_LEVEL_sum -d "$OUT/io_nt" -o run --output-format csv -- python3 tests/perf/host_cpu.py --work c3 --paths dev_walk --threads 1 --reps 1
cp profiles/r05/ab/base.so $LIB
echo "== done"
