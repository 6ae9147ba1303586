#!/usr/bin/env bash
# Round 5: how the GPU fetches registered host memory.  r05p showed the device walk
# issuing 128-B reads for a 32-B mbuf header (4 x 32 B per TCC/EA request).  A/B of
# the registration flags (lab switch UINET_LAB_REGISTER_FLAGS): default fine-grained,
# hipExtHostRegisterUncached (0x80000000), coarse-grained (0x8); 2 alternating rounds
# of the device paths, then the IO counters under the uncached flag.
set -u
OUT=gpurun_out/${TAG:-r05q}; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  echo "   rc=$rc"; grep -v "^[EW]20\|amdgpu.ids" "$OUT/$name.log" | tail -n 1 | cut -c1-200
  case $rc in 0) ;; *) echo FATAL; exit $rc;; esac; }
CMD="python3 tests/perf/host_cpu.py --work c2,c3,hooks --paths dev_walk,zero_copy --threads 1 --reps 3"
for r in 1 2; do
  for f in 0 0x80000000 0x8; do
    export UINET_LAB_REGISTER_FLAGS=$f
    step "flags${f}_r$r" 240 $CMD
  done
done
export UINET_LAB_REGISTER_FLAGS=0x80000000
step io_uc 120 rocprofv3 --pmc TCC_EA0_RDREQ_IO_32B_sum TCC_EA0_RDREQ_IO_CREDIT_STALL_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_LEVEL_sum -d "$OUT/io_uc" -o run --output-format csv -- python3 tests/perf/host_cpu.py --work c3,hooks --paths dev_walk --threads 1 --reps 1
echo "== done"
