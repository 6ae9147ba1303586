#!/usr/bin/env bash
# Round 5: what the hook parse and the walk ask L2 for over the host link --
# EA read sizes (32 / 64 / 128 B), L2 hits and misses, and the memory type of
# the requests (NC / UC / CC / RW) -- on the device-walked config-3 batch and
# the device hooks.  Three PMC passes, one per block group.
set -u
OUT=gpurun_out/${TAG:-r05v}; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -s KILL "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  echo "   rc=$rc"; grep -v "^[EW]20\|amdgpu.ids" "$OUT/$name.log" | tail -n 1 | cut -c1-200
  case $rc in 0) ;; *) echo FATAL; exit $rc;; esac; }
CMD="python3 tests/perf/host_cpu.py --work c3,hooks --paths dev_walk --threads 1 --reps 1"
step sizes 120 rocprofv3 --pmc TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_sum -d "$OUT/sizes" -o run --output-format csv -- $CMD
step hits 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_READ_sum TCC_PROBE_sum -d "$OUT/hits" -o run --output-format csv -- $CMD
step mtype 120 rocprofv3 --pmc TCC_NC_REQ_sum TCC_UC_REQ_sum TCC_CC_REQ_sum TCC_RW_REQ_sum -d "$OUT/mtype" -o run --output-format csv -- $CMD
echo "== done"
