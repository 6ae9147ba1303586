#!/usr/bin/env bash
# Round 5: is the device walk / hook parse bound by host (IO) read requests?
# TCC read requests split DRAM / IO, IO credit stalls, in-flight level (read latency
# = LEVEL / RDREQ), per kernel, on the device-walked config-3 batch and the hooks.
set -u
OUT=gpurun_out/${TAG:-r05p}; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -s KILL "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  echo "   rc=$rc"; grep -v "^[EW]20\|amdgpu.ids" "$OUT/$name.log" | tail -n 1 | cut -c1-300
  case $rc in 0) ;; *) echo FATAL; exit $rc;; esac; }
CMD="python3 tests/perf/host_cpu.py --work c3,hooks --paths dev_walk,zero_copy --threads 1 --reps 1"
step io 120 rocprofv3 --pmc TCC_EA0_RDREQ_IO_32B_sum TCC_EA0_RDREQ_IO_CREDIT_STALL_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_LEVEL_sum -d "$OUT/io" -o run --output-format csv -- $CMD
step dram 120 rocprofv3 --pmc TCC_EA0_RDREQ_DRAM_sum TCC_BUSY_sum GRBM_GUI_ACTIVE -d "$OUT/dram" -o run --output-format csv -- $CMD
step trace 120 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- $CMD
echo "== done"
