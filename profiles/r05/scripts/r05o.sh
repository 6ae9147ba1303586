#!/usr/bin/env bash
# Round 5: what bounds the device walk and the hook parse?  Address-translation
# counters (UTCL1 in the TCP, UTCL2 busy) per kernel, device-walked config-3
# batch and device hooks; one counter pass per block group.
set -u
OUT=gpurun_out/${TAG:-r05o}; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -s KILL "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  echo "   rc=$rc"; grep -v "^[EW]20\|amdgpu.ids" "$OUT/$name.log" | tail -n 1 | cut -c1-300
  case $rc in 0) ;; *) echo FATAL; exit $rc;; esac; }
step tcp 120 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum TCP_UTCL1_STALL_INFLIGHT_MAX_sum -d "$OUT/tcp" -o run --output-format csv -- python3 tests/perf/host_cpu.py --work c3,hooks --paths dev_walk --threads 1 --reps 1
step grbm 120 rocprofv3 --pmc GRBM_UTCL2_BUSY GRBM_GUI_ACTIVE -d "$OUT/grbm" -o run --output-format csv -- python3 tests/perf/host_cpu.py --work c3,hooks --paths dev_walk --threads 1 --reps 1
step tcp_dev 120 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum TCP_UTCL1_STALL_INFLIGHT_MAX_sum -d "$OUT/tcp_dev" -o run --output-format csv -- python3 bench.py --config 3 --steps 3 --warmup 1 --cpu-baseline off
echo "== done"
