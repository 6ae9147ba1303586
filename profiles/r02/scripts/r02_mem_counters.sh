#!/usr/bin/env bash
# Memory-request counters for the span kernel (config 2) and the chain kernel
# (config 3): L1 -> L2 requests per byte, L2 requests / hits, HBM read
# requests.  Tests whether the chain kernel's per-byte request rate (16-B
# lanes over ~110-B segments, duplicate boundary chunks) is what holds it
# below the span kernel's traffic rate.  Usage: TAG=... bash tools/r02_mem_counters.sh
set -u
TAG=${TAG:-r02mem}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 --list-avail > $OUT/list_avail.txt 2>&1; echo "list rc=$?"
for cfg in 2 3; do
  i=0
  for set in "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCC_REQ_sum TCC_HIT_sum" \
             "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum" \
             "TCC_MISS_sum TCC_TAG_STALL_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $set --kernel-trace -d $OUT/c$cfg/p$i -o run --output-format csv -- python3 bench.py --config $cfg --steps 5 --warmup 1 --cpu-baseline off > $OUT/c$cfg.p$i.log 2>&1
    rc=$?; echo "cfg $cfg set $i rc=$rc"; grep -iE "error|invalid|not found" $OUT/c$cfg.p$i.log | grep -v "^W20" | head -3
    case $rc in 124|134|137|139) echo stop; exit $rc;; esac
  done
done
echo done
