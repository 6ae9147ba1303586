#!/usr/bin/env bash
# Round 5: do concurrent misses to one line of registered host memory merge in
# L2?  tools/hbm_read host: one lane per random line loading 1 / 2 / 4 / 8
# chunks of 16 B back to back; time, then the EA read count per kernel.
set -u
OUT=gpurun_out/${TAG:-r05w}; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
echo "== host_read"; timeout -k 10 120 tools/hbm_read host 1572864000 > "$OUT/host_read.log" 2>&1 || exit 1; cat "$OUT/host_read.log"
echo "== pmc"; timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_128B_sum TCC_MISS_sum TCC_HIT_sum -d "$OUT/pmc" -o run --output-format csv -- tools/hbm_read host 1572864000 > "$OUT/pmc.log" 2>&1 || exit 1
echo "== done"
