#!/usr/bin/env bash
# Round 5: the PCIe ceiling for the host-resident paths -- streaming and
# scattered 32-B reads of registered host memory from the GPU, and hipMemcpy
# H2D, over config 2's 1.5 GB (tools/hbm_read host).
set -u
OUT=gpurun_out/${TAG:-r05s}; mkdir -p "$OUT"
echo "== host_read_1"; timeout -k 10 120 tools/hbm_read host 1572864000 > "$OUT/host_read_1.log" 2>&1 || exit 1; cat "$OUT/host_read_1.log"
echo "== host_read_2"; timeout -k 10 120 tools/hbm_read host 1572864000 > "$OUT/host_read_2.log" 2>&1 || exit 1; cat "$OUT/host_read_2.log"
echo "== done"
