#!/usr/bin/env bash
# Round 3: the driver's bench command beside the box's own streaming-read
# ceiling (tools/hbm_read, same 1.57 GB as config 2), so a slow line can be
# told from a slow box; then the driver's command again.
set -u
TAG=${TAG:-r03s2x}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 tools/hbm_read.hip -o /tmp/hbm_read || exit 1
timeout -k 10 120 /tmp/hbm_read 1572864000 > "$OUT/hbm_read_1.log" 2>&1 || exit 1; tail -n 2 "$OUT/hbm_read_1.log"
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/driver_bench.log" 2>&1 || exit 1; grep '^{' "$OUT/driver_bench.log" | cut -c1-200
timeout -k 10 120 /tmp/hbm_read 1572864000 > "$OUT/hbm_read_2.log" 2>&1 || exit 1; tail -n 2 "$OUT/hbm_read_2.log"
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --cpu-baseline off > "$OUT/driver_bench_2.log" 2>&1 || exit 1
echo "== done"
