#!/usr/bin/env bash
# Round 5: SQ counters of the 5tso kernels -- k_chains_wide (auto pick) and the
# tile kernel (chains_wide 1) -- one --pmc pass each (8 SQ counters).
set -u
OUT=gpurun_out/${TAG:-r05widesq}; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
SQ="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY"
timeout -s KILL 120 rocprofv3 --pmc $SQ -d "$OUT/sq_wide" -o run --output-format csv -- python3 bench.py --config 5tso --steps 3 --warmup 1 --cpu-baseline off --host-offload off > "$OUT/sq_wide.log" 2>&1 || exit 1
echo "wide ok"
export UINET_CKSUM_CHAINS_WIDE=1
timeout -s KILL 120 rocprofv3 --pmc $SQ -d "$OUT/sq_tile" -o run --output-format csv -- python3 bench.py --config 5tso --steps 3 --warmup 1 --cpu-baseline off --host-offload off > "$OUT/sq_tile.log" 2>&1 || exit 1
echo "tile ok"
