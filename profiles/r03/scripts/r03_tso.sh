#!/usr/bin/env bash
# Round 3: config 5tso on the 7-wave chain kernel: tile 8 vs 32 (a 32-packet
# tile gives only 4 waves per SIMD at 131 K packets), long-segment threshold,
# grid width; interleaved in one process (tools/ab.py).
set -u
TAG=${TAG:-r03s2y}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 600 python3 tools/ab.py --config 5tso --rounds 8 --variants chains_tile=0 chains_tile=8 chains_long=64 chains_long=256 chains_tile=8,chains_long=64 > $OUT/ab_5tso.log 2>&1 || exit 1
timeout -k 10 600 python3 tools/ab.py --config 3 --rounds 8 --variants chains_tile=0 chains_long=64 chains_long=256 > $OUT/ab_c3.log 2>&1 || exit 1
echo "== done"
