#!/usr/bin/env bash
# Round 5: the tile kernel's tile size on config-3-shaped batches of 96 K to
# 512 K packets (tools/ab.py --packets, in one process each): 32 packets per
# wave (auto from 128 K packets) against 8.  A 32-packet tile gives 4,096
# waves at 128 K packets, 57 % of the 7,168 wave slots.
set -u
OUT=gpurun_out/${TAG:-r05tile}; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for n in 98304 131072 196608 262144 393216 524288; do
  echo "== $n"
  timeout -k 10 300 python3 tools/ab.py --config 3 --packets $n --rounds 8 --variants chains_tile=8 chains_tile=32 chains_tile=8,desc=1 chains_tile=32,desc=1 > "$OUT/ab_c3_$n.log" 2>&1 || exit 1
  grep median_ms "$OUT/ab_c3_$n.log" | tr -d ' \n'; echo
done
echo "== done"
