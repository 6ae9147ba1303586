#!/usr/bin/env bash
# Chains: packets per wave tile (tail balance vs per-tile overhead).
set -u
OUT=gpurun_out/${TAG:-r01n}; mkdir -p $OUT
for c in 3 3tx 5tso; do
  timeout -k 10 300 python tools/ab.py --config $c --variants chains_tile=32 chains_tile=64 chains_tile=16 > $OUT/ab_c$c.json 2> $OUT/ab_c$c.err || exit $?
  python3 -c "import json; d=json.load(open('$OUT/ab_c$c.json')); [print('$c',k,v) for k,v in d['results'].items()]"
done
