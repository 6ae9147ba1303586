#!/usr/bin/env bash
# Historical A/B: chains_variant 2 (k_chains_flat) and 3/4 existed only in the builds of
# the commits that ran it; see profiles/r01/ab/*/NOTES.md for the results.
# Chains: occupancy sensitivity (blocks per CU caps resident waves: 4 waves per
# block, so bpc 8/6/4/2 = 8/6/4/2 waves per SIMD) for the unpipelined (2) and
# pipelined (0) chunk-stream kernels.
set -u
OUT=gpurun_out/${TAG:-r01m}; mkdir -p $OUT
for c in 3 3tx; do
  timeout -k 10 300 python tools/ab.py --config $c --variants \
    chains_variant=2,blocks_per_cu=64 chains_variant=2,blocks_per_cu=8 chains_variant=2,blocks_per_cu=6 \
    chains_variant=2,blocks_per_cu=4 chains_variant=2,blocks_per_cu=2 \
    chains_variant=0,blocks_per_cu=64 chains_variant=0,blocks_per_cu=6 chains_variant=0,blocks_per_cu=4 \
    chains_variant=0,blocks_per_cu=2 > $OUT/ab_c$c.json 2> $OUT/ab_c$c.err || exit $?
  python3 -c "import json; d=json.load(open('$OUT/ab_c$c.json')); [print('$c',k,v) for k,v in d['results'].items()]"
done
