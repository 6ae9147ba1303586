#!/usr/bin/env bash
# Historical A/B: chains_variant 2 (k_chains_flat) and 3/4 existed only in the builds of
# the commits that ran it; see profiles/r01/ab/*/NOTES.md for the results.
# Pipelined chains with the pipelined long-segment stream vs the flat kernel,
# and the long-segment threshold.
set -u
OUT=gpurun_out/${TAG:-r01t}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "chains or config3 or variants or jumbo" > $OUT/pytest.log 2>&1; rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for c in 5tso 3tx 3; do
  timeout -k 10 300 python tools/ab.py --config $c --variants chains_variant=0 chains_variant=2 chains_variant=0,chains_long=64 chains_variant=0,chains_long=32 > $OUT/ab_c$c.json 2> $OUT/ab_c$c.err || exit $?
  python3 -c "import json; d=json.load(open('$OUT/ab_c$c.json')); [print('$c',k,v) for k,v in d['results'].items()]"
done
