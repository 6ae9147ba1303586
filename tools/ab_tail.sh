#!/usr/bin/env bash
# Pipelined chains: share of packets folded in small tiles at the end.
set -u
OUT=gpurun_out/${TAG:-r01p}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "chains or config3 or variants" > $OUT/pytest.log 2>&1; rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for c in 3 3tx; do
  timeout -k 10 300 python tools/ab.py --config $c --variants chains_tail=0 chains_tail=5 chains_tail=10 chains_tail=20 chains_tail=35 chains_tail=0,chains_tile=16 chains_tail=10,chains_tile=16 > $OUT/ab_c$c.json 2> $OUT/ab_c$c.err || exit $?
  python3 -c "import json; d=json.load(open('$OUT/ab_c$c.json')); [print('$c',k,v) for k,v in d['results'].items()]"
done
