#!/usr/bin/env bash
set -u
OUT=gpurun_out/${TAG:-r01u}; mkdir -p $OUT
for c in 3 3tx 5tso; do
  timeout -k 10 300 python tools/ab.py --config $c --variants xcd_remap=0 xcd_remap=1 > $OUT/ab_c$c.json 2> $OUT/ab_c$c.err || exit $?
  python3 -c "import json; d=json.load(open('$OUT/ab_c$c.json')); [print('$c',k,v) for k,v in d['results'].items()]"
done
