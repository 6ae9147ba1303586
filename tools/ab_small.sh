#!/usr/bin/env bash
# Small packets (64 B): grid width (blocks per CU) for the span and strided kernels.
set -u
OUT=gpurun_out/${TAG:-r01z}; mkdir -p $OUT
for api in spans strided; do
  timeout -k 10 300 python tools/ab.py --config 2s --api $api --variants blocks_per_cu=256 blocks_per_cu=64 blocks_per_cu=16 blocks_per_cu=4096 > $OUT/ab_2s_$api.json 2> $OUT/ab_2s_$api.err || exit $?
  python3 -c "import json; d=json.load(open('$OUT/ab_2s_$api.json')); [print('$api',k,v) for k,v in d['results'].items()]"
done
