#!/usr/bin/env bash
# A/B two builds of the engine library (libuinet_amd/alt/libuinet_cksum_{A,B}.so)
# by swapping the in-tree .so between bench runs, interleaved ABAB.
set -u
OUT=gpurun_out/${TAG:-r01ac}; mkdir -p $OUT
cp libuinet_amd/libuinet_cksum.so $OUT/keep.so
for rep in 1 2; do for v in ${VARIANTS:-A B}; do
  cp libuinet_amd/alt/libuinet_cksum_$v.so libuinet_amd/libuinet_cksum.so
  for c in ${CONFIGS:-2 5 3 2s}; do
    timeout -k 10 300 python bench.py --config $c --api ${API:-spans} --cpu-baseline off > $OUT/b_${v}${rep}_c$c.log 2>&1 || { cp $OUT/keep.so libuinet_amd/libuinet_cksum.so; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('$OUT/b_${v}${rep}_c$c.log') if l.startswith('{')][-1]); print('$v$rep', '$c', d['roofline']['kernel_ms_mean'], d['roofline']['achieved'])"
  done
done; done
cp $OUT/keep.so libuinet_amd/libuinet_cksum.so
