#!/usr/bin/env bash
# A/B of several builds of the engine library in separate bench processes,
# alternating (tools/ab_so/<variant>.so copied over the in-tree .so).
# Usage: VARIANTS="base w7 w8" CONFIGS="3 3tx" ROUNDS=3 TAG=... bash tools/ab_lib_multi.sh
set -u
TAG=${TAG:-r03multi}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
LIB=libuinet_amd/libuinet_cksum.so
cp $LIB tools/ab_so/keep.so
for r in $(seq 1 ${ROUNDS:-3}); do for v in ${VARIANTS:-base new}; do for c in ${CONFIGS:-3}; do
  cp tools/ab_so/$v.so $LIB
  timeout -k 10 300 python3 bench.py --config $c ${ARGS:-} --cpu-baseline off > $OUT/$c.$v.$r.log 2>&1 || { cp tools/ab_so/keep.so $LIB; exit 1; }
  python3 -c "import json,sys; l=[x for x in open('$OUT/$c.$v.$r.log') if x.startswith('{')][-1]; j=json.loads(l); print('$c $v $r', j['roofline']['kernel_ms_mean'], j['roofline']['frac'])"
done; done; done
cp tools/ab_so/keep.so $LIB
