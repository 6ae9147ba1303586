#!/usr/bin/env bash
# Round 4: the chain kernel's block size (threads per block: 256 shipped, 128,
# 64): a block exits only when all its waves are done, so waves whose tiles
# finish early leave their slots idle.  Chain parity tests on each build, then
# configs 3 / 3tx / 5tso alternating processes, 3 rounds.
# tools/ab_so/b{256,128,64}.so are built beforehand (UINET_CHAINS_BLOCK).
set -u
TAG=${TAG:-r04cb}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
LIB=libuinet_amd/libuinet_cksum.so
cp $LIB tools/ab_so/keep.so
for v in b128 b64; do
  cp tools/ab_so/$v.so $LIB
  timeout -k 10 300 python3 -u -m pytest tests/test_chains32.py tests/test_chains_dense.py tests/test_variants.py tests/test_gpu_fuzz.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_$v.log 2>&1 || { tail -20 $OUT/pytest_$v.log; cp tools/ab_so/keep.so $LIB; exit 1; }
  echo "$v $(tail -1 $OUT/pytest_$v.log)"
done
for r in 1 2 3; do for v in b256 b128 b64; do for c in 3 3tx 5tso; do
  cp tools/ab_so/$v.so $LIB
  timeout -k 10 300 python3 bench.py --config $c --cpu-baseline off > $OUT/$c.$v.$r.log 2>&1 || { cp tools/ab_so/keep.so $LIB; exit 1; }
  python3 -c "import json; l=[x for x in open('$OUT/$c.$v.$r.log') if x.startswith('{')][-1]; j=json.loads(l); print('$c $v $r', j['roofline']['kernel_ms_mean'], j['roofline']['frac'])"
done; done; done
cp tools/ab_so/keep.so $LIB
