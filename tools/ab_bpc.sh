#!/usr/bin/env bash
# Interleaved A/B of one engine env knob (KNOB, default UINET_CKSUM_BLOCKS_PER_CU)
# on one box: CONFIGS x BPCS x REPS bench lines, kernel mean from HIP events.
set -u
OUT=gpurun_out/${TAG:-abbpc}; mkdir -p $OUT
for rep in $(seq ${REPS:-3}); do for c in ${CONFIGS:-2}; do for b in ${BPCS:-256 4096}; do
  env ${KNOB:-UINET_CKSUM_BLOCKS_PER_CU}=$b timeout -k 10 120 python3 bench.py --config $c ${API:+--api $API} --cpu-baseline off \
    > $OUT/c${c}_b${b}_r$rep.log 2>&1 || exit 1
  grep '^{' $OUT/c${c}_b${b}_r$rep.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read())['roofline']; print('c$c bpc$b r$rep', r['kernel'], r['achieved'])"
done; done; done
