#!/usr/bin/env bash
# The driver's exact bench command, one fresh process per run, alternating
# engine settings by environment: bash tools/drv_ab.sh TAG [REPS]
# (each process builds its workload and measures the 5-warmup / 20-step
# window right after it, as the round-end driver does).
set -u
OUT=gpurun_out/$1; REPS=${2:-4}; mkdir -p $OUT
VARIANTS=${VARIANTS:-"base pipe"}
for rep in $(seq 1 $REPS); do
  for v in $VARIANTS; do
    case $v in
      base) E="UINET_CKSUM_SPANS_PIPE=0";;
      pipe) E="UINET_CKSUM_SPANS_PIPE=1";;
      pipe64x2) E="UINET_CKSUM_SPANS_PIPE=1 UINET_CKSUM_SPANS_GEO=1026";;
      wave) E="UINET_CKSUM_SPANS_PIPE=2";;
      lean) E="UINET_CKSUM_SPANS_PIPE=3";;
      bpc128) E="UINET_CKSUM_SPANS_PIPE=0 UINET_CKSUM_BLOCKS_PER_CU=128";;
      *) echo "unknown variant $v"; exit 2;;
    esac
    env $E timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 --cpu-baseline off > $OUT/${v}_$rep.log 2>&1 || exit 1
    python3 -c "import json; d=json.loads([l for l in open('$OUT/${v}_$rep.log') if l.startswith('{')][-1]); print('$v', $rep, d['ms_per_step'], d['roofline']['frac'])"
  done
done
