#!/usr/bin/env bash
# Round 4: SQ counters of config 3 under the shipped chain kernel and the
# two-batch ping-pong (tools/ab_so/{base,new}.so), one pass each.
set -u
TAG=${TAG:-r04ppm}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
LIB=libuinet_amd/libuinet_cksum.so
cp $LIB tools/ab_so/keep.so
for v in base new; do
  cp tools/ab_so/$v.so $LIB
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY -d "$OUT/sq_c3_$v" -o run --output-format csv -- python3 bench.py --config 3 --steps 3 --warmup 1 --cpu-baseline off > "$OUT/sq_c3_$v.log" 2>&1 || { cp tools/ab_so/keep.so $LIB; exit 1; }
  python3 tools/insts_summary.py "$OUT/sq_c3_$v" --kernel k_chains_pipe --bytes 727743980 > "$OUT/sq_c3_$v.summary.json"
  echo "$v $(cat $OUT/sq_c3_$v.summary.json | tr -d '\n ' | cut -c1-600)"
done
cp tools/ab_so/keep.so $LIB
