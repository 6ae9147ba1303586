#!/usr/bin/env bash
# SQ counters (two passes of 8) and FETCH_SIZE for one bench shape per spec:
# SPECS="3:seglist 3:mbufs" TAG=... bash tools/r06_pmc.sh
set -u
OUT=gpurun_out/${TAG:-r06pmc}; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
SQ1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY"
SQ2="SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_FLAT SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_ACTIVE_INST_MISC"
for spec in ${SPECS:-3:seglist 3:mbufs}; do
  c=${spec%%:*}; f=${spec#*:}; t=c${c}_$f
  A="--config $c --form $f --steps 5 --warmup 2 --cpu-baseline off --host-offload off"
  i=0
  for set in "$SQ1" "$SQ2" "FETCH_SIZE"; do
    i=$((i+1))
    timeout -s KILL 180 rocprofv3 --pmc $set -d "$OUT/${t}_p$i" -o run --output-format csv -- python3 bench.py $A > "$OUT/${t}_p$i.log" 2>&1 || { echo "FAIL $t pass $i"; tail -5 "$OUT/${t}_p$i.log"; exit 1; }
  done
  python3 profiles/r05/scripts/pmc_by_kernel.py $(ls $OUT/${t}_p*/*counter_collection.csv $OUT/${t}_p*/*/*counter_collection.csv 2>/dev/null) > "$OUT/$t.txt" 2>&1
  echo "== $t"; grep -E "k_mbufs|k_chains|SQ_|FETCH" "$OUT/$t.txt" | head -60
done
