#!/usr/bin/env bash
# SQ counter passes for one bench config. Usage: pmc_sets.sh TAG "bench args"
set -u
TAG=$1; shift; ARGS="$*"
OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_LDS" \
           "FETCH_SIZE TA_BUSY_avr TA_FLAT_READ_WAVEFRONTS_sum"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --kernel-trace -d $OUT/p$i -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --cpu-baseline off $ARGS > $OUT/p$i.log 2>&1
  rc=$?; echo "set $i rc=$rc"; grep -iE "error|invalid|not found" $OUT/p$i.log | grep -v "^W20" | head -3
  case $rc in 124|134|137|139) exit $rc;; esac
done
