#!/usr/bin/env bash
# SQ / TA counter sets for the span kernel (config 2) and the chain kernel
# (config 3), same passes, for a side-by-side reading.  One counter set per run.
set -u
TAG=${TAG:-r02e}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT" \
           "TA_BUSY_avr TA_FLAT_READ_WAVEFRONTS_sum GRBM_COUNT" ; do
  i=$((i+1))
  for c in 2 3; do
    timeout -s KILL 90 rocprofv3 --pmc $set --kernel-trace -d "$OUT/c$c/p$i" -o run --output-format csv -- python3 bench.py --config $c --steps 5 --warmup 1 --cpu-baseline off > "$OUT/c${c}_p$i.log" 2>&1
    rc=$?; echo "c$c set $i rc=$rc"; grep -iE "error|invalid" "$OUT/c${c}_p$i.log" | grep -v "^W20\|amdgpu.ids" | head -2
    case $rc in 0) ;; *) exit $rc;; esac
  done
done
for c in 2 3; do python3 tools/pmc_table.py "$OUT/c$c" > "$OUT/c$c/summary.txt"; cat "$OUT/c$c/summary.txt"; done
