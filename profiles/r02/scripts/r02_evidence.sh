#!/usr/bin/env bash
# Round-2 evidence pass:
#  * cold start: per-launch event times + amdsmi clock samples (tools/cold_start.py),
#    and a rocprofv3 kernel trace of exactly the driver's bench command;
#  * SQ counter sets for the current chain kernel on config 3.
set -u
TAG=${TAG:-r02a}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  echo "   rc=$rc"; grep -v "^[EW]20" "$OUT/$name.log" | tail -n 3 | cut -c1-400
  case $rc in 0) ;; *) echo FATAL; exit $rc;; esac; }
step cold_start 300 python3 -u tools/cold_start.py
step driver_bench 300 python3 bench.py --gpus 1 --steps 20 --warmup 5
step driver_trace 300 rocprofv3 --kernel-trace --stats -d "$OUT/driver_trace" -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --cpu-baseline off
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT"; do
  i=$((i+1))
  step sq_c3_p$i 120 rocprofv3 --pmc $set --kernel-trace -d "$OUT/sq_c3/p$i" -o run --output-format csv -- python3 bench.py --config 3 --steps 5 --warmup 1 --cpu-baseline off
done
python3 tools/pmc_table.py "$OUT/sq_c3" > "$OUT/sq_c3/summary.txt"; cat "$OUT/sq_c3/summary.txt"
echo "== done"
