#!/usr/bin/env bash
# Round 5: the tile kernel (k_chains_pipe) with the XCD-banded tile order
# (knob xcd_remap 1) against plain block order (0), in one process
# (tools/ab.py, 3 x 8 rounds) on configs 3 and 3tx, both descriptor forms;
# FETCH_SIZE of config 3 under both; chain parity tests first.
set -u
OUT=gpurun_out/${TAG:-r05tilex}; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  echo "   rc=$rc"; grep -v "^[EW]20\|amdgpu.ids" "$OUT/$name.log" | tail -n 1 | cut -c1-300
  case $rc in 0) ;; *) echo FATAL; exit $rc;; esac; }
step pytest 400 python -u -m pytest tests/test_gpu_parity.py tests/test_chains32.py -k "chains" -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
for r in 1 2 3; do for c in 3 3tx; do
  step ab_${c}_$r 300 python3 tools/ab.py --config $c --rounds 8 --variants xcd_remap=0 xcd_remap=1 xcd_remap=0,desc=1 xcd_remap=1,desc=1
done; done
step pmc_remap1 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$OUT/pmc_remap1" -o run --output-format csv -- python3 bench.py --config 3 --steps 10 --warmup 2 --cpu-baseline off --host-offload off
export UINET_CKSUM_XCD_REMAP=0
step pmc_remap0 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$OUT/pmc_remap0" -o run --output-format csv -- python3 bench.py --config 3 --steps 10 --warmup 2 --cpu-baseline off --host-offload off
echo "== done"
