#!/usr/bin/env bash
# Round 5: k_chains_wide with the XCD-banded packet order (knob xcd_remap, 1 =
# default) against plain block order, in one process (tools/ab.py, 4 x 8
# rounds), 5tso wide and packed; FETCH_SIZE of both orders.
set -u
OUT=gpurun_out/${TAG:-r05wide8}; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  echo "   rc=$rc"; grep -v "^[EW]20\|amdgpu.ids" "$OUT/$name.log" | tail -n 1 | cut -c1-300
  case $rc in 0) ;; *) echo FATAL; exit $rc;; esac; }
step pytest 300 python -u -m pytest tests/test_chains_wide.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider
for r in 1 2 3 4; do
  step ab_$r 300 python3 tools/ab.py --config 5tso --rounds 8 --variants chains_wide=1 chains_wide=2,xcd_remap=0 chains_wide=2,xcd_remap=1 chains_wide=2,xcd_remap=0,desc=1 chains_wide=2,xcd_remap=1,desc=1
done
step pmc_remap1 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$OUT/pmc_remap1" -o run --output-format csv -- python3 bench.py --config 5tso --steps 10 --warmup 2 --cpu-baseline off --host-offload off
export UINET_CKSUM_XCD_REMAP=0
step pmc_remap0 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$OUT/pmc_remap0" -o run --output-format csv -- python3 bench.py --config 5tso --steps 10 --warmup 2 --cpu-baseline off --host-offload off
echo "== done"
