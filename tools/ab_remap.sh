#!/usr/bin/env bash
# A/B of the XCD-banded block order on the span kernels, plus FETCH_SIZE per setting.
set -u
OUT=gpurun_out/${TAG:-abr}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
run() { local name=$1; shift; timeout -k 10 300 python tools/ab.py "$@" > $OUT/$name.json 2> $OUT/$name.err; local rc=$?; echo "$name rc=$rc"; python3 -c "import json,sys; d=json.load(open('$OUT/$name.json')); [print(' ',k,v) for k,v in d['results'].items()]" 2>/dev/null || tail -3 $OUT/$name.err; case $rc in 0) ;; *) exit $rc;; esac; }
run c2_remap --config 2 --rounds 10 --variants xcd_remap=0 xcd_remap=1
run c2s_remap --config 2 --api strided --rounds 10 --variants xcd_remap=0 xcd_remap=1
run c5_remap --config 5 --rounds 10 --variants xcd_remap=0 xcd_remap=1
for r in 0 1; do
  UINET_CKSUM_XCD_REMAP=$r timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$OUT/pmc_r$r" -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --cpu-baseline off > $OUT/pmc_r$r.log 2>&1 || exit $?
  python3 tools/pmc_summary.py "$OUT/pmc_r$r" --bytes 1572864000 | tee $OUT/pmc_r$r.json | grep -E "traffic_over|avg_ns"
done
