#!/usr/bin/env bash
# Grid-size sweep of the config-2 bench (kernel-only numbers from the JSON line).
set -u
OUT=gpurun_out/${1:-sweep}; mkdir -p "$OUT"
for bpc in ${BPCS:-4 8 16 32 64 512}; do
  for api in ${APIS:-spans strided}; do
    UINET_CKSUM_BLOCKS_PER_CU=$bpc timeout -k 10 300 python bench.py --steps 30 --warmup 5 --api $api --cpu-baseline off ${EXTRA:-} > "$OUT/b_${api}_${bpc}.json" 2>/dev/null
    rc=$?; if [[ $rc -ne 0 ]]; then echo "rc=$rc at $bpc $api"; exit $rc; fi
    python3 -c "import json,sys; d=json.load(open('$OUT/b_${api}_${bpc}.json')); r=d['roofline']; print('$api bpc=$bpc', d['value'], 'GiB/s', r['achieved'], 'GB/s', r['frac'], r['kernel_ms_mean'], r['kernel_ms_min'])"
  done
done
