#!/usr/bin/env bash
# Historical A/B: chains_variant 2 (k_chains_flat) and 3/4 existed only in the builds of
# the commits that ran it; see profiles/r01/ab/*/NOTES.md for the results.
# Chains: temporal vs non-temporal loads (variants 3 / 4), time and HBM bytes.
set -u
OUT=gpurun_out/${TAG:-r01i}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for c in 3 3tx 5tso; do
  timeout -k 10 300 python tools/ab.py --config $c --variants chains_variant=3 chains_variant=4 chains_variant=2 > $OUT/ab_c$c.json 2> $OUT/ab_c$c.err || exit $?
  python3 -c "import json; d=json.load(open('$OUT/ab_c$c.json')); [print('$c',k,v) for k,v in d['results'].items()]"
done
for v in 2 3 4; do for c in 3 3tx; do
  UINET_CKSUM_CHAINS=$v timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $OUT/pmc_v${v}_c$c -o run --output-format csv -- python3 bench.py --config $c --steps 10 --warmup 2 --cpu-baseline off > $OUT/pmc_v${v}_c$c.log 2>&1 || exit $?
  python3 tools/pmc_summary.py $OUT/pmc_v${v}_c$c > $OUT/pmc_v${v}_c$c.json; python3 -c "
import json; d=json.load(open('$OUT/pmc_v${v}_c$c.json')); print('v$v c$c', {k: (round(x.get('hbm_read_bytes_per_launch',0)/1e6,1), x.get('dispatches')) for k,x in d.items() if 'chains' in k})"
done; done
