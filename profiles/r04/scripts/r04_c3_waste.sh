#!/usr/bin/env bash
# Round 4: where config 3's HBM bytes above the layout floor come from.
# FETCH_SIZE and time of the chain kernel with 2 / 4 passes per batch (batch
# boundaries every 2 / 4 KiB of chunk list) and tiles of 32 / 8 packets.
set -u
TAG=${TAG:-r04w}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for v in "2 32" "4 32" "2 8"; do set -- $v; P=$1; T=$2; t=p${P}_t${T}
  UINET_CKSUM_CHAINS_PASS=$P UINET_CKSUM_CHAINS_TILE=$T timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$OUT/pmc_$t" -o run --output-format csv -- python3 bench.py --config 3 --steps 10 --warmup 2 --cpu-baseline off > "$OUT/pmc_$t.log" 2>&1 || exit 1
  python3 tools/pmc_summary.py "$OUT/pmc_$t" --bytes 727743980 > "$OUT/pmc_$t.summary.json"
  UINET_CKSUM_CHAINS_PASS=$P UINET_CKSUM_CHAINS_TILE=$T timeout -k 10 120 python3 bench.py --config 3 --cpu-baseline off > "$OUT/bench_$t.log" 2>&1 || exit 1
  echo "$t $(python3 -c "
import json; d=json.load(open('$OUT/pmc_$t.summary.json')); b=json.loads([l for l in open('$OUT/bench_$t.log') if l.startswith('{')][-1])
print([(k, round(e.get('traffic_over_algorithmic',0),4)) for k,e in d.items()], b['roofline']['kernel_ms_mean'], b['roofline']['frac'])")"
done
