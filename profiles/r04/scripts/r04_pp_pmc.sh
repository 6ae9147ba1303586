#!/usr/bin/env bash
# Round 4: HBM bytes (FETCH_SIZE) of config 3 under the shipped chain kernel
# and the two-batch ping-pong (tools/ab_so/{base,new}.so), one pass each.
set -u
TAG=${TAG:-r04ppm}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
LIB=libuinet_amd/libuinet_cksum.so
cp $LIB tools/ab_so/keep.so
for v in base new; do for c in 3 3tx; do
  cp tools/ab_so/$v.so $LIB
  timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$OUT/pmc_c${c}_$v" -o run --output-format csv -- python3 bench.py --config $c --steps 10 --warmup 2 --cpu-baseline off > "$OUT/pmc_c${c}_$v.log" 2>&1 || { cp tools/ab_so/keep.so $LIB; exit 1; }
  B=$(python3 -c "import json; d=json.loads([l for l in open('$OUT/pmc_c${c}_$v.log') if l.startswith('{')][-1]); print(d['config']['algorithmic_bytes_per_gpu'])")
  python3 tools/pmc_summary.py "$OUT/pmc_c${c}_$v" --bytes "$B" > "$OUT/pmc_c${c}_$v.summary.json"
  echo "$c $v $(python3 -c "import json; d=json.load(open('$OUT/pmc_c${c}_$v.summary.json')); print([(k, round(e.get('traffic_over_algorithmic',0),4)) for k,e in d.items()])")"
done; done
cp tools/ab_so/keep.so $LIB
