#!/usr/bin/env bash
# Round 4: chain kernel with the batch's last pass loaded temporal (its last
# line is read again by the next batch) against the shipped all-nt loads:
# chain parity tests on the new build, alternating bench processes, and the
# new build's FETCH_SIZE on configs 3 and 3tx.  tools/ab_so/{base,new}.so.
set -u
TAG=${TAG:-r04tl}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
LIB=libuinet_amd/libuinet_cksum.so
TESTS="tests/test_chains32.py tests/test_chains_dense.py tests/test_variants.py" CONFIGS="3 3tx 5tso" TAG=$TAG bash profiles/r04/scripts/r04_c5.sh || exit 1
cp $LIB tools/ab_so/keep.so; cp tools/ab_so/new.so $LIB
for c in 3 3tx; do
  timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$OUT/pmc_c${c}_new" -o run --output-format csv -- python3 bench.py --config $c --steps 10 --warmup 2 --cpu-baseline off > "$OUT/pmc_c${c}_new.log" 2>&1 || { cp tools/ab_so/keep.so $LIB; exit 1; }
  B=$(python3 -c "import json; d=json.loads([l for l in open('$OUT/pmc_c${c}_new.log') if l.startswith('{')][-1]); print(d['config']['algorithmic_bytes_per_gpu'])")
  python3 tools/pmc_summary.py "$OUT/pmc_c${c}_new" --bytes "$B" > "$OUT/pmc_c${c}_new.summary.json"
  echo "pmc $c new $(python3 -c "import json; d=json.load(open('$OUT/pmc_c${c}_new.summary.json')); print([(k, round(e.get('traffic_over_algorithmic',0),4)) for k,e in d.items()])")"
done
cp tools/ab_so/keep.so $LIB
