#!/usr/bin/env bash
# Packed (6-B) vs wide (12-B) chain descriptors: parity tests, then bench
# interleaved ABAB on the chain configs, then a FETCH_SIZE pass per packed config.
set -u
OUT=gpurun_out/${TAG:-abdesc}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 600 python -u -m pytest tests/test_chains32.py -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for rep in 1 2; do for d in wide packed; do for c in ${CONFIGS:-3 3tx 5tso}; do
  timeout -k 10 300 python bench.py --config $c --desc $d --cpu-baseline off > $OUT/b_${d}${rep}_c$c.log 2>&1 || { tail -5 $OUT/b_${d}${rep}_c$c.log; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('$OUT/b_${d}${rep}_c$c.log') if l.startswith('{')][-1]); print('$d$rep', '$c', d['roofline']['kernel_ms_mean'], d['roofline']['achieved'])"
done; done; done
for c in ${CONFIGS:-3 3tx 5tso}; do
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$OUT/pmc_c$c" -o run --output-format csv -- python3 bench.py --config $c --desc packed --steps 10 --warmup 2 --cpu-baseline off > $OUT/pmc_c$c.log 2>&1 || exit 1
  read B N <<<"$(python3 -c "import json; d=json.loads([l for l in open('$OUT/b_packed1_c$c.log') if l.startswith('{')][-1]); print(d['config']['algorithmic_bytes_per_gpu'], d['config']['packets_per_gpu'])")"
  python3 tools/pmc_summary.py "$OUT/pmc_c$c" --key "k_chains32:config$c:$N" --bytes "$B" --out $OUT/pmc_traffic.json > "$OUT/pmc_c$c.summary.json"
  grep -o '"traffic_over_algorithmic": [0-9.]*' "$OUT/pmc_c$c.summary.json" || true
done
echo done
