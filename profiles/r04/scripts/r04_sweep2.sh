#!/usr/bin/env bash
# Round 4, sweep v2 (early window loads from the raw descriptors, monotone +
# no-hole rounds only): GPU parity, interleaved A/B against the chunk list, and SQ counters of the
# chunk list (chains_sweep 0) vs the sweep (2, 4) on config 3.
set -u
TAG=${TAG:-r04b}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 600 python -u -m pytest tests/test_chains_sweep.py tests/test_chains32.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest_sweep.log 2>&1
rc=$?; tail -n 1 $OUT/pytest_sweep.log; [ $rc -eq 0 ] || { echo FATAL $rc; exit $rc; }
for c in 3 3tx; do
  timeout -k 10 300 python -u tools/ab.py --config $c --rounds 6 --variants chains_sweep=0 chains_sweep=4 chains_sweep=5 chains_sweep=6 \
     chains_sweep=0,desc=1 chains_sweep=5,desc=1 chains_sweep=6,desc=1 > $OUT/ab_c$c.json 2> $OUT/ab_c$c.err
  rc=$?; python3 -c "import json; d=json.load(open('$OUT/ab_c$c.json')); [print('$c', k, v['median_ms']) for k, v in d['results'].items()]"; [ $rc -eq 0 ] || { echo FATAL $rc; tail $OUT/ab_c$c.err; exit $rc; }
done
for sw in 0 5 6; do
  UINET_CKSUM_CHAINS_SWEEP=$sw timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY -d "$OUT/sq_sw$sw" -o run --output-format csv -- python3 bench.py --config 3 --steps 3 --warmup 1 --cpu-baseline off > $OUT/sq_sw$sw.log 2>&1
  rc=$?; echo "sq sweep=$sw rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python3 tools/insts_summary.py $OUT/sq_sw$sw --kernel k_chains_pipe --bytes 727743980 > $OUT/sq_sw$sw.json
  python3 -c "import json; d=json.load(open('$OUT/sq_sw$sw.json')); print('  ', {k: v['per_kib'] for k, v in d.items() if isinstance(v, dict)})"
done
echo "== done"
