#!/usr/bin/env bash
# Round 4: k_chains_sweep (its own kernel, selected by UINET_CKSUM_F_ORDERED)
# against k_chains_pipe: chain GPU parity and smoke, interleaved A/B per chain
# config, SQ counters of both kernels on config 3.
set -u
TAG=${TAG:-r04d}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 600 python -u -m pytest tests/test_chains_sweep.py tests/test_chains32.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest_sweep.log 2>&1
rc=$?; tail -n 1 $OUT/pytest_sweep.log; [ $rc -eq 0 ] || { echo FATAL $rc; exit $rc; }
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?; tail -n 1 $OUT/smoke.log; [ $rc -eq 0 ] || { echo FATAL $rc; exit $rc; }
for c in 3 3tx 5tso; do
  timeout -k 10 300 python -u tools/ab.py --config $c --rounds 6 --variants ordered=0 ordered=1 ordered=0,desc=1 ordered=1,desc=1 > $OUT/ab_c$c.json 2> $OUT/ab_c$c.err
  rc=$?; python3 -c "import json; d=json.load(open('$OUT/ab_c$c.json')); [print('$c', k, v['median_ms']) for k, v in d['results'].items()]"; [ $rc -eq 0 ] || { echo FATAL $rc; tail $OUT/ab_c$c.err; exit $rc; }
done
for o in off on; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY -d "$OUT/sq_$o" -o run --output-format csv -- python3 bench.py --config 3 --ordered $o --steps 3 --warmup 1 --cpu-baseline off > $OUT/sq_$o.log 2>&1
  rc=$?; echo "sq ordered=$o rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python3 tools/insts_summary.py $OUT/sq_$o --kernel k_chains_ --bytes 727743980 > $OUT/sq_$o.json
  python3 -c "import json; d=json.load(open('$OUT/sq_$o.json')); print('  ', d['kernel'], {k: v['per_kib'] for k, v in d.items() if isinstance(v, dict)})"
done
echo "== done"
