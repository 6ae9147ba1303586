#!/usr/bin/env bash
# Round 4: the chain kernel's address sweep (chains_sweep 2 / 4) against the
# chunk-list kernel (chains_sweep 0): chain GPU parity, then one interleaved
# A/B per chain config in one process (tools/ab.py).
set -u
TAG=${TAG:-r04a}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 600 python -u -m pytest tests/test_chains_sweep.py tests/test_host_desc.py tests/test_offload.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest_sweep.log 2>&1
rc=$?; tail -n 3 $OUT/pytest_sweep.log; [ $rc -eq 0 ] || { echo FATAL $rc; exit $rc; }
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?; tail -n 1 $OUT/smoke.log; [ $rc -eq 0 ] || { echo FATAL $rc; exit $rc; }
for c in 3 3tx 5tso; do
  timeout -k 10 300 python -u tools/ab.py --config $c --rounds 6 --variants chains_sweep=0 chains_sweep=2 chains_sweep=3 chains_sweep=4 \
     chains_sweep=0,desc=1 chains_sweep=2,desc=1 chains_sweep=3,desc=1 chains_sweep=4,desc=1 > $OUT/ab_c$c.json 2> $OUT/ab_c$c.err
  rc=$?; cat $OUT/ab_c$c.json; [ $rc -eq 0 ] || { echo FATAL $rc; tail $OUT/ab_c$c.err; exit $rc; }
done
echo "== done"
