#!/usr/bin/env bash
# Full GPU tests, the small-packet (64-B) bench shape, the 3tx long-segment
# threshold, and the host-path scripts from their new place.
set -u
OUT=gpurun_out/${TAG:-r01v}; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1; rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --config 2s > $OUT/bench_c2s.log 2>&1 || exit $?
grep '^{' $OUT/bench_c2s.log
timeout -k 10 600 python bench.py --config 2s --api strided --cpu-baseline off > $OUT/bench_c2s_strided.log 2>&1 || exit $?
grep '^{' $OUT/bench_c2s_strided.log
timeout -k 10 300 python tools/ab.py --config 3tx --rounds 16 --variants chains_long=128 chains_long=64 chains_long=96 > $OUT/ab_long3tx.json 2> $OUT/ab_long3tx.err || exit $?
python3 -c "import json; d=json.load(open('$OUT/ab_long3tx.json')); [print(k,v) for k,v in d['results'].items()]"
timeout -k 10 300 python tests/perf/percall_latency.py > $OUT/percall.json 2> $OUT/percall.err || exit $?
head -3 $OUT/percall.json
