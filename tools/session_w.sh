#!/usr/bin/env bash
set -u
OUT=gpurun_out/${TAG:-r01w}; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "spans or strided or golden or config2 or jumbo or hint" > $OUT/pytest.log 2>&1; rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --config 2s --cpu-baseline off > $OUT/bench_c2s.log 2>&1 || exit $?
grep '^{' $OUT/bench_c2s.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['packets_per_s']/1e9, 'Gpps', d['roofline'])"
timeout -k 10 600 python bench.py --config 2s --api strided --cpu-baseline off > $OUT/bench_c2s_strided.log 2>&1 || exit $?
grep '^{' $OUT/bench_c2s_strided.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['packets_per_s']/1e9, 'Gpps', d['roofline'])"
timeout -k 10 600 python bench.py --cpu-baseline off > $OUT/bench_c2.log 2>&1 || exit $?
grep '^{' $OUT/bench_c2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline'])"
