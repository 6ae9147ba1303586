set -u
OUT=gpurun_out/r01k; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1; rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tests/perf/percall_latency.py > $OUT/percall.json 2>$OUT/percall.err || exit $?
cat $OUT/percall.json
timeout -k 10 300 python tests/perf/offload_rate.py > $OUT/offload.log 2>&1 || exit $?
tail -5 $OUT/offload.log
