set -u
OUT=gpurun_out/${TAG:-r01l}; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "host or golden or pcap or zero_copy or percall or skip" > $OUT/pytest.log 2>&1; rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tests/perf/percall_latency.py > $OUT/percall.json 2>$OUT/percall.err || exit $?
cat $OUT/percall.json
[ -n "${TRACE:-}" ] && export UINET_CKSUM_TRACE_HOST=1
timeout -k 10 600 python tests/perf/host_path.py > $OUT/host_path.log 2>&1 || exit $?
tail -30 $OUT/host_path.log
