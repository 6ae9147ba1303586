# round 6: span path first (packed window, prefetch 128): tests, smoke,
# host CPU table for c2 / c5 at 1 and 16 threads, default bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r06k}; mkdir -p $O
t() { timeout -k 10 "$@"; }
t 900 python -u -m pytest tests/test_span_fast.py tests/test_device_walk.py tests/test_bench_gpu.py tests/test_in6.py tests/test_multi.py tests/test_offload.py tests/test_echo.py -x -q --timeout 200 --timeout-method thread -m gpu > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
t 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
t 500 python -u tests/perf/host_cpu.py --work c2 --threads 1,16 --reps 5 --paths span,dev_walk2 > $O/host_cpu.log 2>&1 || { tail -20 $O/host_cpu.log; exit 1; }
python tools/host_cpu_table.py $O/host_cpu.log | grep -v "—  |"
t 300 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench.json'));print(d['value'],d['roofline']['frac']);print(json.dumps(d['host_resident_cpu']))"
