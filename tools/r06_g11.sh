# round 6: dense span groups copied to HBM by DMA: span tests, smoke, host
# CPU (c2), the driver's bench command twice
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r06n}; mkdir -p $O
t() { timeout -k 10 "$@"; }
t 900 python -u -m pytest tests/test_span_fast.py tests/test_device_walk.py tests/test_bench_gpu.py tests/test_echo.py -x -q --timeout 300 --timeout-method thread -m gpu > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
t 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
t 400 python -u tests/perf/host_cpu.py --work c2 --threads 1,16 --reps 7 --paths span > $O/host_cpu.log 2>&1 || { tail -20 $O/host_cpu.log; exit 1; }
python tools/host_cpu_table.py $O/host_cpu.log | grep "engine, span"
TAG=$(basename $O)/b bash tools/r06_bench3.sh
