# round 6: span path with DMA copies and a lower-bound sleep: span tests, host
# CPU (c2, 3 processes), the driver's bench command twice
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r06p}; mkdir -p $O
t() { timeout -k 10 "$@"; }
t 600 python -u -m pytest tests/test_span_fast.py tests/test_bench_gpu.py -x -q --timeout 300 --timeout-method thread -m gpu > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2 3; do
t 300 python -u tests/perf/host_cpu.py --work c2 --threads 1 --reps 9 --paths span,dev_walk2 > $O/host_cpu$r.log 2>&1 || { tail -20 $O/host_cpu$r.log; exit 1; }
python tools/host_cpu_table.py $O/host_cpu$r.log | grep "engine, span\|dev-walk2" | cut -d'|' -f3,4
done
TAG=$(basename $O)/b bash tools/r06_bench3.sh
