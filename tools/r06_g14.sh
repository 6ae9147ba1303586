# round 6: span_fast 2 (heads read by the GPU) as an option: span tests under
# both forms, ABI, fuzz (host trials draw span_fast 0-2), smoke, bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r06r}; mkdir -p $O
t() { timeout -k 10 "$@"; }
t 900 python -u -m pytest tests/test_span_fast.py tests/test_device_walk.py tests/test_bench_gpu.py tests/test_gpu_fuzz.py -x -q --timeout 300 --timeout-method thread -m gpu > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
t 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
TAG=$(basename $O)/b RUNS=1 bash tools/r06_bench3.sh
