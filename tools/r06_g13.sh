# round 6: span path with the heads read by the GPU (k_span_walk) when the
# mbufs are registered: span / device-walk / bench tests, smoke, host CPU
# (c2: span walk vs host-read span path, 3 processes each), bench twice
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r06q}; mkdir -p $O
t() { timeout -k 10 "$@"; }
t 900 python -u -m pytest tests/test_span_fast.py tests/test_device_walk.py tests/test_bench_gpu.py tests/test_echo.py tests/test_in6.py tests/test_multi.py -x -q --timeout 300 --timeout-method thread -m gpu > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
t 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for r in 1 2 3; do for v in 1 0; do
  UINET_LAB_SPANWALK=$v UINET_CKSUM_TRACE_HOST=1 t 300 python -u tests/perf/host_cpu.py --work c2 --threads 1 --reps 7 --paths span_gpu > $O/h_${v}_${r}.log 2> $O/h_${v}_${r}.err || { tail -20 $O/h_${v}_${r}.err; exit 1; }
  echo "spanwalk=$v r=$r $(python tools/host_cpu_table.py $O/h_${v}_${r}.log | grep "span-gpu\|span_gpu" | cut -d'|' -f4)"
done; done
grep "GPU-read" $O/h_1_1.err | tail -2
TAG=$(basename $O)/b bash tools/r06_bench3.sh
