# round 6: hybrid head reading (every 4th group by the GPU) against host-only
# and GPU-only: span tests, host CPU c2 (span_gpu path: bytes + mbufs
# registered), 3 processes each, bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r06s}; mkdir -p $O
t() { timeout -k 10 "$@"; }
t 600 python -u -m pytest tests/test_span_fast.py -x -q --timeout 300 --timeout-method thread -m gpu > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2 3; do for v in 4 0 3 8; do
  UINET_LAB_GPU_EVERY=$v t 300 python -u tests/perf/host_cpu.py --work c2 --threads 1 --reps 7 --paths span_gpu > $O/h_${v}_${r}.log 2>&1 || { tail -20 $O/h_${v}_${r}.log; exit 1; }
  echo "every=$v r=$r $(python tools/host_cpu_table.py $O/h_${v}_${r}.log | grep 'span-gpu' | cut -d'|' -f4)"
done; done
TAG=$(basename $O)/b RUNS=1 bash tools/r06_bench3.sh
