# round 6: cursor prefetch as the one-thread default: tests, host CPU table
# (c3, hooks, echo; 1 and 16 threads; 2 processes)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r06cursor2}; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_echo.py tests/test_in6.py tests/test_gpu_fuzz.py tests/test_offload.py tests/test_device_walk.py > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  timeout -k 10 300 python -u tests/perf/host_cpu.py --work c3,hooks,echo --threads 1,16 --reps 5 --paths zero_copy,staged > $O/h_$r.log 2>&1 || { tail -5 $O/h_$r.log; exit 1; }
  python3 -c "
import json
d=json.loads([l for l in open('$O/h_$r.log') if l.startswith('{\"threads')][-1])
print('$r', {k:(round(x['wall_ms'],2),round(x['cpu_us_per_1k_pkts'],1)) for k,x in d.items() if isinstance(x,dict) and 'wall_ms' in x})"
done
