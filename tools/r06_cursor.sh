# round 6 lab: host walk cursor prefetch (UINET_WALK_CURSOR=1) against the
# default, zero-copy and staged paths, 1 and 16 threads, alternating processes
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r06cursor}; mkdir -p $O
timeout -k 10 300 env UINET_WALK_CURSOR=1 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_echo.py tests/test_in6.py > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2 3; do for v in 0 1; do
  if [ $v = 1 ]; then export UINET_WALK_CURSOR=1; else unset UINET_WALK_CURSOR; fi
  timeout -k 10 300 python -u tests/perf/host_cpu.py --work c3,echo --threads 1,16 --reps 5 --paths zero_copy,staged > $O/$v.$r.log 2>&1 || { tail -5 $O/$v.$r.log; exit 1; }
  python3 -c "
import json
d=json.loads([l for l in open('$O/$v.$r.log') if l.startswith('{\"threads')][-1])
print('cursor=$v $r', {k:(round(x['wall_ms'],2),round(x['cpu_us_per_1k_pkts'],1)) for k,x in d.items() if isinstance(x,dict) and 'wall_ms' in x and 'reference' not in k})"
done; done
