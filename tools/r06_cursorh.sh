# round 6 lab: cursor prefetch for the hooks too (UINET_WALK_CURSOR_HOOKS=1),
# one thread, zero-copy and staged, alternating processes
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r06cursorh}; mkdir -p $O
timeout -k 10 300 env UINET_WALK_CURSOR_HOOKS=1 UINET_CKSUM_HOST_THREADS=1 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_offload.py tests/test_echo.py > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2 3; do for v in 0 1; do
  if [ $v = 1 ]; then export UINET_WALK_CURSOR_HOOKS=1; else unset UINET_WALK_CURSOR_HOOKS; fi
  timeout -k 10 300 python -u tests/perf/host_cpu.py --work hooks,echo --threads 1 --reps 7 --paths zero_copy,staged > $O/$v.$r.log 2>&1 || { tail -5 $O/$v.$r.log; exit 1; }
  python3 -c "
import json
d=json.loads([l for l in open('$O/$v.$r.log') if l.startswith('{\"threads')][-1])
print('hooks-cursor=$v $r', {k:(round(x['wall_ms'],2),round(x['cpu_us_per_1k_pkts'],1)) for k,x in d.items() if isinstance(x,dict) and 'wall_ms' in x and 'reference' not in k})"
done; done
