# round 6 lab: cursor prefetch at 16 threads, distance / gap sweep (lab build)
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r06cursor16}; mkdir -p $O
for r in 1 2 3; do for v in off 48_8 24_4 32_16; do
  unset UINET_WALK_CURSOR_ANY UINET_CUR_D UINET_CUR_G
  if [ $v != off ]; then export UINET_WALK_CURSOR_ANY=1 UINET_CUR_D=${v%_*} UINET_CUR_G=${v#*_}; fi
  timeout -k 10 300 python -u tests/perf/host_cpu.py --work c3 --threads 16 --reps 7 --paths zero_copy,staged > $O/$v.$r.log 2>&1 || { tail -5 $O/$v.$r.log; exit 1; }
  python3 -c "
import json
d=json.loads([l for l in open('$O/$v.$r.log') if l.startswith('{\"threads')][-1])
print('$v $r', {k:(round(x['wall_ms'],2),round(x['cpu_us_per_1k_pkts'],1)) for k,x in d.items() if isinstance(x,dict) and 'wall_ms' in x and 'reference' not in k})"
done; done
