# round 6 lab: host walk prefetch depth 3 (base.so) vs 7 (new.so), zero-copy
# path, one thread: config 3 and the hooks, alternating processes
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r06walkab}; mkdir -p $O
LIB=libuinet_amd/libuinet_cksum.so
cp $LIB tools/ab_so/keep.so
for r in 1 2 3; do for v in base new; do
  cp tools/ab_so/$v.so $LIB
  timeout -k 10 300 python -u tests/perf/host_cpu.py --work c3,hooks,echo --threads ${THREADS:-1} --reps 5 --paths zero_copy,staged > $O/$v.$r.log 2>&1 || { cp tools/ab_so/keep.so $LIB; tail -5 $O/$v.$r.log; exit 1; }
  python3 -c "
import json
d=json.loads([l for l in open('$O/$v.$r.log') if l.startswith('{\"threads')][-1])
print('$v $r', {k.replace('/1t',''):(round(v['wall_ms'],2),round(v['cpu_us_per_1k_pkts'],1)) for k,v in d.items() if isinstance(v,dict) and 'wall_ms' in v and 'reference' not in k})"
done; done
cp tools/ab_so/keep.so $LIB
