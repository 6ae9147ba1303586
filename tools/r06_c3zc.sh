# round 6: config 3 host walk at one thread (zero-copy and staged), three
# processes, phase trace: is r06final4's 59 ms the code or the box?
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r06c3zc}; mkdir -p $O
for r in 1 2 3; do
  UINET_CKSUM_TRACE_HOST=1 timeout -k 10 200 python -u tests/perf/host_cpu.py --work c3 --threads 1 --reps 5 --paths zero_copy,staged > $O/h_$r.log 2> $O/h_$r.err || { tail -20 $O/h_$r.err; exit 1; }
  python3 -c "
import json,sys
d=json.loads([l for l in open('$O/h_$r.log') if l.startswith('{\"threads')][-1])
print({k:(v['wall_ms'],v['cpu_us_per_1k_pkts']) for k,v in d.items() if isinstance(v,dict) and 'wall_ms' in v})"
  grep 'zero-copy\|zero_copy' $O/h_$r.err | tail -1 | cut -c1-250
done
