# round 6 lab: temporal vs non-temporal packet loads in the span kernels
# (tools/ab_so/lab_t.so vs base.so), over registered host memory (config 2
# host batch, span path, one thread) and device-resident (config 2 bench),
# alternating processes
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r06labt}; mkdir -p $O
LIB=libuinet_amd/libuinet_cksum.so
cp $LIB tools/ab_so/keep.so
for r in 1 2 3; do for v in base lab_t; do
  cp tools/ab_so/$v.so $LIB
  timeout -k 10 200 python -u tests/perf/host_cpu.py --work c2 --threads 1 --reps 7 --paths span > $O/h.$v.$r.log 2>&1 || { cp tools/ab_so/keep.so $LIB; tail -5 $O/h.$v.$r.log; exit 1; }
  echo "host $v $r $(python tools/host_cpu_table.py $O/h.$v.$r.log | grep 'engine, span' | cut -d'|' -f4)"
  timeout -k 10 200 python3 bench.py --cpu-baseline off --host-offload off > $O/b.$v.$r.log 2>&1 || { cp tools/ab_so/keep.so $LIB; tail -5 $O/b.$v.$r.log; exit 1; }
  python3 -c "import json; l=[x for x in open('$O/b.$v.$r.log') if x.startswith('{')][-1]; j=json.loads(l); print('dev $v $r', j['roofline']['kernel_ms_mean'], j['roofline']['frac'])"
done; done
cp tools/ab_so/keep.so $LIB
