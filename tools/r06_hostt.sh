# round 6 lab: temporal vs non-temporal packet loads on the host-resident
# paths (UINET_LAB_HOSTNT=1 = non-temporal), alternating processes: c2 span,
# c3 zero-copy and device walk, hooks device
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r06hostt}; mkdir -p $O
for r in 1 2 3; do for v in t nt; do
  E=""; [ $v = nt ] && E="UINET_LAB_HOSTNT=1"
  env $E timeout -k 10 300 python -u tests/perf/host_cpu.py --work c2,c3,hooks --threads 16 --reps 5 --paths span,zero_copy,dev_walk,dev_walk2 > $O/h.$v.$r.log 2>&1 || { tail -5 $O/h.$v.$r.log; exit 1; }
  echo "== $v $r"; python tools/host_cpu_table.py $O/h.$v.$r.log | grep -v "—  |" | grep engine | cut -d'|' -f2,3,4 | grep -v "| —"
done; done
