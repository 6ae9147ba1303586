# round 6 lab: span path head-mbuf prefetch locality hint (UINET_LAB_PF 0 =
# prefetchnta .. 3 = prefetcht0), config 2, one thread, alternating
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r06pfab}; mkdir -p $O
for r in 1 2 3; do for v in 3 0 1 2; do
  UINET_LAB_PF=$v timeout -k 10 200 python -u tests/perf/host_cpu.py --work c2 --threads 1 --reps 9 --paths span > $O/p_${v}_${r}.log 2>&1 || { tail -20 $O/p_${v}_${r}.log; exit 1; }
  echo "pf=$v r=$r $(python tools/host_cpu_table.py $O/p_${v}_${r}.log | grep 'engine, span' | cut -d'|' -f4)"
done; done
