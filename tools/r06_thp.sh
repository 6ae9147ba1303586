# round 6 lab: span path host CPU with the mbuf pool and arena on 4-KiB vs
# transparent huge pages (UINET_MBUF_HUGEPAGES=1), config 2, one thread
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r06thp}; mkdir -p $O
cat /sys/kernel/mm/transparent_hugepage/enabled /sys/kernel/mm/transparent_hugepage/defrag 2>&1 | tee $O/thp.txt
for r in 1 2; do for v in 0 1; do
  UINET_MBUF_HUGEPAGES=$v timeout -k 10 200 python -u tests/perf/host_cpu.py --work c2 --threads 1 --reps 9 --paths span > $O/h_${v}_${r}.log 2>&1 || { tail -20 $O/h_${v}_${r}.log; exit 1; }
  echo "huge=$v r=$r $(python tools/host_cpu_table.py $O/h_${v}_${r}.log | grep 'engine, span' | cut -d'|' -f4)"
done; done
