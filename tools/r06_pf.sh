set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r06pf}; mkdir -p $O
for d in ${PFS:-48 64 96 128 192 48 64 96 128 192}; do
  UINET_CKSUM_SPAN_PF=$d timeout -k 10 200 python -u tests/perf/host_cpu.py --work c2 --threads 1 --reps 7 --paths span > $O/pf$d.log 2>&1 || { tail -20 $O/pf$d.log; exit 1; }
  echo "pf=$d"; python tools/host_cpu_table.py $O/pf$d.log | grep "engine, span"
done
