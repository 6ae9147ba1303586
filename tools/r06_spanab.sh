# round 6 lab: span path group size and wait granularity (env knobs of a lab
# build), config 2 host batch, one thread, alternating
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r06sab}; mkdir -p $O
for r in 1 2; do for v in "32 65536" "128 65536" "32 262144" "32 16384" "128 262144"; do
  set -- $v
  UINET_WAIT_DIV=$1 UINET_SPAN_G=$2 timeout -k 10 200 python -u tests/perf/host_cpu.py --work c2 --threads 1 --reps 9 --paths span > $O/s_$1_$2_$r.log 2>&1 || { tail -20 $O/s_$1_$2_$r.log; exit 1; }
  echo "div=$1 G=$2 r=$r $(python tools/host_cpu_table.py $O/s_$1_$2_$r.log | grep 'engine, span')"
done; done
