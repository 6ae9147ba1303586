# round 6 lab: span path DMA variants (UINET_LAB_DMA 0 = in place, 1 = H2D from
# the host pointer, 2 = D2D from the device alias, 3 = default kind from the
# alias) and group size, config 2 host batch, one thread, alternating
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r06dma}; mkdir -p $O
for r in 1 2; do for v in "0 65536" "1 65536" "2 65536" "3 65536" "1 262144" "2 262144"; do
  set -- $v
  UINET_LAB_DMA=$1 UINET_LAB_SPAN_G=$2 timeout -k 10 200 python -u tests/perf/host_cpu.py --work c2 --threads 1 --reps 9 --paths span > $O/d_$1_$2_$r.log 2>&1 || { tail -20 $O/d_$1_$2_$r.log; exit 1; }
  echo "dma=$1 G=$2 r=$r $(python tools/host_cpu_table.py $O/d_$1_$2_$r.log | grep 'engine, span' | cut -d'|' -f4)"
done; done
