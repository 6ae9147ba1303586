# round 6 lab: the span path's host pass per packet, cached (64 K packets,
# 16 MB of mbufs) against streaming (1 M packets, 256 MB), one thread
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r06pass}; mkdir -p $O
for np in 65536 1048576 65536 1048576; do
  UINET_CKSUM_TRACE_HOST=1 timeout -k 10 200 python -u tests/perf/host_cpu.py --work c2 --c2-packets $np --threads 1 --reps 9 --paths span > $O/h_$np.log 2> $O/h_$np.err || { tail -20 $O/h_$np.err; exit 1; }
  echo "n=$np $(grep 'uinet_cksum spans' $O/h_$np.err | tail -3 | sed 's/.*| pass \([0-9]*\) us.*/\1/' | tr '\n' ' ') us pass"
done
