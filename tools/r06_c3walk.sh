# round 6 lab: config 3's host walk (zero-copy path, one thread) per packet
# with the mbufs in cache (16 K packets) against DRAM (256 K)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r06c3walk}; mkdir -p $O
for np in 16384 262144 16384 262144; do
  UINET_CKSUM_TRACE_HOST=1 timeout -k 10 200 python -u tests/perf/host_cpu.py --work c3 --c3-packets $np --threads 1 --reps 7 --paths zero_copy > $O/h_$np.log 2> $O/h_$np.err || { tail -20 $O/h_$np.err; exit 1; }
  echo "n=$np $(grep 'zero-copy threads=1' $O/h_$np.err | tail -3 | sed 's/.*pieces=\([0-9]*\).*| walk \([0-9.]*\) .*/\1 \2/' | tr '\n' ' ') (pieces, walk ms)"
done
