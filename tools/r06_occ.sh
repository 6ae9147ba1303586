# round 6: k_mbufs at 6 waves per SIMD (tools/ab_so/new.so, built with
# -DUINET_MBUFS_WAVES=6, launched at 6 blocks per CU) against the shipped 5
# (base.so), alternating bench processes, mbuf forms of 3 / 3tx / 5tso
set -u
O=gpurun_out/${TAG:-r06occ}; mkdir -p $O
LIB=libuinet_amd/libuinet_cksum.so
cp $LIB tools/ab_so/keep.so
for r in 1 2 3; do for v in base new; do for c in ${CONFIGS:-3 3tx 5tso}; do
  cp tools/ab_so/$v.so $LIB
  E=""; [ $v = new ] && E="UINET_CKSUM_BLOCKS_PER_CU=${NEWBPC:-6}"
  env $E timeout -k 10 300 python3 bench.py --config $c --form mbufs --cpu-baseline off --host-offload off > $O/$c.$v.$r.log 2>&1 || { cp tools/ab_so/keep.so $LIB; tail -5 $O/$c.$v.$r.log; exit 1; }
  python3 -c "import json,sys; l=[x for x in open('$O/$c.$v.$r.log') if x.startswith('{')][-1]; j=json.loads(l); print('$c $v $r', j['roofline']['instance'], j['roofline']['kernel_ms_mean'], j['roofline']['frac'])"
done; done; done
cp tools/ab_so/keep.so $LIB
