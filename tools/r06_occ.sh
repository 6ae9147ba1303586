# round 6: k_mbufs variants against the shipped build, alternating bench
# processes, mbuf forms of 3 / 3tx / 5tso.  VARIANTS="base new:6 new2:4": a
# library in tools/ab_so/<name>.so and the blocks per CU it is launched at
# (new: -DUINET_MBUFS_WAVES=6; new2: kLongU 4 at 4 waves)
set -u
O=gpurun_out/${TAG:-r06occ}; mkdir -p $O
LIB=libuinet_amd/libuinet_cksum.so
cp $LIB tools/ab_so/keep.so
for r in 1 2 3; do for vv in ${VARIANTS:-base new:6 new2:4}; do for c in ${CONFIGS:-3 3tx 5tso}; do
  v=${vv%%:*}; bpc=${vv#*:}; [ "$bpc" = "$vv" ] && bpc=0
  cp tools/ab_so/$v.so $LIB
  UINET_CKSUM_BLOCKS_PER_CU=$bpc timeout -k 10 300 python3 bench.py --config $c --form mbufs --cpu-baseline off --host-offload off > $O/$c.$v.$r.log 2>&1 || { cp tools/ab_so/keep.so $LIB; tail -5 $O/$c.$v.$r.log; exit 1; }
  python3 -c "import json,sys; l=[x for x in open('$O/$c.$v.$r.log') if x.startswith('{')][-1]; j=json.loads(l); print('$c $v $r', j['roofline']['instance'], j['roofline']['kernel_ms_mean'], j['roofline']['frac'])"
done; done; done
cp tools/ab_so/keep.so $LIB
