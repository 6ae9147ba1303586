# round 6 lab: k_mbufs grid (blocks per CU cap) on the mbuf forms of 5tso / 3tx
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r06mbgrid}; mkdir -p $O
for c in 5tso 3tx; do for b in 5 3 4 8 16; do
  UINET_CKSUM_BLOCKS_PER_CU=$b timeout -k 10 200 python3 bench.py --config $c --form mbufs --cpu-baseline off --host-offload off > $O/$c.$b.log 2>&1 || { tail -5 $O/$c.$b.log; exit 1; }
  python3 -c "import json; l=[x for x in open('$O/$c.$b.log') if x.startswith('{')][-1]; j=json.loads(l); print('$c bpc=$b', j['roofline']['kernel_ms_mean'], j['roofline']['frac'])"
done; done
