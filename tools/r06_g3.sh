# round 6: k_mbufs with global (not flat) loads -- parity, bench, SQ counters
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r06c}; mkdir -p $O
t() { timeout -k 10 "$@"; }
t 300 python -u -m pytest tests/test_mbufs.py -x -q --timeout 120 --timeout-method thread -m gpu > $O/test_mbufs.log 2>&1 || { tail -40 $O/test_mbufs.log; exit 1; }
tail -1 $O/test_mbufs.log
for c in ${CONFIGS:-3 3tx}; do for f in mbufs; do
t 200 python -u bench.py --config $c --form $f --cpu-baseline off > $O/b${c}_$f.json 2> $O/b${c}_$f.err || { tail -20 $O/b${c}_$f.err; exit 1; }
python -c "import json;d=json.load(open('$O/b${c}_$f.json'));r=d['roofline'];lf=r.get('layout_floor',{});print('$c $f',d['value'],r['kernel_ms_mean'],r['frac'],lf.get('frac'),lf.get('over_algorithmic'))"
done; done
[ -n "${PMC:-}" ] && TAG=${TAG:-r06c}/pmc SPECS="3:mbufs" bash tools/r06_pmc.sh
true
