set -u
# Historical A/B: chains_variant 2 (k_chains_flat) and 3/4 existed only in the builds of
# the commits that ran it; see profiles/r01/ab/*/NOTES.md for the results.
OUT=gpurun_out/${TAG:-r01f}; mkdir -p $OUT
timeout -k 10 900 python -m pytest tests -m gpu -q -x -p no:cacheprovider -k "chains or config3 or spans or golden" > $OUT/pytest.log 2>&1; rc=$?; tail -3 $OUT/pytest.log
case $rc in 0|1) ;; *) exit $rc;; esac
for v in flat serial; do
  UINET_CKSUM_CHAINS=$v timeout -k 10 300 python bench.py --config 3 --steps 20 --warmup 3 --cpu-baseline off > $OUT/c3_$v.json 2>/dev/null || exit $?
  python3 -c "import json; d=json.load(open('$OUT/c3_$v.json')); r=d['roofline']; print('$v', d['value'], r['achieved'], r['frac'], r['kernel_ms_mean'])"
done
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --cpu-baseline off > $OUT/c2.json 2>/dev/null || exit $?
python3 -c "import json; d=json.load(open('$OUT/c2.json')); r=d['roofline']; print('c2', d['value'], r['achieved'], r['frac'], r['kernel_ms_mean'])"
