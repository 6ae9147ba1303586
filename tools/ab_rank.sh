set -u
# Historical A/B: chains_variant 2 (k_chains_flat) and 3/4 existed only in the builds of
# the commits that ran it; see profiles/r01/ab/*/NOTES.md for the results.
OUT=gpurun_out/${TAG:-r01g}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "chains or config3 or variants or 5tso or 3tx" -p no:cacheprovider > $OUT/pytest.log 2>&1; rc=$?; tail -5 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for c in 3 3tx 5tso; do
  timeout -k 10 300 python tools/ab.py --config $c --variants chains_variant=0 chains_variant=2 chains_variant=3 > $OUT/ab_c$c.json 2> $OUT/ab_c$c.err || exit $?
  python3 -c "import json; d=json.load(open('$OUT/ab_c$c.json')); [print('$c',k,v) for k,v in d['results'].items()]"
done
