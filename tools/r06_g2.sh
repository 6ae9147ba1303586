# round 6: k_mbufs with the LDS job ring (longest first) -- tests, config-3
# bench in both forms at the default warmup, the host walk A/B on config 3
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r06b}; mkdir -p $O
t() { timeout -k 10 "$@"; }
t 400 python -u -m pytest tests/test_mbufs.py tests/test_device_walk.py -x -q --timeout 120 --timeout-method thread -m gpu > $O/test_mbufs.log 2>&1 || { tail -40 $O/test_mbufs.log; exit 1; }
tail -1 $O/test_mbufs.log
for c in 3 3tx 5tso; do for f in seglist mbufs; do
t 200 python -u bench.py --config $c --form $f --cpu-baseline off > $O/b${c}_$f.json 2> $O/b${c}_$f.err || { tail -20 $O/b${c}_$f.err; exit 1; }
python -c "import json;d=json.load(open('$O/b${c}_$f.json'));r=d['roofline'];lf=r.get('layout_floor',{});print('$c $f',d['value'],r['kernel_ms_mean'],r['frac'],lf.get('frac'),lf.get('over_algorithmic'))"
done; done
t 300 python -u tests/perf/host_cpu.py --work c3 --threads 16 --reps 5 --paths dev_walk,dev_walk2 > $O/host_cpu.log 2>&1 || { tail -20 $O/host_cpu.log; exit 1; }
python tools/host_cpu_table.py $O/host_cpu.log | grep -v "—"
