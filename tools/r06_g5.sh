# round 6: seg_hint-selected load policy, span path with wide descriptors
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r06h}; mkdir -p $O
t() { timeout -k 10 "$@"; }
t 600 python -u -m pytest tests/test_span_fast.py tests/test_mbufs.py tests/test_device_walk.py tests/test_in6.py tests/test_multi.py tests/test_offload.py -x -q --timeout 120 --timeout-method thread -m gpu > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
t 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -30 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for c in 3 3tx 5tso; do
t 200 python -u bench.py --config $c --form mbufs --cpu-baseline off > $O/b${c}_mbufs.json 2> $O/b${c}_mbufs.err || { tail -20 $O/b${c}_mbufs.err; exit 1; }
python -c "import json;d=json.load(open('$O/b${c}_mbufs.json'));r=d['roofline'];lf=r.get('layout_floor',{});print('$c mbufs',d['value'],r['kernel_ms_mean'],r['frac'],r['instance'],lf.get('frac'))"
done
t 300 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench.json'));print(d['value'],d['roofline']['frac']);print(json.dumps(d['host_resident_cpu']));c=d['cpu_baseline'];print({k:c[k] for k in ('value','one_thread_gibs','all_cores_gibs','host_read_ceiling_gibs','fastest_pass_gibs','within_read_ceiling')})"
