# round 6: A/B of the mbuf kernel's load policy (tools/ab_so), then the
# single-mbuf span path: tests, smoke, default bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r06g}; mkdir -p $O
t() { timeout -k 10 "$@"; }
TAG=$(basename $O)/ab CONFIGS="3 3tx 5tso" ARGS="--form mbufs" bash tools/ab_lib_swap.sh || exit 1
t 600 python -u -m pytest tests/test_span_fast.py tests/test_device_walk.py tests/test_mbufs.py tests/test_in6.py tests/test_multi.py tests/test_offload.py -x -q --timeout 120 --timeout-method thread -m gpu > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
t 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -30 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
t 300 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench.json'));print(d['value'],d['roofline']['frac']);print(json.dumps(d['host_resident_cpu']));c=d['cpu_baseline'];print({k:c[k] for k in ('value','one_thread_gibs','all_cores_gibs','host_read_ceiling_gibs','fastest_pass_gibs','within_read_ceiling')})"
