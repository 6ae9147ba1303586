# round 6: span path (one host thread, descriptors staged to HBM): tests,
# host CPU table for c2 / hooks, default bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r06i}; mkdir -p $O
t() { timeout -k 10 "$@"; }
t 600 python -u -m pytest tests/test_span_fast.py tests/test_bench_gpu.py -x -q --timeout 200 --timeout-method thread -m gpu > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
t 400 python -u tests/perf/host_cpu.py --work c2,hooks --threads 1,16 --reps 5 --paths zero_copy,span,dev_walk > $O/host_cpu.log 2>&1 || { tail -20 $O/host_cpu.log; exit 1; }
python tools/host_cpu_table.py $O/host_cpu.log | grep -v "—  |"
t 300 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench.json'));print(d['value'],d['roofline']['frac']);print(json.dumps(d['host_resident_cpu']));c=d['cpu_baseline'];print({k:c[k] for k in ('value','one_thread_gibs','all_cores_gibs','host_read_ceiling_gibs','fastest_pass_gibs','within_read_ceiling')});print(c['runs_minmax_gibs']);print(c['host_read_max_gibs'])"
