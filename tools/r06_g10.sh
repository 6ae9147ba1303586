# round 6: temporal span loads on the host span path; span / parity / bench
# tests, smoke, host CPU (c2 span), then config 2 profiled again (the
# headline kernel's name gained its load-policy parameter)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r06m}; mkdir -p $O
t() { timeout -k 10 "$@"; }
t 900 python -u -m pytest tests/test_span_fast.py tests/test_spans32.py tests/test_gpu_parity.py tests/test_bench_gpu.py -x -q --timeout 300 --timeout-method thread -m gpu > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
t 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
t 400 python -u tests/perf/host_cpu.py --work c2 --threads 1,16 --reps 7 --paths span > $O/host_cpu.log 2>&1 || { tail -20 $O/host_cpu.log; exit 1; }
python tools/host_cpu_table.py $O/host_cpu.log | grep "engine, span"
TAG=$(basename $O)/prof CONFIGS="2" bash tools/prof_all.sh > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python -c "
import json
l=[x for x in open('$O/prof/bench_c2.log') if x.startswith('{')][-1]; d=json.loads(l)
print(d['value'], d['roofline']['frac'], d['roofline']['instance'])
print(json.dumps(d['host_resident_cpu']))"
