# round 6: host line before the reference passes; bench test, default bench;
# then the k_mbufs 6-wave A/B (tools/r06_occ.sh)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r06l}; mkdir -p $O
t() { timeout -k 10 "$@"; }
t 600 python -u -m pytest tests/test_bench_gpu.py -x -q --timeout 300 --timeout-method thread -m gpu > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
t 300 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench.json'));print(d['value'],d['roofline']['frac']);print(json.dumps(d['host_resident_cpu']))"
TAG=$(basename $O)/occ bash tools/r06_occ.sh
