# round 6, first GPU pass: the HBM mbuf kernel (tests, smoke, bench) and the
# fused device walk behind the host-mbuf batch API and the hooks
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r06a}; mkdir -p $O
t() { timeout -k 10 "$@"; }
t 300 python -u -m pytest tests/test_mbufs.py -x -v --timeout 120 --timeout-method thread -m gpu > $O/test_mbufs.log 2>&1 || { tail -40 $O/test_mbufs.log; exit 1; }
tail -2 $O/test_mbufs.log
t 400 python -u -m pytest tests/test_device_walk.py tests/test_offload.py -x -q --timeout 120 --timeout-method thread -m gpu > $O/test_walk.log 2>&1 || { tail -40 $O/test_walk.log; exit 1; }
tail -2 $O/test_walk.log
t 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -30 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for f in seglist mbufs; do
t 200 python -u bench.py --config 3 --form $f --steps 20 --warmup 20 --cpu-baseline off > $O/b3_$f.json 2> $O/b3_$f.err || { tail -20 $O/b3_$f.err; exit 1; }
python -c "import json;d=json.load(open('$O/b3_$f.json'));r=d['roofline'];print('$f',d['value'],r['kernel_ms_mean'],r['frac'],r.get('layout_floor'))"
done
t 400 python -u tests/perf/host_cpu.py --work c2,c3,hooks --threads 16 --reps 5 --paths dev_walk,dev_walk2 > $O/host_cpu.log 2>&1 || { tail -20 $O/host_cpu.log; exit 1; }
python tools/host_cpu_table.py $O/host_cpu.log
