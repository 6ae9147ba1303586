# round 6: span path copies on their own stream into two stage slots:
# span / fuzz / bench tests, config 2 host wall and CPU (3 processes), bench
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r06cs}; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_span_fast.py tests/test_gpu_fuzz.py tests/test_bench_gpu.py tests/test_in6.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2 3; do
  UINET_CKSUM_TRACE_HOST=1 timeout -k 10 200 python -u tests/perf/host_cpu.py --work c2 --threads 1 --reps 9 --paths span > $O/h_$r.log 2> $O/h_$r.err || { tail -20 $O/h_$r.err; exit 1; }
  python3 -c "
import json
d=json.loads([l for l in open('$O/h_$r.log') if l.startswith('{\"threads')][-1])
v=d['c2/span/1t']; print('c2 span', v['wall_ms'], v['cpu_us_per_1k_pkts'], v['bit_identical'])"
  grep 'uinet_cksum spans' $O/h_$r.err | tail -1
done
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
python3 -c "
import json
d=json.loads([l for l in open('$O/bench.log') if l.startswith('{\"metric')][-1])
h=d['host_resident_cpu']; print('bench', d['roofline']['frac'], h['frac_of_link'], h['wall_ms'], h['host_cpu_us_per_1k_pkts'], h['bit_identical'], h['bytes_only']['frac_of_link'], h['bytes_only']['host_cpu_us_per_1k_pkts'])"
