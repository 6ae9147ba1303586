# round 6: the driver's bench command three times (cpu_baseline read ceiling
# with 20 read passes per setting, one-thread-per-L3 placement), one line each
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r06b3}; mkdir -p $O
for r in ${RUNS:-1 2 3}; do
  timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench$r.json 2> $O/bench$r.err || { tail -20 $O/bench$r.err; exit 1; }
  python -c "
import json;d=json.load(open('$O/bench$r.json'));c=d['cpu_baseline'];h=d['host_resident_cpu']
print($r, d['value'], d['roofline']['frac'], d['roofline']['traffic'], c['value'], c['value_from'], c['one_thread_gibs'], c['all_cores_gibs'], c['fastest_pass_gibs'], c['host_read_ceiling_gibs'], c['within_read_ceiling'], h['frac_of_link'], h['host_cpu_us_per_1k_pkts'], h['host_cpu_us_per_1k_pkts_calls'], h['bytes_only']['host_cpu_us_per_1k_pkts_calls'])
"
done
