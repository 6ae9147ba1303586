# round 6: span path phase times (UINET_CKSUM_TRACE_HOST), config 2, one thread
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r06tr}; mkdir -p $O
UINET_CKSUM_TRACE_HOST=1 timeout -k 10 200 python -u tests/perf/host_cpu.py --work c2 --threads 1 --reps 5 --paths span > $O/host_cpu.log 2> $O/trace.err || { tail -20 $O/trace.err; exit 1; }
python tools/host_cpu_table.py $O/host_cpu.log | grep 'engine, span' | cut -d'|' -f3,4
grep "uinet_cksum spans" $O/trace.err | tail -6
