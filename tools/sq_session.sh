set -u
OUT=gpurun_out/r01q; mkdir -p $OUT
UINET_CKSUM_HOST_THREADS=16 timeout -k 10 600 python tests/perf/host_path.py > $OUT/host_path_t16.log 2>&1 || exit $?
tail -1 $OUT/host_path_t16.log
bash tools/pmc_sets.sh r01q/sq_c2 --config 2 || exit $?
python3 tools/pmc_table.py gpurun_out/r01q/sq_c2 > gpurun_out/r01q/sq_c2/summary.txt
bash tools/pmc_sets.sh r01q/sq_c3 --config 3 || exit $?
python3 tools/pmc_table.py gpurun_out/r01q/sq_c3 > gpurun_out/r01q/sq_c3/summary.txt
cat gpurun_out/r01q/sq_c2/summary.txt gpurun_out/r01q/sq_c3/summary.txt
