set -u
OUT=gpurun_out/r01s; mkdir -p $OUT
for n in 2 4; do
UINET_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus $n --steps 20 --warmup 20 > $OUT/bench_gloo_$n.log 2>&1 || exit $?
grep '^{' $OUT/bench_gloo_$n.log
done
