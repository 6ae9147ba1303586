# round 6: a long fuzz hunt on seeds not run before (device entry points
# incl. uinet_cksum_mbufs, host batches incl. the span path, hooks)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r06hunt}; mkdir -p $O
UINET_FUZZ_TRIALS=${HUNT:-60000} UINET_FUZZ_BASE=${HUNT_BASE:-2000000} timeout -k 10 1100 python -u -m pytest tests/test_gpu_fuzz.py -m gpu -x -q -s --timeout 1000 --timeout-method thread > $O/hunt.log 2>&1 || { tail -40 $O/hunt.log; exit 1; }
grep -E "trials, |passed|failed" $O/hunt.log | tail -8
