# round 6: the whole GPU suite, smoke, then a fuzz hunt on seeds not run before
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r06full}; mkdir -p $O
t() { timeout -k 10 "$@"; }
t 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
t 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
UINET_FUZZ_TRIALS=${HUNT:-6000} UINET_FUZZ_BASE=${HUNT_BASE:-600000} t 1000 python -u -m pytest tests/test_gpu_fuzz.py -m gpu -x -q -s --timeout 900 --timeout-method thread > $O/hunt.log 2>&1 || { tail -40 $O/hunt.log; exit 1; }
grep -E "trials|passed|failed" $O/hunt.log | tail -8
