# round 6: span path with the common-packet run: span / device-walk / fuzz
# tests, then the host pass per packet (cached and streaming)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r06fp}; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_span_fast.py tests/test_device_walk.py tests/test_gpu_fuzz.py tests/test_gpu_parity.py tests/test_in6.py tests/test_echo.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
TAG=${TAG:-r06fp} bash tools/r06_pass.sh
