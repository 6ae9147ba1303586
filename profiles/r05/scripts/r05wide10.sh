#!/usr/bin/env bash
# Round 5: k_chains_wide picked for mean segments of 4-9 KiB (the launcher changed).  (1) chain / wide / host-batch / hook
# GPU tests and the device + host fuzz on new seeds; (2) the chain configs'
# bench + kernel trace + FETCH_SIZE pass (tools/prof_all.sh: cksum_chains.hip
# changed, so their traffic entries are re-measured) and the read ceiling.
set -u
TAG=${TAG:-r05wide10}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  echo "   rc=$rc"; grep -v "^[EW]20\|amdgpu.ids" "$OUT/$name.log" | tail -n 1 | cut -c1-300
  case $rc in 0) ;; *) echo FATAL; exit $rc;; esac; }
step pytest 600 python -u -m pytest tests/test_chains_wide.py tests/test_gpu_parity.py tests/test_chains32.py tests/test_chains_dense.py tests/test_device_walk.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
step fuzz 600 env UINET_FUZZ_TRIALS=9000 UINET_FUZZ_BASE=600000 python -u -m pytest tests/test_gpu_fuzz.py -k "device or host" -m gpu -x -q -s --timeout 500 --timeout-method thread -p no:cacheprovider
TAG=$TAG CONFIGS="5tso 5tso+packed 3 3+packed 3tx 3tx+packed" bash tools/prof_all.sh || exit $?
echo "== hbm_read"
timeout -k 10 300 tools/hbm_read > "$OUT/hbm_read.log" 2>&1 || exit 1
tail -n 3 "$OUT/hbm_read.log"
timeout -k 10 240 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || exit 1
tail -n 1 "$OUT/smoke.log"
echo "== done"
