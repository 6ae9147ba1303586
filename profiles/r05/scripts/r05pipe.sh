#!/usr/bin/env bash
# Round 5: k_chains_wide's pipelined-rounds instantiation (knob chains_wide 3:
# the next round's loads issued before the current one is summed, 123 VGPRs,
# 4 waves) against the one-round kernel (2) and the tile kernel (1) on long
# shapes (tools/chains_cross.py --pipe) and 5tso; parity first.
set -u
OUT=gpurun_out/${TAG:-r05pipe}; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  echo "   rc=$rc"; grep -v "^[EW]20\|amdgpu.ids" "$OUT/$name.log" | tail -n 1 | cut -c1-300
  case $rc in 0) ;; *) echo FATAL; exit $rc;; esac; }
step pytest 300 env UINET_CKSUM_CHAINS_WIDE=3 UINET_TEST_CHAINS_WIDE=3 python -u -m pytest tests/test_gpu_parity.py tests/test_chains_wide.py -k "chains or wide" -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider
step cross 500 python3 tools/chains_cross.py --pipe
step ab_5tso 300 python3 tools/ab.py --config 5tso --rounds 8 --variants chains_wide=1 chains_wide=2 chains_wide=3
echo "== done"
