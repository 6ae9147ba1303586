#!/usr/bin/env bash
# Round 3: k_spans_lean at wide grids (2 steps per wave and fewer) against
# k_spans_pp and the one-shot k_spans, warm (interleaved) and in the
# driver-shaped cold window (after the GPU test suite).
set -u
TAG=${TAG:-r03j}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
step() { local name=$1 secs=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  echo "   rc=$rc"; grep -v "^[EW]20\|amdgpu.ids" "$OUT/$name.log" | tail -n 2 | cut -c1-300
  case $rc in 0) ;; *) echo FATAL; exit $rc;; esac; }
for c in 2 4 5; do
  step ab_c$c 300 python3 tools/ab.py --config $c --rounds 6 --variants spans_pipe=2 spans_pipe=0 spans_pipe=1 spans_pipe=1,blocks_per_cu=256 spans_pipe=1,blocks_per_cu=512 spans_pipe=1,blocks_per_cu=1024 spans_pipe=1,blocks_per_cu=4096
done
step pytest_pre 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
step cold_p1_512 300 env UINET_CKSUM_SPANS_PIPE=1 UINET_CKSUM_BLOCKS_PER_CU=512 python3 tools/cold_start.py --launches 300 --idle-s 1.5
step cold_p1_128 300 env UINET_CKSUM_SPANS_PIPE=1 python3 tools/cold_start.py --launches 300 --idle-s 1.5
step cold_p0 300 env UINET_CKSUM_SPANS_PIPE=0 python3 tools/cold_start.py --launches 300 --idle-s 1.5
step cold_p1_1024 300 env UINET_CKSUM_SPANS_PIPE=1 UINET_CKSUM_BLOCKS_PER_CU=1024 python3 tools/cold_start.py --launches 300 --idle-s 1.5
echo "== done"
