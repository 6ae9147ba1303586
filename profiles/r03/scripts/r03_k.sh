#!/usr/bin/env bash
# Round 3: k_spans_lean with the mask table computed per block (spans_pipe=3,
# lab) vs copied from a global image (1), against pp (2) and one-shot (0).
set -u
TAG=${TAG:-r03k}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
step() { local name=$1 secs=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  echo "   rc=$rc"; grep -v "^[EW]20\|amdgpu.ids" "$OUT/$name.log" | tail -n 2 | cut -c1-300
  case $rc in 0) ;; *) echo FATAL; exit $rc;; esac; }
step pytest_lean 600 env UINET_CKSUM_SPANS_PIPE=3 python -u -m pytest tests/test_gpu_parity.py -x -q -k "spans or strided" --timeout 300 --timeout-method thread -p no:cacheprovider
for c in 2 4 5; do
  step ab_c$c 300 python3 tools/ab.py --config $c --rounds 8 --variants spans_pipe=1 spans_pipe=3 spans_pipe=0 spans_pipe=2 spans_pipe=3,blocks_per_cu=512
done
step cold_p3 300 env UINET_CKSUM_SPANS_PIPE=3 python3 tools/cold_start.py --launches 300 --idle-s 1.5
step cold_p1 300 env UINET_CKSUM_SPANS_PIPE=1 python3 tools/cold_start.py --launches 300 --idle-s 1.5
echo "== done"
