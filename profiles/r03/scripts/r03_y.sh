#!/usr/bin/env bash
# Round 3: k_spans_lean<64> with pipelined rounds (one 9000-B packet per
# wave): parity, then config 5 (and 4 as a control) against k_spans_pp.
set -u
TAG=${TAG:-r03y}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
step() { local name=$1 secs=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  echo "   rc=$rc"; grep -v "^[EW]20\|amdgpu.ids" "$OUT/$name.log" | tail -n 1 | cut -c1-200
  case $rc in 0) ;; *) echo FATAL; exit $rc;; esac; }
step pytest_spans 900 python -u -m pytest tests/test_gpu_parity.py -x -q -k "spans or strided" --timeout 300 --timeout-method thread -p no:cacheprovider
for c in 5 4; do
  step ab_c$c 300 python3 tools/ab.py --config $c --rounds 8 --variants spans_pipe=1 spans_pipe=2 spans_pipe=0 blocks_per_cu=128 blocks_per_cu=512
done
echo "== done"
