#!/usr/bin/env bash
# Round 3: k_spans_quad U = 2 with slot 1 loaded only when a span of the step
# needs it: small-packet parity, then 2s / 2su A/B.
set -u
TAG=${TAG:-r03p}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
step() { local name=$1 secs=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  echo "   rc=$rc"; grep -v "^[EW]20\|amdgpu.ids" "$OUT/$name.log" | tail -n 1 | cut -c1-200
  case $rc in 0) ;; *) echo FATAL; exit $rc;; esac; }
step pytest_spans 900 python -u -m pytest tests/test_gpu_parity.py -x -q -k "spans or strided" --timeout 300 --timeout-method thread -p no:cacheprovider
for c in 2s 2su; do
  step ab_c$c 300 python3 tools/ab.py --config $c --rounds 6 --variants spans_pipe=1 blocks_per_cu=256 spans_geo=65 spans_pipe=0 spans_pipe=0,blocks_per_cu=64
  step ab_c${c}_strided 300 python3 tools/ab.py --config $c --api strided --rounds 6 --variants spans_pipe=1 blocks_per_cu=256 spans_geo=66 spans_pipe=0
done
echo "== done"
