#!/usr/bin/env bash
# Round 3: small packets aligned (2s) and 2 B off alignment (2su): k_spans_quad
# at U = 2 and U = 1 (spans_geo=65) against k_spans, span and strided APIs;
# lean at its new 512 blocks per CU against 128, pp and one-shot.
set -u
TAG=${TAG:-r03n}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
step() { local name=$1 secs=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  echo "   rc=$rc"; grep -v "^[EW]20\|amdgpu.ids" "$OUT/$name.log" | tail -n 1 | cut -c1-200
  case $rc in 0) ;; *) echo FATAL; exit $rc;; esac; }
step pytest_spans 900 python -u -m pytest tests/test_gpu_parity.py -x -q -k "spans or strided" --timeout 300 --timeout-method thread -p no:cacheprovider
for c in 2s 2su; do
  step ab_c$c 300 python3 tools/ab.py --config $c --rounds 6 --variants spans_pipe=0 spans_pipe=0,blocks_per_cu=64 spans_pipe=1 blocks_per_cu=256 spans_geo=65 spans_geo=65,blocks_per_cu=256
  step ab_c${c}_strided 300 python3 tools/ab.py --config $c --api strided --rounds 6 --variants spans_pipe=0 spans_pipe=1 blocks_per_cu=256 spans_geo=65 spans_geo=66
done
step ab_c2 300 python3 tools/ab.py --config 2 --rounds 6 --variants spans_pipe=1 blocks_per_cu=128 spans_pipe=2 spans_pipe=0
echo "== done"
