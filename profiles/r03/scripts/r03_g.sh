#!/usr/bin/env bash
# Round 3: k_spans_quad with super-step descriptors -- parity, then
# interleaved A/B against k_spans<4, *> on config 2s (span and strided APIs).
set -u
TAG=${TAG:-r03h}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
step() { local name=$1 secs=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  echo "   rc=$rc"; grep -v "^[EW]20\|amdgpu.ids" "$OUT/$name.log" | tail -n 2 | cut -c1-300
  case $rc in 0) ;; *) echo FATAL; exit $rc;; esac; }
step pytest_spans 900 python -u -m pytest tests/test_gpu_parity.py -x -q -k "spans or strided" --timeout 300 --timeout-method thread -p no:cacheprovider
step ab_2s 300 python3 tools/ab.py --config 2s --rounds 6 --variants spans_pipe=1 spans_pipe=0 spans_pipe=1,blocks_per_cu=8 spans_pipe=1,blocks_per_cu=64 spans_pipe=1,spans_geo=65
step ab_2s_strided 300 python3 tools/ab.py --config 2s --api strided --rounds 6 --variants spans_pipe=1 spans_pipe=0 spans_pipe=1,blocks_per_cu=8 spans_pipe=1,blocks_per_cu=64
echo "== done"
