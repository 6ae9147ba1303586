#!/usr/bin/env bash
# Round 3: k_spans_lean grid width (blocks per CU) against k_spans_pp,
# interleaved, configs 2 / 4 / 5.
set -u
TAG=${TAG:-r03i}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
step() { local name=$1 secs=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  echo "   rc=$rc"; grep -v "^[EW]20\|amdgpu.ids" "$OUT/$name.log" | tail -n 2 | cut -c1-300
  case $rc in 0) ;; *) echo FATAL; exit $rc;; esac; }
for c in 2 4 5; do
  step ab_c$c 300 python3 tools/ab.py --config $c --rounds 6 --variants spans_pipe=2 spans_pipe=1 spans_pipe=1,blocks_per_cu=8 spans_pipe=1,blocks_per_cu=16 spans_pipe=1,blocks_per_cu=32 spans_pipe=1,blocks_per_cu=64 spans_pipe=1,blocks_per_cu=256 spans_pipe=1,xcd_remap=0
done
echo "== done"
