#!/usr/bin/env bash
# Span-kernel geometry / grid A/B in one process per API (tools/ab.py).
set -u
TAG=${TAG:-r02c}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 python3 tools/ab.py --config 2 --api spans --rounds 8 --launches 20 --variants \
  "spans_geo=0,blocks_per_cu=0" "spans_geo=262,blocks_per_cu=0" "spans_geo=262,blocks_per_cu=128" \
  "spans_geo=262,blocks_per_cu=512" "spans_geo=0,blocks_per_cu=512" "spans_geo=1026,blocks_per_cu=0" \
  > "$OUT/ab_spans.json" 2>&1 || exit $?
timeout -k 10 300 python3 tools/ab.py --config 2 --api strided --rounds 8 --launches 20 --variants \
  "spans_geo=0,blocks_per_cu=0" "spans_geo=262,blocks_per_cu=0" "spans_geo=0,blocks_per_cu=256" \
  > "$OUT/ab_strided.json" 2>&1 || exit $?
cat "$OUT/ab_spans.json" "$OUT/ab_strided.json" | grep -v "^\[W"
