#!/usr/bin/env bash
# Round 5: every config's bench + kernel trace + FETCH_SIZE pass on the final
# tree (tools/prof_all.sh), then the box's pure-read ceiling (tools/hbm_read).
# Two calls: SET=a (span configs), SET=b (chain and small-packet configs).
set -u
TAG=${TAG:-r05set${SET:-a}}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
if [ "${SET:-a}" = a ]; then
  CONFIGS="2 2+packed 2@strided 2rx 4 5 5tso 5tso+packed"
else
  CONFIGS="3 3+packed 3tx 3tx+packed 2s 2s+packed 2su 2su+packed 2su@strided"
fi
TAG=$TAG CONFIGS="$CONFIGS" bash tools/prof_all.sh || exit $?
echo "== hbm_read"
timeout -k 10 300 tools/hbm_read > "$OUT/hbm_read.log" 2>&1 || exit 1
tail -n 3 "$OUT/hbm_read.log"
echo "== done"
