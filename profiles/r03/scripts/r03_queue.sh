#!/usr/bin/env bash
# Round 3 (lab): persistent chain waves with the next tile's range prefetched (chains_queue = 1) --
# parity, then interleaved A/B against the default on configs 3, 3tx.
set -u
TAG=${TAG:-r03s2s}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
step() { local name=$1 secs=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  echo "   rc=$rc"; grep -v "^[EW]20\|amdgpu.ids" "$OUT/$name.log" | tail -n 1 | cut -c1-300
  case $rc in 0) ;; *) echo FATAL; exit $rc;; esac; }
step pytest_queue 300 python -u -m pytest tests/test_chains_queue.py -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider
for c in 3 3tx; do
  step ab_c$c 300 python3 tools/ab.py --config $c --rounds 8 --variants chains_queue=0 chains_queue=1 chains_queue=1,blocks_per_cu=12 chains_queue=1,blocks_per_cu=24
done
echo "== done"
