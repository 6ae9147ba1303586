#!/usr/bin/env bash
# Round 3: the chain kernel's grid width, tile and long-segment threshold
# re-measured with the fixed A/B tool (round 2's choices were made while
# variants leaked knobs), configs 3, 3tx, 5tso.
set -u
TAG=${TAG:-r03w}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
step() { local name=$1 secs=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  echo "   rc=$rc"; grep -v "^[EW]20\|amdgpu.ids" "$OUT/$name.log" | tail -n 1 | cut -c1-200
  case $rc in 0) ;; *) echo FATAL; exit $rc;; esac; }
for c in 3 3tx 5tso; do
  step ab_c$c 300 python3 tools/ab.py --config $c --rounds 8 --variants chains_pass=2 blocks_per_cu=16 blocks_per_cu=32 blocks_per_cu=128 blocks_per_cu=256 chains_tile=8 chains_tile=32 chains_long=64 chains_long=256 chains_long=0
done
echo "== done"
