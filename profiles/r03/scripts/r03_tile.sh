#!/usr/bin/env bash
# Round 3: chain tiles of 64 packets (two bins per lane, the end of the
# tile's segment range by a scalar load) against 32, interleaved in one
# process (the tool checks the results equal).
set -u
TAG=${TAG:-r03s2g}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
step() { local name=$1 secs=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  echo "   rc=$rc"; grep -v "^[EW]20\|amdgpu.ids" "$OUT/$name.log" | tail -n 1 | cut -c1-300
  case $rc in 0) ;; *) echo FATAL; exit $rc;; esac; }
for c in 3tx 3 5tso; do
  step ab_c$c 300 python3 tools/ab.py --config $c --rounds 8 --variants chains_tile=32 chains_tile=64
done
echo "== done"
