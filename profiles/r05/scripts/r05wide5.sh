#!/usr/bin/env bash
# Round 5: k_chains_wide v3 (packed lengths by vector load) against v3s (every
# descriptor read scalar), same box, 3 alternating rounds of tools/ab.py on
# 5tso (tile kernel = chains_wide 1 in each).
set -u
OUT=gpurun_out/${TAG:-r05wide5}; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
LIB=libuinet_amd/libuinet_cksum.so
cp $LIB profiles/r05/ab/head.so
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  echo "   rc=$rc"; grep -v "^[EW]20\|amdgpu.ids" "$OUT/$name.log" | tail -n 1 | cut -c1-300
  case $rc in 0) ;; *) echo FATAL; cp profiles/r05/ab/head.so $LIB; exit $rc;; esac; }
for r in 1 2 3; do for v in v3 v3s; do
  cp profiles/r05/ab/$v.so $LIB
  step ab_${v}_$r 300 python3 tools/ab.py --config 5tso --rounds 8 --variants chains_wide=1 chains_wide=2 chains_wide=1,desc=1 chains_wide=2,desc=1
done; done
cp profiles/r05/ab/head.so $LIB
echo "== done"
