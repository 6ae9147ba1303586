#!/usr/bin/env bash
# Round 5: k_chains_wide variants on 5tso.  w1 = one segment at a time (54
# VGPRs, 8 waves); v3 = a short segment followed by a long one has the long
# one's first round issued before the short one is summed (92 VGPRs, 5 waves);
# v3w7 = v3 held to 7 waves (24 B scratch).  Each library runs tools/ab.py
# in-process (chains_wide 1 = tile kernel against 2 = wave per packet), 2
# alternating rounds; v3's parity tests first.
set -u
OUT=gpurun_out/${TAG:-r05wide2}; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
LIB=libuinet_amd/libuinet_cksum.so
cp $LIB profiles/r05/ab/head.so
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  echo "   rc=$rc"; grep -v "^[EW]20\|amdgpu.ids" "$OUT/$name.log" | tail -n 1 | cut -c1-300
  case $rc in 0) ;; *) echo FATAL; cp profiles/r05/ab/head.so $LIB; exit $rc;; esac; }
cp profiles/r05/ab/v3.so $LIB
step pytest_v3 300 python -u -m pytest tests/test_chains_wide.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider
for r in 1 2; do for v in w1 v3 v3w7; do
  cp profiles/r05/ab/$v.so $LIB
  step ab_${v}_$r 300 python3 tools/ab.py --config 5tso --rounds 8 --variants chains_wide=1 chains_wide=2 chains_wide=1,desc=1 chains_wide=2,desc=1
done; done
cp profiles/r05/ab/head.so $LIB
echo "== done"
