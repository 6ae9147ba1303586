#!/usr/bin/env bash
# Round 5: k_chains_wide variants on 5tso.  v3 = a short segment followed by a
# long one has the long one's first round issued before the short one is
# summed (92 VGPRs, 5 waves); v4 = the same with each round's segment
# descriptors read by one vector load per lane and a scan (108 VGPRs, 4
# waves); v4w6 = v4 held to 6 waves (52 B scratch); v4u6 = v4 with 6 chunks
# per lane per round (78 VGPRs, 6 waves).  Each library runs tools/ab.py
# in-process (chains_wide 1 = tile kernel against 2 = wave per packet), 2
# alternating rounds; v3's parity tests first.
set -u
OUT=gpurun_out/${TAG:-r05wide3}; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
LIB=libuinet_amd/libuinet_cksum.so
cp $LIB profiles/r05/ab/head.so
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  echo "   rc=$rc"; grep -v "^[EW]20\|amdgpu.ids" "$OUT/$name.log" | tail -n 1 | cut -c1-300
  case $rc in 0) ;; *) echo FATAL; cp profiles/r05/ab/head.so $LIB; exit $rc;; esac; }
cp profiles/r05/ab/v4.so $LIB
step pytest_v4 300 python -u -m pytest tests/test_chains_wide.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider
for r in 1 2; do for v in v3 v4 v4w6 v4u6; do
  cp profiles/r05/ab/$v.so $LIB
  step ab_${v}_$r 300 python3 tools/ab.py --config 5tso --rounds 8 --variants chains_wide=1 chains_wide=2 chains_wide=1,desc=1 chains_wide=2,desc=1
done; done
cp profiles/r05/ab/head.so $LIB
echo "== done"
