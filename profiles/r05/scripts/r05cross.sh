#!/usr/bin/env bash
# Round 5: where k_chains_wide beats the tile kernel (tools/chains_cross.py:
# 1, 2, 4 segments of 256 B - 4 KB per packet) and 5tso (tools/ab.py), for
# v3t (the committed kernel: the next descriptor read ahead only for a short
# segment followed by a long one) and v5 (every next descriptor read ahead);
# v5's parity tests first.
set -u
OUT=gpurun_out/${TAG:-r05cross2}; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
LIB=libuinet_amd/libuinet_cksum.so
cp $LIB profiles/r05/ab/head.so
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  echo "   rc=$rc"; grep -v "^[EW]20\|amdgpu.ids" "$OUT/$name.log" | tail -n 1 | cut -c1-300
  case $rc in 0) ;; *) echo FATAL; cp profiles/r05/ab/head.so $LIB; exit $rc;; esac; }
cp profiles/r05/ab/v5.so $LIB
step pytest_v5 300 python -u -m pytest tests/test_chains_wide.py tests/test_gpu_parity.py -k "chains or wide" -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider
for v in v3t v5; do
  cp profiles/r05/ab/$v.so $LIB
  step cross_$v 400 python3 tools/chains_cross.py
  step ab_$v 300 python3 tools/ab.py --config 5tso --rounds 8 --variants chains_wide=1 chains_wide=2 chains_wide=1,desc=1 chains_wide=2,desc=1
done
cp profiles/r05/ab/head.so $LIB
echo "== done"
