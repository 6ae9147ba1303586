#!/usr/bin/env bash
# Round 5: (1) the split-header hook tests and the offload fuzz with header
# splits, plus the span parity suite, on the tree; (2) k_spans_quad<2> taking
# slot 1 from the next quad when packets lie back to back (quad_nb.so = the
# tree) against loading it in every quad (quad_all.so), 3 alternating rounds
# of 2su (span API, wide and packed descriptors) and 2s.  The tree keeps the
# committed build (head.so) until the variant is kept.
set -u
OUT=gpurun_out/${TAG:-r05za}; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
LIB=libuinet_amd/libuinet_cksum.so
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  echo "   rc=$rc"; grep -v "^[EW]20\|amdgpu.ids" "$OUT/$name.log" | tail -n 1 | cut -c1-200
  case $rc in 0) ;; *) echo FATAL; cp profiles/r05/ab/head.so $LIB; exit $rc;; esac; }
cp profiles/r05/ab/quad_nb.so $LIB
step pytest 500 python -u -m pytest tests/test_device_walk.py tests/test_offload.py tests/test_gpu_parity.py tests/test_spans32.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
step fuzz 400 env UINET_FUZZ_TRIALS=2000 python -u -m pytest tests/test_gpu_fuzz.py -m gpu -x -q -s --timeout 380 --timeout-method thread -p no:cacheprovider
for r in 1 2 3; do for v in quad_nb quad_all; do
  cp profiles/r05/ab/$v.so $LIB
  step b2su_${v}_$r 120 python3 bench.py --config 2su --steps 50 --warmup 20 --cpu-baseline off --host-offload off
  step b2sup_${v}_$r 120 python3 bench.py --config 2su --desc packed --steps 50 --warmup 20 --cpu-baseline off --host-offload off
  step b2s_${v}_$r 120 python3 bench.py --config 2s --steps 50 --warmup 20 --cpu-baseline off --host-offload off
done; done
cp profiles/r05/ab/head.so $LIB
echo "== done"
