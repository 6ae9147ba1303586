#!/usr/bin/env bash
# Round 3: the split mask table in k_spans_quad (lab=1): parity (and the lean
# kernel's new default: split table, 256 blocks per CU), then 2s / 2su A/B.
set -u
TAG=${TAG:-r03u}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
step() { local name=$1 secs=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  echo "   rc=$rc"; grep -v "^[EW]20\|amdgpu.ids" "$OUT/$name.log" | tail -n 1 | cut -c1-200
  case $rc in 0) ;; *) echo FATAL; exit $rc;; esac; }
step pytest_spans 900 python -u -m pytest tests/test_gpu_parity.py -x -q -k "spans or strided" --timeout 300 --timeout-method thread -p no:cacheprovider
step pytest_spans_l1 900 env UINET_CKSUM_LAB=1 python -u -m pytest tests/test_gpu_parity.py -x -q -k "spans or strided" --timeout 300 --timeout-method thread -p no:cacheprovider
for c in 2s 2su; do
  step ab_c$c 300 python3 tools/ab.py --config $c --rounds 8 --variants lab=0 lab=1 lab=1,blocks_per_cu=256 spans_pipe=0
  step ab_c${c}_strided 300 python3 tools/ab.py --config $c --api strided --rounds 8 --variants lab=0 lab=1 lab=1,blocks_per_cu=256 spans_pipe=0
done
step ab_c2 300 python3 tools/ab.py --config 2 --rounds 8 --variants spans_pipe=1 spans_pipe=2 spans_pipe=0
echo "== done"
