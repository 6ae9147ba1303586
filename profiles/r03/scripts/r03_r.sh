#!/usr/bin/env bash
# Round 3: chain kernel with 32-B units (chains_unit=32: two chunks per lane
# per pass, one segment lookup and binning scan per 2 KiB): parity, then
# interleaved A/B on configs 3, 3tx, 5tso.
set -u
TAG=${TAG:-r03r}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
step() { local name=$1 secs=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  echo "   rc=$rc"; grep -v "^[EW]20\|amdgpu.ids" "$OUT/$name.log" | tail -n 1 | cut -c1-200
  case $rc in 0) ;; *) echo FATAL; exit $rc;; esac; }
step pytest_chains 900 python -u -m pytest tests/test_gpu_parity.py tests/test_chains32.py -x -q -k "chains" --timeout 300 --timeout-method thread -p no:cacheprovider
for c in 3 3tx 5tso; do
  step ab_c$c 300 python3 tools/ab.py --config $c --rounds 8 --variants chains_unit=16 chains_unit=32 chains_pass=4 chains_unit=32,chains_tile=8
done
echo "== done"
