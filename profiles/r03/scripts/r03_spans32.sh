#!/usr/bin/env bash
# Round 3: packed span descriptors (uinet_cksum_spans32).  Parity tests, then
# interleaved A/B wide vs packed on the small-packet shapes (2s, 2su) and on
# configs 2 / 5, then the measurement set of 2s / 2su on the packed API
# (bench line, rocprofv3 kernel trace, FETCH_SIZE pass).
set -u
TAG=${TAG:-r03s2b}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
step() { local name=$1 secs=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  echo "   rc=$rc"; grep -v "^[EW]20\|amdgpu.ids" "$OUT/$name.log" | tail -n 1 | cut -c1-300
  case $rc in 0) ;; *) echo FATAL; exit $rc;; esac; }
step pytest_spans32 600 python -u -m pytest tests/test_spans32.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
for c in 2s 2su 2 5; do
  step ab_c$c 300 python3 tools/ab.py --config $c --rounds 8 --variants desc=0 desc=1
done
TAG=$TAG CONFIGS="${CONFIGS:-2s+packed 2su+packed}" bash tools/prof_all.sh || exit $?
echo "== done"
