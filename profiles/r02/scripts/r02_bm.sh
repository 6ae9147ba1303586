#!/usr/bin/env bash
# Bitmap segment lookup (chains_variant=2) against the shipped chunk stream:
# chain parity tests, then interleaved A/B on configs 3 / 3tx / 5tso.
set -u
TAG=${TAG:-r02bm}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  echo "   rc=$rc"; grep -v "^[EW]20" "$OUT/$name.log" | tail -n 4 | cut -c1-400
  case $rc in 0) ;; *) echo FATAL; exit $rc;; esac; }
[ -z "${SKIP_TESTS:-}" ] && step pytest_chains 600 python -u -m pytest tests/test_gpu_parity.py tests/test_chains32.py -m gpu -k "chain" -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
for c in ${CONFIGS:-3 3tx 5tso}; do
  step ab_c$c 300 python3 -u tools/ab.py --config $c --rounds 8 --launches 20 --variants ${VARIANTS:-chains_variant=0 chains_variant=2}
done
echo "== done"
