#!/usr/bin/env bash
# Small-packet kernel (k_spans_sm, knob spans_small) against the one-packet-
# per-group k_spans: span parity tests, then interleaved A/B on config 2s
# (16 M x 64 B) through the span and strided APIs.
set -u
TAG=${TAG:-r02small}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  echo "   rc=$rc"; grep -v "^[EW]20" "$OUT/$name.log" | tail -n 4 | cut -c1-400
  case $rc in 0) ;; *) echo FATAL; exit $rc;; esac; }
[ -z "${SKIP_TESTS:-}" ] && step pytest_spans 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -k "small or spans or strided" -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
for api in spans strided; do
  step ab_2s_$api 300 python3 -u tools/ab.py --config 2s --api $api --rounds 8 --launches 20 --variants ${VARIANTS:-spans_small=0 spans_small=1 spans_small=2}
done
echo "== done"
