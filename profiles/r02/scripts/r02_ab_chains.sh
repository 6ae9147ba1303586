#!/usr/bin/env bash
# Chain-kernel variant A/B (tools/ab.py, one process per config) + parity of the
# variant through the chain tests with it forced.
set -u
TAG=${TAG:-r02d}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
VARS=${VARS:-"chains_chunk=16 chains_chunk=32"}
if [ -n "${PARITY_ENV:-}" ]; then
  env $PARITY_ENV timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_chains32.py tests/test_variants.py tests/test_limits.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_variant.log" 2>&1
  rc=$?; tail -2 "$OUT/pytest_variant.log"; [ $rc -eq 0 ] || exit $rc
fi
for c in ${CONFIGS:-3 3tx 5tso}; do
  timeout -k 10 300 python3 tools/ab.py --config $c --rounds 8 --launches 20 --variants $VARS > "$OUT/ab_c$c.json" 2>&1 || exit $?
  python3 -c "import json,sys; t=open('$OUT/ab_c$c.json').read(); d=json.loads(t[t.index('{'):]); print('$c', {k:(v['median_ms'],v['GBps_median']) for k,v in d['results'].items()})"
done
