#!/usr/bin/env bash
# Round 4: small packets through the span API with
# k_spans_quad's address sweep (quad_new.so, the default build) against the
# same library built with -DUINET_QUAD_NOSWEEP (quad_base.so), alternating
# bench processes on one box; span-sweep GPU parity first.
set -u
TAG=${TAG:-r04q}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
LIB=libuinet_amd/libuinet_cksum.so
cp $LIB tools/ab_so/keep.so
timeout -k 10 600 python -u -m pytest tests/test_spans_sweep.py tests/test_spans32.py tests/test_strided_dense.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest_quad.log 2>&1
rc=$?; tail -n 1 $OUT/pytest_quad.log; [ $rc -eq 0 ] || { echo FATAL $rc; exit $rc; }
for r in 1 2; do for v in quad_base quad_new; do for spec in 2s 2su 2s+packed 2su+packed; do
  desc=wide; c=$spec; case $spec in *+packed) desc=packed; c=${spec%+packed};; esac
  cp tools/ab_so/$v.so $LIB
  timeout -k 10 300 python3 bench.py --config $c --desc $desc --cpu-baseline off > $OUT/$spec.$v.$r.log 2>&1 || { cp tools/ab_so/keep.so $LIB; tail -3 $OUT/$spec.$v.$r.log; exit 1; }
  python3 -c "import json; l=[x for x in open('$OUT/$spec.$v.$r.log') if x.startswith('{')][-1]; j=json.loads(l); print('$spec $v $r', j['roofline']['kernel_ms_mean'], j['roofline']['frac'], j['roofline']['instance'])"
done; done; done
cp tools/ab_so/keep.so $LIB
echo "== done"
