#!/usr/bin/env bash
# Round 3: the chain configs through the packed-descriptor API
# (uinet_cksum_chains32) against the wide one, alternating bench processes
# on one box (7-wave chain kernel).
set -u
TAG=${TAG:-r03s3c}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for r in 1 2; do for c in 3 3tx 5tso; do for d in wide packed; do
  timeout -k 10 300 python3 bench.py --config $c --desc $d --cpu-baseline off > $OUT/$c.$d.$r.log 2>&1 || exit 1
  python3 -c "import json; l=[x for x in open('$OUT/$c.$d.$r.log') if x.startswith('{')][-1]; j=json.loads(l); print('$c $d $r', j['roofline']['kernel_ms_mean'], j['roofline']['frac'], j.get('bit_identical'))"
done; done; done
echo "== done"
