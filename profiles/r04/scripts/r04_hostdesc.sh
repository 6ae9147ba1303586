#!/usr/bin/env bash
# Round 4: zero-copy host-mbuf batches with packed 6-B
# chain descriptors (the default) against the same library built with
# -DUINET_HOST_WIDE_DESC (12-B descriptors), alternating processes on one
# box; tools/ab_so/{packed,wide}.so are built here beforehand.
set -u
TAG=${TAG:-r04h}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
LIB=libuinet_amd/libuinet_cksum.so
cp $LIB tools/ab_so/keep.so
for r in 1 2 3; do for v in wide packed; do
  cp tools/ab_so/$v.so $LIB
  timeout -k 10 300 python3 -u tests/perf/host_path.py --shapes c2,c3 --no-reference --reps 7 > $OUT/$v.$r.log 2> $OUT/$v.$r.err || { cp tools/ab_so/keep.so $LIB; tail $OUT/$v.$r.err; exit 1; }
  echo "$v $r $(tail -1 $OUT/$v.$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print({k: (v["staging_gibs"], v["zero_copy_gibs"], v["equal"]) for k, v in d.items()})')"
done; done
cp tools/ab_so/keep.so $LIB
echo "== done"
