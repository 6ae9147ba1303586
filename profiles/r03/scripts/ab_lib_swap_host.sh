#!/usr/bin/env bash
# A/B of two builds of the engine library (tools/ab_so/base.so vs new.so) on
# the host-resident tools, separate processes, alternating, with the
# per-phase host trace.  Usage: TAG=... bash tools/ab_lib_swap_host.sh
set -u
TAG=${TAG:-r02hswap}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
LIB=libuinet_amd/libuinet_cksum.so
cp $LIB tools/ab_so/keep.so
for r in 1 2 3; do for v in base new; do
  cp tools/ab_so/$v.so $LIB
  UINET_CKSUM_TRACE_HOST=1 timeout -k 10 300 python3 -u tests/perf/host_path.py > $OUT/$v.$r.log 2> $OUT/$v.$r.err || { cp tools/ab_so/keep.so $LIB; exit 1; }
  echo "$v $r $(tail -1 $OUT/$v.$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print({k: v["zero_copy_gibs"] for k, v in d.items()})')"
done; done
cp tools/ab_so/keep.so $LIB
