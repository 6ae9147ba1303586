#!/usr/bin/env bash
# Zero-copy host batches: pipeline group size (knob host_group, chunks per
# thread per group) A/B in separate host_path.py processes, alternating, with
# the per-phase trace (UINET_CKSUM_TRACE_HOST).
set -u
TAG=${TAG:-r02hg}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
for r in 1 2; do for g in ${GROUPS_:-1 2 4 16}; do
  UINET_CKSUM_HOST_GROUP=$g UINET_CKSUM_TRACE_HOST=1 timeout -k 10 300 python3 -u tests/perf/host_path.py > $OUT/g$g.$r.log 2> $OUT/g$g.$r.err || exit 1
  echo "g=$g r=$r $(tail -1 $OUT/g$g.$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print({k: v["zero_copy_gibs"] for k, v in d.items()})')"
done; done
