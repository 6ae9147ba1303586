#!/usr/bin/env bash
# Host pool helpers pinned (UINET_CKSUM_HOST_PIN=1) or floating (0): host_path.py
# and offload_rate.py in separate processes, alternating, per-phase trace on.
set -u
TAG=${TAG:-r02pin}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
for r in 1 2 3; do for p in 0 1; do
  UINET_CKSUM_HOST_PIN=$p UINET_CKSUM_TRACE_HOST=1 timeout -k 10 300 python3 -u tests/perf/host_path.py > $OUT/hp$p.$r.log 2> $OUT/hp$p.$r.err || exit 1
  echo "pin=$p r=$r $(tail -1 $OUT/hp$p.$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print({k: (v["staging_gibs"], v["zero_copy_gibs"]) for k, v in d.items()})')"
done; done
for r in 1 2; do for p in 0 1; do
  UINET_CKSUM_HOST_PIN=$p timeout -k 10 300 python3 -u tests/perf/offload_rate.py > $OUT/or$p.$r.log 2>&1 || exit 1
  echo "pin=$p r=$r offload $(tail -1 $OUT/or$p.$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print({k: d[k] for k in ("rx_staged_ms","rx_zero_copy_ms","tx_staged_ms","tx_zero_copy_ms","reference_16thread_rx_ms","reference_16thread_tx_ms")})')"
done; done
