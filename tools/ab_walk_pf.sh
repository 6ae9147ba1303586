#!/usr/bin/env bash
# ABAB of the host walk's software prefetch (UINET_CKSUM_WALK_PF=0 vs on) on
# the host-resident rate tools, same box, same build.
set -u
OUT=gpurun_out/${TAG:-abpf}; mkdir -p $OUT
for rep in $(seq ${REPS:-2}); do for v in ${VARIANTS:-0 1}; do
  export UINET_CKSUM_WALK_PF=$v
  timeout -k 10 300 python tests/perf/host_path.py > $OUT/host_$v$rep.log 2>&1 || exit 1
  timeout -k 10 300 python tests/perf/offload_rate.py > $OUT/offload_$v$rep.log 2>&1 || exit 1
  python3 - "$OUT" "$v$rep" <<'PY'
import json, sys
o, t = sys.argv[1], sys.argv[2]
last = lambda f: json.loads([l for l in open(f) if l.startswith('{')][-1])
h, f = last(f"{o}/host_{t}.log"), last(f"{o}/offload_{t}.log")
print("pf" + t, "c3 staged/zc", h["c3_262144"]["staging_gibs"], h["c3_262144"]["zero_copy_gibs"],
      "c2 staged/zc", h["c2_1048576"]["staging_gibs"], h["c2_1048576"]["zero_copy_gibs"],
      "| offload tx s/zc", f["tx_staged_ms"], f["tx_zero_copy_ms"], "rx s/zc", f["rx_staged_ms"], f["rx_zero_copy_ms"])
PY
done; done
