#!/usr/bin/env bash
# ABAB of two engine builds (libuinet_amd/alt/libuinet_cksum_{A,B}.so) on the
# host-resident rate tools, same box.
set -u
OUT=gpurun_out/${TAG:-abh}; mkdir -p $OUT
cp libuinet_amd/libuinet_cksum.so $OUT/keep.so
for rep in 1 2; do for v in A B; do
  cp libuinet_amd/alt/libuinet_cksum_$v.so libuinet_amd/libuinet_cksum.so
  timeout -k 10 300 python tests/perf/host_path.py > $OUT/host_$v$rep.log 2>&1 || { cp $OUT/keep.so libuinet_amd/libuinet_cksum.so; exit 1; }
  timeout -k 10 300 python tests/perf/offload_rate.py > $OUT/offload_$v$rep.log 2>&1 || { cp $OUT/keep.so libuinet_amd/libuinet_cksum.so; exit 1; }
  timeout -k 10 300 python tests/perf/echo_replay.py > $OUT/echo_$v$rep.log 2>&1 || { cp $OUT/keep.so libuinet_amd/libuinet_cksum.so; exit 1; }
  python3 - "$OUT" "$v$rep" <<'PY'
import json, sys
o, t = sys.argv[1], sys.argv[2]
last = lambda f: json.loads([l for l in open(f) if l.startswith('{')][-1])
h, f, e = last(f"{o}/host_{t}.log"), last(f"{o}/offload_{t}.log"), last(f"{o}/echo_{t}.log")
print(t, "c3 staged/zc", h["c3_262144"]["staging_gibs"], h["c3_262144"]["zero_copy_gibs"],
      "c2 staged/zc", h["c2_1048576"]["staging_gibs"], h["c2_1048576"]["zero_copy_gibs"],
      "| offload tx s/zc", f["tx_staged_ms"], f["tx_zero_copy_ms"], "rx s/zc", f["rx_staged_ms"], f["rx_zero_copy_ms"],
      "| echo s/zc ms", e["gpu_staged"]["total_ms"], e["gpu_zero_copy"]["total_ms"])
PY
done; done
cp $OUT/keep.so libuinet_amd/libuinet_cksum.so
