#!/usr/bin/env bash
# Round 4: the RX / TX hooks with header parsing fused into the batch walk
# (run_jobs_made) against the previous three-pass form: hook, replay, echo and
# fuzz tests on the new build, then tests/perf/offload_rate.py alternating
# builds, 3 rounds, with the phase trace.  tools/ab_so/{base,new}.so.
set -u
TAG=${TAG:-r04hk}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
LIB=libuinet_amd/libuinet_cksum.so
cp $LIB tools/ab_so/keep.so; cp tools/ab_so/new.so $LIB
[ -n "${SKIP_TESTS:-}" ] || timeout -k 10 400 python3 -u -m pytest tests/test_offload.py tests/test_replay.py tests/test_echo.py tests/test_gpu_fuzz.py tests/test_host_desc.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; cp tools/ab_so/keep.so $LIB; exit 1; }
[ -n "${SKIP_TESTS:-}" ] || tail -1 $OUT/pytest.log
for r in $(seq 1 ${ROUNDS:-3}); do for v in base new; do
  cp tools/ab_so/$v.so $LIB
  UINET_CKSUM_TRACE_HOST=1 timeout -k 10 300 python3 -u tests/perf/offload_rate.py --reps 7 > $OUT/rate.$v.$r.log 2> $OUT/trace.$v.$r.log || { cp tools/ab_so/keep.so $LIB; exit 1; }
  echo "$v $r $(tail -1 $OUT/rate.$v.$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print({k: d[k] for k in ("tx_staged_ms","tx_zero_copy_ms","rx_staged_ms","rx_zero_copy_ms","tx_equal_oracle","rx_equal_oracle")})')"
done; done
cp tools/ab_so/keep.so $LIB
