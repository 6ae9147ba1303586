#!/usr/bin/env bash
# Round 5: k_chains_wide as built (short + long segment pair in flight
# together, every descriptor read scalar -- the packed u16 length out of its
# 32-bit word): parity tests, chain parity, fuzz; in-process A/B against the
# tile kernel on 5tso (4 rounds of 8); the 5tso bench line (auto pick) and
# its kernel trace.
set -u
OUT=gpurun_out/${TAG:-r05wide4}; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  echo "   rc=$rc"; grep -v "^[EW]20\|amdgpu.ids" "$OUT/$name.log" | tail -n 1 | cut -c1-300
  case $rc in 0) ;; *) echo FATAL; exit $rc;; esac; }
step pytest 500 python -u -m pytest tests/test_chains_wide.py tests/test_gpu_parity.py -k "chains or wide" -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
step fuzz 400 env UINET_FUZZ_TRIALS=6000 UINET_FUZZ_BASE=500000 python -u -m pytest tests/test_gpu_fuzz.py -k device -m gpu -x -q -s --timeout 380 --timeout-method thread -p no:cacheprovider
for r in 1 2 3 4; do
  step ab_5tso_$r 300 python3 tools/ab.py --config 5tso --rounds 8 --variants chains_wide=1 chains_wide=2 chains_wide=1,desc=1 chains_wide=2,desc=1
done
step bench_c5tso 200 python3 bench.py --config 5tso --steps 50 --warmup 20 --host-offload off
step bench_c5tso_packed 200 python3 bench.py --config 5tso --desc packed --steps 50 --warmup 20 --cpu-baseline off --host-offload off
step trace_c5tso 200 rocprofv3 --kernel-trace --stats -d "$OUT/trace_c5tso" -o run --output-format csv -- python3 bench.py --config 5tso --steps 20 --warmup 5 --cpu-baseline off --host-offload off
echo "== done"
