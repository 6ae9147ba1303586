#!/usr/bin/env bash
# Round 3: lean chain kernel (chains_variant=3) parity + interleaved A/B;
# per-launch series of both span kernels over 300 launches right after the
# GPU test suite (does the lean kernel's fresh-process level ramp?).
set -u
TAG=${TAG:-r03e}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
step() { local name=$1 secs=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  echo "   rc=$rc"; grep -v "^[EW]20\|amdgpu.ids" "$OUT/$name.log" | tail -n 2 | cut -c1-300
  case $rc in 0) ;; *) echo FATAL; exit $rc;; esac; }
step pytest_chains_lean 600 python -u -m pytest tests/test_gpu_parity.py tests/test_chains32.py -x -q -k "chains" --timeout 300 --timeout-method thread -p no:cacheprovider
step pytest_chains_lean_default 900 env UINET_CKSUM_CHAINS=3 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
for c in 3 3tx 5tso; do step ab_c$c 300 python3 tools/ab.py --config $c --rounds 6 --variants chains_variant=0 chains_variant=3 chains_variant=3,blocks_per_cu=128 chains_variant=3,chains_tile=8; done
step pytest_spans_lean 900 env UINET_CKSUM_SPANS_PIPE=3 python -u -m pytest tests/test_gpu_parity.py -x -q -k "spans or strided" --timeout 300 --timeout-method thread -p no:cacheprovider
step pytest_small 600 python -u -m pytest tests/test_gpu_parity.py -x -q -k "small_packets" --timeout 300 --timeout-method thread -p no:cacheprovider
for c in 2 4 5 2s; do step ab_span_c$c 300 python3 tools/ab.py --config $c --rounds 6 --variants spans_pipe=1 spans_pipe=3; done
step ab_span_c2s_strided 300 python3 tools/ab.py --config 2s --api strided --rounds 6 --variants spans_pipe=1 spans_pipe=3 spans_pipe=3,blocks_per_cu=64 spans_pipe=3,blocks_per_cu=8
for k in 1 3; do
  step pytest_pre_p$k 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
  step cold_p$k 300 env UINET_CKSUM_SPANS_PIPE=$k python3 tools/cold_start.py --launches 300 --idle-s 1.5
done
echo "== done"
