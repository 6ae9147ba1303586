#!/usr/bin/env bash
# Round 5: the host wait A/B (sleep-poll ctx_wait = wait.so against the lab
# build -DUINET_WAIT_SPIN = spin.so, spin.so built by "build_lab.sh spin cksum_api -DUINET_WAIT_SPIN"), in
# alternating processes, two rounds of tests/perf/host_cpu.py each; then the
# large-span geometry check (geo64k.py).
set -u
OUT=gpurun_out/${TAG:-r05b}; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
LIB=libuinet_amd/libuinet_cksum.so
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  echo "   rc=$rc"; grep -v "^[EW]20\|amdgpu.ids" "$OUT/$name.log" | tail -n 2 | cut -c1-300
  case $rc in 0) ;; *) echo FATAL; cp profiles/r05/ab/wait.so $LIB; exit $rc;; esac; }
[ -n "${SKIP_TESTS:-}" ] || step pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
for r in 1 2; do for v in wait spin; do
  cp profiles/r05/ab/$v.so $LIB
  step host_cpu_${v}_$r 600 python -u tests/perf/host_cpu.py
done; done
cp profiles/r05/ab/wait.so $LIB
step geo64k 300 python -u profiles/r05/scripts/geo64k.py
echo "== done"
# where a device-walked batch's time goes: walk kernel vs chain fold (c2, c3)
step walk_trace 300 rocprofv3 --kernel-trace --stats -d "$OUT/walk_trace" -o run --output-format csv -- python3 tests/perf/host_cpu.py --work c2,c3 --paths dev_walk --threads 1 --reps 3
python3 tools/pmc_summary.py "$OUT/walk_trace" > "$OUT/walk_trace.summary.json" || true
echo "== done2"
