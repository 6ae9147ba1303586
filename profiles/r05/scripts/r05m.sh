#!/usr/bin/env bash
# Round 5: walk/fold pipeline group count (1, 2, 4, 8 = tree) on the device
# paths, alternating processes, plus the concurrent-threads test and the suite.
set -u
OUT=gpurun_out/${TAG:-r05m}; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
LIB=libuinet_amd/libuinet_cksum.so
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  echo "   rc=$rc"; grep -v "^[EW]20\|amdgpu.ids" "$OUT/$name.log" | tail -n 2 | cut -c1-300
  case $rc in 0) ;; *) echo FATAL; cp profiles/r05/ab/g8.so $LIB; exit $rc;; esac; }
step pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
for r in 1 2; do for v in g8 g1 g2 g4; do
  cp profiles/r05/ab/$v.so $LIB
  step host_cpu_${v}_$r 300 python -u tests/perf/host_cpu.py --work c2,c3,hooks --paths dev_walk --threads 1
done; done
cp profiles/r05/ab/g8.so $LIB
echo "== done"
