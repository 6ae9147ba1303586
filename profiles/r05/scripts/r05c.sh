#!/usr/bin/env bash
# Round 5: the device walk with one-round-trip header loads and the walk/fold
# pipeline (groups8.so = the tree) against the same library walking each batch
# in one group (groups1.so: build_lab.sh groups1 cksum_api -DUINET_WALK_GROUPS=1),
# alternating processes; GPU tests first; kernel trace of the walked batches.
set -u
OUT=gpurun_out/${TAG:-r05c}; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
LIB=libuinet_amd/libuinet_cksum.so
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  echo "   rc=$rc"; grep -v "^[EW]20\|amdgpu.ids" "$OUT/$name.log" | tail -n 2 | cut -c1-300
  case $rc in 0) ;; *) echo FATAL; cp profiles/r05/ab/groups8.so $LIB; exit $rc;; esac; }
step pytest_walk 300 python -u -m pytest tests/test_device_walk.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider
[ -n "${SKIP_TESTS:-}" ] || step pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
for r in 1 2 3; do for v in groups8 groups1; do
  cp profiles/r05/ab/$v.so $LIB
  step host_cpu_${v}_$r 300 python -u tests/perf/host_cpu.py --work c2,c3,hooks,echo --paths dev_walk --threads 1,16
done; done
cp profiles/r05/ab/groups8.so $LIB
step walk_trace 300 rocprofv3 --kernel-trace --stats -d "$OUT/walk_trace" -o run --output-format csv -- python3 tests/perf/host_cpu.py --work c2,c3 --paths dev_walk --threads 1 --reps 3
echo "== done"
