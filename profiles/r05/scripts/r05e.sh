#!/usr/bin/env bash
# Round 5: page size under the device walk.  The walk reads one mbuf header
# per hop at random over the registered mbuf memory; the same batches with the
# mbufs and bytes on transparent huge pages (UINET_MBUF_HUGEPAGES=1:
# libuinet_amd/mbuf.py maps them MADV_HUGEPAGE) against 4-KiB pages,
# alternating processes; kernel traces of both.
set -u
OUT=gpurun_out/${TAG:-r05e}; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  echo "   rc=$rc"; grep -v "^[EW]20\|amdgpu.ids" "$OUT/$name.log" | tail -n 1 | cut -c1-300
  case $rc in 0) ;; *) echo FATAL; exit $rc;; esac; }
for r in 1 2; do
  step pages4k_$r 300 env UINET_MBUF_HUGEPAGES=0 python -u tests/perf/host_cpu.py --work c2,c3,hooks,echo --paths zero_copy,dev_walk --threads 1
  step pages2m_$r 300 env UINET_MBUF_HUGEPAGES=1 python -u tests/perf/host_cpu.py --work c2,c3,hooks,echo --paths zero_copy,dev_walk --threads 1
done
export UINET_MBUF_HUGEPAGES=1
step trace2m 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace2m" -o run --output-format csv -- python3 tests/perf/host_cpu.py --work c2,c3 --paths dev_walk --threads 1 --reps 3
echo "== done"
