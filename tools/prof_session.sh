#!/usr/bin/env bash
# Profiles + the other config shapes.  Each GPU step time-limited; a crash ends it.
set -u
TAG=${1:-r01d}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  echo "   rc=$rc"; grep -v "^[EW]20" "$OUT/$name.log" | tail -n 3
  case $rc in 124|134|137|139) echo FATAL; exit $rc;; esac; }
step prof_trace 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof_trace" -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --cpu-baseline off
step prof_pmc 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace --stats -d "$OUT/prof_pmc" -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --cpu-baseline off
step pmc_calib 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$OUT/pmc_calib" -o run --output-format csv -- tools/hbm_read
step bench_c2rx 300 python3 bench.py --config 2rx --steps 30 --warmup 5
step bench_c5 300 python3 bench.py --config 5 --steps 30 --warmup 5
step bench_c3 600 python3 bench.py --config 3 --steps 20 --warmup 3
step bench_host 300 python3 bench.py --steps 10 --warmup 2 --cpu-baseline off --host-path
echo "== done"
