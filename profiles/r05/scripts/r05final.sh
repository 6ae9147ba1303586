#!/usr/bin/env bash
# Round 5: the round-end driver sequence on the final tree -- GPU suite,
# smoke(), the driver's bench command -- one call.
set -u
OUT=gpurun_out/${TAG:-r05final}; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  echo "   rc=$rc"; grep -v "^[EW]20\|amdgpu.ids" "$OUT/$name.log" | tail -n 1 | cut -c1-300
  case $rc in 0) ;; *) echo FATAL; exit $rc;; esac; }
step pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
step driver_bench 300 python3 bench.py --gpus 1 --steps 20 --warmup 5
echo "== done"
