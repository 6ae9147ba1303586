#!/usr/bin/env bash
# Round 3: is config 4's per-byte gap to config 2 (0.888 vs 0.912) the HBM
# itself at 3.1 GB?  Pure-read ceiling at 1.57 and 3.15 GB, and the lean
# kernel's grid width on config 4.
set -u
TAG=${TAG:-r03s2l}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
step() { local name=$1 secs=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  echo "   rc=$rc"; grep -v "^[EW]20\|amdgpu.ids" "$OUT/$name.log" | tail -n 1 | cut -c1-300
  case $rc in 0) ;; *) echo FATAL; exit $rc;; esac; }
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 tools/hbm_read.hip -o /tmp/hbm_read || exit 1
step hbm_1p5 120 /tmp/hbm_read 1572864000
step hbm_3p1 120 /tmp/hbm_read 3145728000
step ab_c4 300 python3 tools/ab.py --config 4 --rounds 8 --variants blocks_per_cu=0 blocks_per_cu=256 blocks_per_cu=1024
step ab_c2 300 python3 tools/ab.py --config 2 --rounds 8 --variants blocks_per_cu=0 blocks_per_cu=512
echo "== done"
