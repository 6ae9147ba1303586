#!/usr/bin/env bash
# Round 4 measurement set on one box: every config's bench line, rocprofv3
# kernel trace and FETCH_SIZE pass (tools/prof_all.sh, folded into
# profiles/pmc_traffic.json with the kernel's source hash), the chain
# kernel's instruction counters, and the box's pure-read ceiling.
# Usage: TAG=r04x CONFIGS="3 3+packed 3tx" bash profiles/r04/scripts/r04_set.sh
set -u
TAG=${TAG:-r04s}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
step() { local name=$1 secs=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  echo "   rc=$rc"; grep -v "^[EW]20\|amdgpu.ids" "$OUT/$name.log" | tail -n 1 | cut -c1-300
  case $rc in 0) ;; *) echo FATAL; exit $rc;; esac; }
if [ "${HBM:-1}" = 1 ]; then
  /opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 tools/hbm_read.hip -o /tmp/hbm_read || exit 1
  step hbm_read 120 /tmp/hbm_read 1572864000
fi
if [ -n "${INSTS:-}" ]; then  # e.g. INSTS="3 3+packed"
  for spec in $INSTS; do
    desc=wide; case $spec in *+packed) desc=packed; spec=${spec%+packed};; esac
    step insts_c${spec}_$desc 180 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVES SQ_INSTS_LDS -d "$OUT/insts_c${spec}_$desc" -o run --output-format csv -- python3 bench.py --config $spec --desc $desc --steps 3 --warmup 1 --cpu-baseline off
  done
fi
TAG=$TAG CONFIGS="${CONFIGS:-3 3+packed 3tx 5tso}" bash tools/prof_all.sh || exit $?
echo "== done"
