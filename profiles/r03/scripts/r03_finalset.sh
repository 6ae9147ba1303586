#!/usr/bin/env bash
# Round 3, final code: every config's bench line, rocprofv3 kernel trace and
# FETCH_SIZE pass (tools/prof_all.sh), and the box's pure-read ceiling.
set -u
TAG=${TAG:-r03s2p}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 tools/hbm_read.hip -o /tmp/hbm_read || exit 1
timeout -k 10 120 /tmp/hbm_read 1572864000 > "$OUT/hbm_read.log" 2>&1 || exit 1
TAG=$TAG CONFIGS="${CONFIGS:-2 2rx 4 5 2@strided 2s 2s+packed 2su 2su@strided 3 3tx 5tso}" bash tools/prof_all.sh || exit $?
echo "== done"
