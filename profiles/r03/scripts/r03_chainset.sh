#!/usr/bin/env bash
# Round 3: the chain configs' measurement set on the final chain kernel
# (packed 16-bit keys): bench line, rocprofv3 kernel trace, FETCH_SIZE pass.
set -u
TAG=${TAG:-r03s2h}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
TAG=$TAG CONFIGS="${CONFIGS:-3 3tx 5tso 3+packed}" bash tools/prof_all.sh || exit $?
echo "== done"
