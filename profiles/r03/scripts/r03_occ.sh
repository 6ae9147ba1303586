#!/usr/bin/env bash
# Round 3: chain kernel held at 6 (shipped), 7 or 8 waves per SIMD after the
# packed-key change freed registers (7: 36 B of spills, 8: 76 B, all in the
# per-round code, none in the batch loop); alternating bench processes.
set -u
TAG=${TAG:-r03s2d}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
TAG=$TAG VARIANTS="base w7 w8" CONFIGS="3 3tx 5tso" ROUNDS=3 bash tools/ab_lib_multi.sh
echo "== done"
