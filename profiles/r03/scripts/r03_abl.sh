#!/usr/bin/env bash
# Round 3 (lab): where the chain kernel's time goes. Three builds in
# alternating bench processes (tools/ab_lib_multi.sh): base; NOLIST (the
# descriptor rounds and long segments only, no chunk-list batches); NOLOAD
# (everything but the packet-byte loads). Results of the ablations are wrong
# by construction; only their times are read.
set -u
TAG=${TAG:-r03s2t}
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
TAG=$TAG VARIANTS="base nolist noload" CONFIGS="3 3tx 5tso" ROUNDS=2 bash tools/ab_lib_multi.sh
echo "== done"
