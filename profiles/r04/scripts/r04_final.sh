#!/usr/bin/env bash
# Round 4 close: the span measurement set on the final span sources (their
# pmc_traffic.json entries re-measured, folded in on the box), then the
# driver's sequence (every GPU test, smoke, the driver's bench command and
# its trace) reading those entries.
set -u
TAG=${TAG:-r04s4} HBM=1 bash profiles/r04/scripts/r04_spanset.sh || exit 1
TAG=${VTAG:-r04v3} bash profiles/r04/scripts/r04_verify.sh || exit 1
