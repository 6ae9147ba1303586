#!/usr/bin/env bash
# Chain kernel: pipelining across descriptor rounds (chains_variant 2: natural
# VGPRs, 3: capped for occupancy 6) vs the round-local pipeline (0).
set -u
OUT=gpurun_out/${TAG:-abx}; mkdir -p $OUT
for v in 2 3; do
UINET_CKSUM_CHAINS=$v timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "chain or config3 or tso or golden or zero_copy" > $OUT/pytest_v$v.log 2>&1; rc=$?; tail -2 $OUT/pytest_v$v.log; [ $rc -eq 0 ] || exit $rc
done
run() { local name=$1; shift; timeout -k 10 300 python tools/ab.py "$@" > $OUT/$name.json 2> $OUT/$name.err; local rc=$?; echo "$name rc=$rc"; python3 -c "import json,sys; d=json.load(open('$OUT/$name.json')); [print(' ',k,v) for k,v in d['results'].items()]" 2>/dev/null || tail -3 $OUT/$name.err; case $rc in 0) ;; *) exit $rc;; esac; }
run c3_cross --config 3 --rounds 12 --variants chains_variant=0 chains_variant=2 chains_variant=3
run c3tx_cross --config 3tx --rounds 12 --variants chains_variant=0 chains_variant=2 chains_variant=3
run c5tso_cross --config 5tso --rounds 8 --variants chains_variant=0 chains_variant=2 chains_variant=3
