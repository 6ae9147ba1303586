#!/usr/bin/env bash
# Interleaved A/B of passes per batch in the chain kernel (1: 70 VGPRs occ 7,
# 2: 80 occ 6 (default), 3: 96 occ 5) on configs 3 / 3tx / 5tso.
set -u
OUT=gpurun_out/${TAG:-abp}; mkdir -p $OUT
run() { local name=$1; shift; timeout -k 10 300 python tools/ab.py "$@" > $OUT/$name.json 2> $OUT/$name.err; local rc=$?; echo "$name rc=$rc"; python3 -c "import json,sys; d=json.load(open('$OUT/$name.json')); [print(' ',k,v) for k,v in d['results'].items()]" 2>/dev/null || tail -3 $OUT/$name.err; case $rc in 0) ;; *) exit $rc;; esac; }
run c3_pass --config 3 --rounds 12 --variants chains_pass=2 chains_pass=1 chains_pass=3
run c3tx_pass --config 3tx --rounds 12 --variants chains_pass=2 chains_pass=1 chains_pass=3
run c5tso_pass --config 5tso --rounds 8 --variants chains_pass=2 chains_pass=1 chains_pass=3
