#!/usr/bin/env bash
set -u
OUT=gpurun_out/${TAG:-ab}; mkdir -p $OUT
run() { local name=$1; shift; timeout -k 10 300 python tools/ab.py "$@" > $OUT/$name.json 2> $OUT/$name.err; local rc=$?; echo "$name rc=$rc"; cat $OUT/$name.json | python3 -c "import json,sys; d=json.load(sys.stdin); [print(' ',k,v) for k,v in d['results'].items()]" 2>/dev/null || tail -3 $OUT/$name.err; case $rc in 124|134|137|139) exit $rc;; esac; }
run c3_pass --config 3 --variants chains_pass=2 chains_pass=4 chains_pass=8
run c3_bpc --config 3 --variants blocks_per_cu=16 blocks_per_cu=32 blocks_per_cu=64 blocks_per_cu=128
run c2_bpc --config 2 --variants blocks_per_cu=32 blocks_per_cu=64 blocks_per_cu=128 blocks_per_cu=4096
run c5_bpc --config 5 --variants blocks_per_cu=32 blocks_per_cu=64 blocks_per_cu=128 blocks_per_cu=4096
