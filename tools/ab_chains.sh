#!/usr/bin/env bash
# GPU tests, then interleaved A/B of the chain-kernel knobs on configs 3 / 3tx / 5tso.
set -u
OUT=gpurun_out/${TAG:-abc}; mkdir -p $OUT
timeout -k 10 900 python -m pytest tests -m gpu -q -x -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
run() { local name=$1; shift; timeout -k 10 300 python tools/ab.py "$@" > $OUT/$name.json 2> $OUT/$name.err; local rc=$?; echo "$name rc=$rc"; python3 -c "import json,sys; d=json.load(open('$OUT/$name.json')); [print(' ',k,v) for k,v in d['results'].items()]" 2>/dev/null || tail -3 $OUT/$name.err; case $rc in 0) ;; *) exit $rc;; esac; }
run c5tso_long --config 5tso --variants ${C5:-chains_long=0 chains_long=16 chains_long=64}
run c3tx_long --config 3tx --variants ${C3TX:-chains_long=0 chains_long=16 chains_long=32 chains_long=48 chains_long=64 chains_long=128}
run c3_long --config 3 --variants ${C3:-chains_long=0 chains_long=16 chains_long=64}
