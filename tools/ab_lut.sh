#!/usr/bin/env bash
set -u
OUT=gpurun_out/${TAG:-abl}; mkdir -p $OUT
timeout -k 10 600 python -m pytest tests -m gpu -q -x -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -2 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
run() { local name=$1; shift; timeout -k 10 300 python tools/ab.py "$@" > $OUT/$name.json 2> $OUT/$name.err; local rc=$?; echo "$name rc=$rc"; python3 -c "import json,sys; d=json.load(open('$OUT/$name.json')); [print(' ',k,v) for k,v in d['results'].items()]" 2>/dev/null || tail -3 $OUT/$name.err; case $rc in 0) ;; *) exit $rc;; esac; }
run c2_lut --config 2 --rounds 10 --variants spans_lut=0 spans_lut=1
run c2s_lut --config 2 --api strided --rounds 10 --variants spans_lut=0 spans_lut=1
run c2rx_lut --config 2rx --rounds 10 --variants spans_lut=0 spans_lut=1
run c5_lut --config 5 --rounds 10 --variants spans_lut=0 spans_lut=1
timeout -k 10 300 python tools/drift.py --config 2 --launches 400 --variants spans_lut=0 spans_lut=1 spans_lut=0 spans_lut=1 > $OUT/drift.log 2>&1; rc=$?; grep -v "^{" $OUT/drift.log | tail -4; exit $rc
