#!/usr/bin/env bash
# Span kernel: packets in flight per lane group (spans_depth 1 vs 2), parity
# first (every GPU span test with depth forced to 2), then interleaved A/B.
set -u
OUT=gpurun_out/${TAG:-abd}; mkdir -p $OUT
UINET_CKSUM_SPANS_DEPTH=2 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "span or strided or golden or pcap or config2 or config5 or host" > $OUT/pytest_d2.log 2>&1; rc=$?; tail -2 $OUT/pytest_d2.log; [ $rc -eq 0 ] || exit $rc
run() { local name=$1; shift; timeout -k 10 300 python tools/ab.py "$@" > $OUT/$name.json 2> $OUT/$name.err; local rc=$?; echo "$name rc=$rc"; python3 -c "import json,sys; d=json.load(open('$OUT/$name.json')); [print(' ',k,v) for k,v in d['results'].items()]" 2>/dev/null || tail -3 $OUT/$name.err; case $rc in 0) ;; *) exit $rc;; esac; }
run c2s_depth --config 2s --rounds 10 --variants spans_depth=1 spans_depth=2
run c2s_strided_depth --config 2s --api strided --rounds 10 --variants spans_depth=1 spans_depth=2
run c2_depth --config 2 --rounds 8 --variants spans_depth=1 spans_depth=2
run c5_depth --config 5 --rounds 8 --variants spans_depth=1 spans_depth=2
