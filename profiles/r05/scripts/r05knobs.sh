#!/usr/bin/env bash
# Round 5: the whole GPU suite once per forced knob setting (include/
# uinet_cksum.h: knobs never change results): the one-shot span kernels,
# 4-pass chain batches, plain block order, the host walk for registered
# mbufs, 8-packet chain tiles.  No -x: every failure is listed.
set -u
OUT=gpurun_out/${TAG:-r05knobs}; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for kv in UINET_CKSUM_SPANS_PIPE=0 UINET_CKSUM_CHAINS_PASS=4 UINET_CKSUM_XCD_REMAP=0 UINET_CKSUM_WALK_DEVICE=0 UINET_CKSUM_CHAINS_TILE=8; do
  echo "== $kv"
  env $kv timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/${kv%%=*}.log" 2>&1
  rc=$?
  tail -n 3 "$OUT/${kv%%=*}.log"
  case $rc in 0|1) ;; *) echo FATAL rc=$rc; exit $rc;; esac
done
echo "== done"
