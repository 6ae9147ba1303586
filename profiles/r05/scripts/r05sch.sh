#!/usr/bin/env bash
# Round 5: the chain kernel (cksum_chains.hip) built under LLVM's other AMDGPU
# machine schedulers (-mllvm -amdgpu-sched-strategy=...; same 72 VGPRs, 7
# waves, no scratch, different instruction order) against the shipped build
# (head.so), 3 alternating rounds of configs 3 (wide, packed) and 3tx.
set -u
OUT=gpurun_out/${TAG:-r05sch}; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
LIB=libuinet_amd/libuinet_cksum.so
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  echo "   rc=$rc"; grep -o '"ms_per_step": [0-9.]*' "$OUT/$name.log" | tail -n 1
  case $rc in 0) ;; *) echo FATAL; cp profiles/r05/ab/head.so $LIB; exit $rc;; esac; }
for r in 1 2 3; do for v in head max-ilp max-memory-clause iterative-ilp iterative-minreg; do
  cp profiles/r05/ab/$v.so $LIB
  step c3_${v}_$r 150 python3 bench.py --config 3 --steps 50 --warmup 20 --cpu-baseline off --host-offload off
  step c3p_${v}_$r 150 python3 bench.py --config 3 --desc packed --steps 50 --warmup 20 --cpu-baseline off --host-offload off
  step c3tx_${v}_$r 150 python3 bench.py --config 3tx --steps 50 --warmup 20 --cpu-baseline off --host-offload off
done; done
cp profiles/r05/ab/head.so $LIB
echo "== done"
