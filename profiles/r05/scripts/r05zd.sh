#!/usr/bin/env bash
# Round 5: the per-call ABI's fold with AVX2 (percall_avx2.so = the tree)
# against the 64-bit scalar fold (percall_scalar.so), on the GPU box's host CPU:
# tests/perf/percall_bench.c in cache (16 packets cycled) and streaming
# (65,536 packets, 100 MB at 1500 B), 3 alternating rounds; the per-call tests
# on each build first.
set -u
OUT=gpurun_out/${TAG:-r05zd}; mkdir -p "$OUT"
LIB=libuinet_amd/libuinet_cksum.so
cp "$LIB" "$OUT/tree.so.bak"
for v in percall_avx2 percall_scalar; do
  cp profiles/r05/ab/$v.so $LIB
  echo "== pytest $v"
  timeout -k 10 300 python -u -m pytest tests/test_percall_host.py -q -p no:cacheprovider > "$OUT/pytest_$v.log" 2>&1 || { echo FATAL; cp "$OUT/tree.so.bak" $LIB; exit 1; }
  tail -n 1 "$OUT/pytest_$v.log"
done
gcc -O2 -std=c11 -I include tests/perf/percall_bench.c -L libuinet_amd -luinet_cksum \
  -Wl,-rpath,$PWD/libuinet_amd oracle/_ref/libref_cksum.so -Wl,-rpath,$PWD/oracle/_ref \
  -o "$OUT/percall_bench" || { cp "$OUT/tree.so.bak" $LIB; exit 1; }
lscpu | grep -i "model name" > "$OUT/cpu.txt"
for r in 1 2 3; do for v in percall_avx2 percall_scalar; do
  cp profiles/r05/ab/$v.so $LIB
  echo "== $v round $r"
  for len in 64 576 1500 9000; do for np in 16 65536; do
    timeout -k 5 60 taskset -c 2 "$OUT/percall_bench" $len $np >> "$OUT/${v}_$r.jsonl" || { cp "$OUT/tree.so.bak" $LIB; exit 1; }
  done; done
  tail -n 2 "$OUT/${v}_$r.jsonl" | cut -c1-160
done; done
cp "$OUT/tree.so.bak" $LIB
rm -f "$OUT/tree.so.bak" "$OUT/percall_bench"
echo "== done"
