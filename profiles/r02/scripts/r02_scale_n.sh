#!/usr/bin/env bash
# Kernel time against batch size (does a launch carry a fixed tail?).
set -u
TAG=${TAG:-r02f}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for spec in ${SPECS:-"3 262144" "3 1048576" "3 2097152" "3 4194304" "2 1048576" "2 4194304"}; do
  set -- $spec
  timeout -k 10 300 python3 bench.py --config $1 --packets $2 --steps 50 --warmup 100 --cpu-baseline off > "$OUT/c$1_n$2.log" 2>&1 || exit $?
  python3 -c "import json; d=json.loads([l for l in open('$OUT/c$1_n$2.log') if l.startswith('{')][-1]); r=d['roofline']; print('$1 $2', r['kernel_ms_mean'], r['achieved'])"
done
