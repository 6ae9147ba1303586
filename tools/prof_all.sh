#!/usr/bin/env bash
# rocprofv3 kernel-trace (--stats) and a separate FETCH_SIZE pass per config;
# folds the HBM bytes per launch into profiles/pmc_traffic.json (bench reads it).
# Usage: TAG=... CONFIGS="2 3 3tx 5 5tso" tools/prof_all.sh
set -u
TAG=${TAG:-r01p}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  echo "   rc=$rc"; grep -v "^[EW]20" "$OUT/$name.log" | tail -n 2
  case $rc in 0) ;; *) echo FATAL; exit $rc;; esac; }
for spec in ${CONFIGS:-2 3 3tx 5 5tso}; do
  # "C" (spans API) or "C@strided"; a "+packed" suffix selects 6-B descriptors,
  # "+mbufs" the struct mbuf form of a chain config (uinet_cksum_mbufs)
  desc=wide; form=seglist
  case $spec in *+packed) desc=packed; spec=${spec%+packed};; esac
  case $spec in *+mbufs) form=mbufs; spec=${spec%+mbufs};; esac
  c=${spec%@*}; api=spans; [ "$spec" != "$c" ] && api=${spec#*@}
  t=c$c; [ "$api" != spans ] && t=c${c}_$api
  [ "$desc" = packed ] && t=${t}_packed
  [ "$form" = mbufs ] && t=${t}_mbufs
  A="--config $c --api $api --desc $desc --form $form"
  step bench_$t 600 python3 bench.py $A
  step trace_$t 600 rocprofv3 --kernel-trace --stats -d "$OUT/trace_$t" -o run --output-format csv -- python3 bench.py $A --cpu-baseline off
  step pmc_$t 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$OUT/pmc_$t" -o run --output-format csv -- python3 bench.py $A --steps 10 --warmup 2 --cpu-baseline off
  # the key the bench looks its traffic up by (roofline.traffic_source.key)
  read B KEY <<<"$(python3 -c "import json; d=json.loads([l for l in open('$OUT/bench_$t.log') if l.startswith('{')][-1]); print(d['config']['algorithmic_bytes_per_gpu'], d['roofline']['traffic_source']['key'])")"
  python3 tools/pmc_summary.py "$OUT/pmc_$t" --key "$KEY" --bytes "$B" --out profiles/pmc_traffic.json > "$OUT/pmc_$t.summary.json"
  python3 tools/pmc_summary.py "$OUT/trace_$t" > "$OUT/trace_$t.summary.json"
done
cp profiles/pmc_traffic.json "$OUT/pmc_traffic.json"
echo "== done"
