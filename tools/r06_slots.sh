# HBM scattered-header calibration: 32-B reads at 256-B slots (sequential and
# random), timed, then one FETCH_SIZE pass
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r06slots}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 120 ./tools/hbm_read slots 1757364224 > $O/slots.json 2>&1 || { cat $O/slots.json; exit 1; }
cat $O/slots.json
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/pmc -o run --output-format csv -- ./tools/hbm_read slots 1757364224 > $O/pmc.log 2>&1 || { tail $O/pmc.log; exit 1; }
python3 profiles/r05/scripts/pmc_by_kernel.py --per-dispatch $(ls $O/pmc/*counter_collection.csv $O/pmc/*/*counter_collection.csv 2>/dev/null) | sed -n 1,12p
python3 - <<'P'
import csv,glob,collections
rows=[r for f in glob.glob("'$O'/pmc/**/*counter_collection.csv",recursive=True) for r in csv.DictReader(open(f))]
agg=collections.defaultdict(list)
for r in rows: agg[r['Kernel_Name'].split('(')[0]].append(float(r['Counter_Value']))
for k,v in agg.items(): print(k, len(v), sum(v)/len(v), "KB ->", sum(v)/len(v)*1024/6864704, "B per read (x1)")
P
