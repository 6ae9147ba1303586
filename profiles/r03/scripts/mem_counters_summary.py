#!/usr/bin/env python3
"""Per-dispatch medians of the memory-request counters that
tools/r02_mem_counters.sh collects (profiles/r02/mem_counters/)."""
import csv, collections, sys, glob
for cfg in ('2','3'):
    agg = collections.defaultdict(list)
    for p in sorted(glob.glob(f'profiles/r02/mem_counters/c{cfg}/p*.csv')):
        for r in csv.DictReader(open(p)):
            k = r['Kernel_Name']
            if 'k_spans' not in k and 'k_chains' not in k: continue
            agg[(r['Counter_Name'], r['Dispatch_Id'])].append(float(r['Counter_Value']))
    tot = collections.defaultdict(list)
    for (c, d), v in agg.items(): tot[c].append(sum(v))
    print('config', cfg)
    for c, v in sorted(tot.items()):
        v = sorted(v); print(f'  {c:40s} median/dispatch {v[len(v)//2]:.4g}  n={len(v)}')
