"""Average PMC counter values per kernel from rocprofv3 counter_collection.csv files.
Usage: python tools/pmc_summary.py <dir> [kernel-substring ...]"""
import collections
import csv
import os
import re
import sys

root = sys.argv[1]
keys = sys.argv[2:] or ['k_cg_']
acc = collections.defaultdict(list)
for dp, _, fs in os.walk(root):
    for f in fs:
        if f.endswith('counter_collection.csv'):
            for row in csv.DictReader(open(os.path.join(dp, f))):
                m = re.search(r'(k_\w+)', row['Kernel_Name'])
                name = m.group(1) if m else row['Kernel_Name'][:40]
                if any(k in row['Kernel_Name'] for k in keys):
                    acc[name, row['Counter_Name']].append(float(row['Counter_Value']))
kern = sorted({k for k, _ in acc})
for k in kern:
    print(k)
    for (kk, c), v in sorted(acc.items()):
        if kk == k:
            print(f'   {c:24s} {sum(v) / len(v):16.4g}  (n={len(v)})')
