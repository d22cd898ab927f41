"""Shrinks a rocprofv3 output directory to what is committed under profiles/: the kernel stats
CSV as is, and per-kernel PMC means (FETCH_SIZE / WRITE_SIZE per dispatch); the big per-dispatch
trace CSVs are deleted so the gpurun copy-back stays small."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

out = sys.argv[1]
summary = {}
for d in sorted(glob.glob(os.path.join(out, 'pmc_*'))):
    counter = os.path.basename(d)[4:]
    sums, cnts = defaultdict(float), defaultdict(int)
    for f in glob.glob(os.path.join(d, '*counter_collection.csv')):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = row.get('Kernel_Name') or row.get('Kernel-Name') or '?'
                try:
                    sums[k] += float(row.get('Counter_Value') or row.get('Counter-Value') or 0)
                except ValueError:
                    continue
                cnts[k] += 1
    summary[counter] = {k: {'mean_per_dispatch': sums[k] / cnts[k], 'dispatch_rows': cnts[k]} for k in sums}
with open(os.path.join(out, 'pmc_summary.json'), 'w') as fh:
    json.dump(summary, fh, indent=1)
for f in glob.glob(os.path.join(out, '**', '*kernel_trace.csv'), recursive=True) + \
        glob.glob(os.path.join(out, '**', '*counter_collection.csv'), recursive=True):
    os.remove(f)
print('summarized', out)
