"""Per-(kernel, grid size) dispatch durations from a rocprofv3 kernel trace (small-bucket
evidence): the kernel stats CSV groups every k_sum2_tile launch under one name whatever the
bucket size; the grid size tells the sizes apart. Writes <dir>/kernels_by_grid.json and deletes
the per-dispatch trace CSVs so the copy-back stays small.

    python scripts/prof_small.py gpurun_out/<dir>
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

out = sys.argv[1]
groups = defaultdict(list)
header = None
for f in glob.glob(os.path.join(out, '**', '*kernel_trace.csv'), recursive=True):
    with open(f) as fh:
        rd = csv.DictReader(fh)
        header = rd.fieldnames
        for row in rd:
            name = row.get('Kernel_Name') or row.get('Kernel-Name') or '?'
            grid = next((row[k] for k in row if k and k.lower().replace('-', '_') in ('grid_size', 'grid_size_x')), '?')
            try:
                dur = (int(row['End_Timestamp']) - int(row['Start_Timestamp'])) / 1e3
            except (KeyError, ValueError):
                continue
            groups[(name[:120], grid)].append(dur)
res = []
for (name, grid), d in sorted(groups.items(), key=lambda kv: (kv[0][0], int(kv[0][1]) if kv[0][1].isdigit() else 0)):
    d.sort()
    res.append({'kernel': name, 'grid': grid, 'dispatches': len(d), 'mean_us': round(sum(d) / len(d), 3),
                'median_us': round(d[len(d) // 2], 3), 'min_us': round(d[0], 3)})
with open(os.path.join(out, 'kernels_by_grid.json'), 'w') as fh:
    json.dump({'columns': header, 'groups': res}, fh, indent=1)
for f in glob.glob(os.path.join(out, '**', '*kernel_trace.csv'), recursive=True):
    os.remove(f)
print('summarized', out, len(res), 'groups')
