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


def grid_of(row):
    """(x, y) grid size of a trace / counter row (rocprofv3 names the columns Grid_Size_X / _Y,
    older versions Grid_Size)."""
    x = row.get('Grid_Size_X') or row.get('Grid_Size') or row.get('Grid-Size') or '?'
    return f"{x}x{row.get('Grid_Size_Y', '1')}"


# per (kernel, grid) from the kernel trace: the average duration of exactly those dispatches (a bench
# leg is one grid shape: the C4 fold's 2 MiB fp16 chunk is 1025 x 128 lanes, its 8-bucket batch
# 1025 x 128 by 8), and the PMC counters split the same way
by_grid = defaultdict(lambda: {'calls': 0, 'total_ns': 0.0})
for f in glob.glob(os.path.join(out, '**', '*kernel_trace.csv'), recursive=True):
    if '/pmc_' in f:
        continue
    with open(f) as fh:
        for row in csv.DictReader(fh):
            k = row.get('Kernel_Name') or '?'
            if 'ddl::' not in k:
                continue
            try:
                ns = float(row['End_Timestamp']) - float(row['Start_Timestamp'])
            except (KeyError, ValueError):
                continue
            e = by_grid[(k, grid_of(row))]
            e['calls'] += 1
            e['total_ns'] += ns
pmc_grid = defaultdict(lambda: defaultdict(lambda: [0.0, set()]))
for d in sorted(glob.glob(os.path.join(out, 'pmc_*'))):
    counter = os.path.basename(d)[4:]
    for f in glob.glob(os.path.join(d, '*counter_collection.csv')):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = row.get('Kernel_Name') or '?'
                if 'ddl::' not in k:
                    continue
                try:
                    v = float(row.get('Counter_Value') or 0)
                except ValueError:
                    continue
                acc = pmc_grid[(k, grid_of(row))][counter]
                acc[0] += v
                acc[1].add(row.get('Dispatch_Id'))
grid_summary = []
for (k, g), e in sorted(by_grid.items(), key=lambda kv: -kv[1]['total_ns']):
    item = {'kernel': k, 'grid': g, 'calls': e['calls'], 'avg_ns': round(e['total_ns'] / e['calls'], 1)}
    for counter, (tot, ids) in pmc_grid.get((k, g), {}).items():
        item[f'{counter}_per_dispatch'] = tot / max(1, len(ids))
    if 'FETCH_SIZE_per_dispatch' in item and 'WRITE_SIZE_per_dispatch' in item:
        # gfx950: FETCH_SIZE counts half the fetched KiB (MI355X_MICROARCH.md)
        item['hbm_bytes_per_dispatch'] = (2 * item['FETCH_SIZE_per_dispatch'] + item['WRITE_SIZE_per_dispatch']) * 1024
    grid_summary.append(item)
with open(os.path.join(out, 'kernel_by_grid.json'), 'w') as fh:
    json.dump(grid_summary, fh, indent=1)
for f in glob.glob(os.path.join(out, '**', '*kernel_trace.csv'), recursive=True) + \
        glob.glob(os.path.join(out, '**', '*counter_collection.csv'), recursive=True):
    os.remove(f)
print('summarized', out)
