"""Per-kernel summary of rocprofv3 --pmc passes (one directory per pass, each holding a
*counter_collection.csv) for the engine's kernels (names containing 'ddl::'), plus the kernel
trace's average duration: counters summed per dispatch, averaged over dispatches; derived HBM
bytes per dispatch = (2 x FETCH_SIZE + WRITE_SIZE) x 1 KiB (MI355X_MICROARCH.md's gfx950
FETCH_SIZE correction) and the SQ wave-cycle split. Measurement tool (not shipped).
    python tools/pmc_kernel_summary.py <out.json> <trace_kernel_stats.csv> <pass dir> [<pass dir> ...]"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def short(name):
    m = re.search(r'(k_\w+<[^>]*>)', name)
    return m.group(1) if m else name[:80]


def main(out, stats_csv, dirs):
    per = defaultdict(lambda: defaultdict(lambda: defaultdict(float)))  # kernel -> counter -> dispatch -> value
    for d in dirs:
        for f in glob.glob(os.path.join(d, '**', '*counter_collection.csv'), recursive=True):
            with open(f) as fh:
                for row in csv.DictReader(fh):
                    if 'ddl::' not in row['Kernel_Name']:
                        continue
                    per[short(row['Kernel_Name'])][row['Counter_Name']][row['Dispatch_Id']] += float(row['Counter_Value'])
    avg_ns = {}
    if os.path.exists(stats_csv):
        with open(stats_csv) as fh:
            for row in csv.DictReader(fh):
                if 'ddl::' in row['Name']:
                    avg_ns[short(row['Name'])] = (float(row['AverageNs']), int(row['Calls']))
    summary = {}
    for k, counters in per.items():
        s = {c: sum(v.values()) / len(v) for c, v in counters.items()}
        s['dispatches'] = max(len(v) for v in counters.values())
        if 'FETCH_SIZE' in s and 'WRITE_SIZE' in s:
            s['hbm_bytes_per_dispatch'] = (2 * s['FETCH_SIZE'] + s['WRITE_SIZE']) * 1024
        if 'SQ_WAVE_CYCLES' in s:
            wc = s['SQ_WAVE_CYCLES']
            for c, name in (('SQ_WAIT_ANY', 'wait_any_frac'), ('SQ_WAIT_INST_ANY', 'wait_inst_any_frac'),
                            ('SQ_ACTIVE_INST_ANY', 'active_frac')):
                if c in s and wc:
                    s[name] = round(s[c] / wc, 4)
        if k in avg_ns:
            s['avg_ns_kernel_trace'], s['trace_calls'] = avg_ns[k]
        summary[k] = s
    with open(out, 'w') as fh:
        json.dump(summary, fh, indent=1)
    print(json.dumps(summary, indent=1))


if __name__ == '__main__':
    main(sys.argv[1], sys.argv[2], sys.argv[3:])
