#!/usr/bin/env python3
"""Per-kernel statistics (calls, total / average / min / max duration in ns, share of the total)
from a rocprofv3 SQLite output (`rocprofv3 --kernel-trace -d DIR -o NAME -- ...` writes
DIR/NAME_results.db), as the CSV that `--stats --output-format csv` would give.

    python tools/rocpd_stats.py gpurun_out/prof/bench_results.db > profiles/.../kernel_stats.csv
"""
import csv
import sqlite3
import sys


def main(path):
    c = sqlite3.connect(path)
    rows = c.execute('select name, count(*), sum(duration), avg(duration), min(duration), max(duration) '
                     'from kernels group by name order by sum(duration) desc').fetchall()
    total = sum(r[2] for r in rows) or 1
    w = csv.writer(sys.stdout)
    w.writerow(['Name', 'Calls', 'TotalDurationNs', 'AverageNs', 'MinNs', 'MaxNs', 'Percentage'])
    for name, calls, tot, avg, mn, mx in rows:
        w.writerow([name if len(name) < 300 else name[:297] + '...', calls, tot, round(avg, 1), mn, mx,
                    round(100.0 * tot / total, 3)])


if __name__ == '__main__':
    main(sys.argv[1])
