"""Kernel statistics from a rocprofv3 database (the default output format: rocpd SQLite) as the
CSV that `--output-format csv --stats` writes: Name, Calls, TotalDurationNs, AverageNs, Percentage.

    python tools/rocpd_stats.py gpurun_out/<run>/prof/run_results.db > profiles/<name>.csv
"""
import csv
import sqlite3
import sys


def main(path, top=40):
    c = sqlite3.connect(path)
    w = csv.writer(sys.stdout)
    w.writerow(['Name', 'Calls', 'TotalDurationNs', 'AverageNs', 'Percentage'])
    for name, calls, total, avg, pct in c.execute(
            'select name, total_calls, total_duration, average, percentage from top_kernels limit ?', (top,)):
        w.writerow([name, calls, f'{total:.0f}', f'{avg:.1f}', f'{pct:.3f}'])


if __name__ == '__main__':
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 40)
