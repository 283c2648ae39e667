#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace --stats run (rocpd SQLite .db or the
kernel_stats.csv of --output-format csv) as a per-kernel table."""
import csv
import sqlite3
import sys


def from_db(path):
    c = sqlite3.connect(path)
    rows = c.execute("select name, total_calls, total_duration, average, percentage from top_kernels").fetchall()
    return [(n.split("(")[0], int(calls), float(tot), float(avg), float(pct)) for n, calls, tot, avg, pct in rows]


def from_csv(path):
    out = []
    with open(path) as fh:
        for r in csv.DictReader(fh):
            out.append((r["Name"].split("(")[0], int(r["Calls"]), float(r["TotalDurationNs"]) / 1e3,
                        float(r["AverageNs"]) / 1e3, float(r["Percentage"])))
    return out


def main():
    path = sys.argv[1]
    rows = from_db(path) if path.endswith(".db") else from_csv(path)
    print(f"# source: {path}")
    print(f"{'kernel':<40} {'calls':>6} {'total_us':>12} {'avg_us':>10} {'pct':>7}")
    for n, calls, tot, avg, pct in rows:
        print(f"{n:<40} {calls:>6} {tot:>12.1f} {avg:>10.1f} {pct:>7.2f}")


if __name__ == "__main__":
    main()
