"""Summarise a rocprofv3 kernel trace (rocpd SQLite .db or kernel_stats.csv) as a markdown table.

usage: python tools/rocpd_summary.py <run_results.db | kernel_stats.csv> [title] [note]
"""
import csv
import sqlite3
import sys
from collections import defaultdict


def rows_from_db(path):
    c = sqlite3.connect(path)
    acc = defaultdict(lambda: [0, 0.0, 0.0])
    span = c.execute("select min(start), max(end) from kernels").fetchone()
    for name, st, en in c.execute("select name, start, end from kernels"):
        a = acc[name]
        a[0] += 1
        a[1] += en - st
        a[2] = max(a[2], en - st)
    return acc, (span[1] - span[0]) if span[0] is not None else 0


def rows_from_csv(path):
    acc = {}
    for r in csv.DictReader(open(path)):
        acc[r["Name"]] = [int(r["Calls"]), float(r["TotalDurationNs"]), float(r["MaxNs"])]
    return acc, 0


def main():
    path = sys.argv[1]
    acc, span = rows_from_db(path) if path.endswith(".db") else rows_from_csv(path)
    tot = sum(v[1] for v in acc.values())
    out = []
    if len(sys.argv) > 2:
        out += [f"# {sys.argv[2]}", ""]
    if len(sys.argv) > 3:
        out += [sys.argv[3], ""]
    out.append(f"kernel time (sum over streams) {tot / 1e6:.1f} ms; first-start to last-end span {span / 1e6:.1f} ms")
    out += ["", "| kernel | calls | total ms | % | avg us | max us |", "|---|---|---|---|---|---|"]
    for name, (n, t, mx) in sorted(acc.items(), key=lambda kv: -kv[1][1])[:30]:
        out.append(f"| {name[:80]} | {n} | {t / 1e6:.1f} | {100 * t / tot:.1f} | {t / n / 1e3:.1f} | {mx / 1e3:.1f} |")
    print("\n".join(out))


if __name__ == "__main__":
    main()
