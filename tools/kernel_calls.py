"""Per-call durations of the kernels whose name contains PATTERN in a rocprofv3 trace (rocpd
SQLite .db), in launch order, with how much of each call overlapped other kernels.

usage: python tools/kernel_calls.py <run_results.db> PATTERN [max_rows]
"""
import sqlite3
import sys


def main():
    path, pat = sys.argv[1], sys.argv[2]
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 200
    c = sqlite3.connect(path)
    rows = list(c.execute("select name, start, end from kernels order by start"))
    mine = [(st, en) for name, st, en in rows if pat in name]
    other = [(st, en) for name, st, en in rows if pat not in name]
    print(f"{len(mine)} calls of *{pat}*, total {sum(e - s for s, e in mine) / 1e6:.1f} ms")
    print("| # | start ms | us | overlapped by other kernels % |")
    print("|---|---|---|---|")
    t0 = rows[0][1] if rows else 0
    j = 0
    for i, (st, en) in enumerate(mine[:top]):
        while j < len(other) and other[j][1] < st:
            j += 1
        cov, k = 0, j
        while k < len(other) and other[k][0] < en:
            cov += max(0, min(en, other[k][1]) - max(st, other[k][0]))
            k += 1
        print(f"| {i} | {(st - t0) / 1e6:.1f} | {(en - st) / 1e3:.0f} | {100 * min(cov, en - st) / max(1, en - st):.0f} |")


if __name__ == "__main__":
    main()
