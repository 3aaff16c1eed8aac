#!/usr/bin/env python3
"""Per (kernel, grid size) durations from a rocprofv3 --kernel-trace database (rocpd SQLite):
one kernel launched in several modes with different grids (e.g. hevc_sao's statistics /
apply launches) splits into its modes.

    python tools/kgrid.py run_results.db 'hevc_sao|hevc_intra_recon' [--after-ms N]
"""
import argparse
import re
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("pattern")
    ap.add_argument("--after-ms", type=float, default=0.0)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)").fetchall()]
    grid = [k for k in cols if "grid" in k.lower()]
    wg = [k for k in cols if "workgroup" in k.lower() and "size" in k.lower()]
    print("columns:", ", ".join(cols))
    sel = ", ".join(["name", "start", "end"] + grid + wg)
    rows = c.execute(f"select {sel} from kernels order by start").fetchall()
    t0 = rows[0][1] + a.after_ms * 1e6
    pat = re.compile(a.pattern)
    agg: dict = {}
    for r in rows:
        if r[1] < t0 or not pat.search(r[0]):
            continue
        key = (r[0].split("(")[0][:50],) + tuple(r[3:])
        v = agg.setdefault(key, [0, 0.0, 0.0])
        d = (r[2] - r[1]) / 1e6
        v[0] += 1
        v[1] += d
        v[2] = max(v[2], d)
    print(f"| kernel | {' | '.join(grid + wg)} | calls | total ms | avg us | max us |")
    print("|---|" + "---|" * (len(grid) + len(wg)) + "---|---|---|---|")
    for k, (n, tot, mx) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print(f"| {k[0]} | {' | '.join(str(x) for x in k[1:])} | {n} | {tot:.1f} | {1000 * tot / n:.1f} | {1000 * mx:.1f} |")


if __name__ == "__main__":
    main()
