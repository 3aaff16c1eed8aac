#!/usr/bin/env python3
"""Per-kernel summary of a rocprofv3 --kernel-trace database (rocpd SQLite).

    python tools/kstats.py gpurun_out/prof/run_results.db [--last-ms N] [--top K]

Prints calls / total / average per kernel name (sorted by total), plus the busy
span of the whole trace.  ``--after-ms`` restricts to dispatches that start at
least N ms after the first one (e.g. to skip the warmup step).
"""
import argparse
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--after-ms", type=float, default=0.0)
    ap.add_argument("--top", type=int, default=30)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, start, end from kernels order by start").fetchall()
    if not rows:
        print("no kernels")
        return
    t0 = rows[0][1] + a.after_ms * 1e6
    rows = [r for r in rows if r[1] >= t0]
    agg: dict[str, list] = {}
    for name, s, e in rows:
        k = name.split("(")[0][:60]
        v = agg.setdefault(k, [0, 0.0])
        v[0] += 1
        v[1] += (e - s) / 1e6
    tot = sum(v[1] for v in agg.values())
    span = (max(r[2] for r in rows) - min(r[1] for r in rows)) / 1e6
    busy, cur_s, cur_e = 0.0, None, None
    for _, s, e in rows:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += (cur_e - cur_s) / 1e6
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += (cur_e - cur_s) / 1e6
    print(f"{'kernel':60s} {'calls':>7s} {'total ms':>10s} {'avg us':>10s} {'%':>6s}")
    for k, (n, ms) in sorted(agg.items(), key=lambda kv: -kv[1][1])[: a.top]:
        print(f"{k:60s} {n:7d} {ms:10.1f} {ms / n * 1000:10.1f} {100 * ms / tot:6.1f}")
    print(f"kernel total {tot:.1f} ms; trace span {span:.1f} ms, GPU busy {busy:.1f} ms, idle {span - busy:.1f} ms")


if __name__ == "__main__":
    main()
