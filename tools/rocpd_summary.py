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
    if path.endswith(".db"):
        out += timeline(path)
    print("\n".join(out))


def _union(iv):
    """Sorted (start, end) intervals -> merged busy intervals."""
    merged = []
    for st, en in sorted(iv):
        if merged and st <= merged[-1][1]:
            merged[-1][1] = max(merged[-1][1], en)
        else:
            merged.append([st, en])
    return merged


def timeline(path, top=12):
    """Busy share of the device (union of every kernel interval, any queue) and of each queue,
    and the longest idle gaps of the device with their offsets from the first kernel."""
    c = sqlite3.connect(path)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    qcol = next((q for q in ("stream_id", "queue_id") if q in cols), None)
    rows = c.execute(f"select start, end, name{', ' + qcol if qcol else ''} from kernels").fetchall()
    if not rows:
        return []
    t0 = min(r[0] for r in rows)
    t1 = max(r[1] for r in rows)
    span = t1 - t0
    busy = _union([(r[0], r[1]) for r in rows])
    bsum = sum(e - s for s, e in busy)
    out = ["", f"## Timeline: device busy {100.0 * bsum / span:.1f} % of the {span / 1e6:.1f} ms span "
               f"(union of kernel intervals over every queue)", ""]
    if qcol:
        out += [f"| {qcol} | kernels | busy ms | busy % of span |", "|---|---|---|---|"]
        per = defaultdict(list)
        for r in rows:
            per[r[3]].append((r[0], r[1]))
        for q, iv in sorted(per.items(), key=lambda kv: -len(kv[1])):
            u = _union(iv)
            b = sum(e - s for s, e in u)
            out.append(f"| {q} | {len(iv)} | {b / 1e6:.1f} | {100.0 * b / span:.1f} |")
        out.append("")
    gaps = [(busy[i + 1][0] - busy[i][1], busy[i][1]) for i in range(len(busy) - 1)]
    gaps.sort(reverse=True)
    out += [f"Idle gaps: {sum(g for g, _ in gaps) / 1e6:.1f} ms in {len(gaps)} gaps; the longest:", "",
            "| gap ms | at ms (from first kernel) | last kernel before | first kernel after |", "|---|---|---|---|"]
    ends = sorted(rows, key=lambda r: r[1])
    starts = sorted(rows, key=lambda r: r[0])
    import bisect
    end_t = [r[1] for r in ends]
    start_t = [r[0] for r in starts]
    for g, at in gaps[:top]:
        i = bisect.bisect_right(end_t, at) - 1
        j = bisect.bisect_left(start_t, at + g)
        before = ends[i][2][:40] if i >= 0 else "-"
        after = starts[j][2][:40] if j < len(starts) else "-"
        out.append(f"| {g / 1e6:.2f} | {(at - t0) / 1e6:.1f} | {before} | {after} |")
    # steady state: the trailing half of the span (a bench run's timed steps, past its startup
    # and warmup), where a throughput number is measured
    w0 = t1 - span // 2
    clip = [(max(r[0], w0), r[1]) for r in rows if r[1] > w0]
    sb = sum(e - s for s, e in _union(clip))
    out += ["", f"## Steady state (the last {span / 2e6:.1f} ms): device busy {100.0 * sb / (t1 - w0):.1f} %", ""]
    if qcol:
        out += [f"| {qcol} | busy % of the window |", "|---|---|"]
        per = defaultdict(list)
        for r in rows:
            if r[1] > w0:
                per[r[3]].append((max(r[0], w0), r[1]))
        for q, iv in sorted(per.items(), key=lambda kv: -len(kv[1])):
            b = sum(e - s for s, e in _union(iv))
            out.append(f"| {q} | {100.0 * b / (t1 - w0):.1f} |")
    return out


if __name__ == "__main__":
    main()
