#!/usr/bin/env python3
"""Sum rocprofv3 --pmc counters per kernel from a rocpd SQLite database.

    python tools/pmc_summary.py gpurun_out/pmc/run_results.db [--per-dispatch]

Counters are summed over shader engines per dispatch; the mean over dispatches of
each kernel is printed, with instructions per wave (counter / SQ_WAVES when present,
else / workgroups x waves per workgroup).
"""
import collections
import sqlite3
import sys


def main():
    c = sqlite3.connect(sys.argv[1])
    rows = c.execute("select dispatch_id, kernel_name, counter_name, value, grid_size, workgroup_size, duration "
                     "from counters_collection").fetchall()
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    meta = {}
    for d, k, n, v, gs, ws, dur in rows:
        per[(k.split("(")[0], d)][n] += v
        meta[(k.split("(")[0], d)] = (gs, ws, dur)
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for (k, d), cs in per.items():
        gs, ws, dur = meta[(k, d)]
        waves = gs / 64.0
        for n, v in cs.items():
            agg[k][n].append(v)
        agg[k]["_waves"].append(waves)
        agg[k]["_dur_ms"].append(dur / 1e6)
    for k, cs in agg.items():
        n = len(cs["_waves"])
        waves = sum(cs["_waves"]) / n
        print(f"{k}  dispatches={n}  waves={waves:.0f}  dur={sum(cs['_dur_ms']) / n:.3f} ms")
        for name, vs in sorted(cs.items()):
            if name.startswith("_"):
                continue
            m = sum(vs) / len(vs)
            extra = f"  per-wave {m / waves:.1f}" if name.startswith("SQ_INSTS") or name == "SQ_WAVE_CYCLES" else ""
            print(f"  {name:24s} {m:16.0f}{extra}")


if __name__ == "__main__":
    main()
