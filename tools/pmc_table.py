#!/usr/bin/env python3
"""Roofline-style table from the per-pass summaries of tools/gpu/pmc_bench.sh.

    python tools/pmc_table.py gpurun_out/pmc_dir [--top 12] > profiles/xx_pmc.md

Per kernel (mean per dispatch): duration, VALU issue rate as a fraction of the gfx950
VALU issue peak (256 CUs x 4 SIMDs, one wave64 instruction per 2 cycles per SIMD, at
2.4 GHz), LDS instructions and bank-conflict cycles per CU-cycle, MFMA busy, HBM traffic
(FETCH_SIZE + WRITE_SIZE, KiB) and its rate as a fraction of 8 TB/s, and the limiter
read off those numbers.
"""
import argparse
import collections
import os
import re

CUS, CLK = 256, 2.4e9
VALU_PEAK = CUS * 4 * 0.5 * CLK  # wave64 VALU instructions / s
HBM = 8.0e12


def parse(path):
    out = {}
    cur = None
    if not os.path.exists(path):
        return out
    for line in open(path):
        m = re.match(r"^(\S.*?)\s+dispatches=(\d+)\s+waves=(\d+)\s+dur=([\d.]+) ms", line)
        if m:
            cur = m.group(1).replace("void ", "").split("<")[0].replace("mivc::gpu::", "")
            d = out.setdefault(cur, {"disp": int(m.group(2)), "dur_ms": float(m.group(4))})
            continue
        m = re.match(r"^\s+(\w+)\s+([\d.]+)", line)
        if m and cur is not None:
            out[cur][m.group(1)] = float(m.group(2))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--top", type=int, default=12)
    a = ap.parse_args()
    merged = collections.defaultdict(dict)
    for p in ("p1", "p2", "p3", "p4"):
        for k, v in parse(os.path.join(a.dir, f"{p}.summary.txt")).items():
            merged[k].update(v)
    rows = sorted(merged.items(), key=lambda kv: -kv[1].get("dur_ms", 0) * kv[1].get("disp", 0))[: a.top]
    print("| kernel | disp | ms/disp | VALU inst/wave | VALU issue % of peak | MFMA busy % | LDS inst/wave | "
          "LDS conflict % of CU-cycles | HBM MB/disp | HBM % of 8 TB/s | limiter |")
    print("|---|---|---|---|---|---|---|---|---|---|---|")
    for k, v in rows:
        t = v.get("dur_ms", 0) / 1e3
        waves = max(v.get("SQ_WAVES", 1), 1)
        valu = v.get("SQ_INSTS_VALU", 0)
        valu_pct = 100 * valu / t / VALU_PEAK if t else 0
        gui = v.get("GRBM_GUI_ACTIVE", 0)
        mfma = 100 * v.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / (CUS * 4 * t * CLK) if t else 0
        lds = v.get("SQ_INSTS_LDS", 0)
        confl = 100 * v.get("SQ_LDS_BANK_CONFLICT", 0) / (CUS * t * CLK) if t else 0
        mb = (v.get("FETCH_SIZE", 0) + v.get("WRITE_SIZE", 0)) / 1024.0
        hbm = 100 * mb * 1e6 / t / HBM if t else 0
        if hbm > 50:
            lim = "HBM bandwidth"
        elif valu_pct > 40:
            lim = "VALU issue"
        elif confl > 15:
            lim = "LDS bank conflicts"
        elif waves < CUS * 4:
            lim = "occupancy / serial dependence (few waves)"
        else:
            lim = "latency (memory / LDS waits)"
        del gui
        print(f"| {k[:40]} | {v.get('disp', 0)} | {v.get('dur_ms', 0):.3f} | {valu / waves:.0f} | {valu_pct:.1f} | "
              f"{mfma:.2f} | {lds / waves:.0f} | {confl:.1f} | {mb:.1f} | {hbm:.1f} | {lim} |")


if __name__ == "__main__":
    main()
