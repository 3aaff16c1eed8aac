"""Join the per-pass summaries of tools/gpu/pmc_bench.sh (p1..p4.summary.txt: counters per
kernel from tools/pmc_summary.py) into one markdown roofline table of the top kernels.

usage: python tools/pmc_table.py DIR [title] [top]
"""
import os
import re
import sys


def parse(path):
    out, cur = {}, None
    for line in open(path):
        m = re.match(r"^(\S.*?)\s+dispatches=(\d+)\s+waves=(\d+)\s+dur=([\d.]+) ms", line)
        if m:
            cur = m.group(1)
            out.setdefault(cur, {}).update(dispatches=int(m.group(2)), waves=int(m.group(3)), dur=float(m.group(4)))
            continue
        m = re.match(r"^\s+(\w+)\s+(-?[\d.]+)", line)
        if m and cur:
            out[cur][m.group(1)] = float(m.group(2))
    return out


def main():
    d = sys.argv[1]
    title = sys.argv[2] if len(sys.argv) > 2 else d
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 14
    k = {}
    for p in ("p1", "p2", "p3", "p4"):
        f = os.path.join(d, p + ".summary.txt")
        if os.path.exists(f):
            for name, v in parse(f).items():
                k.setdefault(name, {}).update(v)
    rows = sorted(((n, v) for n, v in k.items() if "mivc" in n), key=lambda kv: -kv[1].get("dur", 0) * kv[1].get("dispatches", 0))
    print(f"# {title}\n")
    print("Mean per dispatch of each kernel (counters summed over shader engines).  `VALU active` = "
          "SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES (share of wave cycles issuing VALU); fetched / written "
          "MiB from FETCH_SIZE / WRITE_SIZE (KiB counters).\n")
    print("| kernel | calls | ms / call | waves | VALU / wave | MFMA / wave | LDS / wave | VMEM rd / wave | VALU active % | LDS bank conflicts / wave | fetched MiB / call | written MiB / call |")
    print("|---|---|---|---|---|---|---|---|---|---|---|---|")
    for n, v in rows[:top]:
        w = max(1.0, v.get("waves", 1))
        va = 100.0 * v.get("SQ_ACTIVE_INST_VALU", 0) / max(1.0, v.get("SQ_WAVE_CYCLES", 0)) if v.get("SQ_WAVE_CYCLES") else 0.0
        fetch, wr = v.get("FETCH_SIZE", 0) / 1024.0, v.get("WRITE_SIZE", 0) / 1024.0  # KiB -> MiB
        name = re.sub(r"\(.*", "", n.replace("void ", "").replace("mivc::gpu::", ""))[:48]
        print(f"| `{name}` | {v.get('dispatches', 0)} | {v.get('dur', 0):.3f} | {int(w)} | {v.get('SQ_INSTS_VALU', 0) / w:.0f} | "
              f"{v.get('SQ_INSTS_MFMA', 0) / w:.1f} | {v.get('SQ_INSTS_LDS', 0) / w:.0f} | {v.get('SQ_INSTS_VMEM_RD', 0) / w:.1f} | "
              f"{va:.1f} | {v.get('SQ_LDS_BANK_CONFLICT', 0) / w:.1f} | {fetch:.2f} | {wr:.2f} |")


if __name__ == "__main__":
    main()
