"""BD-rate table from tools/gpu/rd_knob.sh's summary.txt: every knob value against the first.

usage: python tools/bd_knob.py gpurun_out/<outdir>/summary.txt [title]
"""
import collections
import sys

from rd_table import bd_rate  # noqa: E402  (tools/ on sys.path when run as a script)


def main():
    rows = collections.OrderedDict()
    for line in open(sys.argv[1]):
        f = line.split()
        if len(f) < 5:
            continue
        rows.setdefault(f[0], []).append((float(f[1]), float(f[2]), float(f[3]), 0.0, float(f[4])))
    title = sys.argv[2] if len(sys.argv) > 2 else "knob sweep"
    print(f"# {title}\n")
    print("| setting | CRF | kb/s | PSNR-Y dB | fps (64 segments) |")
    print("|---|---|---|---|---|")
    for k, pts in rows.items():
        for crf, kbps, psnr, _, fps in pts:
            print(f"| {k} | {crf:g} | {kbps:.1f} | {psnr:.3f} | {fps:.0f} |")
    keys = list(rows)
    print("\n| setting | BD-rate vs " + keys[0] + " (PSNR-Y) |")
    print("|---|---|")
    for k in keys[1:]:
        print(f"| {k} | {bd_rate(rows[keys[0]], rows[k]):+.2f} % |")


if __name__ == "__main__":
    main()
