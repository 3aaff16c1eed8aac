#!/usr/bin/env python3
"""Build a complete gfx950 kernel library (the ``_hip`` extension) from a modified copy of
``csrc/`` for same-box A/B timing: bench.py loads it through ``MIVC_HIP_LIB`` (with
``--allow-knobs``), so two variants run back to back on one GPU box.

    python tools/build_variant.py NAME 'kernels/bframe.hip:s/old/new/' [more edits ...]
    python tools/build_variant.py NAME --patch my.diff

Each edit is ``FILE:s/REGEX/REPLACEMENT/`` (Python ``re``, applied once per match,
the file relative to csrc/).  Output: ``abso/NAME.so`` (git-ignored, shipped by gpurun).
"""
from __future__ import annotations

import argparse
import os
import re
import shutil
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("name")
    ap.add_argument("edits", nargs="*")
    ap.add_argument("--patch", default=None)
    ap.add_argument("--rev", default=None, help="build csrc/ as of this git revision (e.g. a baseline)")
    ap.add_argument("-j", type=int, default=8)
    a = ap.parse_args()
    from govideocompressor_amd import _build as B

    tmp = tempfile.mkdtemp(prefix=f"variant_{a.name}_")
    try:
        if a.rev:
            os.makedirs(os.path.join(tmp, "csrc"))
            tar = subprocess.run(["git", "-C", ROOT, "archive", a.rev, "csrc"], check=True, capture_output=True).stdout
            subprocess.run(["tar", "-x", "-C", tmp], input=tar, check=True)
        else:
            shutil.copytree(os.path.join(ROOT, "csrc"), os.path.join(tmp, "csrc"))
        for e in a.edits:
            f, sub = e.split(":", 1)
            m = re.fullmatch(r"s/(.*)/(.*)/", sub, re.S)
            if not m:
                raise SystemExit(f"bad edit {e!r}")
            path = os.path.join(tmp, "csrc", f)
            txt = open(path).read()
            new, n = re.subn(m.group(1), m.group(2), txt)
            if n == 0:
                raise SystemExit(f"edit {e!r} matched nothing")
            open(path, "w").write(new)
        if a.patch:
            subprocess.run(["patch", "-p1", "-d", tmp, "-i", os.path.abspath(a.patch)], check=True)
        B.CSRC = os.path.join(tmp, "csrc")
        B.BUILD = os.path.join(tmp, "build")
        out_dir = os.path.join(ROOT, "abso")
        os.makedirs(out_dir, exist_ok=True)
        B.hip_library_path = lambda: os.path.join(out_dir, a.name + ".so")  # noqa: E731
        print(B.build_hip(a.j))
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


if __name__ == "__main__":
    main()
