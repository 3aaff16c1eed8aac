"""In-tree native build driver (no pip, no JIT cache: the .so files land next to
this file so they travel with the repo snapshot to the GPU box).

* ``_host``: host C++ library (bitstream, CAVLC writer, independent decoder, CPU
  reference encoder, Annex-B/MP4 tools) -> g++ -O3, pybind11.
* ``_hip``: gfx950 HIP kernels + their pybind11 launch shims -> hipcc
  --offload-arch=gfx950 (cross-compiles without a GPU).

Usage: ``python -m govideocompressor_amd._build [host|hip|all] [-j N]``.
"""
from __future__ import annotations

import argparse
import glob
import os
import subprocess
import sys
import sysconfig
from concurrent.futures import ThreadPoolExecutor

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(PKG_DIR)
CSRC = os.path.join(REPO, "csrc")
BUILD = os.path.join(REPO, "build", "native")
EXT_SUFFIX = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
GPU_ARCH = os.environ.get("MIVC_GPU_ARCH", "gfx950")


def _pybind_includes() -> list[str]:
    import pybind11

    return [pybind11.get_include(), sysconfig.get_paths()["include"]]


def _headers(*dirs: str) -> list[str]:
    out: list[str] = []
    for d in dirs:
        out += glob.glob(os.path.join(CSRC, d, "*.h"))
    return out


def _stale(target: str, deps: list[str]) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _run(cmd: list[str]) -> None:
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(" ".join(cmd) + "\n" + r.stdout + r.stderr)
        raise RuntimeError(f"native build failed: {os.path.basename(cmd[-1])}")


def _compile_many(jobs: list[tuple[list[str], str, list[str]]], nproc: int) -> None:
    todo = [(cmd, out) for cmd, out, deps in jobs if _stale(out, deps)]
    if not todo:
        return
    with ThreadPoolExecutor(max_workers=max(1, nproc)) as ex:
        list(ex.map(lambda c: _run(c[0]), todo))


def host_library_path() -> str:
    return os.path.join(PKG_DIR, "_host" + EXT_SUFFIX)


def hip_library_path() -> str:
    return os.path.join(PKG_DIR, "_hip" + EXT_SUFFIX)


def sanitized_host_path() -> str:
    """ASan + UBSan build of ``_host`` (outside the package: loaded only through
    ``MIVC_HOST_LIB``, see ops/native.py)."""
    return os.path.join(BUILD, "asan", "_host" + EXT_SUFFIX)


def build_host(nproc: int = 8, sanitize: bool = False) -> str:
    """``sanitize``: -fsanitize=address,undefined -O1 build for the parser hardening runs
    (tools/asan_tests.sh: LD_PRELOAD=libasan, MIVC_HOST_LIB=<this>, the CPU test suite
    and the fuzz tests)."""
    srcs = sorted(glob.glob(os.path.join(CSRC, "host", "*.cc")))
    hdrs = _headers("common", "host")
    sub = "asan" if sanitize else "host"
    os.makedirs(os.path.join(BUILD, sub), exist_ok=True)
    if sanitize:
        # shift-base: the transform/quant arithmetic left-shifts negative values, which is
        # two's-complement-defined since C++20 (and what g++/hipcc emit in C++17 mode)
        flags = ["-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined", "-fno-sanitize=shift-base",
                 "-fno-sanitize-recover=undefined"]
    else:
        flags = ["-O3"]
    flags += ["-std=c++17", "-fPIC", "-fvisibility=hidden", "-Wall", "-Wno-unused-function"]
    flags += [f"-I{p}" for p in _pybind_includes()]
    jobs = []
    objs = []
    for s in srcs:
        o = os.path.join(BUILD, sub, os.path.basename(s) + ".o")
        objs.append(o)
        jobs.append((["g++", *flags, "-c", s, "-o", o], o, [s, *hdrs]))
    _compile_many(jobs, nproc)
    out = sanitized_host_path() if sanitize else host_library_path()
    if _stale(out, objs):
        link = ["-fsanitize=address,undefined"] if sanitize else []
        _run(["g++", "-shared", *link, "-o", out, *objs, "-lpthread"])
    return out


def build_hip(nproc: int = 8) -> str:
    srcs = sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip")))
    binds = sorted(glob.glob(os.path.join(CSRC, "kernels", "*.cc")))
    hdrs = _headers("common", "kernels")
    os.makedirs(os.path.join(BUILD, "hip"), exist_ok=True)
    hip_flags = [
        f"--offload-arch={GPU_ARCH}",
        "-O3",
        "-std=c++17",
        "-fPIC",
        "-fvisibility=hidden",
        "-munsafe-fp-atomics",
        "-Wno-unused-result", "-Wno-unused-value",
    ]
    jobs = []
    objs = []
    for s in srcs:
        o = os.path.join(BUILD, "hip", os.path.basename(s) + ".o")
        objs.append(o)
        jobs.append(([HIPCC, *hip_flags, "-c", s, "-o", o], o, [s, *hdrs]))
    host_flags = ["-O3", "-std=c++17", "-fPIC", "-fvisibility=hidden", "-D__HIP_PLATFORM_AMD__"]
    host_flags += [f"-I{p}" for p in _pybind_includes()] + ["-I/opt/rocm/include"]
    for s in binds:
        o = os.path.join(BUILD, "hip", os.path.basename(s) + ".o")
        objs.append(o)
        jobs.append((["g++", *host_flags, "-c", s, "-o", o], o, [s, *hdrs]))
    _compile_many(jobs, nproc)
    out = hip_library_path()
    if _stale(out, objs):
        _run([HIPCC, f"--offload-arch={GPU_ARCH}", "-shared", "-fPIC", "-o", out, *objs,
              "-L/opt/rocm/lib", "-lamdhip64"])
    return out


def build_all(nproc: int = 8) -> list[str]:
    return [build_host(nproc), build_hip(nproc)]


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("what", nargs="?", default="all", choices=["host", "hip", "all", "asan"])
    ap.add_argument("-j", type=int, default=min(8, os.cpu_count() or 4))
    a = ap.parse_args()
    if a.what in ("host", "all"):
        print(build_host(a.j))
    if a.what in ("hip", "all"):
        print(build_hip(a.j))
    if a.what == "asan":
        print(build_host(a.j, sanitize=True))


if __name__ == "__main__":
    main()
