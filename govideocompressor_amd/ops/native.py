"""Loaders for the in-tree native extensions.

``host()`` -> ``_host`` (C++: bitstream, CAVLC writer, independent decoder, CPU
encoder, Annex-B/MP4 tools).  ``hip()`` -> ``_hip`` (gfx950 kernels).

Both are built by :mod:`govideocompressor_amd._build` (``__graft_entry__.build``).
If a library is missing we try to build it once; on a GPU machine a missing or
unloadable ``_hip`` is a hard error -- there is deliberately no PyTorch/Python
fallback for the GPU encode path.
"""
from __future__ import annotations

import importlib
import importlib.machinery
import importlib.util
import os
import sys
import threading

_lock = threading.Lock()
_cache: dict[str, object] = {}


def _load(name: str, builder):
    with _lock:
        if name in _cache:
            return _cache[name]
        # MIVC_HOST_LIB: e.g. the ASan/UBSan build; MIVC_HIP_LIB: a kernel variant for same-box A/B
        # timing (tools/build_variant.py; bench.py --allow-knobs)
        override = os.environ.get("MIVC_HOST_LIB" if name == "_host" else "MIVC_HIP_LIB")
        if override:  # e.g. the ASan/UBSan build (_build.build_host(sanitize=True))
            full = f"govideocompressor_amd.{name}"
            loader = importlib.machinery.ExtensionFileLoader(full, override)
            spec = importlib.util.spec_from_file_location(full, override, loader=loader)
            mod = importlib.util.module_from_spec(spec)
            loader.exec_module(mod)
            sys.modules[full] = mod
            _cache[name] = mod
            return mod
        try:
            mod = importlib.import_module(f"govideocompressor_amd.{name}")
        except ImportError:
            if os.environ.get("MIVC_NO_AUTOBUILD"):
                raise
            builder()
            mod = importlib.import_module(f"govideocompressor_amd.{name}")
        _cache[name] = mod
        return mod


def host():
    """The host C++ library (always available on CPU)."""
    from .. import _build

    return _load("_host", _build.build_host)


def hip():
    """The gfx950 kernel library.  Raises if it cannot be loaded."""
    from .. import _build

    try:
        return _load("_hip", _build.build_hip)
    except Exception as e:  # pragma: no cover - exercised on broken installs only
        raise RuntimeError(
            "govideocompressor_amd: the gfx950 HIP extension (_hip) is not loadable; "
            "run `python -m govideocompressor_amd._build hip`. No eager fallback exists."
        ) from e


def gpu_available() -> bool:
    try:
        import torch

        return torch.cuda.is_available()
    except Exception:
        return False
