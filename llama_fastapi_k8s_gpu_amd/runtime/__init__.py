"""Native runtime bindings.

``load_hip()`` / ``load_cpu()`` import the in-tree extensions built by
``runtime/build.py``. They fail loudly when the extension is missing instead of
silently falling back to Python (a GPU test that passes on a fallback would be
measuring the wrong code).
"""
from __future__ import annotations

import importlib
import os

_MODS = {}


def _load(name: str, builder: str):
    if name in _MODS:
        return _MODS[name]
    try:
        mod = importlib.import_module(f"{__name__}.{name}")
    except ImportError as e:
        if os.environ.get("LFK_AUTOBUILD", "1") != "0":
            from . import build
            getattr(build, builder)(verbose=False)
            importlib.invalidate_caches()
            mod = importlib.import_module(f"{__name__}.{name}")
        else:
            raise ImportError(f"native extension {name} is not built: run "
                              f"`python -m llama_fastapi_k8s_gpu_amd.runtime.build` ({e})") from e
    _MODS[name] = mod
    return mod


def load_hip():
    # torch first: its libtorch_hip loads the HIP runtime torch ships (soname libamdhip64.so.7,
    # file name libamdhip64.so), and the extension's libamdhip64.so.7 / librccl.so.1 then
    # resolve to those same copies by soname. Loaded the other way round, the extension pulls
    # in /opt/rocm's runtime and torch adds its own by file name - two HIP runtimes in one
    # process, and torch.cuda reports no device.
    if "_hip" not in _MODS:
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
    return _load("_hip", "build_hip")


def load_cpu():
    return _load("_cpu", "build_cpu")
