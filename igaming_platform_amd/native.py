"""Loader for the in-tree native extensions.

``_native`` (host C++ runtime) is required everywhere. ``_hipk`` (gfx950 kernels) is required
whenever a GPU is visible: GPU code paths never silently fall back to PyTorch ops — if the
extension is missing or fails to load on a GPU box, :func:`hipk` raises.
"""
from __future__ import annotations

import importlib
import os
import threading

_lock = threading.Lock()
_native = None
_hipk = None
_hipk_err = None


def _autobuild_enabled() -> bool:
    return os.environ.get("IGP_AUTOBUILD", "1") != "0"


def _load_so(name: str, path: str):
    """Import extension ``name`` from an explicit file (IGP_NATIVE_SO: the ASan/UBSan build)."""
    import importlib.util
    import sys
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    sys.modules[name] = mod
    return mod


def native():
    global _native
    if _native is None:
        with _lock:
            if _native is None:
                so = os.environ.get("IGP_NATIVE_SO")
                if so:
                    _native = _load_so("igaming_platform_amd._native", so)
                    return _native
                try:
                    _native = importlib.import_module("igaming_platform_amd._native")
                except ImportError:
                    if not _autobuild_enabled():
                        raise
                    from . import _build
                    _build.build(only="native")
                    _native = importlib.import_module("igaming_platform_amd._native")
    return _native


def hipk():
    """The HIP kernel module. Raises if it cannot be loaded (no silent fallback)."""
    global _hipk, _hipk_err
    if _hipk is None:
        with _lock:
            if _hipk is None:
                import torch  # noqa: F401  (load torch's HIP runtime first: one runtime per process)
                try:
                    _hipk = importlib.import_module("igaming_platform_amd._hipk")
                except ImportError as e:
                    if _autobuild_enabled():
                        from . import _build
                        _build.build(only="hipk")
                        _hipk = importlib.import_module("igaming_platform_amd._hipk")
                    else:
                        _hipk_err = e
                        raise RuntimeError(
                            "igaming_platform_amd._hipk (gfx950 kernels) is not built; run "
                            "`python -m igaming_platform_amd._build`") from e
    return _hipk


def gpu_available() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False
