"""Build the two in-tree native extensions.

* ``_native``: host runtime (C++17, g++): ONNX reader, CPU executor, tree compiler,
  risk.v1 wire codec, account index. No GPU dependency.
* ``_hipk``: HIP kernels for gfx950 (hipcc) + their launch bindings. Links the HIP runtime
  by soname ``libamdhip64.so.7`` with an rpath to torch's bundled copy, so the process has
  exactly one HIP runtime (torch's) whether torch or the extension is loaded first.

Incremental: objects are rebuilt when the source or any header under ``csrc/`` is newer.
Usage: ``python -m igaming_platform_amd._build [--force] [--only native|hipk] [--sanitize]``.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import os
import subprocess
import sys
import sysconfig
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "igaming_platform_amd")
CSRC = os.path.join(ROOT, "csrc")
BUILD = os.path.join(ROOT, "build")
EXT = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950").split(";")[0]


def _py_includes():
    import pybind11
    return ["-I" + sysconfig.get_paths()["include"], "-I" + pybind11.get_include()]


def _torch_lib():
    import importlib.util
    spec = importlib.util.find_spec("torch")
    if spec is None or not spec.origin:
        return None
    return os.path.join(os.path.dirname(spec.origin), "lib")


def _headers_mtime():
    hs = glob.glob(os.path.join(CSRC, "**", "*.h"), recursive=True)
    hs += glob.glob(os.path.join(CSRC, "**", "*.cuh"), recursive=True)
    return max((os.path.getmtime(h) for h in hs), default=0.0)


def _compile(cmd, src, obj, force):
    if not force and os.path.exists(obj):
        if os.path.getmtime(obj) >= max(os.path.getmtime(src), _headers_mtime()):
            return obj, 0.0, ""
    os.makedirs(os.path.dirname(obj), exist_ok=True)
    t = time.time()
    full = cmd + ["-c", src, "-o", obj]
    p = subprocess.run(full, capture_output=True, text=True)
    if p.returncode != 0:
        raise RuntimeError(f"compile failed: {' '.join(full)}\n{p.stdout}\n{p.stderr}")
    return obj, time.time() - t, p.stderr


def build_native(force=False, sanitize=False, jobs=8):
    srcs = sorted(glob.glob(os.path.join(CSRC, "runtime", "*.cpp")))
    out = os.path.join(PKG, "_native" + EXT)
    flags = ["g++", "-std=c++17", "-O2", "-fPIC", "-fvisibility=hidden", "-Wall", "-Wno-sign-compare",
             "-I" + os.path.join(CSRC, "include")] + _py_includes()
    sub = "native-asan" if sanitize else "native"
    if sanitize:
        flags += ["-fsanitize=address,undefined", "-fno-omit-frame-pointer", "-g"]
        out = os.path.join(BUILD, "asan", "_native" + EXT)
    objs = []
    with cf.ThreadPoolExecutor(jobs) as ex:
        futs = [ex.submit(_compile, flags, s, os.path.join(BUILD, sub, os.path.basename(s) + ".o"), force)
                for s in srcs]
        for f in futs:
            objs.append(f.result()[0])
    if force or not os.path.exists(out) or os.path.getmtime(out) < max(os.path.getmtime(o) for o in objs):
        os.makedirs(os.path.dirname(out), exist_ok=True)
        link = ["g++", "-shared", "-o", out] + objs + (["-fsanitize=address,undefined"] if sanitize else [])
        subprocess.run(link, check=True)
    return out


def build_hipk(force=False, jobs=8):
    srcs = sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip")))
    if not srcs:
        return None
    out = os.path.join(PKG, "_hipk" + EXT)
    tl = _torch_lib()
    flags = ["hipcc", f"--offload-arch={ARCH}", "-std=c++17", "-O3", "-fPIC",
             "-fvisibility=hidden", "-ffp-contract=off",
             "-I" + os.path.join(CSRC, "include")] + _py_includes()
    objs = []
    with cf.ThreadPoolExecutor(jobs) as ex:
        futs = [ex.submit(_compile, flags, s, os.path.join(BUILD, "hipk", os.path.basename(s) + ".o"), force)
                for s in srcs]
        for f in futs:
            objs.append(f.result()[0])
    if force or not os.path.exists(out) or os.path.getmtime(out) < max(os.path.getmtime(o) for o in objs):
        link = ["hipcc", f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", out] + objs
        if tl:
            link += ["-L" + tl, "-Wl,-rpath," + tl]
        subprocess.run(link, check=True)
    return out


def build(force=False, only=None, sanitize=False):
    outs = []
    if only in (None, "native"):
        outs.append(build_native(force=force, sanitize=sanitize))
    if only in (None, "hipk"):
        outs.append(build_hipk(force=force))
    return [o for o in outs if o]


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--only", choices=["native", "hipk"])
    ap.add_argument("--sanitize", action="store_true", help="host runtime with ASan/UBSan")
    a = ap.parse_args(argv)
    for o in build(force=a.force, only=a.only, sanitize=a.sanitize):
        print("built", os.path.relpath(o, ROOT))


if __name__ == "__main__":
    sys.exit(main())
