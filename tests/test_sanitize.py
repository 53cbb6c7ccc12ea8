"""the host C++ runtime (wire codec, ONNX reader / executor, account and link
indexes, CPU scorer) under AddressSanitizer + UndefinedBehaviorSanitizer: the native, C++-backed
engine and gRPC API tests run against the ``--sanitize`` build in a child interpreter with
libasan preloaded. GPU sanitizers are not available on the pool; the kernels are covered by
the bounds checks in their bindings and the GPU numerics tests."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _gcc_lib(name):
    p = subprocess.run(["gcc", f"-print-file-name={name}"], capture_output=True, text=True).stdout.strip()
    return p if p and os.path.isabs(p) and os.path.exists(p) else None


@pytest.mark.timeout(900)
def test_native_runtime_under_asan_ubsan():
    lib, std = _gcc_lib("libasan.so"), _gcc_lib("libstdc++.so.6")
    if lib is None or std is None:
        pytest.skip("no libasan / libstdc++ in this toolchain")
    from igaming_platform_amd import _build
    so = _build.build_native(sanitize=True)
    # libstdc++ preloaded beside the ASan runtime: python itself does not link it, and ASan's
    # __cxa_throw interceptor needs the real symbol at startup (C++ exceptions cross pybind11)
    env = dict(os.environ, LD_PRELOAD=f"{lib} {std}", IGP_NATIVE_SO=so, IGP_AUTOBUILD="0",
               ASAN_OPTIONS="detect_leaks=0:abort_on_error=0:halt_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    tests = ["tests/test_native.py", "tests/test_engine_cpu.py", "tests/test_api.py"]
    # -s: a sanitizer report goes straight to our pipe (pytest's capture would swallow it when
    # halt_on_error ends the child)
    p = subprocess.run([sys.executable, "-m", "pytest", "-x", "-q", "-s", "-p", "no:cacheprovider", "-m", "not gpu",
                        *tests],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=840)
    out = p.stdout + p.stderr
    assert "ERROR: AddressSanitizer" not in out, out[-4000:]
    assert "runtime error:" not in out, out[-4000:]
    assert p.returncode == 0, out[-4000:]
