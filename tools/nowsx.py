#!/usr/bin/env python3
"""Same-box A/B helper: run a script with the split GRU cluster kernel (gru_wsx.hip) off, every
GRU launch on the batch-parallel split kernel (gru_x3). Usage: python tools/nowsx.py SCRIPT ARGS..."""
import os
import runpy
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from igaming_platform_amd.ops import kernels as K  # noqa: E402

_init = K.GruPack.__init__


def _init_nowsx(self, *a, **k):
    _init(self, *a, **k)
    self.wsx_ok = False


K.GruPack.__init__ = _init_nowsx
sys.argv = sys.argv[1:]
runpy.run_path(sys.argv[0], run_name="__main__")
