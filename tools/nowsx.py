#!/usr/bin/env python3
"""Same-box A/B helper for the split GRU cluster kernel (gru_wsx.hip).
Usage: python tools/nowsx.py [--off | --serving-on] SCRIPT ARGS...
  --off         every GRU launch on the batch-parallel split kernel (gru_x3)
  --serving-on  the serving abuse device runs its <= 256-row steps on the clusters
                (AbuseConfig.cluster_kernel = True)"""
import os
import runpy
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

mode = "--off"
if sys.argv[1] in ("--off", "--serving-on"):
    mode = sys.argv.pop(1)
if mode == "--off":
    from igaming_platform_amd.ops import kernels as K

    _init = K.GruPack.__init__

    def _init_off(self, *a, **k):
        _init(self, *a, **k)
        self.wsx_ok = False

    K.GruPack.__init__ = _init_off
else:
    from igaming_platform_amd.engine import acct as A

    _dinit = A.AbuseNativeDevice.__init__

    def _init_on(self, *a, **k):
        k["cluster_kernel"] = True
        _dinit(self, *a, **k)

    A.AbuseNativeDevice.__init__ = _init_on
sys.argv = sys.argv[1:]
runpy.run_path(sys.argv[0], run_name="__main__")
