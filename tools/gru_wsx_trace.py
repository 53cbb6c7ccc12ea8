#!/usr/bin/env python3
"""Per-step phase times of the split weight-stationary GRU clusters (csrc/kernels/gru_wsx.hip):
workgroup 0's layer-2 / K-half-1 wave stamps wall_clock64 (100 MHz) at step start, MFMAs done,
after barrier A (partials combined), own columns written, published (stores acked), counter
reached, gathered. Also the kernel time for a few batch sizes.

Usage: python tools/gru_wsx_trace.py [--rows 32] [--T 100]"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=32)
    ap.add_argument("--T", type=int, default=100)
    a = ap.parse_args()
    import torch
    from igaming_platform_amd.models.plan import compile_onnx, to_device
    from igaming_platform_amd.native import native
    from igaming_platform_amd.ops import kernels as K
    from igaming_platform_amd.onnx import builders
    m = native().OnnxModel.from_bytes(builders.build("gru", seq=a.T, in_dim=16, hidden=256).SerializeToString())
    plan = to_device(compile_onnx(m), "cuda", "fp32")
    gp = K.GruPack([s for s in plan.steps if s.kind == "gru"], plan.steps[-1], "cuda", split=True)
    res = {}
    for rows in sorted({1, 32, 64, 128, a.rows}):
        X = torch.randn(a.T, rows, 16, device="cuda")
        out = torch.zeros(rows, device="cuda")
        for ws, name in ((3, "clusters"), (0, "batch_parallel")):
            for _ in range(3):
                K.gru(gp, rows, a.T, out=out, X=X, ws=ws)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                K.gru(gp, rows, a.T, out=out, X=X, ws=ws)
            e1.record()
            e1.synchronize()
            res[f"{name}_{rows}_us"] = round(e0.elapsed_time(e1) * 100, 1)
    X = torch.randn(a.T, a.rows, 16, device="cuda")
    out = torch.zeros(a.rows, device="cuda")
    tr = torch.zeros(64 * 8 + 4 + 1024, dtype=torch.int64, device="cuda")
    K.gru(gp, a.rows, a.T, out=out, X=X, ws=3, ws_trace=tr)
    torch.cuda.synchronize()
    t = tr[:64 * 8].cpu().numpy().reshape(64, 8).astype(np.float64)
    steps = t[2:62]
    d = np.diff(steps[:, :7], axis=1) / 100.0  # us between consecutive marks
    names = ["mfma", "barrier_A", "combine+own_cols", "publish", "counter", "gather"]
    res["phase_us_median"] = {n: round(float(np.median(d[:, k])), 2) for k, n in enumerate(names)}
    res["step_us_median"] = round(float(np.median(np.diff(steps[:, 0]) / 100.0)), 2)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
