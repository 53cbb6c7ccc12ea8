#!/usr/bin/env python3
"""Write the synthetic random-init ONNX models of the five BASELINE configs (deterministic by
seed; stands in for the reference's missing model-train/export scripts, Makefile:215-225)."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from igaming_platform_amd.onnx import builders, writer  # noqa: E402

MODELS = {
    "cfg1_logistic32.onnx": ("logistic", dict(n_features=32)),
    "cfg2_gbdt100.onnx": ("gbdt", dict(n_trees=100, depth=7, n_features=128)),
    "cfg3_stacked.onnx": ("stacked", dict(n_trees=100, depth=7, n_features=128, k=32)),
    "cfg4_ltv_mlp.onnx": ("ltv_mlp", dict(n_features=256, width=512, layers=4)),
    "cfg5_abuse_gru.onnx": ("gru", dict(seq=100, in_dim=16, hidden=256)),
}


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="models")
    a = ap.parse_args()
    os.makedirs(a.out, exist_ok=True)
    for name, (kind, kw) in MODELS.items():
        p = os.path.join(a.out, name)
        writer.save(builders.build(kind, **kw), p)
        print(f"{p}: {os.path.getsize(p)} bytes")
    return 0


if __name__ == "__main__":
    sys.exit(main())
