#!/usr/bin/env python3
"""cfg 4 LTV chain kernel alone (256 -> 4 x 512 -> 1, bf16), one launch at a time on one stream:
microseconds per launch and TFLOP/s for the one-workgroup kernel (32 / 64 rows per workgroup);
SPLIT=1: the f32-faithful chain at 32 / 64 rows, at several batch sizes. Checks that the
variants agree. Usage: python tools/mlp_bench.py [batches, default 8192,4096,16384]"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    import torch
    from igaming_platform_amd.models.plan import DenseStep, HeadStep
    from igaming_platform_amd.ops import kernels as K
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(0)
    steps = [DenseStep(n=512, k=k, act="relu", w_np=rng.normal(0, 0.05, (512, k)).astype(np.float32),
                       b_np=rng.normal(0, 0.1, 512).astype(np.float32)) for k in (256, 512, 512)]
    steps.append(HeadStep(n1=512, k=512, act1="relu", act2="none",
                          w1_np=rng.normal(0, 0.05, (512, 512)).astype(np.float32),
                          b1_np=rng.normal(0, 0.1, 512).astype(np.float32),
                          w2_np=rng.normal(0, 0.1, 512).astype(np.float32), b2=0.1))
    split = os.environ.get("SPLIT", "0") == "1"  # the f32-faithful chain (hi/lo bf16 pairs)
    pk = K.MlpChainPack(steps, dev, split=split)
    flop_row = 2 * (256 * 512 + 3 * 512 * 512 + 512)
    batches = [int(b) for b in (sys.argv[1] if len(sys.argv) > 1 else "8192,4096,16384").split(",")]
    res = []
    for B in batches:
        X = torch.from_numpy(rng.normal(0, 1, (B, 256)).astype(np.float32)).to(dev)
        ref = None
        variants = ((("split32", "32", False), ("split64", "64", False)) if split else
                    (("wg32", "32", False), ("wg64", "64", False)))
        for name, rows, _ in variants:
            os.environ["IGP_MLP_SPLIT_ROWS" if split else "IGP_MLP_ROWS"] = rows
            ml = torch.zeros(B, device=dev)
            run = lambda: K.mlp_chain(pk, B, X=X, ml=ml)  # noqa: E731
            for _ in range(3):
                run()
            torch.cuda.synchronize()
            if ref is None:
                ref = ml.clone()
            diff = float((ml - ref).abs().max())
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            ts = []
            for _ in range(20):
                e0.record()
                run()
                e1.record()
                e1.synchronize()
                ts.append(e0.elapsed_time(e1) * 1e3)
            us = float(np.median(ts))
            r = dict(batch=B, kernel=name, us=round(us, 2), tflops=round(flop_row * B / us / 1e6, 1),
                     pct_of_2500=round(flop_row * B / us / 1e6 / 25.0, 1), max_diff=diff)
            res.append(r)
            print(json.dumps(r), flush=True)
    with open(os.environ.get("OUT", "gpurun_out/mlp_bench.json"), "w") as f:
        json.dump(res, f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
