#!/usr/bin/env python3
"""Where the 64-row split chain differs from the 32-row one (rows, magnitude, vs fp64)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import torch
    from igaming_platform_amd.models.plan import DenseStep, HeadStep
    from igaming_platform_amd.ops import kernels as K
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(8)
    steps = [DenseStep(n=512, k=k, act="relu", w_np=rng.normal(0, 1 / np.sqrt(k), (512, k)).astype(np.float32),
                       b_np=rng.normal(0, 0.05, 512).astype(np.float32)) for k in (256, 512, 512)]
    steps.append(HeadStep(n1=512, k=512, act1="relu", act2="none",
                          w1_np=rng.normal(0, 1 / np.sqrt(512), (512, 512)).astype(np.float32),
                          b1_np=rng.normal(0, 0.05, 512).astype(np.float32),
                          w2_np=rng.normal(0, 1 / np.sqrt(512), 512).astype(np.float32), b2=0.1))
    pk = K.MlpChainPack(steps, dev, split=True)
    n = 1500
    X = torch.from_numpy(rng.normal(0, 1, (n, 256)).astype(np.float32)).to(dev)
    h = X.double()
    for s in steps[:-1]:
        h = torch.relu(h @ torch.from_numpy(s.w_np).to(dev).double().T + torch.from_numpy(s.b_np).to(dev).double())
    hs = steps[-1]
    z = torch.relu(h @ torch.from_numpy(hs.w1_np).to(dev).double().T + torch.from_numpy(hs.b1_np).to(dev).double())
    ref = (z @ torch.from_numpy(hs.w2_np).to(dev).double() + hs.b2).cpu().numpy()
    outs = {}
    for rows in ("32", "64", "64", "32"):
        os.environ["IGP_MLP_SPLIT_ROWS"] = rows
        ml = torch.full((n,), -7.0, device=dev)
        K.mlp_chain(pk, n, X=X, ml=ml)
        torch.cuda.synchronize()
        o = ml.cpu().numpy()
        print(rows, "err vs fp64", float(np.abs(o - ref).max() / np.abs(ref).max()))
        if rows in outs:
            print(rows, "repeat identical:", bool(np.array_equal(outs[rows], o)))
        outs[rows] = o
    d = np.abs(outs["32"] - outs["64"])
    bad = np.nonzero(d > 0)[0]
    print("differing rows", len(bad), "max", float(d.max()), "first", bad[:20].tolist(),
          "by row%64", np.bincount(bad % 64, minlength=64).tolist())


if __name__ == "__main__":
    main()
