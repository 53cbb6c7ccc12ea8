#!/usr/bin/env python3
"""K2 tree-ensemble sweep on the cfg3 stacked model (100 trees, depth 7, K=32 leaf vectors):
tree groups per row tile, back-to-back launches per variant (launch overhead amortised).
The X rows are real K1 output of a synthetic batch. Checks that every variant reduces to the
same [rows, K] sums. Usage: python tools/tree_bench.py [--batch 8192]"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg3")
    ap.add_argument("--batch", type=int, default=0)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    import torch
    from igaming_platform_amd.ops import kernels as K
    from igaming_platform_amd.utils import benchkit
    from igaming_platform_amd.utils.synth import NOW0
    dev = torch.device("cuda", 0)
    S = benchkit.build(a.config, a.batch, 1 << 20, dev)
    sc, B = S.scorer, S.batch
    v = sc.slab_view(0, B)
    v[:] = S.pool[0]
    v["ts"] = NOW0
    sc._seq += 1
    sc._write_hdr(0, B, NOW0)
    nb = 16 + 48 * B
    sc.dev_slab[:nb].copy_(sc.host_slab[0][:nb])
    K.feature_assemble(sc.store, sc.hdr, sc.cfg_dev, sc.req, sc.X, sc.feat, B, dedup=False)
    torch.cuda.synchronize()
    tree = next(s for s in sc.plan.steps if s.kind == "tree")
    print(f"trees {tree.n_trees} depth {tree.depth} K {tree.k} batch {B} default groups {sc.tree_groups.get(B)}")
    ref = None
    out = []
    for g in (1, 2, 4, 8, 12):
        slab = torch.zeros(g * B * tree.k, dtype=torch.float32, device=dev)
        y = torch.zeros(B, tree.n_out, dtype=torch.float32, device=dev)
        if g == 1:
            run = lambda: K.tree_ensemble(tree, sc.X, y, B)  # noqa: E731
        else:
            run = lambda: K.tree_ensemble(tree, sc.X, None, B, partial=slab, groups=g, no_finish=True)  # noqa: E731
        run()
        torch.cuda.synchronize()
        s = y[:, :tree.k].clone() if g == 1 else slab.view(g, B, tree.k).sum(0)
        if g == 1:
            ref = s
        diff = float((s - ref).abs().max())
        ts = []
        for _ in range(5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.reps):
                run()
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3 / a.reps)
        r = dict(groups=g, us=float(np.median(ts)), max_diff_vs_g1=diff)
        out.append(r)
        print(json.dumps(r), flush=True)
    # phase trace of the default grouping (wall_clock64 at 100 MHz)
    g = sc.tree_groups.get(B, 1)
    slab = torch.zeros(max(g, 2) * B * tree.k, dtype=torch.float32, device=dev)
    tr = torch.zeros(64, dtype=torch.int64, device=dev)
    for _ in range(3):
        K.tree_ensemble(tree, sc.X, None, B, partial=slab, groups=max(g, 2), no_finish=True, trace=tr)
    torch.cuda.synchronize()
    t = tr.cpu().numpy().reshape(8, 8)[:, :6].astype(np.float64)
    t0 = t[t > 0].min()
    print(f"tree trace (groups {max(g, 2)}) us: start / staged / traversed / synced / leaves summed / stored")
    for b in range(8):
        print(f"   group {b // 2} block {64 * (b % 2):3d}", [round((x - t0) / 100.0, 2) if x > 0 else None for x in t[b]])
    return 0


if __name__ == "__main__":
    sys.exit(main())
