#!/usr/bin/env python3
"""K4 GRU tile sweep: rows per workgroup x waves per workgroup x batch, event-ring input
(cfg 5 model: 2x256, T=100, I=16). Checks that every variant gives the same scores."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    import torch
    from igaming_platform_amd.utils import benchkit
    from igaming_platform_amd.ops import kernels as K
    dev = torch.device("cuda", 0)
    S = benchkit.build_model("cfg5", 8192, 1 << 18, dev, use_graphs=False)
    R = S.runner
    res = []
    ref = {}
    batches = [int(b) for b in os.environ.get("GRU_BATCHES", "512,4096,8192").split(",")]
    variants = ((16, 0, 1, 1), (16, 0, 1, 3), (16, 4, 0, 0), (16, 8, 0, 0), (32, 4, 0, 0), (16, 0, 1, 0), (32, 0, 1, 0))
    if os.environ.get("GRU_WS_ONLY"):  # the cluster kernels and the default batch-parallel one
        variants = ((16, 0, 1, 1), (16, 0, 1, 3), (16, 0, 1, 0))
    for B in batches:
        slots = torch.from_numpy(np.random.default_rng(B).integers(0, 1 << 18, B).astype(np.int32)).to(dev)
        for tr, w, pipe, ws in variants:
            if True:
                out = torch.zeros(B, device=dev)
                run = lambda: K.gru(R.gp, B, R.T, out=out, store=R.store, slots=slots, tile_rows=tr, waves=w,  # noqa
                                    pipeline=pipe, ws=ws)
                run()
                torch.cuda.synchronize()
                if B not in ref:
                    ref[B] = out.clone()
                diff = float((out - ref[B]).abs().max())
                ts = []
                for _ in range(10):
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    run()
                    e1.record()
                    e1.synchronize()
                    ts.append(e0.elapsed_time(e1))
                ms = float(np.median(ts[2:]))
                r = dict(batch=B, ws=ws, tile_rows=tr, waves=w, pipeline=pipe, ms=ms, seq_per_s=B / ms * 1e3, us_per_step=ms * 10,
                         max_diff_vs_first=diff, ws_failed=R.gp.ws_failed())
                res.append(r)
                print(json.dumps(r), flush=True)
    with open(os.environ.get("OUT", "gpurun_out/gru_sweep.json"), "w") as f:
        json.dump(res, f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
