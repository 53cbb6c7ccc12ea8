#!/usr/bin/env python3
"""cfg5 f32-faithful GRU (gru_x3_kernel) occupancy sweep: rows per workgroup (16 / 32) x waves
per workgroup (8 / 16) x batch x
concurrent launches on separate streams (1 = the serving rank's single stream, 2-3 = the
bench's per-slot streams). Reports per-launch ms, checks/s and per-CU row rate so the two tile
sizes can be compared on the same box; every variant's scores are compared with the first."""
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
    S = benchkit.build_model("cfg5", 8192, 1 << 18, dev, use_graphs=False, precision="fp32")
    R = S.runner
    assert R.gp.split, "cfg5 fp32 plan must use the split GRU"
    cus = torch.cuda.get_device_properties(dev).multi_processor_count
    res, ref = [], {}
    for B in (4096, 8192):
        for conc in (1, 2, 3):
            streams = [torch.cuda.Stream(dev) for _ in range(conc)]
            slots = [torch.from_numpy(np.random.default_rng(B + i).integers(0, 1 << 18, B).astype(np.int32)).to(dev)
                     for i in range(conc)]
            outs = [torch.zeros(B, device=dev) for _ in range(conc)]
            for tr, nw in ((16, 8), (32, 8), (16, 16), (32, 16)):  # 16 = the default at H = 256
                def run():
                    for s, sl, o in zip(streams, slots, outs):
                        with torch.cuda.stream(s):
                            K.gru(R.gp, B, R.T, out=o, store=R.store, slots=sl, tile_rows=tr, waves=nw, ws=0)
                run()
                torch.cuda.synchronize()
                key = (B, conc)
                if key not in ref:
                    ref[key] = [o.clone() for o in outs]
                diff = max(float((o - r).abs().max()) for o, r in zip(outs, ref[key]))
                ts = []
                for _ in range(6):
                    torch.cuda.synchronize()
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for s in streams:
                        s.wait_event(e0)
                    run()
                    for s in streams:
                        torch.cuda.current_stream().wait_stream(s)
                    e1.record()
                    e1.synchronize()
                    ts.append(e0.elapsed_time(e1))
                ms = float(np.median(ts[1:]))
                wgs = conc * ((B + tr - 1) // tr)
                r = dict(batch=B, concurrent=conc, tile_rows=tr, waves=nw, workgroups=wgs, cus=cus, ms=round(ms, 3),
                         checks_per_s=round(conc * B / ms * 1e3), us_per_step=round(ms * 1e3 / R.T, 2),
                         max_diff_vs_16=diff)
                res.append(r)
                print(json.dumps(r), flush=True)
    with open(os.environ.get("OUT", "gpurun_out/gru_x3_sweep.json"), "w") as f:
        json.dump(res, f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
