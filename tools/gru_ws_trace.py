#!/usr/bin/env python3
"""Phase timeline of the weight-stationary GRU (csrc/kernels/gru_ws.hip), workgroup 0:
per step compute / LDS write+publish / counter wait / gather, in microseconds (wall_clock64,
100 MHz). Usage: python tools/gru_ws_trace.py [batch]"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    import torch
    from igaming_platform_amd.utils import benchkit
    from igaming_platform_amd.ops import kernels as K
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    ws = int(sys.argv[2]) if len(sys.argv) > 2 else 1  # 1: one cluster per CU, 3: two 64-row clusters per CU
    dev = torch.device("cuda", 0)
    S = benchkit.build_model("cfg5", B, 1 << 16, dev, use_graphs=False)
    R = S.runner
    slots = torch.from_numpy(np.random.default_rng(B).integers(0, 1 << 16, B).astype(np.int32)).to(dev)
    out = torch.zeros(B, device=dev)
    tr = torch.zeros(64 * 8 + 4 + 1024, dtype=torch.int64, device=dev)  # phases | clocks | placement
    for _ in range(3):
        K.gru(R.gp, B, R.T, out=out, store=R.store, slots=slots, ws=ws, ws_trace=tr)
    torch.cuda.synchronize()
    raw = tr.cpu().numpy()
    t = raw[:64 * 6].reshape(64, 6).astype(np.float64) / 100.0  # us
    lt = raw[64 * 6:64 * 8].reshape(64, 2).astype(np.float64) / 100.0
    w0, c0, w1, c1 = raw[64 * 8:64 * 8 + 4].astype(np.float64)
    print(json.dumps({"shader_clock_mhz": (c1 - c0) / ((w1 - w0) / 100.0),
                      "layer0_compute_us": float(np.median(lt[2:63, 0] - t[2:63, 0])),
                      "layer1_compute_us": float(np.median(lt[2:63, 1] - t[2:63, 0]))}))
    d = dict(step=np.median(t[2:63, 0][1:] - t[2:62, 0]) if True else 0,
             compute=np.median(t[2:63, 1] - t[2:63, 0]), publish=np.median(t[2:63, 2] - t[2:63, 1]),
             wait=np.median(t[2:63, 3] - t[2:63, 2]), gather=np.median(t[2:63, 4] - t[2:63, 3]))
    print(json.dumps({"batch": B, "median_us": {k: round(float(v), 3) for k, v in d.items()},
                      "ws_failed": R.gp.ws_failed()}))
    for s in range(0, 8):
        print(s, np.round(np.diff(t[s, :5]), 2).tolist())
    if ws == 3:  # which workgroups share a CU (HW_ID: cu_id bits 8..11, sh 12, se 13..15; XCC_ID)
        hw = raw[64 * 8 + 4:64 * 8 + 4 + 1024]
        nwg = ((-(-B // 64) + 7) // 8) * 64  # 64-row clusters, 8 members, groups of 8 clusters
        where = {}
        for b in range(min(nwg, 1024)):
            v = int(hw[b])
            key = (v >> 32, (v >> 13) & 7, (v >> 12) & 1, (v >> 8) & 15)
            where.setdefault(key, []).append(b)
        pairs = [tuple(bs) for bs in where.values() if len(bs) > 1]
        deltas = {}
        for bs in pairs:
            d = bs[1] - bs[0]
            deltas[d] = deltas.get(d, 0) + 1
        print(json.dumps({"cus_used": len(where), "co_resident_pairs": len(pairs),
                          "pair_blockidx_deltas": dict(sorted(deltas.items(), key=lambda kv: -kv[1])[:6]),
                          "first_pairs": pairs[:6]}))
    return 0


if __name__ == "__main__":
    sys.exit(main())
