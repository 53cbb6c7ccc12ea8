#!/usr/bin/env python3
"""Hot-account apply cost (update_multi_kernel on the scorer path): one 8192-row batch where
one account carries N rows (the rest uniform over the population), timed around
update_segments after the batch's dedup insert. The slope over N is the cost per 64-event
chunk, the intercept the batch scan; Zipf(1.2) traffic puts ~1550 rows on its top account.
Prints one JSON line per N."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    import torch
    from igaming_platform_amd.ops import kernels as K
    from igaming_platform_amd.utils import benchkit
    from igaming_platform_amd.utils.synth import NOW0, make_requests
    dev = torch.device("cuda", 0)
    B = 8192
    S = benchkit.build("cfg3", B, 1 << 18, dev, hot_frac=0.0)
    sc, store = S.scorer, S.store
    rng = np.random.default_rng(3)
    res = []
    for N in (0, 65, 128, 512, 1024, 1536, 3072, 6144):
        ts = []
        for it in range(8):
            rows = make_requests(S.pop, B, rng, NOW0, hot_frac=0.0)
            if N:  # the hot account's own devices / ips (a few each), as real traffic
                idx = np.sort(rng.choice(B, N, replace=False))
                rows["slot"][idx] = 7
                P = S.pop.dev_pool.shape[1]
                rows["dev_hash"][idx] = S.pop.dev_pool[7, rng.integers(0, P, N)]
                rows["ip_hash"][idx] = S.pop.ip_pool[7, rng.integers(0, P, N)]
            v = sc.slab_view(0, B)
            v[:] = rows
            sc._seq += 1
            sc._write_hdr(0, B, NOW0 + it)
            nb = 16 + 48 * B
            sc.dev_slab[:nb].copy_(sc.host_slab[0][:nb])
            K.dedup_insert(store, sc.cfg_dev, sc.req, B, sc.hdr)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            K.update_segments(store, sc.cfg_dev, sc.req, B, sc.hdr)
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3)
        r = dict(hot_rows=N, chunks=(N + 63) // 64, update_us=round(float(np.median(ts[2:])), 1),
                 min_us=round(float(np.min(ts[2:])), 1))
        res.append(r)
        print(json.dumps(r), flush=True)
    with open(os.environ.get("OUT", "gpurun_out/hot_apply.json"), "w") as f:
        json.dump(res, f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
