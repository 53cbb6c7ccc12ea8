#!/usr/bin/env python3
"""Host-side cost of one scoring submit (cfg 3, batch 8192): pack, stream contexts, graph
replays, event records, wait. Prints microseconds per operation (medians)."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def med(f, n=200):
    ts = []
    for _ in range(n):
        t = time.perf_counter()
        f()
        ts.append(time.perf_counter() - t)
    return float(np.median(ts)) * 1e6


def main():
    import torch
    from igaming_platform_amd.utils import benchkit
    from igaming_platform_amd.utils.synth import NOW0
    dev = torch.device("cuda", 0)
    S = benchkit.build("cfg3", 0, 1 << 18, dev)
    sc, B = S.scorer, S.batch
    g = sc.graphs[(B, 0)]
    r = {}
    r["pack"] = med(lambda: sc.pack(0, S.pool[0]))
    torch.cuda.synchronize()
    r["stream_ctx"] = med(lambda: torch.cuda.stream(sc.stream).__enter__())
    torch.cuda.set_stream(torch.cuda.default_stream(dev))
    r["event_new_record"] = med(lambda: torch.cuda.Event().record(sc.mstream))
    ev = torch.cuda.Event()
    r["event_record"] = med(lambda: ev.record(sc.mstream))
    r["wait_event"] = med(lambda: sc.stream.wait_event(ev))
    torch.cuda.synchronize()
    r["replay_model_graph"] = med(lambda: g[2].replay(), 50)
    torch.cuda.synchronize()
    r["replay_state_graph"] = med(lambda: g[1].replay(), 50)
    torch.cuda.synchronize()
    r["submit_packed"] = med(lambda: sc.wait(sc.submit_packed(sc.next_slot(), B, NOW0), unpack=False), 50)
    i = [0]

    def loop():
        p = sc.submit_packed(sc.next_slot(), B, NOW0)
        i[0] += 1
        return p
    ps = []
    t = time.perf_counter()
    for k in range(200):
        ps.append(loop())
        if len(ps) >= 3:
            sc.wait(ps.pop(0), unpack=False)
    for p in ps:
        sc.wait(p, unpack=False)
    r["pipelined_submit_no_pack_per_batch"] = (time.perf_counter() - t) / 200 * 1e6
    for k, v in r.items():
        print(f"{k:40s} {v:9.1f} us")


if __name__ == "__main__":
    main()
