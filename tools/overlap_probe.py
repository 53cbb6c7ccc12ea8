#!/usr/bin/env python3
"""Does batch i+1's state graph overlap batch i's model graph? Replays the captured graphs of
the cfg3 scorer without host packing (the slabs are packed once): state-only, model-only and
the two-stream pipeline, each keeping at most DEPTH batches in flight like bench.py."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from igaming_platform_amd.utils import benchkit
    from igaming_platform_amd.utils.synth import NOW0
    dev = torch.device("cuda", 0)
    depth = int(os.environ.get("DEPTH", "3"))
    S = benchkit.build("cfg3", 0, 1 << 20, dev, depth=depth)
    sc, B = S.scorer, S.batch
    for slot in range(depth):
        v = sc.slab_view(slot, B)
        v[:] = S.pool[slot]
        v["ts"] = NOW0
    N = 300

    def run(kind):
        evs = [None] * depth
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(N):
            slot = i % depth
            if evs[slot] is not None:
                evs[slot].synchronize()  # the slot's previous batch is done: its host slab is free
            if kind == "pipeline":
                evs[slot] = sc.submit_packed(slot, B, NOW0).event
                continue
            sc._seq += 1
            sc._write_hdr(slot, B, NOW0)
            st = sc.stream if kind == "state" else sc.mstream
            with torch.cuda.stream(st):
                for gi in ((0, 1) if kind == "state" else (2,)):  # copy+state graphs | model graph
                    sc.graphs[(B, slot)][gi].replay()
                e = torch.cuda.Event()
                e.record(st)
            evs[slot] = e
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / N * 1e6

    def trace(n=40):
        """pipeline with timing events around every graph: per-batch stream intervals"""
        E = lambda: torch.cuda.Event(enable_timing=True)  # noqa: E731
        recs, evs = [], [None] * depth
        torch.cuda.synchronize()
        for i in range(n):
            slot = i % depth
            if evs[slot] is not None:
                evs[slot].synchronize()
            g = sc.graphs[(B, slot)]
            sc._seq += 1
            sc._write_hdr(slot, B, NOW0)
            r = {}
            for name, st, gi, wait in (("copy", sc.cstream, 0, None), ("state", sc.stream, 1, "copy"),
                                       ("model", sc.mstream, 2, "state")):
                with torch.cuda.stream(st):
                    if wait:
                        st.wait_event(r[wait][1])
                    if name == "copy" and i >= 2:
                        st.wait_event(recs[i - 2]["state"][1])
                    if name == "copy" and evs[slot] is not None:
                        st.wait_event(evs[slot])
                    a0, a1 = E(), E()
                    a0.record(st)
                    g[gi].replay()
                    a1.record(st)
                r[name] = (a0, a1)
            evs[slot] = r["model"][1]
            recs.append(r)
        torch.cuda.synchronize()
        base = recs[10]["copy"][0]
        for i in range(10, n):
            line = " ".join(f"{k}[{base.elapsed_time(recs[i][k][0]) * 1e3:7.1f},{base.elapsed_time(recs[i][k][1]) * 1e3:7.1f}]"
                            for k in ("copy", "state", "model"))
            print(f"batch {i:3d} {line}", flush=True)

    sc.store.reset_dedup()
    trace()
    for kind in ("state", "model", "pipeline", "state", "pipeline"):
        torch.cuda.synchronize()
        sc.store.reset_dedup()
        run(kind)
        print(f"{kind:10s} depth={depth} {run(kind):8.1f} us/batch", flush=True)


if __name__ == "__main__":
    main()
