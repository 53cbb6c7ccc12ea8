#!/usr/bin/env python3
"""Per-kernel device time of one scoring step (events around each launch, interleaved rounds
in one process). Usage: python tools/kbench.py [--config cfg3] [--rounds 50]"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg3")
    ap.add_argument("--batch", type=int, default=0)
    ap.add_argument("--accounts", type=int, default=1 << 20)
    ap.add_argument("--rounds", type=int, default=50)
    ap.add_argument("--out", default="")
    ap.add_argument("--hot", type=float, default=0.02, help="fraction of requests on 16 hot accounts")
    ap.add_argument("--only", default="", help="comma-separated op names to run")
    ap.add_argument("--cold", action="store_true",
                    help="rotating K1 batches draw fresh uniform account slots each round (cold state)")
    a = ap.parse_args()
    import torch
    from igaming_platform_amd.ops import kernels as K
    from igaming_platform_amd.utils import benchkit
    from igaming_platform_amd.utils.synth import NOW0
    dev = torch.device("cuda", 0)
    S = benchkit.build(a.config, a.batch, a.accounts, dev, hot_frac=a.hot)
    sc, B = S.scorer, S.batch
    # load a request batch into the device slab once
    slot = 0
    v = sc.slab_view(slot, B)
    v[:] = S.pool[0]
    v["ts"] = NOW0
    sc._seq += 1
    sc._write_hdr(slot, B, NOW0)
    nb = 16 + 48 * B
    sc.dev_slab[:nb].copy_(sc.host_slab[slot][:nb])
    torch.cuda.synchronize()

    steps = sc.plan.steps if sc.plan else []
    tree = next((s for s in steps if s.kind == "tree"), None)
    head = next((s for s in steps if s.kind == "head"), None)
    g = sc.tree_groups.get(B, 1)
    ops = {
        "h2d_slab": lambda: sc.dev_slab[:nb].copy_(sc.host_slab[slot][:nb], non_blocking=True),
        "dedup_insert": lambda: K.dedup_insert(sc.store, sc.cfg_dev, sc.req, B, sc.hdr),
        "feature_assemble+single_update": lambda: K.feature_assemble(sc.store, sc.hdr, sc.cfg_dev, sc.req, sc.X,
                                                                     sc.feat, B, dedup=True),
        "feature_assemble_no_update": lambda: K.feature_assemble(sc.store, sc.hdr, sc.cfg_dev, sc.req, sc.X,
                                                                 sc.feat, B, dedup=False),
        "ensemble": lambda: K.ensemble(sc.hdr, sc.cfg_dev, sc.feat, sc.X, sc.ml, sc.res, B, sc.metrics),
        "update_segments": lambda: K.update_segments(sc.store, sc.cfg_dev, sc.req, B, sc.hdr),
        "d2h_results": lambda: sc.host_res[slot][:B].copy_(sc.res[:B], non_blocking=True),
    }
    if tree is not None:
        ops["tree_ensemble"] = lambda: K.tree_ensemble(tree, sc.X, None if head else sc.step_out[0], B,
                                                        partial=sc.tree_partial, groups=g, no_finish=head is not None)
    if head is not None:
        out = sc.step_out[-1]
        ops["mlp_head"] = lambda: K.mlp_head(head, sc.X, out, B, m_ptr=sc.n_ptr,
                                             tree_partial=(sc.tree_partial, g, tree) if tree else None)
    if sc.graphs:
        gc, gs, gm = sc.graphs[(B, slot)][:3]
        ops["full_step_graph"] = lambda: (gc.replay(), gs.replay(), gm.replay())
    ops_all = dict(ops)
    if a.only:
        keep = set(a.only.split(","))
        ops = {k: v for k, v in ops.items() if k in keep}
    from igaming_platform_amd.native import hipk

    def stall():  # a 300-us device spin ahead of the timed region (the Python launch path takes ~50 us)
        hipk().stall(torch.cuda.current_stream().cuda_stream, 300.0)
    times = {k: [] for k in ops}
    for r in range(a.rounds):
        # a fresh batch sequence number per round, as the scorer does per micro-batch
        sc._seq += 1
        sc._write_hdr(slot, B, NOW0)
        for k, f in ops.items():
            if k == "full_step_graph":  # the graph re-copies the slab: give it its own batch seq
                sc._seq += 1
                sc._write_hdr(slot, B, NOW0)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            stall()  # the device reaches e0 only after the host enqueued the op: device time only
            e0.record()
            f()
            e1.record()
            e1.synchronize()
            times[k].append(e0.elapsed_time(e1) * 1e3)
    # K1 phase trace of 8 sample waves (wall_clock64, 100 MHz -> us from the earliest start)
    trw = torch.zeros(((B + 15) // 16) * 4 * 16, dtype=torch.int64, device=dev)  # every wave: 16 int64
    for dd in (True, False):
        for _ in range(3):
            sc._seq += 1
            sc._write_hdr(slot, B, NOW0)
            sc.dev_slab[:nb].copy_(sc.host_slab[slot][:nb])
            if dd:
                K.dedup_insert(sc.store, sc.cfg_dev, sc.req, B, sc.hdr)
            trw.zero_()
            K.feature_assemble(sc.store, sc.hdr, sc.cfg_dev, sc.req, sc.X, sc.feat, B, dedup=dd, trace=trw)
            torch.cuda.synchronize()
        t = trw.cpu().numpy().reshape(-1, 16)[[w * 293 for w in range(7)]][:, [0, 1, 6, 7, 2, 3, 4, 5]].astype(np.float64)
        t0 = t[t > 0].min()
        print(f"K1 trace (update={dd}) us: start / level1 / live / l2-issued / level2 / compute / stores / end")
        for w in range(7):
            print("   wave", w * 293, [round((x - t0) / 100.0, 2) if x > 0 else None for x in t[w]])
    # K1 with the update on rotating pool batches (the bench's access pattern): event timing
    # of the kernel alone + phase trace of the last one
    # KB_VARIANTS: comma-separated masks (512 = also store the D2H feature images into pinned host
    # memory, as the serving path does; 1024 = a second launch right behind the first)
    fenc_host = torch.zeros((B, 32), dtype=torch.int32).pin_memory()
    modes = [(v, 0) for v in os.environ.get("KB_K1_MODES", "full").split(",") if v not in ("", "-")]
    modes += [("full", int(m)) for m in os.environ.get("KB_VARIANTS", "").split(",") if m]
    for var, abl in modes:  # full | nodedup | noseg
      ts_k1 = []
      for i in range(24):
          vv = sc.slab_view(slot, B)
          vv[:] = S.pool[i % len(S.pool)]
          if a.cold:  # every round a fresh uniform draw over the population: cold account lines
              vv["slot"] = np.random.default_rng(1000 + i).integers(0, a.accounts, B).astype(np.int32)
          vv["ts"] = NOW0 + 1 + i
          sc._seq += 1
          sc._write_hdr(slot, B, NOW0 + 1 + i)
          sc.dev_slab[:nb].copy_(sc.host_slab[slot][:nb])
          if var != "nodedup":
              K.dedup_insert(sc.store, sc.cfg_dev, sc.req, B, sc.hdr)
          trw.zero_()
          e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
          stall()
          e0.record()
          K.feature_assemble(sc.store, sc.hdr, sc.cfg_dev, sc.req, sc.X, sc.feat, B, dedup=var != "nodedup", trace=trw,
                             fenc=fenc_host if abl & 512 else None)
          if abl & 1024:  # the same launch again right behind it (instruction caches warm): 2 launches timed
              K.feature_assemble(sc.store, sc.hdr, sc.cfg_dev, sc.req, sc.X, sc.feat, B, dedup=False,
                                 fenc=fenc_host if abl & 512 else None)
          e1.record()
          e1.synchronize()
          ts_k1.append(e0.elapsed_time(e1) * 1e3)
          if var not in ("nodedup", "noseg"):
              K.update_segments(sc.store, sc.cfg_dev, sc.req, B, sc.hdr)
      full = trw.cpu().numpy().reshape(-1, 16)
      if os.environ.get("KB_TRACE_OUT"):
          np.save(os.environ["KB_TRACE_OUT"] + f"_a{abl}.npy", full)
      print(f"[{var} variant={abl}] K1+update on rotating pool batches: median {np.median(ts_k1[8:]):.1f} us "
            f"(first pass {np.median(ts_k1[:8]):.1f})")
      t = full[[w * 293 for w in range(7)]][:, [0, 1, 6, 7, 2, 3, 4, 5]].astype(np.float64)
      t0 = t[t > 0].min()
      print("K1 trace (update, rotating batches) us: start / level1 / live / l2-issued / level2 / compute / stores / end")
      for w in range(7):
          print("   wave", w * 293, [round((x - t0) / 100.0, 2) if x > 0 else None for x in t[w]])
    # mlp_head (8 sample blocks) phase trace
    tr = torch.zeros(64, dtype=torch.int64, device=dev)
    if head is not None:
        for _ in range(3):
            tr.zero_()
            ops["mlp_head"]() if "mlp_head" in ops else None
            K.mlp_head(head, sc.X, sc.step_out[-1], B, m_ptr=sc.n_ptr,
                       tree_partial=(sc.tree_partial, g, tree) if tree else None, trace=tr)
            torch.cuda.synchronize()
        t = tr.cpu().numpy().reshape(8, 8)[:, :5].astype(np.float64)
        if (t > 0).any():
            t0 = t[t > 0].min()
            print("mlp_head trace us: start / staged / mfma done / synced / stored")
            for b in range(8):
                print("   block", b * 32, [round((x - t0) / 100.0, 2) if x > 0 else None for x in t[b]])
    res = {k: dict(median_us=float(np.median(v[min(5, len(v) - 1):])), min_us=float(np.min(v[min(5, len(v) - 1):])))
           for k, v in times.items()}
    for k, v in res.items():
        print(f"{k:28s} median {v['median_us']:8.1f} us   min {v['min_us']:8.1f} us")
    if a.out:
        with open(a.out, "w") as f:
            json.dump(dict(config=a.config, batch=B, kernels=res), f, indent=1)


if __name__ == "__main__":
    main()
