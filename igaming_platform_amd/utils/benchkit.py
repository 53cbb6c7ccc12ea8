"""Shared setup for the headline bench, the per-kernel microbench and the config benches."""
from __future__ import annotations

from dataclasses import dataclass
from typing import Any, List

import numpy as np

CONFIGS = {
    "cfg3": dict(model="stacked", width=128, batch=8192,
                 desc="cfg3 GBDT(100 trees,d7,128 feat)+MLP(32-256-1) stacked, TreeEnsembleRegressor->Gemm"),
    "cfg2": dict(model="gbdt", width=128, batch=1024,
                 desc="cfg2 GBDT fraud ensemble, 100 trees d7, 128 features, TreeEnsembleClassifier"),
    "cfg1": dict(model="logistic", width=32, batch=8192, desc="cfg1 32-feature logistic (GPU path)"),
    "heuristic": dict(model="heuristic", width=30, batch=8192, desc="reference rules + mockPredict heuristic"),
}


@dataclass
class Setup:
    cfg: Any
    store: Any
    scorer: Any
    pop: Any
    pool: List[Any]
    batch: int
    desc: str
    chunk: int = 0       # data-parallel exchange: chunk capacity C (rows per owner per sender)


def build(config: str, batch: int, accounts: int, dev, rank: int = 0, depth: int = 2,
          use_graphs: bool = True, history_batches: int = 24, n_pool: int = 8,
          hot_frac: float = 0.02, precision: str = "fp32", dp: dict = None, buckets=None,
          sum_mode: str = "sliding") -> Setup:
    """``dp=dict(world=N, comms=[2 RcclComm])``: this rank is one of N ingress ranks of the
    owner-routed exchange (engine/dp.py): its pool entries are (chunks, rows) whose rows are
    spread over every owner uniformly at random, as hash routing spreads real accounts."""
    import torch

    from ..config import Config
    from ..engine.scorer import GpuScorer
    from ..features.device_store import DeviceFeatureStore
    from ..models.plan import compile_onnx, to_device
    from ..native import native
    from ..onnx import builders
    from ..ops import kernels as K
    from .synth import NOW0, make_population, make_requests

    c = CONFIGS[config]
    B = batch or c["batch"]
    cfg = Config()
    cfg.features.width = c["width"]
    cfg.features.sum_mode = sum_mode
    cfg.gpu.buckets = sorted(set(buckets)) if buckets else [B]
    cfg.gpu.max_batch = B
    world = dp["world"] if dp else 1
    C = 0
    if dp:
        from ..parallel.exchange import chunk_capacity
        C = chunk_capacity(B, world)
    # one population layout on every owner in DP mode (rows from any ingress rank match it)
    pop = make_population(accounts, c["width"] - 30, seed=1000 + (0 if dp else rank), fast_hash=True)
    store = DeviceFeatureStore(accounts, cfg.features, dev, events=True, max_events=world * C if dp else B)
    store.set_batch_features(np.arange(accounts), pop.batch)
    if c["width"] > 30:
        store.set_ext(np.arange(accounts), pop.ext)
    for i in range(200):
        store.blacklist.add("device", f"bad-device-{rank}-{i}")
    store.sync_tables()
    plan, model = None, "heuristic"
    if c["model"] != "heuristic":
        m = native().OnnxModel.from_bytes(builders.build(c["model"]).SerializeToString())
        plan = to_device(compile_onnx(m), dev, precision)
        model = "plan"
    if dp:
        from ..engine.dp import DpGpuScorer
        sc = DpGpuScorer(cfg, store, dp["comms"], world, rank, senders=world, cbuckets=[C], plan=plan, model=model,
                         device=dev, pipeline_depth=depth)
    else:
        sc = GpuScorer(cfg, store, plan=plan, model=model, device=dev, pipeline_depth=depth, use_graphs=use_graphs)
    rng = np.random.default_rng(7 + rank)
    for h in range(history_batches):  # ~an hour of history: windows, HLLs, sessions
        r = make_requests(pop, B, rng, NOW0 - 3600 + 150 * h, spread_s=150, hot_frac=0.01)
        t = torch.from_numpy(r.view(np.uint8).copy()).to(dev)
        K.feature_update(store, sc.cfg_dev, t, B, n=B)
    torch.cuda.synchronize(dev)
    sc.capture()
    pool = [make_requests(pop, B, rng, NOW0, hot_frac=hot_frac, unknown_frac=0.001) for _ in range(n_pool)]
    if dp:
        from ..parallel.exchange import build_chunks
        chunks = []
        for rows in pool:
            owners = rng.integers(0, world, len(rows))
            # a row whose owner's chunk is full waits for the next step in a server; the bench
            # drops it from this step and counts only the rows actually sent (P ~ 1e-5 per step)
            keep = np.ones(len(rows), bool)
            for o in range(world):
                idx = np.nonzero(owners == o)[0]
                keep[idx[C:]] = False
            buf = build_chunks(rows[keep], owners[keep], world, C)[0]
            chunks.append((buf, int(keep.sum())))
        pool = chunks
    return Setup(cfg, store, sc, pop, pool, B, c["desc"], C)


# ----------------------------------------------------------------------------- model-service configs
MODEL_CONFIGS = {
    "cfg4": dict(kind="ltv", batch=8192, metric="LTV predictions/sec (whole node)", unit="predictions/s",
                 desc="cfg4 LTV regression MLP 4x512 (256 features = 25 profile + 231 ext, HBM-resident tables) "
                      "+ K9 churn/segment/NBA, streaming micro-batches (hipGraph)"),
    "cfg5": dict(kind="abuse", batch=4096, metric="bonus-abuse checks/sec (whole node)", unit="checks/s",
                 desc="cfg5 bonus-abuse GRU 2x256 over the last 100 player events (HBM event rings, I=16) "
                      "+ Gemm/Sigmoid head, fused K4"),
}


@dataclass
class ModelSetup:
    runner: Any          # LtvGpu | AbuseGpu (submit(slots) / wait(p) / out)
    pool: List[np.ndarray]
    batch: int
    desc: str
    metric: str
    unit: str
    store: Any = None


def build_model(config: str, batch: int, accounts: int, dev, rank: int = 0, depth: int = 2,
                use_graphs: bool = True, n_pool: int = 8, precision: str = "bf16", overlap: bool = True) -> ModelSetup:
    import torch

    from ..config import FeatureConfig
    from ..models.plan import compile_onnx, to_device
    from ..native import native
    from ..onnx import builders

    c = MODEL_CONFIGS[config]
    B = batch or c["batch"]
    rng = np.random.default_rng(11 + rank)
    g = torch.Generator(device=dev)
    g.manual_seed(1234 + rank)
    N = native()
    if c["kind"] == "ltv":
        from ..engine.ltv import LtvGpu
        m = N.OnnxModel.from_bytes(builders.build("ltv_mlp", n_features=256, width=512, layers=4).SerializeToString())
        runner = LtvGpu(dev, accounts, to_device(compile_onnx(m), dev, precision), buckets=[B], use_graphs=use_graphs,
                        depth=depth)
        # synthetic player profiles (same column semantics as golden.ltv.PLAYER_COLUMNS)
        for s in range(0, accounts, 1 << 18):
            n = min(1 << 18, accounts - s)
            pf = torch.rand((n, 25), generator=g, device=dev) * torch.tensor(
                [900, 90, 60, 500, 10, 120, 1e5, 8e4, 3e4, 500, 8, 5e3, 2e5, 1.8e5, 3000, 1, 80, 60, 20, 15, 1,
                 1, 1, 1, 8], device=dev)
            runner.pf_tab[s:s + n].copy_(pf.floor_())
            runner.ext_tab[s:s + n].normal_(generator=g)
        store = None
    else:
        from ..engine.abuse import AbuseGpu
        from ..features.device_store import DeviceFeatureStore
        fc = FeatureConfig()
        store = DeviceFeatureStore(accounts, fc, dev, events=True, max_events=64)
        for s in range(0, accounts, 1 << 16):  # full 100-event histories, ~N(0,1) encoded events
            n = min(1 << 16, accounts - s)
            ev = torch.randn((n, fc.event_ring, fc.event_dim), generator=g, device=dev).to(torch.bfloat16)
            store.ev[s:s + n].copy_(ev.view(torch.int16))
        rt = store.rt.view(-1, store.rt.shape[1])
        from ..layouts import ACCTRT
        head_col = ACCTRT.fields["ev_head"][1] // 4
        cnt_col = ACCTRT.fields["ev_count"][1] // 4
        rt[:, head_col] = torch.randint(0, fc.event_ring, (accounts,), generator=g, device=dev, dtype=torch.int32)
        rt[:, cnt_col] = fc.event_ring
        m = N.OnnxModel.from_bytes(builders.build("gru", seq=100, in_dim=16, hidden=256).SerializeToString())
        runner = AbuseGpu(store, to_device(compile_onnx(m), dev, precision), buckets=[B], use_graphs=use_graphs,
                          depth=depth, overlap=overlap)
    torch.cuda.synchronize(dev)
    runner.capture()
    pool = [rng.integers(0, accounts, B).astype(np.int32) for _ in range(n_pool)]
    return ModelSetup(runner, pool, B, c["desc"], c["metric"], c["unit"], store)
