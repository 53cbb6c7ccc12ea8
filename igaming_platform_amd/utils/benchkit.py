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
    pool: List[np.ndarray]
    batch: int
    desc: str


def build(config: str, batch: int, accounts: int, dev, rank: int = 0, depth: int = 2,
          use_graphs: bool = True, history_batches: int = 24, n_pool: int = 8,
          hot_frac: float = 0.02) -> Setup:
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
    cfg.gpu.buckets = [B]
    cfg.gpu.max_batch = B
    pop = make_population(accounts, c["width"] - 30, seed=1000 + rank, fast_hash=True)
    store = DeviceFeatureStore(accounts, cfg.features, dev, events=True, max_events=B)
    store.set_batch_features(np.arange(accounts), pop.batch)
    if c["width"] > 30:
        store.set_ext(np.arange(accounts), pop.ext)
    for i in range(200):
        store.blacklist.add("device", f"bad-device-{rank}-{i}")
    store.sync_tables()
    plan, model = None, "heuristic"
    if c["model"] != "heuristic":
        m = native().OnnxModel.from_bytes(builders.build(c["model"]).SerializeToString())
        plan = to_device(compile_onnx(m), dev)
        model = "plan"
    sc = GpuScorer(cfg, store, plan=plan, model=model, device=dev, pipeline_depth=depth, use_graphs=use_graphs)
    rng = np.random.default_rng(7 + rank)
    for h in range(history_batches):  # ~an hour of history: windows, HLLs, sessions
        r = make_requests(pop, B, rng, NOW0 - 3600 + 150 * h, spread_s=150, hot_frac=0.01)
        t = torch.from_numpy(r.view(np.uint8).copy()).to(dev)
        K.feature_update(store, sc.cfg_dev, t, B, n=B)
    torch.cuda.synchronize(dev)
    sc.capture()
    pool = [make_requests(pop, B, rng, NOW0, hot_frac=hot_frac, unknown_frac=0.001) for _ in range(n_pool)]
    return Setup(cfg, store, sc, pop, pool, B, c["desc"])
