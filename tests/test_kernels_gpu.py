"""Device kernels vs the golden spec / C++ CPU executor / torch fp32 (run on MI355X)."""
import numpy as np
import pytest

from igaming_platform_amd.config import Config, REASON_BIT
from igaming_platform_amd.golden import ltv as GL
from igaming_platform_amd.utils.hashing import SEED_IP, id_hash

from .helpers import build_world, compare_featrec, golden_score

pytestmark = pytest.mark.gpu

NOW = 1_760_000_000


def _store_and_world(cfg, n_acc=300, seed=1):
    import torch
    from igaming_platform_amd.features.device_store import DeviceFeatureStore
    from igaming_platform_amd.ops import kernels as K
    pop, gold, hist, bl, intel = build_world(cfg, n_acc, seed, NOW)
    store = DeviceFeatureStore(n_acc, cfg.features, "cuda", events=True, max_events=2048)
    store.set_batch_features(np.arange(n_acc), pop.batch)
    if cfg.features.width > 30:
        store.set_ext(np.arange(n_acc), pop.ext)
    for t, v in bl:
        e = store.blacklist.add(t, v, reason="test")
        gold.blacklist[id_hash(v, {"device": 0x44455649, "ip": SEED_IP}[t])] = e.expires_at
    for ip, vpn, proxy, tor in intel:
        store.ipintel.set(ip, vpn, proxy, tor)
        gold.ip_intel[id_hash(ip, SEED_IP)] = (1 if vpn else 0) | (2 if proxy else 0) | (4 if tor else 0)
    store.sync_tables()
    cfg_dev = torch.zeros(176, dtype=torch.uint8, device="cuda")
    from igaming_platform_amd.layouts import score_cfg
    cfg_dev.copy_(torch.from_numpy(score_cfg(cfg, 1, **store.table_params()).view(np.uint8).copy()))
    for r in hist:
        req = torch.from_numpy(r.view(np.uint8).copy()).cuda()
        K.feature_update(store, cfg_dev, req, len(r), n=len(r))
    torch.cuda.synchronize()
    return pop, gold, store


@pytest.mark.parametrize("width,log_mode,sum_mode", [(30, "log1p", "sliding"), (40, "identity", "compat")])
def test_feature_pipeline_matches_golden(width, log_mode, sum_mode):
    from igaming_platform_amd.engine.scorer import GpuScorer
    cfg = Config()
    cfg.features.width = width
    cfg.features.log_transform = log_mode
    cfg.features.sum_mode = sum_mode
    cfg.gpu.buckets = [64, 256, 1024]
    pop, gold, store = _store_and_world(cfg)
    scorer = GpuScorer(cfg, store, plan=None, model="heuristic", update_features=True)
    rng = np.random.default_rng(7)
    from igaming_platform_amd.utils.synth import make_requests, to_events
    for it in range(3):
        now = NOW + 60 * it
        req = make_requests(pop, 700, rng, now, hot_frac=0.2, unknown_frac=0.03)
        req["ts"] = now
        out = scorer.score(req, now=now, want_features=True)
        feats = out["features"]
        for i, row in enumerate(req):
            g = golden_score(cfg, gold, pop, row, now)
            compare_featrec(feats[i], g, i)
            assert out["score"][i] == g["score"], (i, out["score"][i], g["score"])
            assert out["action"][i] == g["action"], i
            assert out["rule_score"][i] == g["rule"], i
            mask = sum(1 << REASON_BIT[r] for r in g["reasons"])
            assert out["reasons"][i] == mask, (i, out["reasons"][i], g["reasons"])
            assert np.float32(out["ml"][i]) == np.float32(g["ml"]), i
        # score-then-update: the golden applies the batch after scoring it
        for ev in to_events(pop, req):
            gold.apply(ev)


def _event_history(store, slot):
    raw = store.ev[slot].cpu().numpy()
    rt = store.read_rt(slot)
    ev = (raw.view(np.uint16).astype(np.uint32) << 16).view(np.float32)
    R = ev.shape[0]
    head, cnt = int(rt["ev_head"]), min(int(rt["ev_count"]), R)
    out = np.zeros_like(ev)
    if cnt:
        out[R - cnt:] = ev[[(head - cnt + i) % R for i in range(cnt)]]
    return out


def test_update_paths_match_golden():
    """Every score-then-update / ingestion path against the golden store: single-event
    accounts (applied inside K1 by the wave), multi-event segments (parallel wave apply),
    segments spanning more than a TTL (ordered serial apply) and accounts with more events
    than a dedup list holds (ordered batch scan)."""
    import torch
    from igaming_platform_amd.engine.scorer import GpuScorer
    from igaming_platform_amd.ops import kernels as K
    from igaming_platform_amd.utils.synth import make_requests, to_events
    cfg = Config()
    cfg.gpu.buckets = [512]
    pop, gold, store = _store_and_world(cfg, n_acc=80, seed=11)
    scorer = GpuScorer(cfg, store, plan=None, model="heuristic", update_features=True)
    rng = np.random.default_rng(5)
    # scorer path (all events at the batch time): account 5 x100 (list overflow -> scan),
    # account 6 x20 (parallel segment), the rest random (singles + small segments)
    for it in range(2):
        now = NOW + 30 * it
        req = make_requests(pop, 400, rng, now)
        req["slot"][:100] = 5
        req["slot"][100:120] = 6
        out = scorer.score(req, now=now, want_features=True)
        for i, row in enumerate(req):
            compare_featrec(out["features"][i], golden_score(cfg, gold, pop, row, now), i)
        for ev in to_events(pop, req):
            gold.apply(ev)
    # ingestion path with spread timestamps: account 7 spans 3 h (> every TTL but the HLL's:
    # serial), account 8 has 90 events (scan), account 9 spans 2 min (parallel)
    req = make_requests(pop, 300, rng, NOW + 100)
    req["slot"][:40], req["ts"][:40] = 7, NOW + 100 + np.sort(rng.integers(0, 3 * 3600, 40))
    req["slot"][40:130], req["ts"][40:130] = 8, NOW + 100 + np.arange(90)
    req["slot"][130:150], req["ts"][130:150] = 9, NOW + 100 + np.sort(rng.integers(0, 120, 20))
    req["ts"][150:] = NOW + 200
    t = torch.from_numpy(req.view(np.uint8).copy()).cuda()
    with torch.cuda.stream(scorer.stream):
        K.feature_update(store, scorer.cfg_dev, t, len(req), n=len(req))
    torch.cuda.synchronize()
    for ev in to_events(pop, req):
        gold.apply(ev)
    now = NOW + 4 * 3600
    probe = make_requests(pop, 80, rng, now)
    probe["slot"] = np.arange(80)
    out = scorer.score(probe, now=now, want_features=True)
    for i, row in enumerate(probe):
        compare_featrec(out["features"][i], golden_score(cfg, gold, pop, row, now), i)
    for ev in to_events(pop, probe):
        gold.apply(ev)
    for a in range(80):  # the ring stores bf16 (golden.encode_event is f32)
        g = torch.from_numpy(gold.event_history(pop.ids[a])).to(torch.bfloat16).float().numpy()
        np.testing.assert_array_equal(_event_history(store, a), g, err_msg=str(a))


def test_normalized_inputs_match_golden():
    import torch
    from igaming_platform_amd.engine.scorer import GpuScorer
    cfg = Config()
    cfg.features.width = 40
    cfg.gpu.buckets = [512]
    pop, gold, store = _store_and_world(cfg, n_acc=200, seed=3)
    scorer = GpuScorer(cfg, store, plan=None, model="heuristic", update_features=False, use_graphs=False)
    rng = np.random.default_rng(9)
    from igaming_platform_amd.utils.synth import make_requests
    req = make_requests(pop, 500, rng, NOW, hot_frac=0.1)
    scorer.score(req, now=NOW)
    X = scorer.X[:500].cpu().numpy()
    for i, row in enumerate(req):
        g = golden_score(cfg, gold, pop, row, NOW)
        np.testing.assert_allclose(X[i], g["x"], rtol=2e-7, atol=0, err_msg=f"row {i}")


def test_graph_replay_equals_eager():
    from igaming_platform_amd.engine.scorer import GpuScorer
    cfg = Config()
    cfg.gpu.buckets = [128, 1024]
    pop, gold, store = _store_and_world(cfg, n_acc=256, seed=5)
    sa = GpuScorer(cfg, store, plan=None, model="heuristic", update_features=False, use_graphs=False)
    sb = GpuScorer(cfg, store, plan=None, model="heuristic", update_features=False, use_graphs=True)
    sb.capture()
    from igaming_platform_amd.utils.synth import make_requests
    rng = np.random.default_rng(11)
    for n in (1, 77, 128, 900):
        req = make_requests(pop, n, rng, NOW)
        a = sa.score(req, now=NOW)
        b = sb.score(req, now=NOW)
        for k in ("score", "action", "reasons", "rule_score", "ml"):
            np.testing.assert_array_equal(a[k], b[k])


# ----------------------------------------------------------------------------- trees
def _tree_case(kind, **kw):
    import torch
    from igaming_platform_amd.models.plan import compile_onnx, to_device
    from igaming_platform_amd.native import native
    from igaming_platform_amd.onnx import builders
    N = native()
    m = N.OnnxModel.from_bytes(builders.build(kind, **kw).SerializeToString())
    plan = to_device(compile_onnx(m), "cuda")
    return N, m, plan


@pytest.mark.parametrize("kind,kw,groups", [
    ("gbdt", dict(n_trees=100, depth=7), 1), ("gbdt", dict(n_trees=100, depth=7), 6),
    ("gbdt", dict(n_trees=37, depth=5, mixed_modes=True), 3),
])
def test_tree_kernel_matches_cpu_executor(kind, kw, groups):
    import torch
    from igaming_platform_amd.ops import kernels as K
    N, m, plan = _tree_case(kind, **kw)
    ts = plan.steps[0]
    rng = np.random.default_rng(0)
    for rows in (1, 63, 1000, 4096):
        X = rng.uniform(0, 1, (rows, 128)).astype(np.float32)
        X[rng.uniform(0, 1, X.shape) < 0.01] = np.nan
        X[:, 5] = ts.nodes_np[0, 0, 0] if ts.nodes_np.size else 0.5  # hit a threshold exactly
        ref = N.Executor(m).run({"input": X})["output"]
        Xd = torch.from_numpy(X).cuda()
        out = torch.zeros((rows, ts.n_out), dtype=torch.float32, device="cuda")
        part = torch.zeros(max(groups, 1) * rows * ts.k, dtype=torch.float32, device="cuda")
        K.tree_ensemble(ts, Xd, out, rows, partial=part, groups=groups)
        np.testing.assert_allclose(out.cpu().numpy(), ref, rtol=1e-5, atol=2e-6)


def test_stacked_tree_embedding_matches_cpu():
    import torch
    from igaming_platform_amd.ops import kernels as K
    from igaming_platform_amd.onnx import builders, writer
    from igaming_platform_amd.native import native
    N = native()
    # regressor-only model (the embedding part of cfg 3)
    full = builders.stacked(n_trees=50, depth=6, k=32)
    g = full.graph
    nodes = [g.node[0]]
    nodes[0].output[0] = "output"
    reg = writer.model(nodes, [g.input[0]], [writer.value_info("output", 1, ["N", 32])], name="emb")
    m = N.OnnxModel.from_bytes(reg.SerializeToString())
    from igaming_platform_amd.models.plan import compile_onnx, to_device
    plan = to_device(compile_onnx(m), "cuda")
    ts = plan.steps[0]
    X = np.random.default_rng(1).uniform(0, 1, (2048, 128)).astype(np.float32)
    ref = N.Executor(m).run({"input": X})["output"]
    out = torch.zeros((2048, 32), dtype=torch.float32, device="cuda")
    part = torch.zeros(4 * 2048 * 32, dtype=torch.float32, device="cuda")
    for groups in (1, 4):
        K.tree_ensemble(ts, torch.from_numpy(X).cuda(), out, 2048, partial=part, groups=groups)
        np.testing.assert_allclose(out.cpu().numpy(), ref, rtol=1e-5, atol=1e-5)


# ----------------------------------------------------------------------------- dense / MFMA
@pytest.mark.parametrize("precision", ["fp32", "bf16"])
@pytest.mark.parametrize("M,N,Kd,act,xbf", [
    (1, 32, 32, "relu", False), (37, 256, 32, "relu", False), (4096, 512, 256, "relu", True),
    (8192, 256, 32, "none", False), (1000, 768, 16, "none", True), (333, 1, 256, "sigmoid", False),
    (5000, 512, 512, "tanh", True),
])
def test_dense_mfma_matches_torch_fp32(M, N, Kd, act, xbf, precision):
    """fp32 weights (f32 MFMA) vs a true fp32 torch reference; bf16 weights vs the same
    reference with the error bf16 operands imply (and tightly vs bf16-rounded operands)."""
    import torch
    from igaming_platform_amd.models.plan import _bf16_padded, _f32_padded
    from igaming_platform_amd.ops import kernels as K
    g = torch.Generator().manual_seed(M + N + Kd)
    X = torch.randn(M, Kd, generator=g)
    if xbf:
        X = X.to(torch.bfloat16).float()  # the producer hands bf16 activations: exact in both
    W = torch.randn(N, Kd, generator=g) / Kd ** 0.5     # [N, K] = output rows
    b = torch.randn(N, generator=g) * 0.1
    Xd = (X.to(torch.bfloat16) if xbf else X).cuda()
    Wd = (_f32_padded if precision == "fp32" else _bf16_padded)(W.numpy()).cuda()
    Y = torch.zeros(M, N, dtype=torch.float32, device="cuda")
    K.dense(Xd, Wd, b.cuda(), Y, M, N, Kd, act=act)
    f = {"relu": torch.relu, "sigmoid": torch.sigmoid, "tanh": torch.tanh, "none": lambda t: t}[act]
    ref32 = f(X.double() @ W.double().T + b.double()).float()
    if precision == "fp32":
        torch.testing.assert_close(Y.cpu(), ref32, rtol=1e-5, atol=2e-5)
    else:
        refb = f(X.to(torch.bfloat16).float() @ W.to(torch.bfloat16).float().T + b)
        torch.testing.assert_close(Y.cpu(), refb, rtol=2e-3, atol=2e-3)
        torch.testing.assert_close(Y.cpu(), ref32, rtol=3e-2, atol=3e-2)


def test_dense_respects_live_rows():
    import torch
    from igaming_platform_amd.models.plan import _bf16_padded
    from igaming_platform_amd.ops import kernels as K
    X = torch.randn(256, 64).cuda()
    Wd = _bf16_padded(np.random.default_rng(0).standard_normal((128, 64)).astype(np.float32)).cuda()
    Y = torch.full((256, 128), 7.0, device="cuda")
    m = torch.tensor([100], dtype=torch.int32, device="cuda")
    K.dense(X, Wd, None, Y, 256, 128, 64, m_ptr=m)
    assert torch.all(Y[100:] == 7.0)
    assert not torch.all(Y[:100] == 7.0)


# ----------------------------------------------------------------------------- full model plans
@pytest.mark.parametrize("kind,width,precision", [("logistic", 32, "fp32"), ("gbdt", 128, "fp32"),
                                                ("stacked", 128, "fp32"), ("stacked", 128, "bf16")])
def test_scorer_with_model_matches_executor_and_golden(kind, width, precision):
    """fp32 (the default, the ONNX model's f32 contract): on 10240 requests the device's score,
    action and reason mask are EXACTLY the golden rules + ensemble fed by the C++ fp32
    executor run on the golden feature vectors (no device value reused), and ml agrees to
    1e-5. bf16 (opt-in): ml within 2e-2 and the ensemble exact given the device's own ml."""
    from igaming_platform_amd.engine.scorer import GpuScorer
    from igaming_platform_amd.golden import scoring as GS
    from igaming_platform_amd.models.plan import compile_onnx, to_device
    from igaming_platform_amd.native import native
    from igaming_platform_amd.onnx import builders
    cfg = Config()
    cfg.features.width = width
    cfg.gpu.buckets = [256, 1024]
    pop, gold, store = _store_and_world(cfg, n_acc=3000, seed=2)
    N = native()
    m = N.OnnxModel.from_bytes(builders.build(kind).SerializeToString())
    plan = to_device(compile_onnx(m), "cuda", precision)
    sc = GpuScorer(cfg, store, plan=plan, model="plan", update_features=False)
    sc.capture()
    rng = np.random.default_rng(4)
    from igaming_platform_amd.utils.synth import make_requests
    n_rows = 10240 if precision == "fp32" else 1024
    req = make_requests(pop, n_rows, rng, NOW, hot_frac=0.1)
    outs = [sc.score(req[i:i + 1024], now=NOW) for i in range(0, n_rows, 1024)]
    out = {k: np.concatenate([o[k] for o in outs]) for k in ("ml", "score", "action", "reasons")}
    gs = [golden_score(cfg, gold, pop, row, NOW, model="none") for row in req]
    Xg = np.stack([g["x"] for g in gs]).astype(np.float32)
    ref = N.Executor(m).run({"input": Xg})["output"]
    ml_ref = np.array([GS.clamp01_f32(v) for v in ref[:, plan.ml_col]], np.float32)
    if precision == "fp32":
        np.testing.assert_allclose(out["ml"], ml_ref, atol=1e-5, rtol=0)
    else:
        np.testing.assert_allclose(out["ml"], ml_ref, atol=2e-2)
    bad = []
    for i, g in enumerate(gs):
        ml = float(ml_ref[i]) if precision == "fp32" else float(out["ml"][i])
        score, action, reasons, _ = GS.ensemble(cfg.scoring, g["rule"], g["reasons"], ml)
        mask = sum(1 << REASON_BIT[r] for r in reasons)
        if (out["score"][i], out["action"][i], out["reasons"][i]) != (score, action, mask):
            bad.append((i, out["score"][i], score, out["action"][i], action))
    assert not bad, f"{len(bad)} of {n_rows} decisions differ: {bad[:5]}"


# ----------------------------------------------------------------------------- LTV
def test_ltv_kernel_matches_golden():
    import torch
    from igaming_platform_amd.ops import kernels as K
    rng = np.random.default_rng(3)
    n = 3000
    rows = []
    for i in range(n):
        f = GL.PlayerFeatures(
            days_since_registration=int(rng.integers(0, 400)), days_since_last_deposit=int(rng.integers(0, 60)),
            days_since_last_bet=int(rng.integers(0, 60)), sessions_per_week=float(np.float32(rng.uniform(0, 8))),
            total_deposits=float(np.float32(rng.uniform(0, 5e4))), total_withdrawals=float(np.float32(rng.uniform(0, 5e4))),
            net_revenue=float(np.float32(rng.normal(500, 3000))), deposit_frequency=float(np.float32(rng.uniform(0, 6))),
            bet_count=int(rng.integers(0, 300)), games_played=int(rng.integers(0, 20)),
            bonuses_claimed=int(rng.integers(0, 6)), bonus_conversion_rate=float(np.float32(rng.uniform(0, 1))),
            push_enabled=bool(rng.integers(0, 2)), email_opt_in=bool(rng.integers(0, 2)),
            has_vip_manager=bool(rng.integers(0, 2)), support_tickets=int(rng.integers(0, 6)))
        rows.append(f)
    pf = torch.tensor(np.array([f.row() for f in rows], np.float32)).cuda()
    out = torch.zeros((n, 6), dtype=torch.float32, device="cuda")
    K.ltv(pf, out)
    o = out.cpu().numpy()
    for i, f in enumerate(rows):
        p = GL.predict(f)
        assert np.float32(o[i, 0]) == np.float32(p.predicted_ltv), i
        assert np.float32(o[i, 1]) == np.float32(p.churn_risk), i
        assert int(o[i, 2]) == p.survival_days and int(o[i, 4]) == p.segment, i
        assert np.float32(o[i, 3]) == np.float32(p.confidence), i
        assert GL.NBA_CODES[int(o[i, 5])] == p.next_best_action, i


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
@pytest.mark.parametrize("M,K,N1,act1,act2,xbf", [
    (8192, 32, 256, "relu", "sigmoid", False), (100, 512, 512, "relu", "none", True),
    (1, 64, 64, "tanh", "sigmoid", False), (4097, 256, 130, "relu", "sigmoid", True),
])
def test_mlp_head_matches_torch_fp32(M, K, N1, act1, act2, xbf, precision):
    import torch
    from igaming_platform_amd.models.plan import HeadStep, to_device, Plan
    from igaming_platform_amd.ops import kernels as K_
    g = torch.Generator().manual_seed(M + K + N1)
    X = torch.randn(M, K, generator=g)
    if xbf:
        X = X.to(torch.bfloat16).float()
    W1 = torch.randn(N1, K, generator=g) / K ** 0.5
    b1 = torch.randn(N1, generator=g) * 0.1
    w2 = torch.randn(N1, generator=g) / N1 ** 0.5
    hs = HeadStep(n1=N1, k=K, act1=act1, act2=act2, w1_np=W1.numpy(), b1_np=b1.numpy(), w2_np=w2.numpy(), b2=0.3)
    to_device(Plan("t", K, [hs], 1, 0, {}, "input", "output"), "cuda", precision)
    Y = torch.zeros(M, 1, device="cuda")
    K_.mlp_head(hs, (X.to(torch.bfloat16) if xbf else X).cuda(), Y, M)
    f = {"relu": torch.relu, "sigmoid": torch.sigmoid, "tanh": torch.tanh, "none": lambda t: t}
    h32 = f[act1](X.double() @ W1.double().T + b1.double())
    ref32 = f[act2](h32 @ w2.double() + 0.3).float()
    if precision == "fp32":
        torch.testing.assert_close(Y[:, 0].cpu(), ref32, rtol=1e-5, atol=1e-5)
    else:
        h = f[act1](X.to(torch.bfloat16).float() @ W1.to(torch.bfloat16).float().T + b1)
        ref = f[act2](h @ w2 + 0.3)
        torch.testing.assert_close(Y[:, 0].cpu(), ref, rtol=3e-3, atol=3e-3)
