"""K4 fused GRU kernel vs the C++ CPU executor (fp32 ONNX GRU semantics)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _model(**kw):
    from igaming_platform_amd.models.plan import compile_onnx, to_device
    from igaming_platform_amd.native import native
    from igaming_platform_amd.onnx import builders
    N = native()
    m = N.OnnxModel.from_bytes(builders.build("gru", **kw).SerializeToString())
    plan = to_device(compile_onnx(m), "cuda")
    return N, m, plan


@pytest.mark.parametrize("kw", [
    dict(seq=20, hidden=256, layers=2, linear_before_reset=1, head=True),
    dict(seq=12, hidden=64, layers=1, linear_before_reset=0, head=False),
    dict(seq=16, hidden=128, layers=2, linear_before_reset=0, head=True, in_dim=40),
])
def test_gru_dense_input_matches_executor(kw):
    import torch
    from igaming_platform_amd.engine.runner import DeviceModel
    N, m, plan = _model(**kw)
    T, I = kw["seq"], kw.get("in_dim", 16)
    rng = np.random.default_rng(1)
    for rows in (5, 100, 6200):
        X = rng.standard_normal((T, rows, I)).astype(np.float32)
        ref = N.Executor(m).run({"input": X})["output"]
        dm = DeviceModel(plan, "cuda", [rows])
        out = dm.run(torch.from_numpy(X).cuda(), rows)
        got = out[:rows].cpu().numpy().reshape(ref.shape)
        np.testing.assert_allclose(got, ref, rtol=0, atol=1e-2)
        assert np.abs(got - ref).mean() < 2e-3


def test_gru_event_ring_input_matches_executor():
    import torch
    from igaming_platform_amd.config import FeatureConfig
    from igaming_platform_amd.features.device_store import DeviceFeatureStore
    from igaming_platform_amd.layouts import ACCTRT
    from igaming_platform_amd.ops import kernels as K
    N, m, plan = _model(seq=100, hidden=256, layers=2, linear_before_reset=1, head=True)
    fc = FeatureConfig()
    C, R, D = 500, fc.event_ring, fc.event_dim
    store = DeviceFeatureStore(C, fc, "cuda", events=True, max_events=64)
    rng = np.random.default_rng(2)
    ev = rng.standard_normal((C, R, D)).astype(np.float32)
    ev_bf = torch.from_numpy(ev).to(torch.bfloat16)
    store.ev.copy_(ev_bf.view(torch.int16).cuda())
    rt = np.zeros(C, ACCTRT)
    rt["ev_head"] = rng.integers(0, R, C)
    rt["ev_count"] = rng.integers(0, R + 1, C)
    rt["ev_count"][:5] = R
    store.rt.copy_(torch.from_numpy(rt.view(np.int32).reshape(C, -1).copy()).cuda())
    rows = 300
    slots = rng.integers(0, C, rows).astype(np.int32)
    slots[::17] = -1
    # host gather: oldest first, right-aligned, zeros before the first event
    evq = ev_bf.float().numpy()
    X = np.zeros((R, rows, D), np.float32)
    for b, s in enumerate(slots):
        if s < 0:
            continue
        cnt, head = int(rt["ev_count"][s]), int(rt["ev_head"][s])
        for t in range(R - cnt, R):
            X[t, b] = evq[s, (head - R + t) % R]
    ref = N.Executor(m).run({"input": X})["output"].reshape(-1)
    gp = K.GruPack([s for s in plan.steps if s.kind == "gru"], plan.steps[-1], "cuda")
    out = torch.zeros(rows, dtype=torch.float32, device="cuda")
    K.gru(gp, rows, R, out=out, store=store, slots=torch.from_numpy(slots).cuda())
    got = out.cpu().numpy()
    np.testing.assert_allclose(got, ref, rtol=0, atol=1e-2)


def test_gru_respects_live_rows():
    import torch
    from igaming_platform_amd.engine.runner import DeviceModel
    N, m, plan = _model(seq=8, hidden=64, layers=1, linear_before_reset=1, head=True)
    dm = DeviceModel(plan, "cuda", [256])
    X = torch.randn(8, 256, 16, device="cuda")
    dm.out.fill_(-7.0)
    n = torch.tensor([100], dtype=torch.int32, device="cuda")
    dm.run(X, 256, m_ptr=n)
    o = dm.out.cpu().numpy().reshape(-1)
    assert np.all(o[100:] == -7.0) and np.all(o[:100] != -7.0)
