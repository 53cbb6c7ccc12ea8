"""K3 fused MLP chain (csrc/kernels/mlp_fused.hip) against a plain PyTorch fp32 reference of the
same bf16 numerics (bf16 weights / activations, f32 accumulation), and the fused LTV path (table
gather + chain + K9 in one kernel) against the unfused layer-kernel path."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _bf(t):
    import torch
    return t.to(torch.bfloat16).to(torch.float32)


def test_mlp_chain_dense_input_matches_reference():
    import torch
    from igaming_platform_amd.models.plan import DenseStep, HeadStep
    from igaming_platform_amd.ops import kernels as K
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(0)
    dims = [(200, 128), (128, 192)]   # input 200 (padded to 256 inside), hidden 128 -> 192
    steps = [DenseStep(n=n, k=k, act="relu", w_np=rng.normal(0, 0.1, (n, k)).astype(np.float32),
                       b_np=rng.normal(0, 0.1, n).astype(np.float32)) for k, n in dims]
    steps.append(HeadStep(n1=64, k=192, act1="relu", act2="sigmoid",
                          w1_np=rng.normal(0, 0.1, (64, 192)).astype(np.float32),
                          b1_np=rng.normal(0, 0.1, 64).astype(np.float32),
                          w2_np=rng.normal(0, 0.3, 64).astype(np.float32), b2=0.1))
    pk = K.MlpChainPack(steps, dev)
    n = 300                                             # not a multiple of the 32-row tile
    X = torch.from_numpy(rng.normal(0, 1, (n, 200)).astype(np.float32)).to(dev)
    ml = torch.full((n,), -1.0, device=dev)
    m_ptr = torch.tensor([n - 5], dtype=torch.int32, device=dev)   # 5 padded rows: not computed
    K.mlp_chain(pk, n, X=X, ml=ml, m_ptr=m_ptr)
    torch.cuda.synchronize()
    h = _bf(X)
    for s in steps[:-1]:
        w = _bf(torch.from_numpy(s.w_np).to(dev))
        h = _bf(torch.relu(h @ w.T + torch.from_numpy(s.b_np).to(dev)))
    hs = steps[-1]
    z = torch.relu(h @ _bf(torch.from_numpy(hs.w1_np).to(dev)).T + torch.from_numpy(hs.b1_np).to(dev))
    ref = torch.sigmoid(z @ torch.from_numpy(hs.w2_np).to(dev) + hs.b2)
    got = ml.cpu().numpy()
    np.testing.assert_allclose(got[:n - 5], ref.cpu().numpy()[:n - 5], atol=2e-3, rtol=2e-3)


def _ltv_gpu(fused: bool, plan, dev, cap):
    from igaming_platform_amd.engine.ltv import LtvGpu
    old = os.environ.get("IGP_MLP_FUSED")
    os.environ["IGP_MLP_FUSED"] = "1" if fused else "0"
    try:
        g = LtvGpu(dev, cap, plan, buckets=[256, 2048])
    finally:
        if old is None:
            os.environ.pop("IGP_MLP_FUSED")
        else:
            os.environ["IGP_MLP_FUSED"] = old
    assert (g.chain is not None) == fused
    return g


def test_fused_ltv_matches_layer_kernels():
    import torch
    from igaming_platform_amd.models.plan import compile_onnx, to_device
    from igaming_platform_amd.native import native
    from igaming_platform_amd.onnx import builders
    dev = torch.device("cuda", 0)
    m = native().OnnxModel.from_bytes(builders.build("ltv_mlp", n_features=256, width=512, layers=4).SerializeToString())
    plan = to_device(compile_onnx(m), dev, "bf16")
    cap = 4096
    rng = np.random.default_rng(1)
    pf = np.floor(rng.uniform(0, 1, (cap, 25)) * np.array(
        [900, 90, 60, 500, 10, 120, 1e5, 8e4, 3e4, 500, 8, 5e3, 2e5, 1.8e5, 3000, 1, 80, 60, 20, 15, 1, 1, 1, 1, 8]))
    ext = rng.normal(0, 1, (cap, 231)).astype(np.float32)
    outs = []
    for fused in (True, False):
        g = _ltv_gpu(fused, plan, dev, cap)
        g.set_rows(np.arange(cap), pf.astype(np.float32), ext)
        slots = rng.integers(0, cap, 1500).astype(np.int32) if not outs else slots  # noqa: F821
        slots[::97] = -1
        outs.append(g.predict_slots(slots))
    a, b = outs
    np.testing.assert_array_equal(a[:, 1:4], b[:, 1:4])           # churn, survival, confidence
    np.testing.assert_allclose(a[:, 0], b[:, 0], rtol=2e-2, atol=1e-2)   # learned LTV (bf16 chain)
    assert np.mean(a[:, 4] == b[:, 4]) > 0.98                     # segment (threshold flips allowed)
