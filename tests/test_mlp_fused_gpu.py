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


def test_mlp_chain_64_row_tiles_match_32(monkeypatch):
    """64 rows x 8 waves per workgroup (4 x 4 MFMA tiles per wave) computes every row with the
    same bf16 operands in the same k order as the 32-row tiles: bit-identical outputs, also
    with a live count that ends inside a tile."""
    import torch
    from igaming_platform_amd.models.plan import DenseStep, HeadStep
    from igaming_platform_amd.ops import kernels as K
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(5)
    dims = [(256, 512), (512, 512), (512, 512), (512, 512)]
    steps = [DenseStep(n=n, k=k, act="relu", w_np=rng.normal(0, 0.05, (n, k)).astype(np.float32),
                       b_np=rng.normal(0, 0.1, n).astype(np.float32)) for k, n in dims[:-1]]
    steps.append(HeadStep(n1=512, k=512, act1="relu", act2="none",
                          w1_np=rng.normal(0, 0.05, (512, 512)).astype(np.float32),
                          b1_np=rng.normal(0, 0.1, 512).astype(np.float32),
                          w2_np=rng.normal(0, 0.1, 512).astype(np.float32), b2=0.2))
    pk = K.MlpChainPack(steps, dev)
    assert pk.waves() == 8
    n = 1000
    X = torch.from_numpy(rng.normal(0, 1, (n, 256)).astype(np.float32)).to(dev)
    m_ptr = torch.tensor([n - 23], dtype=torch.int32, device=dev)
    outs = {}
    for rows in ("32", "64"):
        monkeypatch.setenv("IGP_MLP_ROWS", rows)
        ml = torch.full((n,), -7.0, device=dev)
        K.mlp_chain(pk, n, X=X, ml=ml, m_ptr=m_ptr)
        torch.cuda.synchronize()
        outs[rows] = ml.cpu()
    assert torch.equal(outs["32"], outs["64"])
    assert torch.all(outs["64"][n - 23:] == -7.0) and not torch.any(outs["64"][:n - 23] == -7.0)


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


def test_mlp_chain_split_mode_matches_fp32_reference():
    """The f32-faithful split mode (bf16 hi/lo pairs, three MFMAs per product) against a plain
    PyTorch fp32 (no bf16 anywhere) reference of the same chain: ~1e-5, where the bf16 mode
    is ~1e-3 off."""
    import torch
    from igaming_platform_amd.models.plan import DenseStep, HeadStep
    from igaming_platform_amd.ops import kernels as K
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(3)
    dims = [(256, 512), (512, 512), (512, 512)]
    steps = [DenseStep(n=n, k=k, act="relu", w_np=rng.normal(0, 1 / np.sqrt(k), (n, k)).astype(np.float32),
                       b_np=rng.normal(0, 0.05, n).astype(np.float32)) for k, n in dims]
    steps.append(HeadStep(n1=512, k=512, act1="relu", act2="none",
                          w1_np=rng.normal(0, 1 / np.sqrt(512), (512, 512)).astype(np.float32),
                          b1_np=rng.normal(0, 0.05, 512).astype(np.float32),
                          w2_np=rng.normal(0, 1 / np.sqrt(512), 512).astype(np.float32), b2=0.1))
    n = 4100
    X = torch.from_numpy(rng.normal(0, 1, (n, 256)).astype(np.float32)).to(dev)
    h = X.double()
    for s in steps[:-1]:
        h = torch.relu(h @ torch.from_numpy(s.w_np).to(dev).double().T + torch.from_numpy(s.b_np).to(dev).double())
    hs = steps[-1]
    z = torch.relu(h @ torch.from_numpy(hs.w1_np).to(dev).double().T + torch.from_numpy(hs.b1_np).to(dev).double())
    ref = (z @ torch.from_numpy(hs.w2_np).to(dev).double() + hs.b2).cpu().numpy()
    errs = {}
    for split in (True, False):
        pk = K.MlpChainPack(steps, dev, split=split)
        ml = torch.full((n,), -1.0, device=dev)
        K.mlp_chain(pk, n, X=X, ml=ml)
        torch.cuda.synchronize()
        errs[split] = float(np.abs(ml.cpu().numpy() - ref).max() / np.abs(ref).max())
    assert errs[True] < 1e-4, errs
    assert errs[True] < errs[False] / 20, errs   # the split mode is far closer to fp32 than bf16


def test_mlp_chain_split_64_row_tiles_match_32(monkeypatch):
    """The f32-faithful split chain at 64 rows per workgroup (hi + lo tiles in LDS once, each
    overwritten in place after every wave read it) equals the 32-row split chain bit for bit."""
    import torch
    from igaming_platform_amd.models.plan import DenseStep, HeadStep
    from igaming_platform_amd.ops import kernels as K
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(8)
    steps = [DenseStep(n=512, k=k, act="relu", w_np=rng.normal(0, 1 / np.sqrt(k), (512, k)).astype(np.float32),
                       b_np=rng.normal(0, 0.05, 512).astype(np.float32)) for k in (256, 512, 512)]
    steps.append(HeadStep(n1=512, k=512, act1="relu", act2="none",
                          w1_np=rng.normal(0, 1 / np.sqrt(512), (512, 512)).astype(np.float32),
                          b1_np=rng.normal(0, 0.05, 512).astype(np.float32),
                          w2_np=rng.normal(0, 1 / np.sqrt(512), 512).astype(np.float32), b2=0.1))
    pk = K.MlpChainPack(steps, dev, split=True)
    n = 1500
    X = torch.from_numpy(rng.normal(0, 1, (n, 256)).astype(np.float32)).to(dev)
    m_ptr = torch.tensor([n - 29], dtype=torch.int32, device=dev)
    outs = {}
    for rows in ("32", "64"):
        monkeypatch.setenv("IGP_MLP_SPLIT_ROWS", rows)
        ml = torch.full((n,), -7.0, device=dev)
        K.mlp_chain(pk, n, X=X, ml=ml, m_ptr=m_ptr)
        torch.cuda.synchronize()
        outs[rows] = ml.cpu()
    assert torch.equal(outs["32"], outs["64"])
    assert torch.all(outs["64"][n - 29:] == -7.0) and not torch.any(outs["64"][:n - 29] == -7.0)


def test_ltv_fp32_plan_runs_the_split_chain_and_matches_the_executor():
    """An fp32 LTV plan takes the fused chain in split mode; over 12288 players (table gather in
    the kernel) its model output matches the C++ fp32 executor of the ONNX model (the reference
    contract, onnx_model.go:369-399) to 1e-4 relative, and the K9 segments / next-best actions
    equal the golden LTV rules fed with the executor's output."""
    import torch
    from igaming_platform_amd.engine.ltv import LtvGpu
    from igaming_platform_amd.golden import ltv as GL
    from igaming_platform_amd.models.plan import compile_onnx, to_device
    from igaming_platform_amd.native import native
    from igaming_platform_amd.onnx import builders
    from igaming_platform_amd.ops import kernels as K
    dev = torch.device("cuda", 0)
    N = native()
    m = N.OnnxModel.from_bytes(builders.build("ltv_mlp", n_features=256, width=512, layers=4).SerializeToString())
    plan = to_device(compile_onnx(m), dev, "fp32")
    cap = 12288
    rng = np.random.default_rng(5)
    pf = np.floor(rng.uniform(0, 1, (cap, 25)) * np.array(
        [900, 90, 60, 500, 10, 120, 1e5, 8e4, 3e4, 500, 8, 5e3, 2e5, 1.8e5, 3000, 1, 80, 60, 20, 15, 1, 1, 1, 1, 8]))
    pf = pf.astype(np.float32)
    ext = rng.normal(0, 1, (cap, 231)).astype(np.float32)
    g = LtvGpu(dev, cap, plan, buckets=[4096])
    assert g.chain is not None and g.chain.split
    g.set_rows(np.arange(cap), pf, ext)
    slots = torch.arange(cap, dtype=torch.int32, device=dev)
    ml = torch.zeros(cap, device=dev)
    out = torch.zeros((cap, 6), device=dev)
    K.mlp_chain(g.chain, cap, slots=slots, pf_tab=g.pf_tab, ext_tab=g.ext_tab, ml=ml, ltv_out=out)
    torch.cuda.synchronize()
    X = np.concatenate([np.sign(pf) * np.log1p(np.abs(pf)), ext], 1).astype(np.float32)
    ref = N.Executor(m).run({"input": X})["output"].reshape(-1)
    got = ml.cpu().numpy()
    assert float(np.abs(got - ref).max()) / float(np.abs(ref).max()) < 1e-4
    o = out.cpu().numpy()
    want = [GL.predict(GL.PlayerFeatures.from_row(pf[i]), ltv_override=float(ref[i])) for i in range(cap)]
    assert [int(x) for x in o[:, 4]] == [w.segment for w in want]


def test_ltv_chain_host_outputs_equal_device_outputs(monkeypatch):
    """IGP_LTV_HOST_OUT=1: the chain's K9 epilogue stores the rows into the slot's pinned host
    buffer (no D2H copy); IGP_LTV_HOST_IN=1 also reads [n | slots] from the pinned slab (no
    H2D); results equal the device-buffer + copy path, batch by batch."""
    import torch
    from igaming_platform_amd.models.plan import compile_onnx, to_device
    from igaming_platform_amd.native import native
    from igaming_platform_amd.onnx import builders
    dev = torch.device("cuda", 0)
    m = native().OnnxModel.from_bytes(builders.build("ltv_mlp", n_features=256, width=512, layers=4).SerializeToString())
    plan = to_device(compile_onnx(m), dev, "fp32")
    cap = 4096
    rng = np.random.default_rng(4)
    pf = np.floor(rng.uniform(0, 1, (cap, 25)) * 700).astype(np.float32)
    ext = rng.normal(0, 1, (cap, 231)).astype(np.float32)
    batches = [rng.integers(0, cap, 1000 + 300 * i).astype(np.int32) for i in range(4)]
    outs = {}
    for host in ("0", "1", "in"):
        monkeypatch.setenv("IGP_LTV_HOST_OUT", "0" if host == "0" else "1")
        monkeypatch.setenv("IGP_LTV_HOST_IN", "1" if host == "in" else "0")
        g = _ltv_gpu(True, plan, dev, cap)
        assert g._host_out == (host != "0") and g._host_in == (host == "in")
        g.set_rows(np.arange(cap), pf, ext)
        outs[host] = [g.predict_slots(s) for s in batches]
    for a, b, c in zip(outs["0"], outs["1"], outs["in"]):
        np.testing.assert_array_equal(a, b)
        np.testing.assert_array_equal(a, c)
