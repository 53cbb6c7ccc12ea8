"""General TreeEnsembles on the GPU vs the C++ executor (fp32, 1e-5): K2b on the pointer
layout for sklearn GradientBoosting at depth 16, fully grown (unbalanced) RandomForests with
AVERAGE / MIN / MAX and PROBIT; the complete-tree kernel with the post transforms it gained
(SOFTMAX_ZERO, binary SOFTMAX / PROBIT, PROBIT regressor); single- and multi-group launches."""
import os

import numpy as np
import pytest

from tests import tree_models as TM

pytestmark = pytest.mark.gpu


def _device_run(m, X, groups=None):
    import torch
    from igaming_platform_amd.engine.runner import DeviceModel
    from igaming_platform_amd.models.plan import compile_onnx, to_device
    from igaming_platform_amd.native import native
    dev = torch.device("cuda", 0)
    plan = to_device(compile_onnx(native().OnnxModel.from_bytes(m.SerializeToString())), dev)
    n = X.shape[0]
    B = -(-n // 64) * 64
    Xp = np.zeros((B, X.shape[1]), np.float32)
    Xp[:n] = X
    old = os.environ.get("IGP_TREE_GROUPS")
    if groups is not None:
        os.environ["IGP_TREE_GROUPS"] = str(groups)
    try:
        dm = DeviceModel(plan, dev, [B])
    finally:
        if groups is not None:
            if old is None:
                os.environ.pop("IGP_TREE_GROUPS")
            else:
                os.environ["IGP_TREE_GROUPS"] = old
    out = dm.run(torch.from_numpy(Xp).to(dev), B)
    torch.cuda.synchronize()
    return plan, out[:n].cpu().numpy(), dm.tree_groups[B]


@pytest.mark.parametrize("kind", TM.SKLEARN)
@pytest.mark.parametrize("groups", [1, None])
def test_sparse_tree_kernel_matches_executor(kind, groups):
    m, X = TM.build(kind)
    plan, got, g = _device_run(m, X, groups)
    assert plan.steps[0].layout == "sparse"
    assert (g == 1) if groups == 1 else (g > 1)
    ref, _ = TM.executor_output(m, X)
    np.testing.assert_allclose(got.reshape(ref.shape), ref, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("kind", TM.SYNTHETIC)
def test_tree_post_transforms_match_executor(kind):
    m, X = TM.build(kind)
    plan, got, _ = _device_run(m, X)
    ref, _ = TM.executor_output(m, X)
    np.testing.assert_allclose(got.reshape(ref.shape), ref, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("kind", ["softmax_zero4", "binary_softmax", "probit_reg4"])
def test_forced_sparse_post_transforms_match_executor(kind, monkeypatch):
    monkeypatch.setenv("IGP_TREE_LAYOUT", "sparse")
    m, X = TM.build(kind)
    plan, got, _ = _device_run(m, X)
    assert plan.steps[0].layout == "sparse"
    ref, _ = TM.executor_output(m, X)
    np.testing.assert_allclose(got.reshape(ref.shape), ref, rtol=1e-5, atol=1e-5)
