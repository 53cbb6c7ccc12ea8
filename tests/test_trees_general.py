"""General TreeEnsembles on the device path, CPU side: the plan now lowers every TreeEnsemble
(depth > 12 and unbalanced trees on the pointer layout, MIN / MAX aggregates, all five post
transforms) instead of dropping it to the CPU executor; the pointer layout evaluated by its
host twin equals the executor; corrupted layouts are rejected before upload."""
import numpy as np
import pytest

from tests import tree_models as TM


def _plan(m):
    from igaming_platform_amd.models.plan import compile_onnx
    from igaming_platform_amd.native import native
    return compile_onnx(native().OnnxModel.from_bytes(m.SerializeToString()))


@pytest.mark.parametrize("kind", TM.SKLEARN)
def test_sklearn_ensembles_lower_to_the_sparse_layout_and_match_the_executor(kind):
    m, X = TM.build(kind)
    plan = _plan(m)
    (ts,) = [s for s in plan.steps if s.kind == "tree"]
    assert ts.layout == "sparse", plan.describe()
    if kind == "gb_d16":
        assert ts.depth > 12
    if kind in ("rf_min", "rf_max"):
        assert ts.aggregate == {"rf_min": 2, "rf_max": 3}[kind]
    ref, _ = TM.executor_output(m, X)
    got = TM.sparse_eval(ts, X)
    np.testing.assert_allclose(got.reshape(ref.shape), ref, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("kind", TM.SYNTHETIC)
def test_post_transforms_lower_to_the_device(kind):
    m, X = TM.build(kind)
    plan = _plan(m)
    (ts,) = [s for s in plan.steps if s.kind == "tree"]
    want_post = {"softmax_zero4": 3, "softmax3": 2, "probit_reg4": 4, "binary_softmax": 2, "binary_probit": 4}[kind]
    assert ts.post == want_post
    # K = 3 has no complete-kernel instance: it goes to the pointer layout
    assert ts.layout == ("sparse" if kind == "softmax3" else "complete")


@pytest.mark.parametrize("kind", ["softmax3", "softmax_zero4", "binary_probit"])
def test_forced_sparse_layout_matches_executor(kind, monkeypatch):
    monkeypatch.setenv("IGP_TREE_LAYOUT", "sparse")
    m, X = TM.build(kind)
    (ts,) = [s for s in _plan(m).steps if s.kind == "tree"]
    assert ts.layout == "sparse"
    ref, _ = TM.executor_output(m, X)
    np.testing.assert_allclose(TM.sparse_eval(ts, X), ref, rtol=1e-5, atol=1e-5)


def test_balanced_gbdt_keeps_the_complete_layout():
    from igaming_platform_amd.onnx import builders
    plan = _plan(builders.build("gbdt"))
    assert plan.steps[0].layout == "complete"
    plan = _plan(builders.build("stacked"))
    assert plan.steps[0].layout == "complete"


def test_validate_sparse_rejects_bad_layouts():
    import copy
    from igaming_platform_amd.models.plan import PlanError, validate_sparse
    m, _ = TM.build("rf_unbalanced")
    (ts,) = [s for s in _plan(m).steps if s.kind == "tree"]
    validate_sparse(ts)
    nodes = ts.nodes_np.reshape(-1, 4)
    inner = np.nonzero(((nodes[:, 0].view(np.uint32) >> 16) & 7) != 7)[0]
    bad = copy.copy(ts)
    bad.nodes_np = ts.nodes_np.copy()
    bad.nodes_np.reshape(-1, 4)[inner[0], 3] = nodes.shape[0] + 5          # child out of range
    with pytest.raises(PlanError):
        validate_sparse(bad)
    bad.nodes_np = ts.nodes_np.copy()
    bad.nodes_np.reshape(-1, 4)[inner[1], 2] = ts.roots_np[0]               # cycle back to a root
    with pytest.raises(PlanError):
        validate_sparse(bad)
    bad = copy.copy(ts)
    bad.depth = 2                                                           # path longer than depth
    with pytest.raises(PlanError):
        validate_sparse(bad)


@pytest.mark.parametrize("kind", ["gb_d16", "rf_unbalanced"])
def test_feature_importance_of_sparse_layout_ensembles(kind):
    """GetFeatureImportance (onnx_model.go:329-345) of deep / unbalanced ensembles that lower to
    the pointer layout: split counts per input column, equal to the sklearn trees' own."""
    from igaming_platform_amd.features.store_ops import input_names, plan_importance
    from igaming_platform_amd.models.plan import compile_onnx
    from igaming_platform_amd.native import native
    from tests import tree_models as TM
    m, _ = TM.build(kind)
    plan = compile_onnx(native().OnnxModel.from_bytes(m.SerializeToString()))
    assert any(s.kind == "tree" and s.layout == "sparse" for s in plan.steps)
    imp = plan_importance(plan, TM.N_FEAT)
    # sklearn's own split features
    from sklearn.ensemble import GradientBoostingClassifier, RandomForestRegressor
    X, y, _ = TM.data()
    if kind == "gb_d16":
        est = GradientBoostingClassifier(n_estimators=25, max_depth=16, learning_rate=0.2, random_state=0).fit(X, y > 0)
        trees = [e[0].tree_ for e in est.estimators_]
    else:
        est = RandomForestRegressor(n_estimators=30, max_depth=None, max_features=0.5, random_state=0).fit(X, y)
        trees = [e.tree_ for e in est.estimators_]
    cnt = np.zeros(TM.N_FEAT)
    for t in trees:
        f = t.feature[t.feature >= 0]
        cnt += np.bincount(f, minlength=TM.N_FEAT)
    names = input_names(TM.N_FEAT)
    got = np.array([imp.get(n, 0.0) for n in names])
    np.testing.assert_allclose(got, cnt / cnt.sum(), rtol=1e-12)
