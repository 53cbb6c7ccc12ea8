"""ai.onnx.ml linear models / preprocessing and DAG-shaped models.

* C++ executor (csrc/runtime/executor.cpp): LinearClassifier, LinearRegressor, Scaler,
  Normalizer, ZipMap against numpy implementations of the operator definitions (ORT is not
  available offline: ORT parity is unpinned; these pin the ai.onnx.ml definitions).
* Plan lowering (models/plan.py): Scaler folds into the next layer, LinearClassifier becomes a
  dense layer / the fused head, Add / Concat of two branches become join steps. The lowered
  plan is evaluated with numpy on the host and compared with the executor - the same math the
  device kernels run (tests/test_onnx_ml_gpu.py runs it on the device).
"""
import numpy as np
import pytest
from scipy.special import erfinv

from igaming_platform_amd.models.plan import PlanError, compile_onnx, executor_output, step_inputs
from igaming_platform_amd.native import native
from igaming_platform_amd.onnx import builders
from igaming_platform_amd.onnx import schema as S
from igaming_platform_amd.onnx.writer import ML_DOMAIN, model, node, value_info

N = native()


def _run(m, X, out="output"):
    return N.Executor(N.OnnxModel.from_bytes(m.SerializeToString())).run({"input": np.ascontiguousarray(X, np.float32)})


def _post(z, post):
    z = np.asarray(z, np.float64)
    if post == "LOGISTIC":
        return 1 / (1 + np.exp(-z))
    if post in ("SOFTMAX", "SOFTMAX_ZERO"):
        keep = np.ones_like(z, bool) if post == "SOFTMAX" else z != 0
        m = np.where(keep, z, -np.inf).max(axis=1, keepdims=True)
        e = np.where(keep, np.exp(z - np.where(np.isfinite(m), m, 0)), 0)
        tot = e.sum(axis=1, keepdims=True)
        return e / np.where(tot > 0, tot, 1)  # an all-zero row stays zero
    if post == "PROBIT":
        return np.sqrt(2) * erfinv(2 * z - 1)
    return z


def _attrs(m, op):
    n = next(n for n in m.graph.node if n.op_type == op)
    out = {}
    for a in n.attribute:
        out[a.name] = (np.asarray(a.floats) if a.floats else np.asarray(a.ints) if a.ints
                       else [s.decode() for s in a.strings] if a.strings else a.s.decode() if a.s else a.i)
    return out


def _scaled(m, X):
    a = _attrs(m, "Scaler")
    return (X.astype(np.float64) - a["offset"]) * a["scale"]


@pytest.mark.parametrize("classes,post", [(2, "NONE"), (2, "LOGISTIC"), (3, "NONE"), (3, "LOGISTIC"),
                                          (3, "SOFTMAX"), (4, "SOFTMAX_ZERO"), (2, "SOFTMAX")])
def test_linear_classifier_matches_numpy(classes, post):
    m = builders.sklearn_linear(n_features=12, classes=classes, post=post, zipmap=classes != 4)
    X = np.random.default_rng(1).standard_normal((300, 12)).astype(np.float32)
    y = _run(m, X)
    a = _attrs(m, "LinearClassifier")
    E = len(a["intercepts"])
    raw = _scaled(m, X) @ a["coefficients"].reshape(E, -1).T + a["intercepts"]
    z = np.concatenate([-raw, raw], 1) if E == 1 else raw
    want = _post(z, post)
    np.testing.assert_allclose(y["output"], want, atol=1e-5, rtol=1e-5)
    lab = (raw[:, 0] > 0).astype(np.int64) if E == 1 else raw.argmax(1)
    np.testing.assert_array_equal(y["label"], lab)


def test_linear_classifier_string_labels_softmax_zero_and_probit():
    # string class labels: the executor's label tensor carries the class index
    m = builders.sklearn_linear(n_features=6, classes=3, post="NONE", string_labels=True)
    X = np.random.default_rng(2).standard_normal((50, 6)).astype(np.float32)
    y = _run(m, X)
    a = _attrs(m, "LinearClassifier")
    raw = _scaled(m, X) @ a["coefficients"].reshape(3, -1).T + a["intercepts"]
    np.testing.assert_array_equal(y["label"], raw.argmax(1))
    # SOFTMAX_ZERO leaves exact-zero scores at zero; PROBIT maps probabilities through erfinv
    coef = np.array([[1, 0], [0, 1], [0, 0]], np.float32)
    for post, X2 in (("SOFTMAX_ZERO", np.array([[0.5, 0.0], [0.0, 0.0], [2.0, -1.0]], np.float32)),
                     ("PROBIT", np.array([[0.2, 0.7], [0.9, 0.4]], np.float32))):
        g = model([node("LinearClassifier", ["input"], ["label", "output"], domain=ML_DOMAIN,
                        coefficients=coef.ravel(), intercepts=np.zeros(3, np.float32), post_transform=post,
                        classlabels_ints=np.array([5, 6, 7], np.int64))],
                  [value_info("input", S.FLOAT, ["N", 2])],
                  [value_info("label", S.INT64, ["N"]), value_info("output", S.FLOAT, ["N", 3])])
        y = _run(g, X2)
        np.testing.assert_allclose(y["output"], _post(X2.astype(np.float64) @ coef.T, post), atol=1e-5)
        np.testing.assert_array_equal(y["label"], np.array([5, 6, 7])[(X2 @ coef.T).argmax(1)])


@pytest.mark.parametrize("targets,post", [(1, "NONE"), (3, "NONE"), (2, "LOGISTIC")])
def test_linear_regressor_matches_numpy(targets, post):
    m = builders.linear_regressor(n_features=10, targets=targets, post=post)
    X = np.random.default_rng(3).standard_normal((200, 10)).astype(np.float32)
    a = _attrs(m, "LinearRegressor")
    want = _post(_scaled(m, X) @ a["coefficients"].reshape(targets, -1).T + a["intercepts"], post)
    np.testing.assert_allclose(_run(m, X)["output"], want, atol=1e-5, rtol=1e-5)


@pytest.mark.parametrize("norm", ["MAX", "L1", "L2"])
def test_normalizer_and_scalar_scaler(norm):
    X = np.random.default_rng(4).standard_normal((64, 9)).astype(np.float32)
    X[3] = 0.25  # scales to an all-zero row: left unchanged
    g = model([node("Scaler", ["input"], ["s"], domain=ML_DOMAIN, offset=[0.25], scale=[2.0]),
               node("Normalizer", ["s"], ["output"], domain=ML_DOMAIN, norm=norm)],
              [value_info("input", S.FLOAT, ["N", 9])], [value_info("output", S.FLOAT, ["N", 9])])
    s = (X.astype(np.float64) - 0.25) * 2.0
    d = {"MAX": s.max(1, keepdims=True), "L1": np.abs(s).sum(1, keepdims=True),
         "L2": np.sqrt((s * s).sum(1, keepdims=True))}[norm]
    want = np.where(d != 0, s / np.where(d == 0, 1, d), s)
    np.testing.assert_allclose(_run(g, X)["output"], want, atol=1e-5, rtol=1e-5)


# ------------------------------------------------------------------ lowering
ACT = {"none": lambda v: v, "relu": lambda v: np.maximum(v, 0), "sigmoid": lambda v: 1 / (1 + np.exp(-v)),
       "tanh": np.tanh}


def run_plan_numpy(plan, X):
    """The lowered plan evaluated on the host: what K3 dense / head and join compute."""
    vals = []

    def val(k):
        return X.astype(np.float64) if k < 0 else vals[k]
    for i, s in enumerate(plan.steps):
        if s.kind == "join":
            a, b = val(s.a)[:, :s.na], val(s.b)[:, :s.nb]
            y = a + b if s.op == "add" else np.concatenate([a, b], 1)
        elif s.kind == "dense":
            x = val(step_inputs(plan.steps, i)[0])[:, :s.k]
            y = ACT[s.act](x @ s.w_np.T.astype(np.float64) + (0 if s.b_np is None else s.b_np))
        elif s.kind == "head":
            x = val(step_inputs(plan.steps, i)[0])[:, :s.k]
            h = ACT[s.act1](x @ s.w1_np.T.astype(np.float64) + (0 if s.b1_np is None else s.b1_np))
            y = ACT[s.act2](h @ s.w2_np + s.b2)[:, None]
        else:
            raise AssertionError(s.kind)
        vals.append(y)
    return vals[-1]


CASES = [("sklearn_linear", dict(n_features=16, classes=2, post="LOGISTIC"), ["dense"]),
         ("sklearn_linear", dict(n_features=16, classes=2, post="NONE", zipmap=False), ["dense"]),
         ("sklearn_linear", dict(n_features=16, classes=2, post="SOFTMAX"), ["dense"]),
         ("sklearn_linear", dict(n_features=16, classes=3, post="LOGISTIC"), ["dense"]),
         ("linear_regressor", dict(n_features=16, targets=2), ["dense"]),
         ("mlp_classifier", dict(n_features=16, hidden=64), ["head"]),
         ("wide_deep", dict(n_features=16), ["dense", "dense", "dense", "join", "dense"]),
         ("residual_mlp", dict(n_features=16, width=64, blocks=2),
          ["dense", "dense", "dense", "join", "dense", "dense", "join", "dense"])]


@pytest.mark.parametrize("kind,kw,kinds", CASES, ids=[f"{c[0]}-{i}" for i, c in enumerate(CASES)])
def test_plan_lowering_matches_executor(kind, kw, kinds):
    m = builders.build(kind, **kw)
    om = N.OnnxModel.from_bytes(m.SerializeToString())
    plan = compile_onnx(om)
    assert [s.kind for s in plan.steps] == kinds, plan.describe()
    X = np.random.default_rng(5).standard_normal((257, kw["n_features"])).astype(np.float32)
    ref = np.asarray(N.Executor(om).run({"input": X})["output"]).reshape(len(X), -1)
    got = run_plan_numpy(plan, X)
    np.testing.assert_allclose(got[:, plan.ml_col], ref[:, plan.executor_col], atol=1e-5, rtol=1e-5)
    assert executor_output(om) == (plan.executor_col, "output")
    if kind in ("sklearn_linear", "mlp_classifier") and kw.get("classes", 2) == 2:
        # a binary classifier runs as one positive-class column on the device
        assert plan.out_width == 1 and plan.ml_col == 0 and plan.executor_col == 1
    if kind in ("wide_deep", "residual_mlp"):
        assert not plan.is_chain
        joins = [s for s in plan.steps if s.kind == "join"]
        assert {s.op for s in joins} == ({"concat"} if kind == "wide_deep" else {"add"})


def test_plan_folds_constant_arithmetic_into_layers():
    """Sub / Mul / Div by constants around dense layers fold into weights and biases (no extra
    step), and a scaling that cannot fold (after a Relu with another reader) materialises."""
    rng = np.random.default_rng(6)
    from igaming_platform_amd.onnx.writer import tensor
    w1 = rng.standard_normal((8, 16)).astype(np.float32)
    w2 = rng.standard_normal((16, 1)).astype(np.float32)
    c = rng.uniform(0.5, 1.5, 8).astype(np.float32)
    g = model([node("Sub", ["input", "c"], ["a"]), node("Div", ["a", "two"], ["b"]),
               node("MatMul", ["b", "W1"], ["h"]), node("Mul", ["h", "half"], ["h2"]), node("Relu", ["h2"], ["r"]),
               node("Mul", ["r", "three"], ["r3"]), node("Add", ["r3", "r"], ["j"]),
               node("MatMul", ["j", "W2"], ["o"]), node("Sigmoid", ["o"], ["output"])],
              [value_info("input", S.FLOAT, ["N", 8])], [value_info("output", S.FLOAT, ["N", 1])],
              [tensor("c", c), tensor("two", np.array([2.0], np.float32)), tensor("half", np.array([0.5], np.float32)),
               tensor("three", np.array([3.0], np.float32)), tensor("W1", w1), tensor("W2", w2)])
    om = N.OnnxModel.from_bytes(g.SerializeToString())
    plan = compile_onnx(om)
    # Sub / Div fold into W1, Mul 0.5 folds into W1 too (before the Relu); Mul 3 after the Relu
    # has another reader (the Add) -> one diagonal layer; the Add of two branches -> join
    assert [s.kind for s in plan.steps] == ["dense", "dense", "join", "dense"], plan.describe()
    X = rng.standard_normal((64, 8)).astype(np.float32)
    ref = np.asarray(N.Executor(om).run({"input": X})["output"])
    np.testing.assert_allclose(run_plan_numpy(plan, X), ref, atol=1e-5, rtol=1e-5)


def test_plan_refuses_what_the_device_cannot_run():
    for m, msg in [(builders.sklearn_linear(n_features=8, classes=3, post="SOFTMAX"), "CPU-only"),
                   (model([node("Normalizer", ["input"], ["output"], domain=ML_DOMAIN, norm="L2")],
                          [value_info("input", S.FLOAT, ["N", 8])], [value_info("output", S.FLOAT, ["N", 8])]),
                    "not lowered")]:
        om = N.OnnxModel.from_bytes(m.SerializeToString())
        with pytest.raises(PlanError, match=msg):
            compile_onnx(om)
    # the label output is not a device value
    m = builders.sklearn_linear(n_features=8, classes=2)
    with pytest.raises(PlanError, match="score"):
        compile_onnx(N.OnnxModel.from_bytes(m.SerializeToString()), output_name="label")
    # a binary classifier the device cannot run still reports its positive column to the executor path
    g = model([node("Normalizer", ["input"], ["n"], domain=ML_DOMAIN, norm="L2"),
               node("LinearClassifier", ["n"], ["label", "output"], domain=ML_DOMAIN,
                    coefficients=np.ones(8, np.float32), intercepts=np.zeros(1, np.float32),
                    post_transform="LOGISTIC", classlabels_ints=np.array([0, 1], np.int64))],
              [value_info("input", S.FLOAT, ["N", 8])],
              [value_info("label", S.INT64, ["N"]), value_info("output", S.FLOAT, ["N", 2])])
    assert executor_output(N.OnnxModel.from_bytes(g.SerializeToString())) == (1, "output")


@pytest.mark.parametrize("backend", ["cpu", "golden"])
def test_engine_scores_an_sklearn_pipeline_with_the_positive_class(backend):
    """A Scaler -> LinearClassifier -> ZipMap fraud model in the engine: ml_score is the
    positive-class probability - the same scores as the equivalent core-ONNX graph
    (Sub -> Mul -> Gemm -> Sigmoid) on the same traffic."""
    from igaming_platform_amd.config import Config
    from igaming_platform_amd.engine.risk_engine import RiskEngine
    from igaming_platform_amd.onnx.writer import tensor
    from tests.test_engine_cpu import NOW, _txs
    m = builders.sklearn_linear(n_features=30, classes=2, post="LOGISTIC")
    sa, la = _attrs(m, "Scaler"), _attrs(m, "LinearClassifier")
    core = model([node("Sub", ["input", "off"], ["a"]), node("Mul", ["a", "sc"], ["b"]),
                  node("Gemm", ["b", "W", "B"], ["z"]), node("Sigmoid", ["z"], ["output"])],
                 [value_info("input", S.FLOAT, ["N", 30])], [value_info("output", S.FLOAT, ["N", 1])],
                 [tensor("off", sa["offset"].astype(np.float32)), tensor("sc", sa["scale"].astype(np.float32)),
                  tensor("W", la["coefficients"].astype(np.float32).reshape(30, 1)),
                  tensor("B", la["intercepts"].astype(np.float32))])
    txs = _txs(60, np.random.default_rng(7))
    scores = []
    for fm in (m, core):
        eng = RiskEngine(Config(), backend=backend, capacity=64, fraud_model=fm.SerializeToString())
        scores.append(np.array([r["ml_score"] for r in eng.score(txs, now=NOW)], np.float64))
        eng.close()
    assert np.all((scores[0] > 0) & (scores[0] < 1)) and np.ptp(scores[0]) > 0.01
    np.testing.assert_allclose(scores[0], scores[1], atol=1e-6)
