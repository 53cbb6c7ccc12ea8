"""Deterministic random-init ONNX models for the five BASELINE configs.

There is no network for trained checkpoints (BASELINE.json: "random-init model weights"),
so each config's model is generated from a fixed seed with the architecture the config
names. Input name ``input`` / primary output ``output`` follow ``onnx_model.go:37-38``.

* cfg1 ``logistic``: input[N,32] -> Gemm -> Sigmoid -> output[N,1]
* cfg2 ``gbdt``:     input[N,128] -> TreeEnsembleClassifier(100 trees, LOGISTIC)
                      -> label[N], output[N,2]
* cfg3 ``stacked``:  input[N,128] -> TreeEnsembleRegressor(100 trees, n_targets=32)
                      -> Gemm(32x256) -> Relu -> Gemm(256x1) -> Sigmoid -> output[N,1]
* cfg4 ``ltv_mlp``:  input[N,256] -> (Gemm -> Relu) x4 (width 512) -> Gemm -> output[N,1]
* cfg5 ``gru``:      input[T=100,N,16] -> GRU(256) -> Squeeze -> GRU(256) -> Y_h
                      -> Reshape[N,256] -> Gemm -> Sigmoid -> output[N,1]
"""
from __future__ import annotations

from typing import Dict

import numpy as np

from . import schema as S
from .writer import ML_DOMAIN, model, node, tensor, tree_attrs, value_info

MODES = ["BRANCH_LEQ", "BRANCH_LT", "BRANCH_GTE", "BRANCH_GT"]


def random_complete_tree(rng: np.random.Generator, depth: int, n_features: int, k: int,
                         leaf_scale: float = 0.1, mixed_modes: bool = False,
                         feature_lo: int = 0) -> Dict[str, np.ndarray]:
    """Complete binary tree in BFS order: node i has children 2i+1 (true) / 2i+2 (false)."""
    n_int = (1 << depth) - 1
    n = (1 << (depth + 1)) - 1
    feature = np.full(n, -1, np.int64)
    feature[:n_int] = rng.integers(feature_lo, n_features, n_int)
    threshold = np.zeros(n, np.float32)
    threshold[:n_int] = rng.uniform(0.05, 0.95, n_int).astype(np.float32)
    left = np.zeros(n, np.int64)
    right = np.zeros(n, np.int64)
    left[:n_int] = 2 * np.arange(n_int) + 1
    right[:n_int] = 2 * np.arange(n_int) + 2
    if mixed_modes:
        mode = [MODES[i] for i in rng.integers(0, 4, n)]
    else:
        mode = ["BRANCH_LEQ"] * n
    missing = rng.integers(0, 2, n).astype(np.int64)
    leaf_values = np.zeros((n, k), np.float32)
    leaf_values[n_int:] = (rng.standard_normal((n - n_int, k)) * leaf_scale).astype(np.float32)
    return dict(feature=feature, threshold=threshold, left=left, right=right, mode=mode,
                missing_true=missing, leaf_values=leaf_values)


def logistic(n_features: int = 32, seed: int = 1):
    rng = np.random.default_rng(seed)
    w = (rng.standard_normal((n_features, 1)) * 0.5).astype(np.float32)
    b = np.array([-1.0], np.float32)
    nodes = [node("Gemm", ["input", "W", "B"], ["logit"]), node("Sigmoid", ["logit"], ["output"])]
    return model(nodes, [value_info("input", S.FLOAT, ["N", n_features])],
                 [value_info("output", S.FLOAT, ["N", 1])], [tensor("W", w), tensor("B", b)],
                 name="fraud_logistic", metadata={"family": "logistic", "features": str(n_features)})


def gbdt(n_trees: int = 100, depth: int = 7, n_features: int = 128, seed: int = 2,
         mixed_modes: bool = False):
    rng = np.random.default_rng(seed)
    trees = []
    for _ in range(n_trees):
        t = random_complete_tree(rng, depth, n_features, 1, leaf_scale=0.15, mixed_modes=mixed_modes)
        t["class_offset"] = 1   # weights on class 1 only: ORT's binary case
        trees.append(t)
    a = tree_attrs(trees, "class")
    nodes = [node("TreeEnsembleClassifier", ["input"], ["label", "output"], domain=ML_DOMAIN,
                  post_transform="LOGISTIC", classlabels_int64s=np.array([0, 1], np.int64),
                  base_values=np.array([-0.5], np.float32), **a)]
    return model(nodes, [value_info("input", S.FLOAT, ["N", n_features])],
                 [value_info("label", S.INT64, ["N"]), value_info("output", S.FLOAT, ["N", 2])],
                 name="fraud_gbdt",
                 metadata={"family": "gbdt", "trees": str(n_trees), "depth": str(depth)})


def stacked(n_trees: int = 100, depth: int = 7, n_features: int = 128, k: int = 32,
            hidden: int = 256, seed: int = 3):
    rng = np.random.default_rng(seed)
    trees = [random_complete_tree(rng, depth, n_features, k, leaf_scale=0.1) for _ in range(n_trees)]
    a = tree_attrs(trees, "target")
    w1 = (rng.standard_normal((k, hidden)) * np.sqrt(2.0 / k)).astype(np.float32)
    b1 = (rng.standard_normal(hidden) * 0.01).astype(np.float32)
    w2 = (rng.standard_normal((hidden, 1)) * np.sqrt(1.0 / hidden)).astype(np.float32)
    b2 = np.array([-0.25], np.float32)
    nodes = [
        node("TreeEnsembleRegressor", ["input"], ["emb"], domain=ML_DOMAIN, n_targets=k,
             aggregate_function="SUM", post_transform="NONE",
             base_values=np.zeros(k, np.float32), **a),
        node("Gemm", ["emb", "W1", "B1"], ["h1"]),
        node("Relu", ["h1"], ["a1"]),
        node("Gemm", ["a1", "W2", "B2"], ["logit"]),
        node("Sigmoid", ["logit"], ["output"]),
    ]
    return model(nodes, [value_info("input", S.FLOAT, ["N", n_features])],
                 [value_info("output", S.FLOAT, ["N", 1])],
                 [tensor("W1", w1), tensor("B1", b1), tensor("W2", w2), tensor("B2", b2)],
                 name="fraud_stacked",
                 metadata={"family": "stacked", "trees": str(n_trees), "targets": str(k)})


def ltv_mlp(n_features: int = 256, width: int = 512, layers: int = 4, seed: int = 4):
    rng = np.random.default_rng(seed)
    nodes, inits = [], []
    prev, cur = n_features, "input"
    for i in range(layers):
        w = (rng.standard_normal((prev, width)) * np.sqrt(2.0 / prev)).astype(np.float32)
        b = (rng.standard_normal(width) * 0.01).astype(np.float32)
        inits += [tensor(f"W{i}", w), tensor(f"B{i}", b)]
        nodes += [node("Gemm", [cur, f"W{i}", f"B{i}"], [f"h{i}"]), node("Relu", [f"h{i}"], [f"a{i}"])]
        prev, cur = width, f"a{i}"
    w = (rng.standard_normal((prev, 1)) * np.sqrt(1.0 / prev)).astype(np.float32)
    inits += [tensor("Wout", w), tensor("Bout", np.array([50.0], np.float32))]
    nodes.append(node("Gemm", [cur, "Wout", "Bout"], ["output"]))
    return model(nodes, [value_info("input", S.FLOAT, ["N", n_features])],
                 [value_info("output", S.FLOAT, ["N", 1])], inits, name="ltv_mlp",
                 metadata={"family": "mlp", "layers": str(layers), "width": str(width)})


def _gru_weights(rng, in_dim: int, hidden: int):
    s = 1.0 / np.sqrt(hidden)
    w = rng.uniform(-s, s, (1, 3 * hidden, in_dim)).astype(np.float32)
    r = rng.uniform(-s, s, (1, 3 * hidden, hidden)).astype(np.float32)
    b = rng.uniform(-s, s, (1, 6 * hidden)).astype(np.float32)
    return w, r, b


def gru(seq: int = 100, in_dim: int = 16, hidden: int = 256, seed: int = 5, layers: int = 2,
        linear_before_reset: int = 1, head: bool = True, direction: str = "forward", layout: int = 0):
    """GRU sequence classifier. ``direction`` forward / reverse / bidirectional (one layer),
    ``layout`` 0 ([seq, N, in]) or 1 (batch-major [N, seq, in])."""
    rng = np.random.default_rng(seed)
    D = 2 if direction == "bidirectional" else 1
    if D == 2 and layers != 1:
        raise ValueError("bidirectional: one layer")

    def weights(i):
        ws = [_gru_weights(rng, i, hidden) for _ in range(D)]
        return tuple(np.concatenate([w[k] for w in ws], 0) for k in range(3))
    w1, r1, b1 = weights(in_dim)
    wh = (rng.standard_normal((D * hidden, 1)) * np.sqrt(1.0 / (D * hidden))).astype(np.float32)
    bh = np.array([0.0], np.float32)
    lbr = int(linear_before_reset)
    attrs = dict(hidden_size=hidden, linear_before_reset=lbr)
    if direction != "forward":
        attrs["direction"] = direction
    if layout:
        attrs["layout"] = int(layout)
    nodes = [node("GRU", ["input", "W1", "R1", "B1"], ["Y1", "Yh1"], **attrs)]
    # Y: layout 0 [seq, D, N, H] -> squeeze axis 1; layout 1 [N, seq, D, H] -> squeeze axis 2
    inits = [tensor("W1", w1), tensor("R1", r1), tensor("B1", b1),
             tensor("ax1", np.array([2 if layout else 1], np.int64)),
             tensor("shp", np.array([-1, D * hidden], np.int64))]
    last_h = "Yh1"
    if layers == 2:
        w2, r2, b2 = weights(hidden)
        nodes += [node("Squeeze", ["Y1", "ax1"], ["X2"]),
                  node("GRU", ["X2", "W2", "R2", "B2"], ["Y2", "Yh2"], **attrs)]
        inits += [tensor("W2", w2), tensor("R2", r2), tensor("B2", b2)]
        last_h = "Yh2"
    if D == 2 and not layout:  # Y_h [2, N, H] -> [N, 2, H] -> [N, 2H]
        nodes.append(node("Transpose", [last_h], ["hT"], perm=[1, 0, 2]))
        last_h = "hT"
    if head:
        nodes += [node("Reshape", [last_h, "shp"], ["h"]), node("Gemm", ["h", "Wh", "Bh"], ["logit"]),
                  node("Sigmoid", ["logit"], ["output"])]
        inits += [tensor("Wh", wh), tensor("Bh", bh)]
        out_vi = value_info("output", S.FLOAT, ["N", 1])
    else:
        nodes.append(node("Reshape", [last_h, "shp"], ["output"]))
        out_vi = value_info("output", S.FLOAT, ["N", D * hidden])
    x_dims = ["N", seq, in_dim] if layout else [seq, "N", in_dim]
    return model(nodes, [value_info("input", S.FLOAT, x_dims)], [out_vi], inits, name="abuse_gru",
                 metadata={"family": "gru", "layers": str(layers), "hidden": str(hidden), "seq": str(seq),
                           "direction": direction, "layout": str(layout)})


def _scaler(rng, n_features: int):
    """sklearn StandardScaler as ai.onnx.ml Scaler: (x - mean) * (1 / std)."""
    mean = rng.uniform(-0.5, 0.5, n_features).astype(np.float32)
    scale = rng.uniform(0.5, 2.0, n_features).astype(np.float32)
    return node("Scaler", ["input"], ["scaled"], domain=ML_DOMAIN, offset=mean, scale=scale)


def sklearn_linear(n_features: int = 32, classes: int = 2, post: str = "LOGISTIC", seed: int = 6,
                   scaler: bool = True, zipmap: bool = True, string_labels: bool = False):
    """sklearn-onnx style linear pipeline: [Scaler] -> LinearClassifier -> [ZipMap].
    ``classes`` 2 writes one coefficient row (sklearn's binary LogisticRegression); more write
    one row per class."""
    rng = np.random.default_rng(seed)
    E = 1 if classes == 2 else classes
    coef = (rng.standard_normal((E, n_features)) * 0.3).astype(np.float32)
    icpt = (rng.standard_normal(E) * 0.1).astype(np.float32)
    labels = (dict(classlabels_strings=[f"c{i}" for i in range(classes)]) if string_labels
              else dict(classlabels_ints=np.arange(classes, dtype=np.int64)))
    nodes = [_scaler(rng, n_features)] if scaler else []
    x = "scaled" if scaler else "input"
    probs = "probabilities" if zipmap else "output"
    nodes.append(node("LinearClassifier", [x], ["label", probs], domain=ML_DOMAIN, coefficients=coef.ravel(),
                      intercepts=icpt, post_transform=post, multi_class=0, **labels))
    if zipmap:
        zl = (dict(classlabels_strings=labels["classlabels_strings"]) if string_labels
              else dict(classlabels_int64s=np.arange(classes, dtype=np.int64)))
        nodes.append(node("ZipMap", [probs], ["output"], domain=ML_DOMAIN, **zl))
    return model(nodes, [value_info("input", S.FLOAT, ["N", n_features])],
                 [value_info("label", S.INT64, ["N"]), value_info("output", S.FLOAT, ["N", classes])],
                 name="sklearn_linear", metadata={"family": "linear", "classes": str(classes)})


def linear_regressor(n_features: int = 32, targets: int = 1, post: str = "NONE", seed: int = 7):
    rng = np.random.default_rng(seed)
    coef = (rng.standard_normal((targets, n_features)) * 0.3).astype(np.float32)
    icpt = (rng.standard_normal(targets) * 0.1).astype(np.float32)
    nodes = [_scaler(rng, n_features),
             node("LinearRegressor", ["scaled"], ["output"], domain=ML_DOMAIN, coefficients=coef.ravel(),
                  intercepts=icpt, targets=targets, post_transform=post)]
    return model(nodes, [value_info("input", S.FLOAT, ["N", n_features])],
                 [value_info("output", S.FLOAT, ["N", targets])], name="linear_regressor",
                 metadata={"family": "linear"})


def mlp_classifier(n_features: int = 32, hidden: int = 64, seed: int = 8):
    """sklearn MLPClassifier-style pipeline: Scaler -> Gemm -> Relu -> LinearClassifier (binary,
    LOGISTIC) -> ZipMap. On the device: the Scaler folds into the first layer's weights and the
    two layers run as one fused head."""
    rng = np.random.default_rng(seed)
    w = (rng.standard_normal((n_features, hidden)) * np.sqrt(2.0 / n_features)).astype(np.float32)
    b = (rng.standard_normal(hidden) * 0.01).astype(np.float32)
    coef = (rng.standard_normal(hidden) * np.sqrt(1.0 / hidden)).astype(np.float32)
    nodes = [_scaler(rng, n_features), node("Gemm", ["scaled", "W", "B"], ["h"]), node("Relu", ["h"], ["a"]),
             node("LinearClassifier", ["a"], ["label", "probabilities"], domain=ML_DOMAIN, coefficients=coef,
                  intercepts=np.array([-0.1], np.float32), post_transform="LOGISTIC",
                  classlabels_ints=np.array([0, 1], np.int64)),
             node("ZipMap", ["probabilities"], ["output"], domain=ML_DOMAIN,
                  classlabels_int64s=np.array([0, 1], np.int64))]
    return model(nodes, [value_info("input", S.FLOAT, ["N", n_features])],
                 [value_info("label", S.INT64, ["N"]), value_info("output", S.FLOAT, ["N", 2])],
                 [tensor("W", w), tensor("B", b)], name="mlp_classifier", metadata={"family": "mlp"})


def wide_deep(n_features: int = 32, hidden: int = 128, deep_out: int = 64, wide: int = 16, seed: int = 9):
    """DAG: a deep tower (Gemm -> Relu -> Gemm -> Relu) and a wide linear branch read the same
    input; Concat -> Gemm -> Sigmoid."""
    rng = np.random.default_rng(seed)

    def lin(k, n, name):
        return [tensor(f"W{name}", (rng.standard_normal((k, n)) * np.sqrt(2.0 / k)).astype(np.float32)),
                tensor(f"B{name}", (rng.standard_normal(n) * 0.01).astype(np.float32))]
    inits = lin(n_features, hidden, "d1") + lin(hidden, deep_out, "d2") + lin(n_features, wide, "w") + \
        lin(deep_out + wide, 1, "o")
    nodes = [node("Gemm", ["input", "Wd1", "Bd1"], ["d1"]), node("Relu", ["d1"], ["a1"]),
             node("Gemm", ["a1", "Wd2", "Bd2"], ["d2"]), node("Relu", ["d2"], ["a2"]),
             node("Gemm", ["input", "Ww", "Bw"], ["wide"]),
             node("Concat", ["a2", "wide"], ["cat"], axis=1),
             node("Gemm", ["cat", "Wo", "Bo"], ["logit"]), node("Sigmoid", ["logit"], ["output"])]
    return model(nodes, [value_info("input", S.FLOAT, ["N", n_features])],
                 [value_info("output", S.FLOAT, ["N", 1])], inits, name="wide_deep", metadata={"family": "mlp"})


def residual_mlp(n_features: int = 32, width: int = 128, blocks: int = 2, seed: int = 10):
    """DAG: h = Relu(x W0 + b0); per block h = h + Relu(Relu(h W1 + b1) W2 + b2) (MatMul + Add
    pairs); head Gemm -> Sigmoid."""
    rng = np.random.default_rng(seed)
    inits = [tensor("W0", (rng.standard_normal((n_features, width)) * np.sqrt(2.0 / n_features)).astype(np.float32)),
             tensor("B0", np.zeros(width, np.float32))]
    nodes = [node("Gemm", ["input", "W0", "B0"], ["z0"]), node("Relu", ["z0"], ["h0"])]
    h = "h0"
    for i in range(blocks):
        for j in (1, 2):
            inits += [tensor(f"W{i}_{j}", (rng.standard_normal((width, width)) * np.sqrt(1.0 / width)).astype(np.float32)),
                      tensor(f"B{i}_{j}", (rng.standard_normal(width) * 0.01).astype(np.float32))]
        nodes += [node("MatMul", [h, f"W{i}_1"], [f"m{i}_1"]), node("Add", [f"m{i}_1", f"B{i}_1"], [f"z{i}_1"]),
                  node("Relu", [f"z{i}_1"], [f"a{i}_1"]),
                  node("MatMul", [f"a{i}_1", f"W{i}_2"], [f"m{i}_2"]), node("Add", [f"m{i}_2", f"B{i}_2"], [f"z{i}_2"]),
                  node("Relu", [f"z{i}_2"], [f"a{i}_2"]),
                  node("Add", [h, f"a{i}_2"], [f"h{i + 1}"])]
        h = f"h{i + 1}"
    inits += [tensor("Wh", (rng.standard_normal((width, 1)) * np.sqrt(1.0 / width)).astype(np.float32)),
              tensor("Bh", np.array([-0.2], np.float32))]
    nodes += [node("Gemm", [h, "Wh", "Bh"], ["logit"]), node("Sigmoid", ["logit"], ["output"])]
    return model(nodes, [value_info("input", S.FLOAT, ["N", n_features])],
                 [value_info("output", S.FLOAT, ["N", 1])], inits, name="residual_mlp", metadata={"family": "mlp"})


BUILDERS = {"logistic": logistic, "gbdt": gbdt, "stacked": stacked, "ltv_mlp": ltv_mlp, "gru": gru,
            "sklearn_linear": sklearn_linear, "linear_regressor": linear_regressor,
            "mlp_classifier": mlp_classifier, "wide_deep": wide_deep, "residual_mlp": residual_mlp}


def build(kind: str, **kw):
    return BUILDERS[kind](**kw)
