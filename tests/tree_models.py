"""TreeEnsemble models for the general-tree tests (CPU layout twin + GPU parity): sklearn
fits exported by onnx/convert.py (deep GradientBoosting, fully grown unbalanced RandomForest,
MIN / MAX aggregates, PROBIT) and synthetic classifiers for the post transforms the complete
kernel now runs (SOFTMAX, SOFTMAX_ZERO, binary SOFTMAX, PROBIT)."""
import numpy as np

N_FEAT = 16


def data(n=3000, seed=0, nan_frac=0.002):
    rng = np.random.default_rng(seed)
    X = rng.standard_normal((n, N_FEAT)).astype(np.float32)
    y = X[:, 0] * 2 - X[:, 3] ** 2 + np.sin(3 * X[:, 5]) + rng.standard_normal(n) * 0.3
    Xq = X.copy()
    Xq[rng.uniform(0, 1, Xq.shape) < nan_frac] = np.nan  # missing values follow the false branch
    return X, y, Xq


def _synthetic(kind, seed=7):
    from igaming_platform_amd.onnx import schema as S
    from igaming_platform_amd.onnx.builders import random_complete_tree
    from igaming_platform_amd.onnx.writer import ML_DOMAIN, model, node, tree_attrs, value_info
    rng = np.random.default_rng(seed)
    if kind in ("softmax_zero4", "softmax3", "probit_reg4"):
        k = {"softmax_zero4": 4, "softmax3": 3, "probit_reg4": 4}[kind]
        trees = []
        for _ in range(30):
            t = random_complete_tree(rng, 6, N_FEAT, k, leaf_scale=0.4, mixed_modes=True)
            t["threshold"] = (t["threshold"] * 2 - 1).astype(np.float32)
            if kind == "softmax_zero4":  # some leaves leave a class at exactly 0
                t["leaf_values"][rng.uniform(0, 1, t["leaf_values"].shape) < 0.3] = 0.0
            if kind == "probit_reg4":
                t["leaf_values"] = (np.abs(t["leaf_values"]) * 0.02).astype(np.float32)
            trees.append(t)
        if kind == "probit_reg4":
            a = tree_attrs(trees, "target")
            nd = node("TreeEnsembleRegressor", ["input"], ["output"], domain=ML_DOMAIN, n_targets=k,
                      aggregate_function="SUM", post_transform="PROBIT", base_values=np.full(k, 0.1, np.float32), **a)
            outs = [value_info("output", S.FLOAT, ["N", k])]
        else:
            a = tree_attrs(trees, "class")
            post = "SOFTMAX_ZERO" if kind == "softmax_zero4" else "SOFTMAX"
            nd = node("TreeEnsembleClassifier", ["input"], ["label", "output"], domain=ML_DOMAIN,
                      post_transform=post, classlabels_int64s=np.arange(k, dtype=np.int64), **a)
            outs = [value_info("label", S.INT64, ["N"]), value_info("output", S.FLOAT, ["N", k])]
        return model([nd], [value_info("input", S.FLOAT, ["N", N_FEAT])], outs, name=kind)
    if kind in ("binary_softmax", "binary_probit"):
        trees = []
        for _ in range(25):
            t = random_complete_tree(rng, 5, N_FEAT, 1, leaf_scale=0.02, mixed_modes=True)
            t["threshold"] = (t["threshold"] * 2 - 1).astype(np.float32)
            t["leaf_values"] = np.abs(t["leaf_values"]).astype(np.float32)
            t["class_offset"] = 1
            trees.append(t)
        a = tree_attrs(trees, "class")
        post = "SOFTMAX" if kind == "binary_softmax" else "PROBIT"
        nd = node("TreeEnsembleClassifier", ["input"], ["label", "output"], domain=ML_DOMAIN, post_transform=post,
                  classlabels_int64s=np.array([0, 1], np.int64), base_values=np.array([0.05], np.float32), **a)
        return model([nd], [value_info("input", S.FLOAT, ["N", N_FEAT])],
                     [value_info("label", S.INT64, ["N"]), value_info("output", S.FLOAT, ["N", 2])], name=kind)
    raise ValueError(kind)


def build(kind):
    """-> (ONNX ModelProto, X to score)."""
    from igaming_platform_amd.onnx import convert
    X, y, Xq = data()
    if kind == "gb_d16":
        from sklearn.ensemble import GradientBoostingClassifier
        est = GradientBoostingClassifier(n_estimators=25, max_depth=16, learning_rate=0.2, random_state=0)
        est.fit(X, y > 0)
        return convert.gradient_boosting(est, N_FEAT), Xq
    if kind.startswith("rf_"):
        from sklearn.ensemble import RandomForestRegressor
        yy = 1 / (1 + np.exp(-y)) if kind == "rf_probit" else y
        est = RandomForestRegressor(n_estimators=30, max_depth=None, max_features=0.5, random_state=0).fit(X, yy)
        agg, post = {"rf_unbalanced": ("AVERAGE", "NONE"), "rf_min": ("MIN", "NONE"), "rf_max": ("MAX", "NONE"),
                     "rf_probit": ("AVERAGE", "PROBIT")}[kind]
        return convert.random_forest(est, N_FEAT, aggregate=agg, post_transform=post), Xq
    return _synthetic(kind), Xq


SKLEARN = ["gb_d16", "rf_unbalanced", "rf_min", "rf_max", "rf_probit"]
SYNTHETIC = ["softmax_zero4", "softmax3", "probit_reg4", "binary_softmax", "binary_probit"]


def executor_output(m, X):
    from igaming_platform_amd.native import native
    N = native()
    om = N.OnnxModel.from_bytes(m.SerializeToString())
    return np.asarray(N.Executor(om).run({"input": X})["output"], np.float32), om


def sparse_eval(step, X):
    """Host twin of the K2b kernel on the pointer layout (the CPU test of the layout builder)."""
    nodes = step.nodes_np.reshape(-1, 4)
    meta = nodes[:, 0].view(np.uint32)
    thr = nodes[:, 1].view(np.float32)
    mode, feat, miss = (meta >> 16) & 7, meta & 0xFFFF, (meta >> 19) & 1
    n, K, agg = X.shape[0], step.k, step.aggregate
    acc = np.full((n, K), np.inf if agg == 2 else -np.inf if agg == 3 else 0.0, np.float32)
    for t in range(step.n_trees):
        cur = np.full(n, step.roots_np[t], np.int64)
        for _ in range(step.depth + 1):
            idx = np.nonzero(mode[cur] != 7)[0]
            if idx.size == 0:
                break
            c = cur[idx]
            x, th, mm = X[idx, feat[c]], thr[c], mode[c]
            with np.errstate(invalid="ignore"):
                cond = np.select([mm == 0, mm == 1, mm == 2, mm == 3, mm == 4],
                                 [x <= th, x < th, x >= th, x > th, x == th], x != th)
            cond |= (miss[c] == 1) & np.isnan(x)
            cur[idx] = np.where(cond, nodes[c, 2], nodes[c, 3])
        leaf = nodes[cur, 2]
        w, h = step.leaf_w_np[leaf], step.leaf_has_np[leaf].astype(bool)
        if agg < 2:
            acc += w
        elif agg == 2:
            acc = np.where(h, np.minimum(acc, w), acc)
        else:
            acc = np.where(h, np.maximum(acc, w), acc)
    if agg >= 2:
        acc[np.isinf(acc)] = 0
    if agg == 1:
        acc /= step.n_trees
    if step.base_np is not None:
        acc += step.base_np[: acc.shape[1]]
    return post(step, acc)


def _erfinv(x):
    from scipy.special import erfinv
    return erfinv(x).astype(np.float32)


def post(step, s):
    p = step.post
    if step.binary_class >= 0:
        v, c = s[:, 0], step.binary_class
        z = np.zeros((len(v), 2), np.float32)
        if p == 1:
            z[:, c], z[:, 1 - c] = 1 / (1 + np.exp(-v)), 1 / (1 + np.exp(v))
            return z
        z[:, c] = v
        z[:, 1 - c] = 1 - v if step.all_positive else -v
        if p == 4:
            z = np.sqrt(2) * _erfinv(2 * z - 1)
        elif p in (2, 3):
            e = np.exp(z - z.max(1, keepdims=True))
            z = e / e.sum(1, keepdims=True)
        return z.astype(np.float32)
    z = s.astype(np.float32).copy()
    if p == 1:
        return 1 / (1 + np.exp(-z))
    if p in (2, 3):
        mask = (z != 0) if p == 3 else np.ones_like(z, bool)
        m = np.where(mask, z, -np.inf).max(1, keepdims=True)
        e = np.where(mask, np.exp(z - m), 0)
        sm = e.sum(1, keepdims=True)
        return np.where(sm > 0, e / np.where(sm > 0, sm, 1), 0).astype(np.float32)
    if p == 4:
        return (np.sqrt(2) * _erfinv(2 * z - 1)).astype(np.float32)
    return z
