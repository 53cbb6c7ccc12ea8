"""scikit-learn tree ensembles -> ONNX ``ai.onnx.ml`` TreeEnsemble models.

Stands in for the reference's missing model export scripts (Makefile:215-225
``model-train``/``model-export``; the scripts are not in the repository) and is the
independent oracle for the tree kernels: a model fitted by sklearn,
exported here, must score identically in the C++ executor and on the GPU.
"""
from __future__ import annotations

from typing import List

import numpy as np

from . import schema as S
from .writer import model, node, tree_attrs, value_info


def _tree_dict(tree, scale: float, k_index: int = 0, n_targets: int = 1):
    t = tree.tree_
    n = t.node_count
    feat = np.where(t.children_left < 0, -1, t.feature).astype(np.int64)
    vals = np.zeros((n, n_targets), np.float32)
    vals[:, k_index] = t.value[:, 0, 0] * scale if t.value.ndim == 3 else t.value[:, 0] * scale
    return dict(feature=feat, threshold=t.threshold.astype(np.float32), left=t.children_left, right=t.children_right,
                mode=["BRANCH_LEQ"] * n, missing_true=np.zeros(n, np.int64), leaf_values=vals)


def gradient_boosting(est, n_features: int, input_name: str = "input", output_name: str = "output"):
    """GradientBoostingRegressor / binary GradientBoostingClassifier -> ONNX.

    Regressor: TreeEnsembleRegressor (n_targets=1, base = init prediction).
    Binary classifier: TreeEnsembleRegressor on the log-odds + Sigmoid -> P(class 1) [N, 1].
    sklearn sends ``x <= threshold`` left, which is ONNX BRANCH_LEQ with the true branch left.
    """
    lr = float(est.learning_rate)
    trees: List[dict] = [_tree_dict(t[0], lr) for t in est.estimators_]
    X0 = np.zeros((1, n_features), np.float32)
    base = float(np.asarray(est._raw_predict_init(X0)).ravel()[0])
    a = tree_attrs(trees, "target")
    a.update(n_targets=1, aggregate_function="SUM", post_transform="NONE", base_values=np.array([base], np.float32))
    is_clf = hasattr(est, "classes_")
    if is_clf and len(est.classes_) != 2:
        raise ValueError("only binary classifiers are converted")
    nodes = [node("TreeEnsembleRegressor", [input_name], ["raw" if is_clf else output_name], domain="ai.onnx.ml", **a)]
    if is_clf:
        nodes.append(node("Sigmoid", ["raw"], [output_name]))
    return model(nodes, [value_info(input_name, S.FLOAT, ["N", n_features])],
                 [value_info(output_name, S.FLOAT, ["N", 1])], name="sklearn_gbdt",
                 metadata={"family": "gbdt", "source": "sklearn"})


def random_forest(est, n_features: int, input_name: str = "input", output_name: str = "output",
                  aggregate: str = "AVERAGE", post_transform: str = "NONE"):
    """RandomForestRegressor -> TreeEnsembleRegressor with AVERAGE aggregation (``aggregate``
    MIN / MAX / SUM and a ``post_transform`` give the other TreeEnsemble variants over the same
    fitted trees: the device parity tests use them)."""
    trees = [_tree_dict(t, 1.0) for t in est.estimators_]
    a = tree_attrs(trees, "target")
    a.update(n_targets=1, aggregate_function=aggregate, post_transform=post_transform)
    return model([node("TreeEnsembleRegressor", [input_name], [output_name], domain="ai.onnx.ml", **a)],
                 [value_info(input_name, S.FLOAT, ["N", n_features])],
                 [value_info(output_name, S.FLOAT, ["N", 1])], name="sklearn_rf", metadata={"family": "gbdt"})
