"""Minimal ONNX model construction helpers (no ``onnx`` package in the image)."""
from __future__ import annotations

from typing import Dict, Iterable, List, Optional, Sequence

import numpy as np

from . import schema as S

_NP2ONNX = {np.dtype(np.float32): S.FLOAT, np.dtype(np.int64): S.INT64,
            np.dtype(np.int32): S.INT32, np.dtype(np.float64): S.DOUBLE,
            np.dtype(np.uint8): S.UINT8, np.dtype(np.int8): S.INT8, np.dtype(np.bool_): S.BOOL}
ML_DOMAIN = "ai.onnx.ml"


def tensor(name: str, arr: np.ndarray, raw: bool = True):
    arr = np.ascontiguousarray(arr)
    t = S.TensorProto(name=name, data_type=_NP2ONNX[arr.dtype])
    t.dims.extend(int(d) for d in arr.shape)
    if raw:
        t.raw_data = arr.tobytes()
    elif arr.dtype == np.float32:
        t.float_data.extend(arr.ravel().tolist())
    elif arr.dtype == np.int64:
        t.int64_data.extend(arr.ravel().tolist())
    else:
        t.raw_data = arr.tobytes()
    return t


def attr(name: str, value):
    a = S.AttributeProto(name=name)
    if isinstance(value, float):
        a.type, a.f = S.A_FLOAT, value
    elif isinstance(value, (bool, int, np.integer)):
        a.type, a.i = S.A_INT, int(value)
    elif isinstance(value, (str, bytes)):
        a.type, a.s = S.A_STRING, value.encode() if isinstance(value, str) else value
    elif isinstance(value, np.ndarray) and value.dtype.kind == "f":
        a.type = S.A_FLOATS
        a.floats.extend(value.astype(np.float32).ravel().tolist())
    elif isinstance(value, np.ndarray) and value.dtype.kind in "iu":
        a.type = S.A_INTS
        a.ints.extend(int(v) for v in value.ravel())
    elif isinstance(value, (list, tuple)) and value and isinstance(value[0], (str, bytes)):
        a.type = S.A_STRINGS
        a.strings.extend(v.encode() if isinstance(v, str) else v for v in value)
    elif isinstance(value, (list, tuple)) and value and isinstance(value[0], float):
        a.type = S.A_FLOATS
        a.floats.extend(value)
    elif isinstance(value, (list, tuple)):
        a.type = S.A_INTS
        a.ints.extend(int(v) for v in value)
    else:
        raise TypeError(f"attribute {name}: unsupported value {type(value)}")
    return a


def node(op: str, inputs: Sequence[str], outputs: Sequence[str], name: str = "",
         domain: str = "", **attrs):
    n = S.NodeProto(op_type=op, name=name or f"{op}_{outputs[0]}", domain=domain)
    n.input.extend(inputs)
    n.output.extend(outputs)
    for k, v in attrs.items():
        n.attribute.append(attr(k, v))
    return n


def value_info(name: str, elem_type: int, shape: Sequence):
    v = S.ValueInfoProto(name=name)
    tt = v.type.tensor_type
    tt.elem_type = elem_type
    for d in shape:
        dim = tt.shape.dim.add()
        if isinstance(d, str):
            dim.dim_param = d
        else:
            dim.dim_value = int(d)
    return v


def model(nodes, inputs, outputs, initializers: Iterable = (), name: str = "graph",
          opset: int = 17, ml_opset: int = 3, metadata: Optional[Dict[str, str]] = None):
    g = S.GraphProto(name=name)
    g.node.extend(nodes)
    g.input.extend(inputs)
    g.output.extend(outputs)
    g.initializer.extend(initializers)
    m = S.ModelProto(ir_version=8, producer_name="igaming_platform_amd", producer_version="0.1",
                     graph=g)
    m.opset_import.add(domain="", version=opset)
    if any(n.domain == ML_DOMAIN for n in nodes):
        m.opset_import.add(domain=ML_DOMAIN, version=ml_opset)
    for k, v in (metadata or {}).items():
        m.metadata_props.add(key=k, value=v)
    return m


def save(m, path: str) -> None:
    with open(path, "wb") as f:
        f.write(m.SerializeToString())


def load(path: str):
    with open(path, "rb") as f:
        return S.ModelProto.FromString(f.read())


def tree_attrs(trees: List[Dict[str, np.ndarray]], prefix: str) -> Dict[str, object]:
    """Flatten per-tree arrays into TreeEnsemble attributes.

    Each tree dict: ``feature`` (int, -1 for leaf), ``threshold`` (f32), ``left``/``right``
    (child node ids; true branch = left), ``mode`` (str per node), ``missing_true`` (0/1),
    ``leaf_values`` ([n_nodes, K] for leaves; rows of internal nodes ignored).
    ``prefix`` is ``target`` (regressor) or ``class`` (classifier).
    """
    tids, nids, fids, vals, modes, tn, fn, miss = [], [], [], [], [], [], [], []
    lt, ln, lid, lw = [], [], [], []
    for t, tr in enumerate(trees):
        n = len(tr["feature"])
        for i in range(n):
            leaf = tr["feature"][i] < 0
            tids.append(t)
            nids.append(i)
            fids.append(0 if leaf else int(tr["feature"][i]))
            vals.append(0.0 if leaf else float(tr["threshold"][i]))
            modes.append("LEAF" if leaf else tr["mode"][i])
            tn.append(0 if leaf else int(tr["left"][i]))
            fn.append(0 if leaf else int(tr["right"][i]))
            miss.append(0 if leaf else int(tr["missing_true"][i]))
            if leaf:
                off = int(tr.get("class_offset", 0))
                for k, w in enumerate(np.atleast_1d(tr["leaf_values"][i])):
                    lt.append(t)
                    ln.append(i)
                    lid.append(k + off)
                    lw.append(float(w))
    return {
        "nodes_treeids": np.array(tids, np.int64), "nodes_nodeids": np.array(nids, np.int64),
        "nodes_featureids": np.array(fids, np.int64), "nodes_values": np.array(vals, np.float32),
        "nodes_modes": modes, "nodes_truenodeids": np.array(tn, np.int64),
        "nodes_falsenodeids": np.array(fn, np.int64),
        "nodes_missing_value_tracks_true": np.array(miss, np.int64),
        f"{prefix}_treeids": np.array(lt, np.int64), f"{prefix}_nodeids": np.array(ln, np.int64),
        f"{prefix}_ids": np.array(lid, np.int64), f"{prefix}_weights": np.array(lw, np.float32),
    }
