"""ONNX graph -> device execution plan.

The C++ reader parses the file; this module walks the (single-input) chain from the model
input to the primary output and lowers it to fused device steps:

* ``TreeStep``   TreeEnsemble{Classifier,Regressor} (+ a following Sigmoid folded into the
                 post transform) -> K2 ``tree_ensemble`` on the complete-tree layout, or K2b
                 ``tree_sparse`` on the pointer layout for deep (> 12) or very unbalanced trees,
                 MIN / MAX aggregates and target counts the complete kernel is not built for.
                 Every post transform (NONE, LOGISTIC, SOFTMAX, SOFTMAX_ZERO, PROBIT) runs on
                 the device.
* ``DenseStep``  Gemm / MatMul(+Add) with a following Relu/Sigmoid/Tanh fused into the
                 epilogue -> K3 ``gemm`` (MFMA) or ``gemv`` (N == 1).
* ``GRUStep``    ONNX GRU (forward, layout 0) -> K4 (cfg 5).
* Identity / Flatten / Squeeze / Reshape to 2-D are folded away.

Anything else raises :class:`PlanError`; the engine then runs that model through the C++
CPU executor (explicitly, with a warning) rather than silently substituting torch ops.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional

import numpy as np

from ..native import native

ML_DOMAIN = "ai.onnx.ml"
POST = {0: "NONE", 1: "LOGISTIC", 2: "SOFTMAX", 3: "SOFTMAX_ZERO", 4: "PROBIT"}


class PlanError(RuntimeError):
    pass


@dataclass
class TreeStep:
    n_trees: int
    depth: int
    k: int
    n_out: int
    post: int            # kernel post code (POST): 0 none, 1 logistic, 2 softmax, 3 softmax_zero, 4 probit
    average: int
    binary_class: int    # -1 unless the classifier binary case
    all_positive: int
    max_feature: int
    nodes_np: np.ndarray  # complete: [T][2^D-1][2] f32; sparse: [N][4] int32
    leaves_np: Optional[np.ndarray]  # complete: [T][2^D][K]; sparse: None
    base_np: Optional[np.ndarray]
    classifier: bool = False
    layout: str = "complete"   # complete (K2) | sparse (K2b pointer layout)
    aggregate: int = 0         # 0 sum, 1 average, 2 min, 3 max
    roots_np: Optional[np.ndarray] = None     # sparse: [T] root node index
    leaf_w_np: Optional[np.ndarray] = None    # sparse: [L][K]
    leaf_has_np: Optional[np.ndarray] = None  # sparse: [L][K] uint8
    nodes: Any = None
    leaves: Any = None
    base: Any = None
    roots: Any = None
    leaf_w: Any = None
    leaf_has: Any = None
    kind: str = "tree"

    @property
    def out_width(self) -> int:
        return self.n_out

    @property
    def all_leq(self) -> bool:
        """Every node is BRANCH_LEQ (sklearn-style ensembles; missing-value tracks allowed): the
        kernel then skips decoding the comparison mode per node."""
        if self.layout != "complete":
            return False
        meta = self.nodes_np.reshape(-1, 2)[:, 1].view(np.uint32)
        return bool(np.all(((meta >> 16) & 0x7) == 0))


COMPLETE_K = (1, 2, 4, 8, 16, 32, 64)   # target counts the complete-tree kernel is built for
SPARSE_MAX_K = 64


def choose_tree_layout(info: Dict[str, Any], depth_limit: int = 12) -> str:
    """complete (K2) when the ensemble fits it without much padding, else sparse (K2b).
    ``IGP_TREE_LAYOUT=complete|sparse`` forces one (the complete layout still needs SUM /
    AVERAGE, depth <= ``depth_limit`` and a supported K)."""
    import os
    D, T, N, K = int(info["depth"]), int(info["n_trees"]), int(info["n_nodes"]), int(info["k"])
    fits = int(info["aggregate"]) in (0, 1) and D <= depth_limit and K in COMPLETE_K
    forced = os.environ.get("IGP_TREE_LAYOUT", "auto")
    if forced == "sparse" or not fits:
        return "sparse"
    if forced == "complete":
        return "complete"
    # the complete layout stores 2^(D+1) - 1 slots per tree: keep it when that is within 8x
    # of the real node count (balanced GBDTs are ~1x; a few deep paths blow it up)
    return "complete" if T * ((1 << (D + 1)) - 1) <= 8 * max(N, 1) + 64 * T else "sparse"


@dataclass
class DenseStep:
    n: int
    k: int
    act: str
    w_np: np.ndarray     # [N, K] float32 (logical)
    b_np: Optional[np.ndarray]
    w: Any = None        # bf16 [N_pad, K_pad] device
    b: Any = None
    kind: str = "dense"

    @property
    def out_width(self) -> int:
        return self.n


@dataclass
class HeadStep:
    """dense(K -> N1, act1) + dense(N1 -> 1, act2) fused into one kernel (K3 mlp_head)."""
    n1: int
    k: int
    act1: str
    act2: str
    w1_np: np.ndarray    # [N1, K]
    b1_np: Optional[np.ndarray]
    w2_np: np.ndarray    # [N1]
    b2: float
    w1: Any = None
    b1: Any = None
    w2: Any = None
    kind: str = "head"

    @property
    def out_width(self) -> int:
        return 1


@dataclass
class GRUStep:
    hidden: int
    in_dim: int
    linear_before_reset: int
    w_np: np.ndarray     # [3H, I]
    r_np: np.ndarray     # [3H, H]
    b_np: np.ndarray     # [6H]
    seq: int = 0
    dev: Dict[str, Any] = field(default_factory=dict)
    kind: str = "gru"
    reverse: bool = False      # direction=reverse: the sequence is read last step first
    layout: int = 0            # ONNX layout attribute (1: batch-major X / Y / Y_h)
    bidirectional: bool = False
    w_rev_np: Optional[np.ndarray] = None  # bidirectional: the reverse direction's W / R / B
    r_rev_np: Optional[np.ndarray] = None
    b_rev_np: Optional[np.ndarray] = None

    @property
    def out_width(self) -> int:
        return self.hidden * (2 if self.bidirectional else 1)

    def direction(self, d: int) -> "GRUStep":
        """One direction of a bidirectional layer as a unidirectional step (d = 1: reverse)."""
        if d == 0:
            return GRUStep(self.hidden, self.in_dim, self.linear_before_reset, self.w_np, self.r_np, self.b_np,
                           seq=self.seq, layout=self.layout)
        return GRUStep(self.hidden, self.in_dim, self.linear_before_reset, self.w_rev_np, self.r_rev_np,
                       self.b_rev_np, seq=self.seq, reverse=True, layout=self.layout)


@dataclass
class Plan:
    family: str
    in_width: int
    steps: List[Any]
    out_width: int
    ml_col: int
    metadata: Dict[str, str]
    input_name: str
    output_name: str
    seq_input: bool = False
    precision: str = "fp32"   # dense / head weights on device: fp32 (reference, f32 MFMA) | bf16

    def describe(self) -> str:
        parts = []
        for s in self.steps:
            if s.kind == "tree":
                parts.append(f"tree(T={s.n_trees},D={s.depth},K={s.k},post={s.post},{s.layout})")
            elif s.kind == "dense":
                parts.append(f"dense({s.k}->{s.n},{s.act})")
            elif s.kind == "head":
                parts.append(f"head({s.k}->{s.n1},{s.act1}->1,{s.act2})")
            else:
                parts.append(f"gru(I={s.in_dim},H={s.hidden})")
        return " -> ".join(parts)


def _consumers(nodes, name):
    return [n for n in nodes if name in n["inputs"]]


def compile_onnx(model, input_name: str = "input", output_name: str = "output",
                 depth_limit: int = 12, fuse_heads: bool = True) -> Plan:
    """``model``: _native.OnnxModel. Returns a host-side Plan (upload with :func:`to_device`)."""
    N = native()
    ex = N.Executor(model)
    nodes = model.nodes()
    index = {id(n): i for i, n in enumerate(nodes)}
    inputs = {v[0]: v for v in model.inputs()}
    if input_name not in inputs:
        if len(inputs) == 1:
            input_name = next(iter(inputs))
        else:
            raise PlanError(f"model has no input named {input_name!r}")
    outs = [v[0] for v in model.outputs()]
    if output_name not in outs:
        output_name = outs[-1]
    in_vi = inputs[input_name]
    dims = in_vi[2]
    seq_input = len(dims) == 3
    in_width = int(dims[-1]) if dims and dims[-1] > 0 else -1
    inits = set(model.initializer_names())

    def const(name):
        return model.initializer(name)

    steps: List[Any] = []
    cur = input_name
    width = in_width
    ml_col = 0
    visited = set()
    bidir_pending = False  # a layout-0 bidirectional Y_h still in [D, N, H] order
    while cur != output_name:
        cons = [n for n in _consumers(nodes, cur) if id(n) not in visited]
        if len(cons) != 1:
            raise PlanError(f"value {cur!r} feeds {len(cons)} nodes; only chains are lowered")
        n = cons[0]
        visited.add(id(n))
        op, a = n["op_type"], n["attrs"]
        if op in ("TreeEnsembleClassifier", "TreeEnsembleRegressor"):
            info = ex.tree_info(index[id(n)])
            if int(info["k"]) > SPARSE_MAX_K:
                raise PlanError(f"TreeEnsemble with {info['k']} targets (> {SPARSE_MAX_K}) is CPU-only")
            layout = choose_tree_layout(info, depth_limit)
            c = (ex.tree_complete(index[id(n)], depth_limit) if layout == "complete"
                 else ex.tree_sparse(index[id(n)]))
            post = int(c["post"])
            binary = bool(c["binary_case"])
            k = int(c["k"])
            n_out = int(c["n_outputs"]) if c["classifier"] else k
            base = np.asarray(c["base_values"], np.float32)
            if binary:
                base = base[:1] if len(base) == 1 else (base[c["binary_class"]:c["binary_class"] + 1]
                                                        if len(base) == 2 else None)
            elif len(base):  # targets past the given base values get 0 (executor semantics)
                base = np.pad(base[:k], (0, max(0, k - len(base))))
            sparse = layout == "sparse"
            ts = TreeStep(n_trees=int(c["n_trees"]), depth=int(c["depth"]), k=k, n_out=n_out, post=post,
                          average=int(c["aggregate"] == 1), binary_class=int(c["binary_class"]) if binary else -1,
                          all_positive=int(bool(c["weights_all_positive"])), max_feature=int(c["max_feature"]),
                          nodes_np=np.ascontiguousarray(c["nodes"], np.int32 if sparse else np.float32),
                          leaves_np=None if sparse else np.ascontiguousarray(c["leaves"], np.float32),
                          base_np=None if base is None or len(base) == 0 else np.asarray(base, np.float32),
                          classifier=bool(c["classifier"]), layout=layout, aggregate=int(c["aggregate"]),
                          roots_np=np.ascontiguousarray(c["roots"], np.int32) if sparse else None,
                          leaf_w_np=np.ascontiguousarray(c["leaf_w"], np.float32) if sparse else None,
                          leaf_has_np=np.ascontiguousarray(c["leaf_has"], np.uint8) if sparse else None)
            steps.append(ts)
            width = n_out
            if c["classifier"]:
                # outputs: (label, probabilities); continue on the probability tensor
                prob = n["outputs"][1] if len(n["outputs"]) > 1 else n["outputs"][0]
                ml_col = 1 if n_out == 2 else 0
                cur = prob
            else:
                cur = n["outputs"][0]
            continue
        if op in ("Gemm", "MatMul"):
            w = const(n["inputs"][1]) if n["inputs"][1] in inits else None
            if w is None:
                raise PlanError(f"{op}: weight must be an initializer")
            w = np.asarray(w, np.float32)
            if op == "Gemm":
                if int(a.get("transA", 0)):
                    raise PlanError("Gemm transA=1 is not lowered")
                if int(a.get("transB", 0)):
                    w = w.T
                alpha = float(a.get("alpha", 1.0))
                beta = float(a.get("beta", 1.0))
                w = w * alpha
                b = None
                if len(n["inputs"]) > 2 and n["inputs"][2]:
                    b = np.asarray(const(n["inputs"][2]), np.float32).ravel() * beta
                    if b.size == 1 and w.shape[1] > 1:
                        b = np.full(w.shape[1], b[0], np.float32)
            else:
                b = None
            out_name = n["outputs"][0]
            if op == "MatMul":
                nxt = _consumers(nodes, out_name)
                if len(nxt) == 1 and nxt[0]["op_type"] == "Add" and id(nxt[0]) not in visited:
                    other = [i for i in nxt[0]["inputs"] if i != out_name][0]
                    if other in inits:
                        b = np.asarray(const(other), np.float32).ravel()
                        visited.add(id(nxt[0]))
                        out_name = nxt[0]["outputs"][0]
            act = "none"
            nxt = _consumers(nodes, out_name)
            if len(nxt) == 1 and nxt[0]["op_type"] in ("Relu", "Sigmoid", "Tanh") and id(nxt[0]) not in visited:
                act = nxt[0]["op_type"].lower()
                visited.add(id(nxt[0]))
                out_name = nxt[0]["outputs"][0]
            if width > 0 and w.shape[0] != width:
                raise PlanError(f"{op}: weight rows {w.shape[0]} != input width {width}")
            steps.append(DenseStep(n=int(w.shape[1]), k=int(w.shape[0]), act=act,
                                   w_np=np.ascontiguousarray(w.T, np.float32), b_np=b))
            width = int(w.shape[1])
            ml_col = 0
            cur = out_name
            continue
        if op in ("Relu", "Sigmoid", "Tanh"):
            last = steps[-1] if steps else None
            if isinstance(last, DenseStep) and last.act == "none":
                last.act = op.lower()
            elif isinstance(last, TreeStep) and op == "Sigmoid" and last.post == 0:
                last.post = 1
            else:
                raise PlanError(f"standalone {op} is not lowered")
            cur = n["outputs"][0]
            continue
        if op in ("Identity", "Flatten"):
            cur = n["outputs"][0]
            continue
        if op in ("Squeeze", "Reshape", "Unsqueeze"):
            # shape-only between GRU layers / before the head (validated by the CPU executor)
            if op == "Reshape" and bidir_pending:
                raise PlanError("bidirectional GRU: Y_h [2, N, H] must be transposed to [N, 2, H] before reshaping")
            cur = n["outputs"][0]
            continue
        if op == "Transpose":
            # only the direction <-> batch swap of a layout-0 GRU's Y_h ([D, N, H] -> [N, D, H])
            perm = [int(x) for x in a.get("perm", [])]
            if not steps or steps[-1].kind != "gru" or steps[-1].layout != 0 or perm != [1, 0, 2]:
                raise PlanError("Transpose is lowered only as perm [1, 0, 2] on a GRU's final states")
            bidir_pending = False
            cur = n["outputs"][0]
            continue
        if op == "GRU":
            direction = a.get("direction", "forward")
            layout = int(a.get("layout", 0))
            if direction not in ("forward", "reverse", "bidirectional") or layout not in (0, 1):
                raise PlanError(f"GRU: direction {direction!r} / layout {layout} is not lowered")
            if len(n["inputs"]) > 4 and n["inputs"][4]:
                raise PlanError("GRU: sequence_lens is not lowered")
            if len(n["inputs"]) > 5 and n["inputs"][5]:
                raise PlanError("GRU: initial_h is not lowered (the device starts every sequence at zero)")
            prev = [s for s in steps if s.kind == "gru"]
            if prev and (direction == "bidirectional" or prev[0].bidirectional
                         or prev[0].reverse != (direction == "reverse") or prev[0].layout != layout):
                raise PlanError("GRU: stacked layers must share direction and layout (bidirectional: one layer)")
            Wa = np.asarray(const(n["inputs"][1]), np.float32)
            Ra = np.asarray(const(n["inputs"][2]), np.float32)
            H = int(a.get("hidden_size", Ra.shape[-1]))
            D = 2 if direction == "bidirectional" else 1
            Ba = (np.asarray(const(n["inputs"][3]), np.float32).reshape(D, 6 * H)
                  if len(n["inputs"]) > 3 and n["inputs"][3] else np.zeros((D, 6 * H), np.float32))
            if Wa.shape[0] != D or Ra.shape[0] != D:
                raise PlanError("GRU: weight direction count does not match the direction attribute")
            seq = dims[1] if layout == 1 else dims[0]
            steps.append(GRUStep(hidden=H, in_dim=int(Wa.shape[2]),
                                 linear_before_reset=int(a.get("linear_before_reset", 0)),
                                 w_np=Wa[0], r_np=Ra[0], b_np=Ba[0], seq=int(seq) if seq > 0 else 0,
                                 reverse=direction == "reverse", layout=layout, bidirectional=D == 2,
                                 w_rev_np=Wa[1] if D == 2 else None, r_rev_np=Ra[1] if D == 2 else None,
                                 b_rev_np=Ba[1] if D == 2 else None))
            width = H * D
            # continue on Y (chained GRU) or Y_h (head)
            y, yh = n["outputs"][0], (n["outputs"][1] if len(n["outputs"]) > 1 else "")
            y_used = bool(y) and any(id(c) not in visited for c in _consumers(nodes, y))
            if D == 2 and y_used:
                raise PlanError("bidirectional GRU: only the final states (Y_h) are lowered")
            bidir_pending = D == 2 and layout == 0
            cur = y if y_used else yh
            continue
        raise PlanError(f"op {op} is not lowered to the device")
    fam = model.metadata.get("family", "")
    if not fam:
        kinds = [s.kind for s in steps]
        fam = ("gbdt" if kinds == ["tree"] else "stacked" if kinds and kinds[0] == "tree"
               else "gru" if "gru" in kinds else "mlp")
    plan = Plan(family=fam, in_width=in_width, steps=steps, out_width=width, ml_col=ml_col,
                metadata=dict(model.metadata), input_name=input_name, output_name=output_name,
                seq_input=seq_input)
    return fuse(plan) if fuse_heads else plan


def fuse(plan: Plan) -> Plan:
    """Fusion pass: dense(N>1) followed by dense(N=1) -> HeadStep (no hidden tensor in HBM)."""
    out = []
    i = 0
    st = plan.steps
    while i < len(st):
        s = st[i]
        if (s.kind == "dense" and s.n > 1 and i + 1 < len(st) and st[i + 1].kind == "dense"
                and st[i + 1].n == 1 and s.n <= 4096 and s.k <= 1024):
            t = st[i + 1]
            out.append(HeadStep(n1=s.n, k=s.k, act1=s.act, act2=t.act, w1_np=s.w_np, b1_np=s.b_np,
                                w2_np=np.ascontiguousarray(t.w_np[0], np.float32),
                                b2=float(t.b_np[0]) if t.b_np is not None else 0.0))
            i += 2
            continue
        out.append(s)
        i += 1
    plan.steps = out
    return plan


def _bf16_padded(w: np.ndarray, n_mult: int = 128, k_mult: int = 64):
    import torch
    n, k = w.shape
    npad = -(-n // n_mult) * n_mult
    kpad = -(-k // k_mult) * k_mult
    buf = np.zeros((npad, kpad), np.float32)
    buf[:n, :k] = w
    return torch.from_numpy(buf).to(torch.bfloat16)


def _f32_padded(w: np.ndarray, n_mult: int = 128, k_mult: int = 64):
    import torch
    n, k = w.shape
    buf = np.zeros((-(-n // n_mult) * n_mult, -(-k // k_mult) * k_mult), np.float32)
    buf[:n, :k] = w
    return torch.from_numpy(buf)


PRECISIONS = ("fp32", "bf16")


def validate_sparse(s: TreeStep) -> None:
    """Host check of a pointer-layout ensemble before it reaches the device: every child / root
    index is a node, every leaf row exists, and no root-to-leaf path is longer than ``depth``
    (the kernel's traversal bound), so K2b can only read inside its arrays."""
    nodes = s.nodes_np.reshape(-1, 4)
    N, L = nodes.shape[0], s.leaf_w_np.shape[0]
    if s.leaf_w_np.shape != (L, s.k) or s.leaf_has_np.shape != (L, s.k):
        raise PlanError("sparse trees: leaf tables must be [L, K]")
    if s.roots_np.shape != (s.n_trees,) or (s.roots_np < 0).any() or (s.roots_np >= N).any():
        raise PlanError("sparse trees: root index out of range")
    mode = (nodes[:, 0].view(np.uint32) >> 16) & 7
    leaf = mode == 7
    if ((nodes[leaf, 2] < 0) | (nodes[leaf, 2] >= L)).any():
        raise PlanError("sparse trees: leaf row out of range")
    ch = nodes[~leaf][:, 2:4]
    if ((ch < 0) | (ch >= N)).any():
        raise PlanError("sparse trees: child index out of range")
    if (nodes[~leaf, 0].view(np.uint32) & 0xFFFF).max(initial=0) > s.max_feature:
        raise PlanError("sparse trees: feature id above max_feature")
    # longest path by level expansion from the roots (bounded by depth + 1 levels)
    frontier = s.roots_np.astype(np.int64)
    for _ in range(s.depth + 1):
        inner = frontier[~leaf[frontier]]
        if inner.size == 0:
            return
        frontier = np.unique(np.concatenate([nodes[inner, 2], nodes[inner, 3]]).astype(np.int64))
    raise PlanError("sparse trees: a path is longer than the declared depth (cycle?)")


def to_device(plan: Plan, device, precision: str = "fp32") -> Plan:
    """Upload the plan's tensors. ``precision`` selects the dense / head weight format:
    ``fp32`` (default) keeps the ONNX model's f32 numerics end to end (f32 MFMA,
    onnx_model.go:221-238 contract); ``bf16`` runs the dense layers on the bf16 MFMA path
    (f32 accumulate). Trees are always f32; GRU weights are always bf16 (K4)."""
    import torch
    if precision not in PRECISIONS:
        raise ValueError(f"precision must be one of {PRECISIONS}, got {precision!r}")
    plan.precision = precision
    pad = _f32_padded if precision == "fp32" else _bf16_padded
    for s in plan.steps:
        if s.kind == "tree":
            s.nodes = torch.from_numpy(s.nodes_np).to(device)
            s.base = None if s.base_np is None else torch.from_numpy(s.base_np).to(device)
            if s.layout == "sparse":
                validate_sparse(s)
                s.roots = torch.from_numpy(s.roots_np).to(device)
                s.leaf_w = torch.from_numpy(s.leaf_w_np).to(device)
                s.leaf_has = torch.from_numpy(s.leaf_has_np).to(device)
            else:
                s.leaves = torch.from_numpy(s.leaves_np).to(device)
        elif s.kind == "dense":
            s.w = pad(s.w_np).to(device)
            s.b = None if s.b_np is None else torch.from_numpy(np.ascontiguousarray(s.b_np)).to(device)
        elif s.kind == "head":
            # f32 head: K padded to 32 only (the f32 MFMA k-step is 16; the specialised kernel is
            # built for k_pad 32 / 64), so a 32-wide tree embedding runs no all-zero k-steps
            s.w1 = (_f32_padded(s.w1_np, k_mult=32) if precision == "fp32" else pad(s.w1_np)).to(device)
            s.b1 = None if s.b1_np is None else torch.from_numpy(np.ascontiguousarray(s.b1_np)).to(device)
            s.w2 = torch.from_numpy(s.w2_np).to(device)
    return plan


def gru_device_weights(s: GRUStep, device) -> Dict[str, Any]:
    import torch
    H = s.hidden
    d = {
        "R": torch.from_numpy(np.ascontiguousarray(s.r_np)).to(torch.bfloat16).to(device),
        "bias": torch.from_numpy(np.ascontiguousarray(s.b_np, np.float32)).to(device),
        # input projection as a dense layer [3H, I] (W rows are output columns already)
        "W": _bf16_padded(np.ascontiguousarray(s.w_np)).to(device),
        "Wb": torch.from_numpy(np.ascontiguousarray(s.b_np[:3 * H], np.float32)).to(device),
    }
    return d
