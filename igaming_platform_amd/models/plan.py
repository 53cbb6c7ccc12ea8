"""ONNX graph -> device execution plan.

The C++ reader parses the file; this module lowers the nodes the primary output depends on
(one model input; chains and DAGs whose branches meet in an Add / Concat) to fused device
steps:

* ``TreeStep``   TreeEnsemble{Classifier,Regressor} (+ a following Sigmoid folded into the
                 post transform) -> K2 ``tree_ensemble`` on the complete-tree layout, or K2b
                 ``tree_sparse`` on the pointer layout for deep (> 12) or very unbalanced trees,
                 MIN / MAX aggregates and target counts the complete kernel is not built for.
                 Every post transform (NONE, LOGISTIC, SOFTMAX, SOFTMAX_ZERO, PROBIT) runs on
                 the device.
* ``DenseStep``  Gemm / MatMul(+Add) with a following Relu/Sigmoid/Tanh fused into the
                 epilogue -> K3 ``gemm`` (MFMA) or ``gemv`` (N == 1).
* ``GRUStep``    ONNX GRU (forward / reverse / bidirectional, layout 0 / 1) -> K4 (cfg 5).
* ``JoinStep``   Add / Concat of two branches (residual blocks, wide & deep) -> ``join``.
* ai.onnx.ml ``LinearClassifier`` / ``LinearRegressor`` (post NONE / LOGISTIC; a two-class
  SOFTMAX as sigmoid(s1 - s0)) -> a dense layer, so an sklearn pipeline
  Scaler -> LinearClassifier -> ZipMap, or an MLP ending in one, runs on the fused head.
* ``Scaler`` and constant Add / Sub / Mul / Div fold into a neighbouring dense layer's
  weights; Identity / Flatten / Squeeze / Reshape / ZipMap / Cast(float) are folded away.

Anything else raises :class:`PlanError`; the engine then runs that model through the C++
CPU executor (explicitly, with a warning) rather than silently substituting torch ops.
"""
from __future__ import annotations

from dataclasses import dataclass, field, replace
from typing import Any, Dict, List, Optional, Tuple

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
    src: Optional[int] = None  # producing step of the input (None: the previous step; -1: model input)

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
    src: Optional[int] = None

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
    src: Optional[int] = None

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
    src: Optional[int] = None
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
    cpu_col: Optional[int] = None  # score column in the CPU executor's output (None: ml_col)

    @property
    def executor_col(self) -> int:
        """Column of the model score in the C++ executor's output tensor (a binary classifier
        lowered to its positive column has ml_col 0 on the device, 1 in the executor)."""
        return self.ml_col if self.cpu_col is None else self.cpu_col

    @property
    def is_chain(self) -> bool:
        return all(s.kind != "join" and getattr(s, "src", None) is None for s in self.steps)

    def describe(self) -> str:
        parts = []
        for s in self.steps:
            if s.kind == "tree":
                parts.append(f"tree(T={s.n_trees},D={s.depth},K={s.k},post={s.post},{s.layout})")
            elif s.kind == "dense":
                parts.append(f"dense({s.k}->{s.n},{s.act})")
            elif s.kind == "head":
                parts.append(f"head({s.k}->{s.n1},{s.act1}->1,{s.act2})")
            elif s.kind == "join":
                parts.append(f"{s.op}(#{s.a},#{s.b})")
            else:
                parts.append(f"gru(I={s.in_dim},H={s.hidden})")
        return " -> ".join(parts)


@dataclass
class JoinStep:
    """Add / Concat of two branch values (join.hip): ``a`` / ``b`` are the producing steps'
    indices (-1: the model input). Residual blocks and wide & deep towers lower to one per
    join; everything else in the branches stays on the fused dense / tree / head kernels."""
    op: str      # add | concat
    a: int
    b: int
    na: int
    nb: int
    kind: str = "join"

    @property
    def out_width(self) -> int:
        return self.na if self.op == "add" else self.na + self.nb


def step_inputs(steps, i: int) -> Tuple[int, ...]:
    """Indices of the steps whose outputs step ``i`` reads (-1: the model input)."""
    s = steps[i]
    if s.kind == "join":
        return (s.a, s.b)
    src = getattr(s, "src", None)
    return (i - 1 if src is None else src,)


def step_consumers(steps) -> List[List[int]]:
    cons: List[List[int]] = [[] for _ in steps]
    for i in range(len(steps)):
        for j in step_inputs(steps, i):
            if j >= 0:
                cons[j].append(i)
    return cons


@dataclass
class _Val:
    """A graph value during lowering: the step producing it plus what is still pending on it."""
    step: int                 # producing step (-1: the model input)
    width: int                # columns (-1: unknown, a symbolic model input)
    scale: Optional[np.ndarray] = None   # pending per-column affine x * scale + shift (Scaler,
    shift: Optional[np.ndarray] = None   # Add / Sub / Mul / Div by a constant), folded into a neighbour
    exclusive: bool = True    # derived from the step's output through single-use values only
    ml_col: int = 0           # model-score column of the value on the device
    cpu_col: int = 0          # ... and in the CPU executor's output of the same value
    narrowed: bool = False    # a binary classifier lowered to its positive column only
    label: bool = False       # a classifier's label output (not lowered)
    gru_y: bool = False       # a GRU's per-step outputs (only another GRU layer reads them)
    bidir_pending: bool = False  # a layout-0 bidirectional Y_h still in [D, N, H] order


ALIAS_OPS = ("Identity", "Flatten", "Squeeze", "Unsqueeze", "Reshape", "ZipMap", "Cast")
ACT_OPS = ("Relu", "Sigmoid", "Tanh")
LINEAR_POST = {"NONE": "none", "LOGISTIC": "sigmoid"}


def compile_onnx(model, input_name: str = "input", output_name: str = "output",
                 depth_limit: int = 12, fuse_heads: bool = True) -> Plan:
    """``model``: _native.OnnxModel. Returns a host-side Plan (upload with :func:`to_device`).

    The nodes the primary output depends on are lowered in dependency order; each value is
    tracked as (producing step, pending affine). Linear ops fold into their neighbours:
    Scaler / constant Add, Sub, Mul, Div into the next dense layer's weights (or the previous
    one's, when it has no activation), a constant Add after MatMul into its bias, Relu /
    Sigmoid / Tanh into the dense epilogue. Two branches meet in a :class:`JoinStep`."""
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

    # the nodes the output depends on, in dependency order: a depth-first post-order from the
    # output, so each branch's nodes stay contiguous (a dense layer and the N=1 layer reading it
    # end up adjacent for the head fusion)
    prod = {o: n for n in nodes for o in n["outputs"] if o}
    if output_name not in prod:
        raise PlanError(f"output {output_name!r} is not computed by a node")
    order, live = [], set()
    stack = [(prod[output_name], 0)]
    while stack:
        n, k = stack.pop()
        if id(n) in live:
            continue
        if k < len(n["inputs"]):
            stack.append((n, k + 1))
            name = n["inputs"][k]
            p = prod.get(name)
            if p is not None and id(p) not in live:
                stack.append((p, 0))
            elif p is None and name and name not in inits and name != input_name:
                raise PlanError(f"the output depends on graph input {name!r} besides the model input")
            continue
        live.add(id(n))
        order.append(n)

    def root(name):  # the value an alias chain (Identity / Reshape / ZipMap ...) starts from
        n = prod.get(name)
        while n is not None and id(n) in live and n["op_type"] in ALIAS_OPS:
            name = n["inputs"][0]
            n = prod.get(name)
        return name

    uses: Dict[str, int] = {}
    for n in order:
        if n["op_type"] in ALIAS_OPS:
            continue
        for i in set(n["inputs"]):
            if i and i not in inits:
                uses[root(i)] = uses.get(root(i), 0) + 1
    uses[root(output_name)] = uses.get(root(output_name), 0) + 1

    def single_use(name):
        return uses.get(root(name), 0) == 1

    steps: List[Any] = []
    vals: Dict[str, _Val] = {input_name: _Val(-1, in_width)}

    def emit(step, src: int) -> int:
        if step.kind != "join":
            step.src = src
        steps.append(step)
        return len(steps) - 1

    def get(name, what):
        v = vals.get(name)
        if v is None:
            raise PlanError(f"{what}: value {name!r} is not computed by a lowered node")
        if v.label:
            raise PlanError(f"{what}: a classifier's label output is not lowered (the device computes scores)")
        if v.narrowed:
            raise PlanError(f"{what}: reads a binary classifier's scores (lowered to the positive column)")
        if v.gru_y:
            raise PlanError(f"{what}: a GRU's per-step outputs are lowered only into another GRU layer")
        return v

    def plain(name, what) -> _Val:
        """The value with its pending affine applied: folded into the producing dense layer when
        that has no activation and nothing else reads its output, else one diagonal layer."""
        v = get(name, what)
        if v.scale is None:
            return v
        w = v.width if v.width > 0 else max(len(v.scale), len(v.shift))
        if w <= 1 and v.width <= 0:
            raise PlanError(f"{what}: scaling of a value of unknown width")
        sc = np.broadcast_to(v.scale, (w,)).astype(np.float64)
        sh = np.broadcast_to(v.shift, (w,)).astype(np.float64)
        st = steps[v.step] if v.step >= 0 else None
        if st is not None and st.kind == "dense" and st.act == "none" and v.exclusive:
            st.w_np = np.ascontiguousarray(st.w_np * sc[:, None], np.float32)
            b = np.zeros(st.n) if st.b_np is None else st.b_np.astype(np.float64)
            st.b_np = (b * sc + sh).astype(np.float32)
            nv = _Val(v.step, w, ml_col=v.ml_col, cpu_col=v.cpu_col)
        else:
            i = emit(DenseStep(n=w, k=w, act="none", w_np=np.diag(sc).astype(np.float32),
                               b_np=sh.astype(np.float32)), v.step)
            nv = _Val(i, w)
        vals[name] = nv
        return nv

    def linear(name, w, b, what):
        """(step, w, b) of ``x @ w + b`` for x = ``name`` (w [K, N]): x's pending affine is
        folded into w / b (scale rows of w, shift through w into b)."""
        v = get(name, what)
        if v.width > 0 and w.shape[0] != v.width:
            raise PlanError(f"{what}: weight rows {w.shape[0]} != input width {v.width}")
        if v.scale is not None:
            K = w.shape[0]
            sc = np.broadcast_to(v.scale, (K,)).astype(np.float64)
            sh = np.broadcast_to(v.shift, (K,)).astype(np.float64)
            b64 = (np.zeros(w.shape[1]) if b is None else b.astype(np.float64)) + sh @ w.astype(np.float64)
            w = (sc[:, None] * w.astype(np.float64)).astype(np.float32)
            b = b64.astype(np.float32)
        return v.step, w, b

    def affine(name, out, what, scale=None, shift=None):
        v = get(name, what)
        s0 = np.ones(1) if v.scale is None else v.scale
        t0 = np.zeros(1) if v.shift is None else v.shift
        sc = np.ones(1) if scale is None else np.asarray(scale, np.float64).ravel()
        sh = np.zeros(1) if shift is None else np.asarray(shift, np.float64).ravel()
        w = v.width
        for x in (s0, t0, sc, sh):
            if len(x) > 1:
                if w > 0 and len(x) != w:
                    raise PlanError(f"{what}: {len(x)} per-column constants for width {w}")
                w = len(x)
        vals[out] = replace(v, width=w, scale=s0 * sc, shift=t0 * sc + sh,
                            exclusive=v.exclusive and single_use(name))

    for n in order:
        op, a = n["op_type"], n["attrs"]
        ins = n["inputs"]
        x = ins[0] if ins else ""
        if op in ("TreeEnsembleClassifier", "TreeEnsembleRegressor"):
            v = plain(x, op)
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
            idx = emit(ts, v.step)
            if c["classifier"]:
                col = 1 if n_out == 2 else 0
                vals[n["outputs"][0]] = _Val(idx, 1, label=True)
                if len(n["outputs"]) > 1:
                    vals[n["outputs"][1]] = _Val(idx, n_out, ml_col=col, cpu_col=col)
                else:  # a single output holds the probabilities
                    vals[n["outputs"][0]] = _Val(idx, n_out, ml_col=col, cpu_col=col)
            else:
                vals[n["outputs"][0]] = _Val(idx, k)
            continue
        if op in ("Gemm", "MatMul"):
            if len(ins) < 2 or ins[1] not in inits:
                raise PlanError(f"{op}: weight must be an initializer")
            w = np.asarray(const(ins[1]), np.float32)
            if w.ndim != 2:
                raise PlanError(f"{op}: weight must be 2-D")
            b = None
            if op == "Gemm":
                if int(a.get("transA", 0)):
                    raise PlanError("Gemm transA=1 is not lowered")
                if int(a.get("transB", 0)):
                    w = w.T
                w = w * float(a.get("alpha", 1.0))
                if len(ins) > 2 and ins[2]:
                    if ins[2] not in inits:
                        raise PlanError("Gemm: bias must be an initializer")
                    b = np.asarray(const(ins[2]), np.float32).ravel() * float(a.get("beta", 1.0))
                    if b.size == 1 and w.shape[1] > 1:
                        b = np.full(w.shape[1], b[0], np.float32)
                    if b.size != w.shape[1]:
                        raise PlanError("Gemm: bias length differs from the output width")
            src, w, b = linear(x, w, b, op)
            idx = emit(DenseStep(n=int(w.shape[1]), k=int(w.shape[0]), act="none",
                                 w_np=np.ascontiguousarray(w.T, np.float32), b_np=b), src)
            vals[n["outputs"][0]] = _Val(idx, int(w.shape[1]))
            continue
        if op in ("Add", "Sub", "Mul", "Div"):
            dyn = [i for i in ins if i not in inits]
            if op == "Add" and len(dyn) == 2:
                va, vb = plain(dyn[0], op), plain(dyn[1], op)
                if va.width <= 0 or va.width != vb.width:
                    raise PlanError(f"Add join: widths {va.width} and {vb.width} must be equal and known")
                idx = emit(JoinStep("add", va.step, vb.step, va.width, vb.width), -1)
                vals[n["outputs"][0]] = _Val(idx, va.width)
                continue
            if len(dyn) != 1:
                raise PlanError(f"{op}: only a constant operand or an Add of two branches is lowered")
            xd = dyn[0]
            cst = np.asarray(const([i for i in ins if i != xd][0]), np.float64).ravel()
            first = ins[0] == xd
            v = get(xd, op)
            st = steps[v.step] if v.step >= 0 else None
            if (op == "Add" and v.scale is None and st is not None and st.kind == "dense" and st.act == "none"
                    and v.exclusive and single_use(xd) and cst.size in (1, st.n)):
                # MatMul + Add (and any constant added to a linear layer): the layer's bias
                b = np.zeros(st.n) if st.b_np is None else st.b_np.astype(np.float64)
                st.b_np = (b + np.broadcast_to(cst, (st.n,))).astype(np.float32)
                vals[n["outputs"][0]] = replace(v)
            elif op == "Add":
                affine(xd, n["outputs"][0], op, shift=cst)
            elif op == "Sub":
                affine(xd, n["outputs"][0], op, shift=-cst) if first else affine(xd, n["outputs"][0], op,
                                                                                  scale=-1.0, shift=cst)
            elif op == "Mul":
                affine(xd, n["outputs"][0], op, scale=cst)
            elif first:
                affine(xd, n["outputs"][0], op, scale=1.0 / cst)
            else:
                raise PlanError("Div of a constant by a value is not lowered")
            continue
        if op == "Concat":
            if int(a.get("axis", 0)) not in (1, -1) or any(i in inits for i in ins) or len(ins) < 2:
                raise PlanError("Concat is lowered along the feature axis of two or more branches")
            acc = plain(ins[0], op)
            for nxt in ins[1:]:
                vb = plain(nxt, op)
                if acc.width <= 0 or vb.width <= 0:
                    raise PlanError("Concat: branch widths must be known")
                idx = emit(JoinStep("concat", acc.step, vb.step, acc.width, vb.width), -1)
                acc = _Val(idx, acc.width + vb.width)
            vals[n["outputs"][0]] = acc
            continue
        if op in ACT_OPS:
            v = plain(x, op)
            st = steps[v.step] if v.step >= 0 else None
            if st is not None and st.kind == "dense" and st.act == "none" and v.exclusive and single_use(x):
                st.act = op.lower()
            elif (st is not None and st.kind == "tree" and op == "Sigmoid" and st.post == 0 and st.binary_class < 0
                  and v.exclusive and single_use(x)):
                st.post = 1
            else:
                raise PlanError(f"standalone {op} is not lowered")
            vals[n["outputs"][0]] = replace(v)
            continue
        if op in ALIAS_OPS:
            if x not in vals:
                raise PlanError(f"{op}: value {x!r} is not computed by a lowered node")
            v = vals[x]
            if op == "Reshape" and v.bidir_pending:
                raise PlanError("bidirectional GRU: Y_h [2, N, H] must be transposed to [N, 2, H] before reshaping")
            if op == "Cast" and int(a.get("to", 1)) != 1:
                raise PlanError("Cast to a non-float type is not lowered")
            vals[n["outputs"][0]] = v
            continue
        if op == "Transpose":
            # only the direction <-> batch swap of a layout-0 GRU's Y_h ([D, N, H] -> [N, D, H])
            v = vals.get(x)
            perm = [int(p) for p in a.get("perm", [])]
            if (v is None or v.step < 0 or steps[v.step].kind != "gru" or steps[v.step].layout != 0
                    or perm != [1, 0, 2]):
                raise PlanError("Transpose is lowered only as perm [1, 0, 2] on a GRU's final states")
            vals[n["outputs"][0]] = replace(v, bidir_pending=False)
            continue
        if op == "GRU":
            v = vals.get(x)
            if v is None or v.scale is not None or (v.step >= 0 and not v.gru_y):
                raise PlanError("GRU: the input must be the model input or the previous layer's Y")
            direction = a.get("direction", "forward")
            layout = int(a.get("layout", 0))
            if direction not in ("forward", "reverse", "bidirectional") or layout not in (0, 1):
                raise PlanError(f"GRU: direction {direction!r} / layout {layout} is not lowered")
            if len(ins) > 4 and ins[4]:
                raise PlanError("GRU: sequence_lens is not lowered")
            if len(ins) > 5 and ins[5]:
                raise PlanError("GRU: initial_h is not lowered (the device starts every sequence at zero)")
            prev = [s for s in steps if s.kind == "gru"]
            if prev and (direction == "bidirectional" or prev[0].bidirectional
                         or prev[0].reverse != (direction == "reverse") or prev[0].layout != layout):
                raise PlanError("GRU: stacked layers must share direction and layout (bidirectional: one layer)")
            Wa = np.asarray(const(ins[1]), np.float32)
            Ra = np.asarray(const(ins[2]), np.float32)
            H = int(a.get("hidden_size", Ra.shape[-1]))
            D = 2 if direction == "bidirectional" else 1
            Ba = (np.asarray(const(ins[3]), np.float32).reshape(D, 6 * H)
                  if len(ins) > 3 and ins[3] else np.zeros((D, 6 * H), np.float32))
            if Wa.shape[0] != D or Ra.shape[0] != D:
                raise PlanError("GRU: weight direction count does not match the direction attribute")
            seq = dims[1] if layout == 1 else dims[0]
            idx = emit(GRUStep(hidden=H, in_dim=int(Wa.shape[2]),
                               linear_before_reset=int(a.get("linear_before_reset", 0)),
                               w_np=Wa[0], r_np=Ra[0], b_np=Ba[0], seq=int(seq) if seq > 0 else 0,
                               reverse=direction == "reverse", layout=layout, bidirectional=D == 2,
                               w_rev_np=Wa[1] if D == 2 else None, r_rev_np=Ra[1] if D == 2 else None,
                               b_rev_np=Ba[1] if D == 2 else None), v.step)
            y, yh = n["outputs"][0], (n["outputs"][1] if len(n["outputs"]) > 1 else "")
            if D == 2 and y and uses.get(y, 0) > 0:
                raise PlanError("bidirectional GRU: only the final states (Y_h) are lowered")
            if y:
                vals[y] = _Val(idx, H * D, gru_y=True)
            if yh:
                vals[yh] = _Val(idx, H * D, bidir_pending=D == 2 and layout == 0)
            continue
        if op in ("LinearClassifier", "LinearRegressor"):
            coef = np.asarray(a.get("coefficients", []), np.float64).ravel()
            icpt = np.asarray(a.get("intercepts", []), np.float64).ravel()
            post = str(a.get("post_transform", "NONE"))
            if op == "LinearRegressor":
                E = int(a.get("targets", 1))
            else:
                E = len(icpt) if len(icpt) else max(1, coef.size // max(vals[x].width, 1) if x in vals else 1)
            if E < 1 or coef.size % E:
                raise PlanError(f"{op}: coefficients do not split into {E} rows")
            w = coef.reshape(E, coef.size // E).T           # [C, E]
            b = icpt if len(icpt) else np.zeros(E)
            if len(b) != E:
                raise PlanError(f"{op}: {len(b)} intercepts for {E} rows")
            col = cpu = 0
            narrowed = False
            if op == "LinearClassifier" and E == 2 and post == "SOFTMAX":
                # softmax over two scores: p1 = sigmoid(s1 - s0), one column
                w, b, act = w[:, 1:] - w[:, :1], b[1:] - b[:1], "sigmoid"
                narrowed, cpu = True, 1
            elif op == "LinearClassifier" and E == 1 and post == "SOFTMAX":
                # one row: softmax over [-s, s] -> p1 = sigmoid(2 s)
                w, b, act = 2 * w, 2 * b, "sigmoid"
                narrowed, cpu = True, 1
            elif post in LINEAR_POST:
                act = LINEAR_POST[post]
                if op == "LinearClassifier" and E == 1:
                    narrowed, cpu = True, 1   # executor scores [-s, s] (LOGISTIC: sigmoid of both)
                elif op == "LinearClassifier" and E == 2:
                    col = cpu = 1
            else:
                raise PlanError(f"{op}: post_transform {post} with {E} rows is CPU-only")
            src, w32, b32 = linear(x, w.astype(np.float32), b.astype(np.float32), op)
            idx = emit(DenseStep(n=int(w32.shape[1]), k=int(w32.shape[0]), act=act,
                                 w_np=np.ascontiguousarray(w32.T, np.float32), b_np=b32), src)
            scores = _Val(idx, int(w32.shape[1]), ml_col=col, cpu_col=cpu, narrowed=narrowed)
            if op == "LinearClassifier":
                vals[n["outputs"][0]] = _Val(idx, 1, label=True)
                if len(n["outputs"]) > 1:
                    vals[n["outputs"][1]] = scores
            else:
                vals[n["outputs"][0]] = scores
            continue
        if op == "Scaler":
            off = np.asarray(a.get("offset", [0.0]), np.float64).ravel()
            sc = np.asarray(a.get("scale", [1.0]), np.float64).ravel()
            if len(off) > 1 and len(sc) == 1:
                sc = np.full(len(off), sc[0])
            if len(sc) > 1 and len(off) == 1:
                off = np.full(len(sc), off[0])
            affine(x, n["outputs"][0], op, scale=sc, shift=-off * sc)
            continue
        raise PlanError(f"op {op} is not lowered to the device")

    fv = vals.get(output_name)
    if fv is None or fv.label:
        raise PlanError("the primary output must be a score / probability tensor")
    if fv.scale is not None:
        fv = plain(output_name, "output")
    if not steps or fv.step != len(steps) - 1:
        raise PlanError("the output must be computed by the last lowered step")
    if any(s.kind == "gru" for s in steps) and any(s.kind == "join" or s.src != i - 1
                                                   for i, s in enumerate(steps)):
        raise PlanError("sequence models are lowered as chains (GRU layers + head) only")
    fam = model.metadata.get("family", "")
    if not fam:
        kinds = [s.kind for s in steps]
        fam = ("gbdt" if kinds == ["tree"] else "stacked" if kinds and kinds[0] == "tree"
               else "gru" if "gru" in kinds else "mlp")
    plan = Plan(family=fam, in_width=in_width, steps=steps, out_width=fv.width, ml_col=fv.ml_col,
                metadata=dict(model.metadata), input_name=input_name, output_name=output_name,
                seq_input=seq_input, cpu_col=fv.cpu_col)
    return fuse(plan) if fuse_heads else fuse(plan, heads=False)


def executor_output(model, default_output: str = "output") -> Tuple[int, str]:
    """(score column, output name) of the model's primary output in the C++ CPU executor -
    also for models the device cannot run (the plan's view when it compiles; otherwise the
    last graph output, column 1 for a two-class classifier's probabilities)."""
    try:
        p = compile_onnx(model, output_name=default_output)
        return p.executor_col, p.output_name
    except Exception:  # PlanError, or a graph the lowering cannot even walk: the executor still runs it
        pass
    outs = [v[0] for v in model.outputs()]
    name = default_output if default_output in outs else outs[-1]
    nodes = model.nodes()
    prod = {o: n for n in nodes for o in n["outputs"] if o}
    n = prod.get(name)
    while n is not None and n["op_type"] in ALIAS_OPS:
        n = prod.get(n["inputs"][0])
    col = 0
    if n is not None and n["op_type"] == "LinearClassifier":
        icpt = np.asarray(n["attrs"].get("intercepts", []))
        col = 1 if len(icpt) in (1, 2) else 0
    elif n is not None and n["op_type"] == "TreeEnsembleClassifier":
        col = 1 if len(np.asarray(n["attrs"].get("classlabels_int64s", n["attrs"].get("classlabels_strings", [])))) == 2 else 0
    return col, name


def fuse(plan: Plan, heads: bool = True) -> Plan:
    """Fusion pass: dense(N>1) followed by dense(N=1) that alone reads it -> HeadStep (no
    hidden tensor in HBM). Step inputs are then renumbered and stored implicitly (``src`` None)
    wherever a step reads its predecessor."""
    st = plan.steps
    ins = [step_inputs(st, i) for i in range(len(st))]
    cons = step_consumers(st)
    out, origin, remap = [], [], {-1: -1}
    i = 0
    while i < len(st):
        s = st[i]
        if (heads and s.kind == "dense" and s.n > 1 and i + 1 < len(st) and st[i + 1].kind == "dense"
                and st[i + 1].n == 1 and ins[i + 1] == (i,) and cons[i] == [i + 1]
                and s.n <= 4096 and s.k <= 1024):
            t = st[i + 1]
            out.append(HeadStep(n1=s.n, k=s.k, act1=s.act, act2=t.act, w1_np=s.w_np, b1_np=s.b_np,
                                w2_np=np.ascontiguousarray(t.w_np[0], np.float32),
                                b2=float(t.b_np[0]) if t.b_np is not None else 0.0))
            origin.append(i)
            remap[i] = remap[i + 1] = len(out) - 1
            i += 2
            continue
        out.append(s)
        origin.append(i)
        remap[i] = len(out) - 1
        i += 1
    for j, (s, oi) in enumerate(zip(out, origin)):
        if s.kind == "join":
            s.a, s.b = remap[s.a], remap[s.b]
        else:
            src = remap[ins[oi][0]]
            s.src = None if src == j - 1 else src
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
