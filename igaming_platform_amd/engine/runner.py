"""Device execution of a compiled :class:`Plan` (tree / dense / fused head / GRU steps).

Owns the per-step activation buffers (sized for the largest bucket), the tree-partial slab
used by the tree->head fusion and the per-bucket tree group counts. Launches are eager on the
current stream; callers (the fraud scorer, the LTV and abuse services) capture them in
their own hipGraphs together with their copies, so a model step never re-captures.
"""
from __future__ import annotations

import os

from typing import Dict, List, Optional, Sequence

import torch

from ..models.plan import Plan, step_consumers, step_inputs
from ..ops import kernels as K


def tree_groups(step, bucket: int) -> int:
    """Split the trees of one ensemble into ``g`` groups so a small batch still fills the
    256 CUs, without shrinking a group below 8 trees: >= 384 workgroups (3 groups at 8192 rows).
    Round 5 moved the target from 512 to 256 workgroups (at 8192 rows 2 groups instead of 4
    left more of the chip to K1 / the dedup insert: engine_only 151 vs 139 M, profiles/r5/eng/
    groups). After round 6's LDS traversal rework and at serving depth 6, 3 groups measured best
    (same box, interleaved: 2 / 3 / 4 groups engine_only 149.4 / 151.0 / 147.5 M, serving
    120.1 / 127.1 / 127.0 M, profiles/r6/al; 3 pairs 2 vs 3 groups: serving 119.7 / 122.8 / 122.7
    vs 125.5 / 126.4 / 127.1 M, engine_only flat, profiles/r6/am); 1 group drops to 91 M."""
    forced = int(os.environ.get("IGP_TREE_GROUPS", "0"))  # same-box A/B override
    if forced > 0:
        return max(1, min(forced, step.n_trees))
    tiles = -(-bucket // 64)
    return max(1, min(max(1, step.n_trees // 8), -(-384 // tiles)))


class GruModel:
    """The GRU part of a plan on the device (K4, csrc/kernels/gru*.hip):

    * forward or reverse layers (1-2, stacked): one launch, the N=1 head fused in its epilogue;
    * one bidirectional layer: a forward and a reverse launch, each writing its final state
      into its half of a [rows, 2H] buffer (the ONNX Y_h in [N, 2, H] order), then the N=1
      head as a dense launch.

    Input: dense X f32 [T, rows, I] (the ONNX layout-0 order; layout-1 plans are fed the same,
    see :meth:`DeviceModel.run`) or the store's event rings for ``slots``."""

    def __init__(self, steps, device, split: bool, bmax: int):
        n = 0
        while n < len(steps) and steps[n].kind == "gru":
            n += 1
        head = steps[n] if n < len(steps) and steps[n].kind == "dense" and steps[n].n == 1 else None
        if n == 0 or n + (head is not None) != len(steps):
            raise ValueError("sequence model must be GRU layers followed by at most an N=1 head")
        g = steps[0]
        self.H = g.hidden
        self.seq = g.seq
        self.bidirectional = g.bidirectional
        self.head = head
        if g.bidirectional:
            if n != 1:
                raise ValueError("bidirectional GRU: one layer")
            self.packs = [K.GruPack([g.direction(0)], None, device, split=split),
                          K.GruPack([g.direction(1)], None, device, split=split, reverse=True)]
            self.yh = [torch.zeros((bmax, self.H), dtype=torch.float32, device=device) for _ in range(2)]
            self.cat = torch.zeros((bmax, 2 * self.H), dtype=torch.float32, device=device)
        else:
            self.packs = [K.GruPack(steps[:n], head, device, split=split, reverse=g.reverse)]

    @property
    def has_head(self) -> bool:
        return self.head is not None

    @property
    def split(self) -> bool:
        """f32-faithful (bf16 hi/lo, three MFMAs per product) weights."""
        return self.packs[0].split

    def run(self, n_rows: int, T: int, out: torch.Tensor, X: Optional[torch.Tensor] = None, store=None,
            slots: Optional[torch.Tensor] = None, m_ptr: Optional[torch.Tensor] = None) -> None:
        """``out``: [rows] probabilities with a head, else [rows, H * directions] final states."""
        if not self.bidirectional:
            gp = self.packs[0]
            if self.head is not None:
                K.gru(gp, n_rows, T, out=out, X=X, store=store, slots=slots, m_ptr=m_ptr)
            else:
                K.gru(gp, n_rows, T, yh=out, X=X, store=store, slots=slots, m_ptr=m_ptr)
            return
        for gp, yh in zip(self.packs, self.yh):
            K.gru(gp, n_rows, T, yh=yh, X=X, store=store, slots=slots, m_ptr=m_ptr)
        dst = self.cat if self.head is not None else out
        torch.cat([self.yh[0][:n_rows], self.yh[1][:n_rows]], dim=1, out=dst[:n_rows])
        if self.head is not None:
            h = self.head
            K.dense(self.cat, h.w, h.b, out, n_rows, 1, 2 * self.H, act=h.act, m_ptr=m_ptr)


class DeviceModel:
    def __init__(self, plan: Plan, device, buckets: Sequence[int]):
        self.plan = plan
        self.device = K.as_device(device)
        self.buckets = sorted(set(int(b) for b in buckets))
        B = self.buckets[-1]
        self.step_out: List[torch.Tensor] = []
        self.tree_partial: Optional[torch.Tensor] = None
        self.tree_groups: Dict[int, int] = {}
        steps = plan.steps
        self.consumers = step_consumers(steps)
        for i, s in enumerate(steps):
            last = i == len(steps) - 1
            cons = self.consumers[i]
            feeds_mma = (not last) and bool(cons) and all(steps[j].kind in ("dense", "head", "join") for j in cons)
            # bf16 plans hand bf16 activations to the MFMA layers reading them; fp32 plans stay f32
            dt = (torch.bfloat16 if (s.kind in ("dense", "gru", "join") and feeds_mma and plan.precision == "bf16")
                  else torch.float32)
            self.step_out.append(torch.zeros((B, s.out_width), dtype=dt, device=self.device))
            if s.kind == "tree":
                need = 0
                for b in self.buckets:
                    g = tree_groups(s, b)
                    self.tree_groups[b] = g
                    need = max(need, g * b * s.k)
                self.tree_partial = torch.zeros(max(need, 1), dtype=torch.float32, device=self.device)
        # tree -> head pairs that run as one launch (trees.hip tree_head_kernel) need one ticket
        # counter per 64-row tile (the kernel returns them to zero)
        self.tile_cnt = torch.zeros(-(-B // 64), dtype=torch.int32, device=self.device)
        # sequence models: the GRU layers (+ an N=1 head) run as ONE fused K4 launch
        # (a bidirectional layer: two launches + the head, GruModel)
        self.gru: Optional[GruModel] = None
        self.gru_steps = 0
        if any(s.kind == "gru" for s in steps):
            self.gru = GruModel(steps, self.device, plan.precision != "bf16", B)
            self.gru_steps = len(steps)
            self.seq_len = steps[0].seq
        self.out = self.step_out[-1] if self.step_out else None

    @property
    def out_width(self) -> int:
        return self.plan.out_width

    def fuses_ensemble(self, bucket: Optional[int] = None) -> bool:
        """Whether :meth:`run` can run the scorer's K5 ensemble in the epilogue of its last step:
        an N=1 MLP head whose output column is the model score, or (for ``bucket``) a
        complete-layout tree ensemble as the only step, launched in groups, whose finish kernel
        then runs K5 (IGP_FUSE_TREE_ENS=0 keeps the standalone ensemble there)."""
        steps = self.plan.steps
        if self.gru is not None or not steps:
            return False
        if steps[-1].kind == "head":
            return self.plan.ml_col == 0
        return (bucket is not None and len(steps) == 1 and steps[0].kind == "tree"
                and steps[0].layout != "sparse" and self.tree_groups.get(bucket, 1) > 1
                and os.environ.get("IGP_FUSE_TREE_ENS", "1") != "0")

    def run(self, X: torch.Tensor, bucket: int, m_ptr: Optional[torch.Tensor] = None,
            ens: Optional[dict] = None) -> torch.Tensor:
        """X: [rows, in] f32 (or [T, rows, I] for a GRU model); returns the last step's buffer.
        ``ens`` (only when :meth:`fuses_ensemble`): K5 arguments for the fused head epilogue."""
        steps = self.plan.steps
        if ens is not None and not self.fuses_ensemble(bucket):
            raise ValueError("this plan cannot fuse the ensemble")
        if self.gru is not None:
            if self.plan.steps[0].layout == 1:  # batch-major model input [rows, T, I]
                X = X.transpose(0, 1).contiguous()
            self.gru.run(bucket, X.shape[0], self.out, X=X, m_ptr=m_ptr)
            return self.out
        cur = X
        fused_partial = None
        skip = -1
        one_launch = os.environ.get("IGP_TREE_HEAD", "1") != "0"

        def value(k):
            return X if k < 0 else self.step_out[k]
        for i, (s, out) in enumerate(zip(steps, self.step_out)):
            if i == skip:
                cur = out
                continue
            if s.kind == "join":  # two branches of a DAG model meet
                K.join(s.op, value(s.a), value(s.b), out, bucket, s.na, s.nb, m_ptr=m_ptr)
                fused_partial = None
                cur = out
                continue
            cur = value(step_inputs(steps, i)[0])
            if s.kind == "tree" and s.layout == "sparse":
                K.tree_sparse(s, cur, out, bucket, partial=self.tree_partial, groups=self.tree_groups.get(bucket, 1))
                fused_partial = None
            elif s.kind == "tree":
                g = self.tree_groups.get(bucket, 1)
                fuse = (g > 1 and i + 1 < len(steps) and steps[i + 1].kind == "head" and s.post == 0
                        and s.binary_class < 0 and steps[i + 1].k == s.k and self.consumers[i] == [i + 1]
                        and step_inputs(steps, i + 1) == (i,))
                if fuse and one_launch and K.tree_head_ok(s, steps[i + 1], g):
                    # the head (and the K5 of a last head) in the tree kernel's last-arriving blocks
                    K.tree_head(s, steps[i + 1], cur, self.step_out[i + 1], bucket, self.tree_partial, g,
                                self.tile_cnt, m_ptr=m_ptr, ens=ens if i + 1 == len(steps) - 1 else None)
                    skip = i + 1
                    cur = out
                    continue
                K.tree_ensemble(s, cur, None if fuse else out, bucket, partial=self.tree_partial,
                                groups=g, no_finish=fuse, ens=ens if i == len(steps) - 1 else None)
                fused_partial = (self.tree_partial, g, s) if fuse else None
            elif s.kind == "dense":
                K.dense(cur, s.w, s.b, out, bucket, s.n, s.k, act=s.act, m_ptr=m_ptr)
            elif s.kind == "head":
                K.mlp_head(s, cur, out, bucket, m_ptr=m_ptr, tree_partial=fused_partial,
                           ens=ens if i == len(steps) - 1 else None)
                fused_partial = None
            cur = out
        return cur
