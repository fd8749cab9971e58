"""Hungarian matching of predicted to target segments, reference models/matcher.py:14-101.

Cost = cost_segment * L1(centre, length) + cost_giou * (-gIoU) on the device; the assignment is
scipy's ``linear_sum_assignment`` on the host, as in the reference.  The reference makes one
device->host copy per call (``.cpu()`` :86) plus two syncing asserts (utils/box_ops.py:59-60), once
per decoder level; ``match_levels`` builds every level's cost matrix and the well-formedness flags
on the device and moves them in ONE copy."""
from collections.abc import Sequence

import numpy as np
import torch
from scipy.optimize import linear_sum_assignment
from torch import nn

from ..utils.box_ops import generalized_box_iou_unchecked, segment_cl_to_xy

__all__ = ["HungarianMatcher", "build_matcher"]


class HungarianMatcher(nn.Module):
    def __init__(self, cost_class=1., cost_segment=1., cost_giou=1., cost_alpha=0.25, cost_gamma=2.0):
        super().__init__()
        self.cost_class = cost_class
        self.cost_segment = cost_segment
        self.cost_giou = cost_giou
        self.cost_alpha = cost_alpha
        self.cost_gamma = cost_gamma
        assert cost_class != 0 or cost_segment != 0 or cost_giou != 0, "Costs cant be 0."

    @torch.no_grad()
    def forward(self, outputs, targets):
        """outputs["pred_segments"] (B, Q, 2); targets: list of {"segments": (n_b, 2)} ->
        [(pred_idx int64, tgt_idx int64)] per clip (reference :43-94)."""
        return self.match_levels([outputs], targets)[0]

    @torch.no_grad()
    def match_levels(self, outputs_list, targets):
        """``forward`` for several outputs (decoder levels) against the same targets."""
        costs, meta = self.level_costs(outputs_list, targets)
        return self.solve_levels(costs.cpu(), meta)  # the one device->host copy

    @torch.no_grad()
    def level_costs(self, outputs_list, targets):
        """The device half of ``match_levels``: every level's cost matrix and the well-formedness
        flags packed in one fp64 device tensor (a graph-captured step copies it to the host),
        plus the host metadata ``solve_levels`` needs."""
        tgt_segments = torch.cat([v["segments"] for v in targets])
        tgt_xy = segment_cl_to_xy(tgt_segments)
        sizes = [len(v["segments"]) for v in targets]
        shapes = [tuple(o["pred_segments"].shape[:2]) for o in outputs_list]
        if len(outputs_list) > 1 and len(set(shapes)) == 1 and len(set(o["pred_segments"].dtype
                                                                      for o in outputs_list)) == 1:
            # every level's rows in one matrix: the costs are row-wise (cdist p=1, gIoU), so each
            # element is the per-level one and the flattened (levels * B * Q, n) matrix is the
            # concatenation of the per-level flattened costs — a few launches instead of ~20 a level
            out_segments = torch.stack([o["pred_segments"] for o in outputs_list]).flatten(0, 2)
            out_xy = segment_cl_to_xy(out_segments)
            c = (self.cost_segment * torch.cdist(out_segments, tgt_segments, p=1)
                 - self.cost_giou * generalized_box_iou_unchecked(out_xy, tgt_xy))
            flags = (out_xy[:, 1] >= out_xy[:, 0]).view(len(outputs_list), -1).all(1)
            flags = torch.cat([flags, (tgt_xy[:, 1] >= tgt_xy[:, 0]).all().reshape(1)])
            return (torch.cat([c.reshape(-1).double(), flags.double()]),
                    (shapes, sizes, len(tgt_segments), len(outputs_list) + 1))
        costs, flags, shapes = [], [], []
        for outputs in outputs_list:
            B, Q = outputs["pred_segments"].shape[:2]
            out_segments = outputs["pred_segments"].flatten(0, 1)
            out_xy = segment_cl_to_xy(out_segments)
            cost_segment = torch.cdist(out_segments, tgt_segments, p=1)
            cost_giou = -generalized_box_iou_unchecked(out_xy, tgt_xy)
            c = self.cost_segment * cost_segment + self.cost_giou * cost_giou
            costs.append(c.reshape(-1).double())  # exact for fp32 costs; scipy solves in fp64
            flags.append((out_xy[:, 1] >= out_xy[:, 0]).all().reshape(1))
            shapes.append((B, Q))
        flags.append((tgt_xy[:, 1] >= tgt_xy[:, 0]).all().reshape(1))
        return torch.cat(costs + [torch.cat(flags).double()]), (shapes, sizes, len(tgt_segments), len(flags))

    @staticmethod
    def solve_levels(host, meta):
        """The host half: the reference's syncing asserts (utils/box_ops.py:59-60) and scipy's
        linear_sum_assignment per clip and level (reference :86-94), on numpy views of the one
        copied buffer (the per-clip torch indexing and conversions were most of the host step)."""
        res = HungarianMatcher.solve_levels_into(host, meta, None)
        return res.materialize() if isinstance(res, _LevelPairs) else res  # a plain list leaves the public API

    @staticmethod
    def solve_levels_into(host, meta, idx_out):
        """``solve_levels``; with ``idx_out`` (an int64 (levels, 2, n_tgt) array) also writes every
        level's get_src_permutation_idx (clip, prediction) lists into it.  Every clip's matching in ONE
        native call (include/host_lsa.h: scipy's algorithm and tie rules) where the levels share their
        shapes and no clip has more targets than predictions; scipy per clip otherwise (or with
        MFL_HOST_LSA=0)."""
        import os
        shapes, sizes, n_tgt, n_flags = meta
        h = host.numpy() if isinstance(host, torch.Tensor) else np.asarray(host)
        ok = h[-n_flags:]
        assert bool(ok[:-1].all()), "Segment start > Segment end (from output)"
        assert bool(ok[-1]), "Segment start > Segment end (from target)"
        bounds = np.cumsum([0] + list(sizes)).astype(np.int64)
        if (os.environ.get("MFL_HOST_LSA", "1") != "0" and shapes and len(set(shapes)) == 1
                and h.dtype in (np.float32, np.float64) and max(sizes, default=0) <= shapes[0][1]
                and n_tgt == int(bounds[-1])):
            from .. import _native
            lib = _native.load_library()
            L = len(shapes)
            B, Q = shapes[0]
            cost = np.ascontiguousarray(h[:L * B * Q * n_tgt], dtype=np.float64)  # (scipy solves in float64)
            src = np.empty((L, n_tgt), np.int64)
            tgt = np.empty((L, n_tgt), np.int64)
            idx = idx_out if idx_out is not None else np.empty((L, 2, n_tgt), np.int64)
            rc = lib.mfl_lsa_levels(cost.ctypes.data, L, B, Q, n_tgt, bounds.ctypes.data, src.ctypes.data,
                                    tgt.ctypes.data, idx.ctypes.data)
            if rc == 2:
                raise ValueError("matrix contains invalid numeric entries")
            if rc == 3:
                raise ValueError("cost matrix is infeasible")
            if rc != 0:
                raise RuntimeError(f"mfl_lsa_levels failed (status {rc})")
            return _LevelPairs(src, tgt, bounds, L, B)
        result, off = [], 0
        for B, Q in shapes:
            n = B * Q * n_tgt
            cost = h[off:off + n].reshape(B, Q, n_tgt)
            off += n
            level = []
            for b in range(B):
                i, j = linear_sum_assignment(cost[b, :, bounds[b]:bounds[b + 1]])
                level.append((torch.from_numpy(i.astype(np.int64)), torch.from_numpy(j.astype(np.int64))))
            result.append(level)
        if idx_out is not None:
            for lvl, ind in enumerate(result):
                off = 0
                for b, (s_, t_) in enumerate(ind):
                    sv, tv = s_.numpy(), t_.numpy()
                    k = len(sv)
                    idx_out[lvl, 0, off:off + k] = b
                    idx_out[lvl, 1, off:off + k] = sv[np.argsort(tv, kind="stable")]
                    off += k
        return result


class _LevelPairs(Sequence):
    """solve_levels_into's result ([level][clip] -> (prediction indices, target indices) int64 tensors)
    over the native call's flat arrays, built when first read: a replayed DVC step reads only the index
    lists the call also wrote (the ~200 small tensors cost more host time than the matching).  A
    read-only Sequence, not a list subclass (C-level list operations would see the empty storage);
    the public ``solve_levels`` hands out ``materialize()``'s plain list."""

    def __init__(self, src, tgt, bounds, L, B):
        self._args = (src, tgt, bounds, L, B)
        self._levels = None

    def materialize(self):
        if self._levels is None:
            src, tgt, bounds, L, B = self._args
            st, tt = torch.from_numpy(src), torch.from_numpy(tgt)
            self._levels = [[(st[lvl, bounds[b]:bounds[b + 1]], tt[lvl, bounds[b]:bounds[b + 1]]) for b in range(B)]
                            for lvl in range(L)]
        return self._levels

    def __getitem__(self, i):
        return self.materialize()[i]

    def __len__(self):
        return self._args[3]

    def __eq__(self, other):
        return self.materialize() == (other.materialize() if isinstance(other, _LevelPairs) else other)

    def __repr__(self):
        return repr(self.materialize())


def build_matcher(args):
    """reference :97-101"""
    return HungarianMatcher(cost_class=args.cost_class, cost_segment=args.cost_segment, cost_giou=args.cost_giou,
                            cost_alpha=args.cost_alpha, cost_gamma=args.cost_gamma)
