"""Helpers the deformable path uses from the reference's ``models/modules/misc_modules.py``."""
from typing import Optional

import torch
from torch import Tensor

__all__ = ["inverse_sigmoid", "predict_event_num", "predict_event_num_with_depth", "NestedTensor"]


def inverse_sigmoid(x, eps=1e-5):
    """reference misc_modules.py:28-32"""
    x = x.clamp(min=0, max=1)
    x1 = x.clamp(min=eps)
    x2 = (1 - x).clamp(min=eps)
    return torch.log(x1 / x2)


def predict_event_num(counter, query_features):
    """reference misc_modules.py:35-39: max-pool over queries, then the count head."""
    query_features_pool = torch.max(query_features, dim=1, keepdim=False)[0]
    return counter(query_features_pool)


def predict_event_num_with_depth(counter, query_features):
    """reference misc_modules.py:41-45"""
    query_features_pool = torch.max(query_features, dim=2, keepdim=False)[0]
    return counter(query_features_pool)


def level_heads(core, hs):
    """Class / segment / count heads on every decoder level of hs (depth, B, Q, d), stacked over
    levels (reference unimodal_deformable_dvc.py:197-203, heads applied per level).  The reference
    builds the per-level heads as ONE shared module (:72-74), so here each head runs once over the
    stacked levels (row-wise layers: the same numbers, a sixth of the launches, and no per-level
    select whose backward writes a full-size zero gradient per level); distinct per-level heads
    run level by level."""
    heads = (core.class_embedding, core.segment_embedding, core.count_head)
    if all(all(m is h[0] for m in h) for h in heads):
        return (core.class_embedding[0](hs).softmax(dim=-1), core.segment_embedding[0](hs).sigmoid(),
                predict_event_num_with_depth(core.count_head[0], hs))
    classes, segments, counts = [], [], []
    for lvl, h in enumerate(hs.unbind(0)):
        classes.append(core.class_embedding[lvl](h).softmax(dim=-1))
        segments.append(core.segment_embedding[lvl](h).sigmoid())
        counts.append(predict_event_num(core.count_head[lvl], h))
    return torch.stack(classes), torch.stack(segments), torch.stack(counts)


class NestedTensor(object):
    """reference misc_modules.py:47-70: tensors + padding mask (+ clip durations)."""

    def __init__(self, tensors, mask: Optional[Tensor], duration=None):
        self.tensors = tensors
        self.mask = mask
        self.duration = duration

    def to(self, device, non_blocking=False):
        cast_tensor = self.tensors.to(device, non_blocking=non_blocking)
        cast_mask = self.mask.to(device, non_blocking=non_blocking) if self.mask is not None else None
        return NestedTensor(cast_tensor, cast_mask)  # the reference drops duration here too

    def decompose(self):
        return self.tensors, self.mask

    def __repr__(self):
        return str(self.tensors)
