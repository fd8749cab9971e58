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
