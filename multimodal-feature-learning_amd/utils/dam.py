"""Sparse-DETR decoder attention map, same functions and signatures as the reference's
``utils/dam.py`` (used by the criterion's mask-prediction loss and correlation metric,
models/criterion.py:246-309).

``attn_map_to_flat_grid`` is the scatter-add hot spot: it runs on the HIP kernel
``msda_hip_dam_flat_grid`` (one workgroup per (batch*layer, head) row, the row accumulated in
LDS).  Like every op of this package it has no CPU implementation and raises for host tensors.
``idx_to_flat_grid`` / ``compute_corr`` are a one-hot scatter and a few sums: plain torch.
"""
import torch

from .. import _native
from .. import msda as _msda

__all__ = ["attn_map_to_flat_grid", "idx_to_flat_grid", "compute_corr"]


def idx_to_flat_grid(temporal_shapes, idx):
    """(rows, S) one-hot of the selected token indices (reference utils/dam.py:12-17)."""
    shapes, _ = _msda.host_levels(temporal_shapes)
    flat_grid = torch.zeros((idx.shape[0], sum(shapes)), device=idx.device, dtype=torch.float32)
    flat_grid.scatter_(1, idx.to(torch.int64), 1)
    return flat_grid


def attn_map_to_flat_grid(temporal_shapes, level_start_index, sampling_locations, attention_weights):
    """(B, num_layers, num_heads, S) attention mass per token (reference utils/dam.py:20-73).

    sampling_locations (B, NL, Lq, M, L, P[, 1]), attention_weights (B, NL, Lq, M, L, P)."""
    loc = sampling_locations
    if loc.dim() == 7:
        loc = loc[..., 0]
    if loc.dim() != 6 or tuple(loc.shape) != tuple(attention_weights.shape):
        raise ValueError(f"sampling_locations {tuple(sampling_locations.shape)} / attention_weights "
                         f"{tuple(attention_weights.shape)}: expected (B, NL, Lq, M, L, P[, 1])")
    if not (loc.is_cuda and attention_weights.is_cuda):
        raise RuntimeError("attn_map_to_flat_grid: ROCm device tensors required (HIP kernel, no CPU path)")
    shapes, starts = _msda.host_levels(temporal_shapes, level_start_index)
    B, NL, Lq, M, L, P = loc.shape
    if len(shapes) != L:
        raise ValueError(f"{len(shapes)} level shapes for {L} levels")
    loc = loc.to(torch.float32).contiguous()
    aw = attention_weights.to(torch.float32).contiguous()
    out = torch.empty((B, NL, M, sum(shapes)), dtype=torch.float32, device=loc.device)
    lib = _native.load_library()
    rc = lib.msda_hip_dam_flat_grid(loc.data_ptr(), aw.data_ptr(), _native.host_i64_array(shapes),
                                    _native.host_i64_array(starts), L, B * NL, Lq, M, P, out.data_ptr(),
                                    _native.stream_handle(loc.device))
    _native.check(rc, "msda_hip_dam_flat_grid")
    return out


def compute_corr(flat_grid_topk, flat_grid_attn_map, temporal_shapes):
    """Overall and per-level fraction of attention mass on the top-k tokens
    (reference utils/dam.py:76-93)."""
    if flat_grid_topk.dim() == 1:
        flat_grid_topk = flat_grid_topk.unsqueeze(0)
        flat_grid_attn_map = flat_grid_attn_map.unsqueeze(0)
    corr = [(flat_grid_topk * flat_grid_attn_map).sum(-1) / flat_grid_attn_map.sum(-1)]
    shapes, _ = _msda.host_levels(temporal_shapes)
    start = 0
    for t in shapes:
        sl = slice(start, start + t)
        corr.append((flat_grid_topk[:, sl] * flat_grid_attn_map[:, sl]).sum(-1) / flat_grid_attn_map[:, sl].sum(-1))
        start += t
    return corr
