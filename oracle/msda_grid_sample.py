"""ORACLE — test infrastructure, never product code.

Restatement of the reference's live MSDA core as the reference computes it: per level a
``torch.nn.functional.grid_sample`` (bilinear, border, align_corners=False) on a
(B*M, D, T_l, 1) image at grid (x = -1, y = 2*loc - 1), the per-level samples stacked
into a (B*M, D, Lq, L*P) tensor, multiplied by the attention weights and summed
(reference models/modules/attention.py:331-383).  Autograd gives the backward
(ATen grid_sampler_2d_backward + stack/mul/sum).

Used by bench.py's ``cpu_baseline`` leg (the reference's pure-PyTorch CPU path, timed on
the GPU box's host cores) and by the CPU tests that run this package's transformer
modules with the core swapped for this function (``cpu_model.oracle_core``).
"""
import torch
import torch.nn.functional as F

__all__ = ["msda_core_grid_sample"]


def _host_shapes(value_temporal_shapes):
    cached = getattr(value_temporal_shapes, "_mfl_host", None)
    if cached is not None:
        return [int(t) for t in cached]
    if isinstance(value_temporal_shapes, torch.Tensor):
        return [int(t) for t in value_temporal_shapes.reshape(-1).tolist()]
    return [int(t) for t in value_temporal_shapes]


def msda_core_grid_sample(value, value_temporal_shapes, sampling_locations, attention_weights,
                          return_value=False):
    """Same signature / result as reference ``ms_deform_attn_core_pytorch``."""
    shapes = _host_shapes(value_temporal_shapes)
    if sampling_locations.dim() == 6:
        sampling_locations = sampling_locations[..., 0]
    B, _, M, D = value.shape
    Lq, L, P = sampling_locations.shape[1], sampling_locations.shape[3], sampling_locations.shape[4]
    per_level_values = value.split(shapes, dim=1)
    grid_y = 2 * sampling_locations - 1
    sampled = []
    for lvl, T in enumerate(shapes):
        img = per_level_values[lvl].flatten(2).transpose(1, 2).reshape(B * M, D, T, 1)
        gy = grid_y[:, :, :, lvl].transpose(1, 2).flatten(0, 1).reshape(B * M, 1, Lq * P)
        grid = torch.stack([-torch.ones_like(gy), gy], dim=-1)
        s = F.grid_sample(img, grid, mode="bilinear", padding_mode="border", align_corners=False)
        sampled.append(s.reshape(B * M, D, Lq, P))
    stacked = torch.stack(sampled, dim=-2)                       # (B*M, D, Lq, L, P)
    if return_value:
        return stacked
    w = attention_weights.transpose(1, 2).reshape(B * M, 1, Lq, L * P)
    out = (stacked.flatten(-2) * w).sum(-1).view(B, M * D, Lq)
    return out.transpose(1, 2).contiguous()
