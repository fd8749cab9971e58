"""reference models/ops/modules/ms_deform_attn.py (and ms_deform_attn_for_caption.py):
the extension-backed MSDeformAttn variant that lifts the 1-D locations to the 2-D
(H = 1, W = T; y = 0.5) layout of the native op and zero-initialises the attention
weights (:72-73, unlike models/modules/attention.py:437)."""
import math
import warnings

import torch
import torch.nn.functional as F
from torch import nn
from torch.nn.init import constant_, xavier_uniform_

from .... import msda as _msda
from ..functions import MSDeformAttnFunction, ms_deform_attn_core_pytorch
from ...modules.linear import Linear

__all__ = ["MSDeformAttn", "MSDeformAttnCap", "stack_sampled_values"]


def _is_power_of_2(n):
    if (not isinstance(n, int)) or (n < 0):
        raise ValueError("invalid input for _is_power_of_2: {} (type: {})".format(n, type(n)))
    return (n & (n - 1) == 0) and n != 0


def stack_sampled_values(value, shapes, starts, loc, attention_weights, padding_mode):
    """Per-sample interpolated values stacked as (B*M, D, Lq, L, P) — the ``return_value``
    result of the reference cores (attention.py:376-378, ms_deform_attn_func.py:66-67).
    Computed by L*P kernel launches with one-hot attention weights."""
    B, S, M, D = value.shape
    Lq, L, P = loc.shape[1], loc.shape[3], loc.shape[4]
    cols = []
    for li in range(L):
        for pi in range(P):
            onehot = torch.zeros_like(attention_weights)
            onehot[:, :, :, li, pi] = 1
            cols.append(_msda.msda_apply(value, shapes, starts, loc, onehot, padding_mode).view(B, Lq, M, D))
    st = torch.stack(cols, -1).view(B, Lq, M, D, L, P)
    return st.permute(0, 2, 3, 1, 4, 5).reshape(B * M, D, Lq, L, P)


class MSDeformAttn(nn.Module):
    def __init__(self, d_model=256, n_levels=4, n_heads=8, n_points=4):
        super().__init__()
        if d_model % n_heads != 0:
            raise ValueError('d_model must be divisible by n_heads, but got {} and {}'.format(d_model, n_heads))
        if not _is_power_of_2(d_model // n_heads):
            warnings.warn("You'd better set d_model in MSDeformAttn to make the dimension of each attention "
                          "head a power of 2 which is more efficient in our CUDA implementation.")
        self.im2col_step = 64
        self.d_model = d_model
        self.n_levels = n_levels
        self.n_heads = n_heads
        self.n_points = n_points
        self.sampling_offsets = Linear(d_model, n_heads * n_levels * n_points)
        self.attention_weights = Linear(d_model, n_heads * n_levels * n_points)
        self.value_proj = Linear(d_model, d_model)
        self.output_proj = Linear(d_model, d_model)
        self._reset_parameters()

    def _reset_parameters(self):
        constant_(self.sampling_offsets.weight.data, 0.)
        thetas = torch.arange(self.n_heads, dtype=torch.float32) * (2 * math.pi / self.n_heads)
        grid_init = torch.stack([thetas.cos(), thetas.sin()], -1)
        grid_init = (grid_init / grid_init.abs().max(-1, keepdim=True)[0]).view(self.n_heads, 1, 1, 2)
        grid_init = grid_init[..., 0].repeat(1, self.n_levels, self.n_points)
        for i in range(self.n_points):
            grid_init[:, :, i] *= i + 1
        with torch.no_grad():
            self.sampling_offsets.bias = nn.Parameter(grid_init.view(-1))
        constant_(self.attention_weights.weight.data, 0.)
        constant_(self.attention_weights.bias.data, 0.)
        xavier_uniform_(self.value_proj.weight.data)
        constant_(self.value_proj.bias.data, 0.)
        xavier_uniform_(self.output_proj.weight.data)
        constant_(self.output_proj.bias.data, 0.)

    def _locations(self, query, reference_points, input_flatten, input_spatial_shapes, input_padding_mask):
        N, Len_q, _ = query.shape
        N, Len_in, _ = input_flatten.shape
        shapes, _ = _msda.host_levels(input_spatial_shapes)
        assert sum(shapes) == Len_in
        value = self.value_proj(input_flatten)
        if input_padding_mask is not None:
            value = value.masked_fill(input_padding_mask[..., None], float(0))
        value = value.view(N, Len_in, self.n_heads, self.d_model // self.n_heads)
        off = self.sampling_offsets(query).view(N, Len_q, self.n_heads, self.n_levels, self.n_points)
        aw = self.attention_weights(query).view(N, Len_q, self.n_heads, self.n_levels * self.n_points)
        aw = F.softmax(aw, -1).view(N, Len_q, self.n_heads, self.n_levels, self.n_points)
        if reference_points.shape[-1] == 1:
            norm = input_spatial_shapes if isinstance(input_spatial_shapes, torch.Tensor) else \
                torch.as_tensor(shapes, dtype=torch.long, device=query.device)
            loc = reference_points[:, :, None, :, None, 0] + off / norm.reshape(-1)[None, None, None, :, None]
        elif reference_points.shape[-1] == 2:
            loc = reference_points[:, :, None, :, None, 0] \
                + off / self.n_points * reference_points[:, :, None, :, None, 1] * 0.5
        else:
            raise ValueError(
                'Last dim of reference_points must be 1 or 2, but get {} instead.'.format(reference_points.shape[-1]))
        # 1-D -> 2-D lift (H = 1, W = T_l; y = 0.5), reference ms_deform_attn.py:114-117
        loc = torch.stack((loc, 0.5 * loc.new_ones(loc.shape)), -1)
        shapes2d = torch.as_tensor([[1, t] for t in shapes], dtype=torch.long, device=query.device)
        shapes2d._mfl_host = tuple(shapes)  # read by msda.host_levels instead of the device tensor
        return value, shapes2d, loc, aw

    def forward(self, query, reference_points, input_flatten, input_spatial_shapes, input_level_start_index,
                input_padding_mask=None):
        value, shapes2d, loc, aw = self._locations(query, reference_points, input_flatten, input_spatial_shapes,
                                                   input_padding_mask)
        output = MSDeformAttnFunction.apply(value, shapes2d, input_level_start_index, loc, aw, self.im2col_step)
        return self.output_proj(output)


class MSDeformAttnCap(MSDeformAttn):
    """reference ms_deform_attn_for_caption.py: returns the per-sample values
    (``return_value=True`` of the 2-D border core) instead of the weighted sum.

    Differs from ``MSDeformAttn`` as the reference does: the offset / weight projections read
    2*d_model queries (:54-55) and the offset grid is centred over the points (:67)."""

    def __init__(self, d_model=256, n_levels=4, n_heads=8, n_points=4):
        nn.Module.__init__(self)
        if d_model % n_heads != 0:
            raise ValueError('d_model must be divisible by n_heads, but got {} and {}'.format(d_model, n_heads))
        if not _is_power_of_2(d_model // n_heads):
            warnings.warn("You'd better set d_model in MSDeformAttn to make the dimension of each attention "
                          "head a power of 2 which is more efficient in our CUDA implementation.")
        self.im2col_step = 64
        self.d_model = d_model
        self.n_levels = n_levels
        self.n_heads = n_heads
        self.n_points = n_points
        self.sampling_offsets = Linear(2 * d_model, n_heads * n_levels * n_points)
        self.attention_weights = Linear(2 * d_model, n_heads * n_levels * n_points)
        self.value_proj = Linear(d_model, d_model)
        self.output_proj = Linear(d_model, d_model)
        self._reset_parameters()

    def _reset_parameters(self):
        super()._reset_parameters()
        with torch.no_grad():
            grid = self.sampling_offsets.bias.view(self.n_heads, self.n_levels, self.n_points)
            grid.sub_(grid.mean(2, keepdim=True))

    def forward(self, query, reference_points, input_flatten, input_spatial_shapes, input_level_start_index,
                input_padding_mask=None):
        value, shapes2d, loc, aw = self._locations(query, reference_points, input_flatten, input_spatial_shapes,
                                                   input_padding_mask)
        return ms_deform_attn_core_pytorch(value, shapes2d, loc, aw, return_value=True)
