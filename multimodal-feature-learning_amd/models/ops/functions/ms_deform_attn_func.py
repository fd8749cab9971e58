"""reference models/ops/functions/ms_deform_attn_func.py: the autograd Function over the
native extension, plus the 2-D-form pure core, both on the HIP kernel."""
import torch
from torch.autograd import Function
from torch.autograd.function import once_differentiable

from .... import MultiScaleDeformableAttention as MSDA
from .... import msda as _msda

__all__ = ["MSDeformAttnFunction", "ms_deform_attn_core_pytorch"]


class MSDeformAttnFunction(Function):
    """``apply(value, value_spatial_shapes, value_level_start_index, sampling_locations,
    attention_weights, im2col_step)`` -> (B, Lq, M*D); reference
    ms_deform_attn_func.py:23-41 (and its twin models/modules/attention.py:310-328).
    Backward returns ``(grad_value, None, None, grad_sampling_loc, grad_attn_weight, None)``."""

    @staticmethod
    def forward(ctx, value, value_spatial_shapes, value_level_start_index, sampling_locations,
                attention_weights, im2col_step):
        ctx.im2col_step = im2col_step
        output = MSDA.ms_deform_attn_forward(value, value_spatial_shapes, value_level_start_index,
                                             sampling_locations, attention_weights, ctx.im2col_step)
        ctx.save_for_backward(value, value_spatial_shapes, value_level_start_index, sampling_locations,
                              attention_weights)
        return output

    @staticmethod
    @once_differentiable
    def backward(ctx, grad_output):
        value, shapes, starts, loc, aw = ctx.saved_tensors
        grad_value, grad_loc, grad_aw = MSDA.ms_deform_attn_backward(
            value, shapes, starts, loc, aw, grad_output.contiguous(), ctx.im2col_step,
            need_value=ctx.needs_input_grad[0], need_loc=ctx.needs_input_grad[3],
            need_attn=ctx.needs_input_grad[4])
        return grad_value, None, None, grad_loc, grad_aw, None


def ms_deform_attn_core_pytorch(value, value_spatial_shapes, sampling_locations, attention_weights,
                                return_value=False):
    """2-D-form border core, reference ms_deform_attn_func.py:44-71 (``(L, 2)`` [H, W]
    shapes, ``(…, 2)`` [x, y] locations, grid_sample border / align_corners=False).

    Temporal maps only (H == 1): on a one-row map the border clamp pins y to row 0 with a
    zero y-gradient, so this is the 1-D border kernel along x."""
    shapes, starts = _msda.host_levels(value_spatial_shapes)
    if sampling_locations.dim() != 6 or sampling_locations.shape[-1] != 2:
        raise ValueError("expected (B, Lq, M, L, P, 2) sampling locations")
    x = sampling_locations[..., 0]
    y_dead = sampling_locations[..., 1] * 0  # keeps y in the graph with its (zero) gradient
    if return_value:
        from ..modules.ms_deform_attn import stack_sampled_values
        return stack_sampled_values(value, shapes, starts, x + y_dead, attention_weights, "border")
    return _msda.msda_apply(value, shapes, starts, x + y_dead, attention_weights, "border")
