"""Mirror of the reference's pybind extension module ``MultiScaleDeformableAttention``
(models/ops/setup.py:53, models/ops/src/vision.cpp:13-16), backed by libmsda_hip.so.

``ms_deform_attn_forward(value, spatial_shapes, level_start_index, sampling_loc,
attn_weight, im2col_step)`` and ``ms_deform_attn_backward(..., grad_output, im2col_step)``
keep the reference's argument order, layouts and semantics: the extension kernel's
zero padding (ms_deform_im2col_cuda.cuh:34-85, samples with the image coordinate
outside (-1, T) skipped), ``spatial_shapes`` as (L, 2) ``[H, W]`` with sampling
locations (…, 2) ``[x, y]`` — restricted here to H == 1, the temporal lift of
models/ops/modules/ms_deform_attn.py:114-117 — or the native 1-D forms (L,) / (…, 1) /
5-D.  Checks raise ``RuntimeError`` like the reference's ``AT_ASSERTM``
(ms_deform_attn_cuda.cu:28-52); a CPU tensor raises like ``AT_ERROR("Not implemented
on the CPU")`` (ms_deform_attn.h:38).
"""
import torch

from . import msda as _msda

__all__ = ["ms_deform_attn_forward", "ms_deform_attn_backward"]


def _check_like_reference(value, spatial_shapes, level_start_index, sampling_loc, attn_weight, im2col_step,
                          grad_output=None):
    named = [("value", value), ("sampling_loc", sampling_loc), ("attn_weight", attn_weight)]
    if grad_output is not None:
        named.append(("grad_output", grad_output))
    for name, t in named:
        if not t.is_cuda:
            raise RuntimeError("Not implemented on the CPU")
        if not t.is_contiguous():
            raise RuntimeError(f"{name} tensor has to be contiguous")
    batch = int(value.shape[0])
    step = min(batch, int(im2col_step))
    if step <= 0 or batch % step != 0:
        raise RuntimeError(f"batch({batch}) must divide im2col_step({step})")


def _row_weight_h1(y):
    """Weight of row 0 and its y-derivative for a bilinear tap on an H == 1 map with
    zero padding: h = y*1 - 0.5; rows floor(h), floor(h)+1, only row 0 exists."""
    h = y - 0.5
    live = (h > -1) & (h < 1)
    upper = h >= 0                     # row 0 is the low row: weight 1 - (h - 0)
    rw = torch.where(upper, 1 - h, h + 1)
    drw = torch.where(upper, -torch.ones_like(h), torch.ones_like(h))
    zero = torch.zeros_like(h)
    return torch.where(live, rw, zero), torch.where(live, drw, zero)


def split_locations(sampling_loc, attn_weight):
    """Return (x_loc (B,Lq,M,L,P), effective attn weight, row_weight, drow_dy, layout).

    layout: '5d', '6d1' (trailing 1) or '6d2' (2-D [x, y] with H == 1)."""
    if sampling_loc.dim() == 5:
        return sampling_loc, attn_weight, None, None, "5d"
    if sampling_loc.dim() == 6 and sampling_loc.shape[-1] == 1:
        return sampling_loc[..., 0], attn_weight, None, None, "6d1"
    if sampling_loc.dim() == 6 and sampling_loc.shape[-1] == 2:
        x = sampling_loc[..., 0]
        rw, drw = _row_weight_h1(sampling_loc[..., 1])
        return x, attn_weight * rw.to(attn_weight.dtype), rw, drw, "6d2"
    raise ValueError(f"sampling_loc must be (B,Lq,M,L,P[,1|2]); got {tuple(sampling_loc.shape)}")


def _prep(value, spatial_shapes, level_start_index, sampling_loc, attn_weight):
    shapes, starts = _msda.host_levels(spatial_shapes, level_start_index)
    x, aw_eff, rw, drw, layout = split_locations(sampling_loc, attn_weight)
    cd = torch.float64 if value.dtype == torch.float64 else torch.float32
    return shapes, starts, x.to(cd).contiguous(), aw_eff.to(cd).contiguous(), rw, drw, layout


def ms_deform_attn_forward(value, spatial_shapes, level_start_index, sampling_loc, attn_weight, im2col_step):
    """-> output (B, Lq, M*D)  (reference ms_deform_attn_cuda.cu:20-80)"""
    _check_like_reference(value, spatial_shapes, level_start_index, sampling_loc, attn_weight, im2col_step)
    shapes, starts, x, aw_eff, _, _, _ = _prep(value, spatial_shapes, level_start_index, sampling_loc, attn_weight)
    return _msda.msda_forward(value, shapes, starts, x, aw_eff, "zeros")


def ms_deform_attn_backward(value, spatial_shapes, level_start_index, sampling_loc, attn_weight, grad_output,
                            im2col_step, need_value=True, need_loc=True, need_attn=True):
    """-> [grad_value, grad_sampling_loc, grad_attn_weight]  (reference ms_deform_attn_cuda.cu:83-153)

    grad_sampling_loc has the layout of ``sampling_loc``; for the 2-D form its y
    component is height * d(row weight)/dy * attn * sum_c(grad * sample), as the
    extension's col2im computes it (ms_deform_im2col_cuda.cuh:88-160)."""
    _check_like_reference(value, spatial_shapes, level_start_index, sampling_loc, attn_weight, im2col_step,
                          grad_output)
    shapes, starts, x, aw_eff, rw, drw, layout = _prep(value, spatial_shapes, level_start_index, sampling_loc,
                                                       attn_weight)
    need_ga = need_attn or (need_loc and layout == "6d2")
    gv, gx, ga = _msda.msda_backward(value, shapes, starts, x, aw_eff, grad_output, "zeros",
                                     need_value=need_value, need_loc=need_loc, need_aw=need_ga)
    g_attn = None
    if need_attn:
        g_attn = ga if rw is None else ga * rw.to(ga.dtype)
        g_attn = g_attn.to(attn_weight.dtype)
    g_loc = None
    if need_loc:
        if layout == "5d":
            g_loc = gx
        elif layout == "6d1":
            g_loc = gx.unsqueeze(-1)
        else:
            gy = attn_weight.to(ga.dtype) * drw.to(ga.dtype) * ga
            g_loc = torch.stack([gx, gy], -1)
        g_loc = g_loc.to(sampling_loc.dtype)
    return [gv, g_loc, g_attn]
