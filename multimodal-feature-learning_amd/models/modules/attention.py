"""MSDA interface of the reference's ``models/modules/attention.py``, backed by the HIP kernel.

Drop-in for the three MSDA symbols the reference's transformers import
(``from ..modules.attention import MSDeformAttn`` — reference
models/deformable/unimodal_deformable_transformer.py:10 and friends):

* ``ms_deform_attn_core_pytorch``  — reference attention.py:331-383 (live core).
  Same signature and result; computed by ``msda_hip_forward`` / ``msda_hip_backward``
  in border mode instead of per-level ``F.grid_sample``.
* ``MSDeformAttnFunction``          — reference attention.py:310-328 (dormant call
  into the CUDA extension).  Same ``apply`` signature; zero-padding semantics of the
  extension kernel (ms_deform_im2col_cuda.cuh:34-85).
* ``MSDeformAttn``                  — reference attention.py:394-511.  Same constructor,
  parameter names / init and forward signature, including ``is_sparse``.
* ``CrossAttention``                — reference attention.py:213-306 (caption decoder).

There is no CPU path (see ``msda.py``).
"""
import math
import warnings

import torch
import torch.nn.functional as F
from torch import nn
from torch.autograd.function import once_differentiable
from torch.nn.init import constant_, xavier_uniform_

from ... import msda as _msda
from ...utils.preds_postprocess import SegmentMemory
from .seg_attention import segment_attention, segment_key_mask
from .value_proj import linear_group, linear_group_supported
from ..ops.functions.ms_deform_attn_func import MSDeformAttnFunction  # reference attention.py:310-328
from ..ops.modules.ms_deform_attn import stack_sampled_values
from .linear import (Linear, _AutocastLinear, _accum_group, _addmm, _bias_grad, _claim_group, _defer, _mm_nn,
                     _weight_grad, grad_sum_mm, grad_sum_tagged, linear_pair)

__all__ = ["MSDeformAttnFunction", "ms_deform_attn_core_pytorch", "MSDeformAttn", "CrossAttention",
           "masked_scores_softmax", "mask_padding_rows", "mha_self_attention", "joint_supported"]


def _loc5(sampling_locations):
    """(B,Lq,M,L,P) or the live module's (B,Lq,M,L,P,1) form -> (B,Lq,M,L,P)."""
    if sampling_locations.dim() == 6 and sampling_locations.shape[-1] == 1:
        return sampling_locations[..., 0]
    if sampling_locations.dim() == 5:
        return sampling_locations
    raise ValueError(f"sampling_locations must be (B,Lq,M,L,P[,1]); got {tuple(sampling_locations.shape)}")


def ms_deform_attn_core_pytorch(value, value_temporal_shapes, sampling_locations, attention_weights,
                                return_value=False):
    """Live MSDA core, reference attention.py:331-383 (border padding, align_corners=False).

    :param value (batch_size, sum of tokens over levels, n_heads, d_model/n_heads)
    :param value_temporal_shapes (n_levels,) or (n_levels, 1)
    :param sampling_locations (batch_size, Lq, n_heads, n_levels, n_points[, 1])
    :param attention_weights (batch_size, Lq, n_heads, n_levels, n_points)
    :return (batch_size, Lq, n_heads * d_model/n_heads), contiguous
    """
    shapes, starts = _msda.host_levels(value_temporal_shapes)
    loc = _loc5(sampling_locations)
    if return_value:
        # reference attention.py:376-378: per-sample values stacked (B*M, D, Lq, L, P); unused by the models
        return stack_sampled_values(value, shapes, starts, loc, attention_weights, "border")
    return _msda.msda_apply(value, shapes, starts, loc, attention_weights, "border")


def _is_power_of_2(n):
    if (not isinstance(n, int)) or (n < 0):
        raise ValueError("invalid input for _is_power_of_2: {} (type: {})".format(n, type(n)))
    return (n & (n - 1) == 0) and n != 0


def _rows_view(a, b):
    """[a; b] (rows of a, then rows of b) as a view when b's storage follows a's (the trainer lays
    paired parameters out that way, ``MSDeformAttn.flat_groups``), else a copy."""
    if (a.is_contiguous() and b.is_contiguous() and a.dtype == b.dtype and a.shape[1:] == b.shape[1:]
            and a.untyped_storage().data_ptr() == b.untyped_storage().data_ptr()
            and b.storage_offset() == a.storage_offset() + a.numel()):
        return a.new_empty(0).set_(a.untyped_storage(), a.storage_offset(), (a.shape[0] + b.shape[0],) + a.shape[1:])
    return torch.cat((a, b), 0)


class _QueryPrologue(torch.autograd.Function):
    """``sampling_offsets`` and ``attention_weights`` of MSDeformAttn (attention.py:468-470) as ONE
    GEMM into rows of [offsets | logits], and the prologue (softmax + locations, :471-483) reading
    those rows in place (``msda_hip_prologue_forward_ex``).  Backward: the prologue backward writes
    both gradients into one buffer of the same rows, which is the input of ONE dgrad GEMM against
    [W_off; W_aw] and of the weight-gradient product (queued with the short-K layers' when the
    query rows are few).  Against the two-projection form (linear_pair + MSDAPrologueFunction): one
    GEMM instead of two each way and no concatenation of the two gradients.  The arithmetic is the
    same: each output column is its own dot product over the input, in the GEMM's dtype."""

    @staticmethod
    def forward(ctx, x, wa, ba, wb, bb, wca, bca, wcb, bcb, ref, shapes, dims, layout=0):
        from ... import _trace
        _trace.hit("query_prologue")
        B, Lq, M, L, P = dims
        wc, bc = _rows_view(wca, wcb), _rows_view(bca, bcb)
        x2 = x.reshape(-1, x.shape[-1])
        y = _addmm(bc, x2, wc)
        loc, aw = _msda.prologue_forward_rows(y, B, Lq, M, L, P, ref, shapes, layout)
        ctx.save_for_backward(x2, wc, y, aw, ref)
        ctx.shapes, ctx.x_shape, ctx.layout = shapes, x.shape, layout
        ctx.gsum = grad_sum_tagged(x)
        ctx.params = (wa, ba, wb, bb)
        return loc, aw

    @staticmethod
    @once_differentiable
    def backward(ctx, grad_loc, grad_aw):
        x2, wc, y, aw, ref = ctx.saved_tensors
        nig = ctx.needs_input_grad
        g2, g_ref = _msda.prologue_backward_rows(grad_loc, grad_aw, aw, y, ref, ctx.shapes, need_ref=nig[9],
                                                 layout=ctx.layout)
        return _prologue_grads(ctx, nig, g2, x2, wc) + (None, None, None, None, g_ref, None, None, None)


def _prologue_grads(ctx, nig, g2, x2, wc):
    """(gx, g W_off, g b_off, g W_aw, g b_aw) of a query prologue from its [offsets | logits] rows' gradient
    g2: one dgrad GEMM, the weight / bias products queued with the short-K layers' or written into the
    trainer's flat views (_QueryPrologue, _QueryPrologueJoint)."""
    gx = grad_sum_mm(ctx.gsum, x2, g2, wc, ctx.x_shape) if nig[0] else None
    wa, ba, wb, bb = ctx.params
    na = wa.shape[0]
    if all(nig[1:5]) and _defer((g2[:, :na], x2, wa, 0, ba), (g2[:, na:], x2, wb, 0, bb)):
        return (gx, None, None, None, None)
    gwa = gwb = gba = gbb = None
    # [W_off; W_aw] and [b_off; b_aw] lie back to back in the trainer's flat gradient buffer
    # (flat_groups): the products are written straight into those views when they can be claimed
    # (a module called several times in one backward — the multimodal encoder's shared
    # self-attention: a later call adds its products into the view an earlier one claimed)
    if nig[1] or nig[3]:
        acc = _accum_group((wa, wb)) if nig[1] and nig[3] else None
        if acc is not None:
            _weight_grad(g2, x2, acc, accumulate=True)
        else:
            gw = _weight_grad(g2, x2, _claim_group((wa, wb)) if nig[1] and nig[3] else None)
            gwa, gwb = gw[:na], gw[na:]
    if nig[2] or nig[4]:
        acc = _accum_group((ba, bb)) if nig[2] and nig[4] else None
        if acc is not None:
            _bias_grad(g2, acc, accumulate=True)
        else:
            gbias = _bias_grad(g2, _claim_group((ba, bb)) if nig[2] and nig[4] else None)
            gba, gbb = gbias[:na], gbias[na:]
    return (gx, gwa, gba, gwb, gbb)


class _QueryPrologueJoint(torch.autograd.Function):
    """_QueryPrologue over the rows of several MSDA calls of one module at once (the multimodal
    encoder's video and audio streams, MSDeformAttn.forward_joint): ONE [offsets | logits] GEMM over
    all the query rows, then each call's prologue on its row range (its reference points and its value
    pyramid's level shapes); backward: each call's prologue backward into its rows of one gradient
    buffer, ONE dgrad GEMM and one weight / bias product.  ``metas``: per call (q0, q1, B, Lq, shapes,
    layout); ``refs``: the calls' reference points.  Returns loc_0, aw_0, loc_1, aw_1, ..."""

    @staticmethod
    def forward(ctx, x, wa, ba, wb, bb, wca, bca, wcb, bcb, dims, metas, *refs):
        from ... import _trace
        _trace.hit("query_prologue")
        _trace.hit("query_prologue_joint")
        M, L, P = dims
        wc, bc = _rows_view(wca, wcb), _rows_view(bca, bcb)
        x2 = x.reshape(-1, x.shape[-1])
        y = _addmm(bc, x2, wc)
        outs, saved = [], []
        for (q0, q1, B, Lq, shapes, layout), ref in zip(metas, refs):
            loc, aw = _msda.prologue_forward_rows(y[q0:q1], B, Lq, M, L, P, ref, shapes, layout)
            outs += [loc, aw]
            saved.append(aw)
        ctx.save_for_backward(x2, wc, y, *saved, *refs)
        ctx.metas, ctx.x_shape, ctx.n = metas, x.shape, len(metas)
        ctx.gsum = grad_sum_tagged(x)
        ctx.params = (wa, ba, wb, bb)
        return tuple(outs)

    @staticmethod
    @once_differentiable
    def backward(ctx, *grads):
        x2, wc, y = ctx.saved_tensors[:3]
        n = ctx.n
        aws, refs = ctx.saved_tensors[3:3 + n], ctx.saved_tensors[3 + n:]
        nig = ctx.needs_input_grad
        g2 = torch.empty_like(y)
        g_refs = []
        for i, (q0, q1, B, Lq, shapes, layout) in enumerate(ctx.metas):
            _, g_ref = _msda.prologue_backward_rows(grads[2 * i], grads[2 * i + 1], aws[i], y[q0:q1], refs[i], shapes,
                                                    need_ref=nig[11 + i], layout=layout, g2_out=g2[q0:q1])
            g_refs.append(g_ref)
        return _prologue_grads(ctx, nig, g2, x2, wc) + (None,) * 6 + tuple(g_refs)


class _JointMSDA(torch.autograd.Function):
    """Several MSDA calls on row ranges of ONE projected value (B rows first within each range) writing
    row ranges of ONE output (MSDeformAttn.forward_joint): the calls' value ranges cover the value rows
    once, so the backward writes every row of one grad_value (each call its range, no adds).  ``metas``:
    per call (q0, q1, v0, v1, B, Lq, S, shapes, starts, layout); ``coords``: loc_0, aw_0, loc_1, aw_1, ..."""

    @staticmethod
    def forward(ctx, value, heads, n_rows, metas, *coords):
        from ... import _trace
        M, Dh = heads
        out = torch.empty((n_rows, M * Dh), dtype=value.dtype, device=value.device)
        tiles = []
        for i, (q0, q1, v0, v1, B, Lq, S, shapes, starts, layout) in enumerate(metas):
            _trace.hit("msda_" + str(value.dtype).replace("torch.", ""))
            if layout == _msda.LEVEL_MAJOR:
                _trace.hit("msda_level_major")
            _, t = _msda.msda_forward(value[v0:v1].view(B, S, M, Dh), shapes, starts, coords[2 * i], coords[2 * i + 1],
                                      "border", want_tiles=True, layout=layout, out=out[q0:q1].view(B, Lq, M * Dh))
            tiles.append(t)
        _trace.hit("msda_joint")
        ctx.tiles, ctx.metas, ctx.heads = tiles, metas, heads
        ctx.save_for_backward(value, *coords)
        return out

    @staticmethod
    @once_differentiable
    def backward(ctx, grad_out):
        value, *coords = ctx.saved_tensors
        M, Dh = ctx.heads
        nig = ctx.needs_input_grad
        gv = torch.empty_like(value) if nig[0] else None
        grads = []
        for i, (q0, q1, v0, v1, B, Lq, S, shapes, starts, layout) in enumerate(ctx.metas):
            vi = value[v0:v1].view(B, S, M, Dh)
            _, gl, ga = _msda.msda_backward(vi, shapes, starts, coords[2 * i], coords[2 * i + 1],
                                            grad_out[q0:q1].view(B, Lq, M * Dh), "border", need_value=nig[0],
                                            need_loc=nig[4 + 2 * i], need_aw=nig[5 + 2 * i], tiles=ctx.tiles[i],
                                            layout=layout, gv_out=None if gv is None else gv[v0:v1].view(vi.shape))
            grads += [gl, ga]
        ctx.tiles = None
        if gv is not None:
            gv._mfl_private = True  # fresh, referenced by nothing else (attention.private_grad)
        return (gv, None, None, None) + tuple(grads)


class MSDeformAttn(nn.Module):
    """Multi-scale temporal deformable attention, reference attention.py:394-511.

    Parameters, their names (``sampling_offsets``, ``attention_weights``,
    ``value_proj``, ``output_proj``) and their initialisation follow the reference
    (attention.py:426-442: xavier attention weights, not the ops module's zero init),
    so reference state_dicts load unchanged.
    """

    def __init__(self, d_model=256, n_levels=4, n_heads=8, n_points=4):
        super().__init__()
        if d_model % n_heads != 0:
            raise ValueError('d_model must be divisible by n_heads, but got {} and {}'.format(d_model, n_heads))
        _d_per_head = d_model // n_heads
        if not _is_power_of_2(_d_per_head):
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

    def flat_groups(self):
        """Parameters a flat-buffer trainer should lay out back to back (train_step.py): the two
        query projections' weights and biases, so that [W_off; W_aw] is a view (_QueryPrologue)."""
        return [(self.sampling_offsets.weight, self.attention_weights.weight),
                (self.sampling_offsets.bias, self.attention_weights.bias)]

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
        xavier_uniform_(self.attention_weights.weight.data)
        constant_(self.attention_weights.bias.data, 0.)
        xavier_uniform_(self.value_proj.weight.data)
        constant_(self.value_proj.bias.data, 0.)
        xavier_uniform_(self.output_proj.weight.data)
        constant_(self.output_proj.bias.data, 0.)

    def forward_joint(self, query, value_in, padding_mask, calls):
        """Several calls of this module on joint row tensors (``_forward_joint``)."""
        return _forward_joint(self, query, value_in, padding_mask, calls)

    def forward(self, query, reference_points, input_flatten, input_spatial_shapes,
                input_level_start_index, input_padding_mask=None, is_sparse=False, value=None):
        """
        :param query                   (N, Len_q, C)
        :param reference_points        (N, Len_q, n_levels, 1) in [0, 1], or (N, Len_q, n_levels, 2) (centre, length)
        :param input_flatten           (N, sum_l T_l, C)
        :param input_spatial_shapes    (n_levels,) [T_0, ..., T_{L-1}]
        :param input_level_start_index (n_levels,)
        :param input_padding_mask      (N, sum_l T_l) bool, True = padding
        :param value                   optional (N, sum_l T_l, C): this module's projected, padding-masked
                                       value, already computed (the decoder computes every layer's at once,
                                       models/modules/value_proj.py); input_flatten is then not projected
        :return output (N, Len_q, C)  [, sampling_locations (N,Len_q,M,L,P,1), attention_weights (N,Len_q,M,L,P)]
        """
        N, Len_q, _ = query.shape
        N, Len_in, _ = input_flatten.shape
        shapes, starts = _msda.host_levels(input_spatial_shapes, input_level_start_index)
        assert sum(shapes) == Len_in  # attention.py:458, without the device sync

        if value is None:
            value = self.value_proj(input_flatten)
            if input_padding_mask is not None:
                value = mask_padding_rows(value, input_padding_mask)
        dest = getattr(value, "_mfl_grad_dest", None)  # (value_proj.layer_values' gradient slot)
        if dest is not None:  # one consumer per slot: a second call on the same value writes its own
            if getattr(value, "_mfl_grad_dest_taken", False):
                dest = None
            else:
                value._mfl_grad_dest_taken = True
        value = value.view(N, Len_in, self.n_heads, self.d_model // self.n_heads)
        if dest is not None:
            value._mfl_grad_dest = dest.view(value.shape)

        a, b = self.sampling_offsets, self.attention_weights
        dt = a._autocast_dtype(query) if isinstance(a, Linear) else None
        if (dt == torch.bfloat16 and isinstance(b, Linear) and a.bias is not None and b.bias is not None
                and reference_points.shape[-1] in (1, 2)
                and _msda.prologue_supported(self.n_heads, self.n_levels, self.n_points)):
            # both query projections as one GEMM read in place by the prologue kernel, one
            # backward GEMM each way (_QueryPrologue)
            wca, bca = a._low(dt)
            wcb, bcb = b._low(dt)
            if wca is None or wcb is None:
                wca, bca, wcb, bcb = a.weight.to(dt), a.bias.to(dt), b.weight.to(dt), b.bias.to(dt)
            # the coordinates stay level-major between the prologue, the MSDA kernels and their
            # backward (whole 128-B lines per row block, include/msda_hip.h MSDA_COORD_LEVEL_MAJOR)
            # where the call takes the row-block backward; the is_sparse returns keep the
            # reference layout
            layout = (_msda.LEVEL_MAJOR if not is_sparse and torch.is_grad_enabled()
                      and _msda.level_major_ok(value, shapes, Len_q, self.n_points) else 0)
            with torch.autocast("cuda", enabled=False):
                sampling_locations, attention_weights = _QueryPrologue.apply(
                    query.to(dt), a.weight, a.bias, b.weight, b.bias, wca, bca, wcb, bcb,
                    reference_points.float().contiguous(), tuple(int(t) for t in shapes),
                    (N, Len_q, self.n_heads, self.n_levels, self.n_points), layout)
            if layout:
                output = _msda.msda_apply(value, shapes, starts, sampling_locations, attention_weights, "border",
                                          layout=layout)
            else:
                output = ms_deform_attn_core_pytorch(value, shapes, sampling_locations, attention_weights)
            output = self.output_proj(output)
            if is_sparse:
                return output, sampling_locations.unsqueeze(-1), attention_weights
            return output

        # one input cast and one fused backward for the two query projections
        sampling_offsets, attention_weights = linear_pair(query, self.sampling_offsets, self.attention_weights)
        sampling_offsets = sampling_offsets.view(N, Len_q, self.n_heads, self.n_levels, self.n_points)
        attention_weights = attention_weights.view(N, Len_q, self.n_heads, self.n_levels * self.n_points)
        if (query.is_cuda and reference_points.shape[-1] in (1, 2) and reference_points.device == query.device
                and attention_weights.dtype == sampling_offsets.dtype
                and _msda.prologue_supported(self.n_heads, self.n_levels, self.n_points)):
            # softmax + location arithmetic in one HIP kernel each way
            sampling_locations, attention_weights = _msda.msda_prologue_apply(
                sampling_offsets, attention_weights, reference_points, shapes)
            output = ms_deform_attn_core_pytorch(value, shapes, sampling_locations, attention_weights)
            output = self.output_proj(output)
            if is_sparse:
                return output, sampling_locations.unsqueeze(-1), attention_weights
            return output
        attention_weights = F.softmax(attention_weights, -1).view(N, Len_q, self.n_heads, self.n_levels, self.n_points)

        if reference_points.shape[-1] == 1:
            normalizer = _shape_tensor(input_spatial_shapes, shapes, query.device)
            sampling_locations = reference_points[:, :, None, :, None, 0] \
                + sampling_offsets / normalizer[None, None, None, :, None]
        elif reference_points.shape[-1] == 2:
            sampling_locations = reference_points[:, :, None, :, None, 0] \
                + sampling_offsets / self.n_points * reference_points[:, :, None, :, None, 1] * 0.5
        else:
            raise ValueError(
                'Last dim of reference_points must be 1 or 2, but get {} instead.'.format(reference_points.shape[-1]))

        # host-side T_l tuple: no (L,1) device tensor, no .split() sync (attention.py:346,495)
        output = ms_deform_attn_core_pytorch(value, shapes, sampling_locations, attention_weights)
        output = self.output_proj(output)
        if is_sparse:
            return output, sampling_locations.unsqueeze(-1), attention_weights
        return output


def joint_supported(attn, query, value_in):
    """Whether MSDeformAttn.forward_joint runs fused for these joint rows (bf16 autocast on the GPU, the
    bf16 query prologue, D = d / M)."""
    a, b = attn.sampling_offsets, attn.attention_weights
    return (query.is_cuda and value_in.is_cuda and query.dim() == 2 and value_in.dim() == 2
            and isinstance(a, Linear) and isinstance(b, Linear) and a.bias is not None and b.bias is not None
            and a._autocast_dtype(query) == torch.bfloat16
            and _msda.prologue_supported(attn.n_heads, attn.n_levels, attn.n_points))


def _forward_joint(self, query, value_in, padding_mask, calls):
    """Several calls of this module at once, on ONE tensor of query rows and ONE tensor of value-input
    rows (the multimodal encoder's video and audio streams, models/deformable/multimodal_deformable_
    transformer.py): ``value_proj`` and the masking once over all the value rows, the two query
    projections as one GEMM over all the query rows (_QueryPrologueJoint), each call's MSDA on its row
    ranges into one output (_JointMSDA), ``output_proj`` once.  The same arithmetic as one ``forward``
    per call (reference attention.py:446-511; each GEMM output element is its own dot product).

    query (Rq, C) bf16 rows, value_in (Rv, C) rows, padding_mask (Rv,) bool or None; ``calls``: per call
    (q0, q1, v0, v1, B, reference_points (B, Lq, L, 1|2), level shapes, level starts) — query rows
    [q0, q1) = B x Lq, value rows [v0, v1) = B x sum(shapes), the value ranges covering [0, Rv) once."""
    M, L, P = self.n_heads, self.n_levels, self.n_points
    Dh = self.d_model // M
    value = self.value_proj(value_in)
    if padding_mask is not None:
        value = mask_padding_rows(value, padding_mask)
    cover = sorted((c[2], c[3]) for c in calls)
    if cover[0][0] != 0 or cover[-1][1] != value.shape[0] or any(x[1] != y[0] for x, y in zip(cover, cover[1:])):
        raise ValueError("MSDeformAttn.forward_joint: the calls' value ranges must cover the value rows once")
    a, b = self.sampling_offsets, self.attention_weights
    dt = torch.bfloat16
    wca, bca = a._low(dt)
    wcb, bcb = b._low(dt)
    if wca is None or wcb is None:
        wca, bca, wcb, bcb = a.weight.to(dt), a.bias.to(dt), b.weight.to(dt), b.bias.to(dt)
    pmetas, mmetas, refs = [], [], []
    for q0, q1, v0, v1, B, ref, shapes, starts in calls:
        shapes = tuple(int(t) for t in shapes)
        starts = tuple(int(t) for t in starts)
        Lq, S = (q1 - q0) // B, (v1 - v0) // B
        layout = (_msda.LEVEL_MAJOR if torch.is_grad_enabled()
                  and _msda.level_major_ok(value[v0:v1].view(B, S, M, Dh), shapes, Lq, P) else 0)
        pmetas.append((q0, q1, B, Lq, shapes, layout))
        mmetas.append((q0, q1, v0, v1, B, Lq, S, shapes, starts, layout))
        refs.append(ref.float().contiguous())
    with torch.autocast("cuda", enabled=False):
        coords = _QueryPrologueJoint.apply(query.to(dt), a.weight, a.bias, b.weight, b.bias, wca, bca, wcb, bcb,
                                           (M, L, P), tuple(pmetas), *refs)
        out = _JointMSDA.apply(value.contiguous(), (M, Dh), query.shape[0], tuple(mmetas), *coords)
    return self.output_proj(out)


def private_grad(grad):
    """Whether ``grad`` (or the tensor it views) is a gradient the MSDA backward just allocated and
    nothing else references (msda.MSDAFunction tags it): a second consumer of the value gives a
    fresh sum instead, so only then may the gradient be written in place."""
    base = grad if grad._base is None else grad._base
    return base._base is None and getattr(base, "_mfl_private", False) and grad.is_contiguous()


class _ZeroPaddingRows(torch.autograd.Function):
    """In-place ``value.masked_fill_(mask[..., None], 0)`` through ``mfl_zero_masked_rows``: only
    padding rows are written (an all-valid batch reads the mask and nothing else); the backward
    zeroes the same rows of the incoming gradient in place when the MSDA backward produced it and
    nothing else holds it (``private_grad``), else out of place (``masked_fill``).  A hook on the
    masked value that keeps the gradient it is given sees the zeroed rows (not supported)."""

    @staticmethod
    def forward(ctx, value, mask):
        from ... import _trace
        _trace.hit("zero_rows")
        _zero_rows(value, mask)
        ctx.mark_dirty(value)
        ctx.save_for_backward(mask)
        return value

    @staticmethod
    def backward(ctx, grad):
        (mask,) = ctx.saved_tensors
        if not private_grad(grad):
            return grad.masked_fill(mask[..., None], 0), None
        _zero_rows(grad, mask)
        return grad, None


def _zero_rows(x, mask):
    from ... import _native
    lib = _native.load_library()
    rows = mask.numel()
    rc = lib.mfl_zero_masked_rows(x.data_ptr(), rows, x.numel() * x.element_size() // max(rows, 1),
                                  mask.data_ptr(), _native.stream_handle(x.device))
    if rc != 0:
        raise RuntimeError("mfl_zero_masked_rows failed: " + lib.mfl_relu_dropout_last_error().decode())


def mask_padding_rows(value, mask):
    """``value.masked_fill(mask[..., None], 0)`` for value (N, Len_in, C) and a bool mask (N, Len_in)
    (reference attention.py:462-463).  On the GPU, for a contiguous value whose rows are a multiple
    of 16 bytes, the fill is done in place on the value projection's fresh output (the projection
    keeps its input, not its output, for the backward)."""
    if (value.is_cuda and value.is_contiguous() and mask.dtype == torch.bool and mask.is_contiguous()
            and mask.device == value.device and mask.shape == value.shape[:-1]
            and (value.shape[-1] * value.element_size()) % 16 == 0 and value.data_ptr() % 16 == 0
            and value.numel() > 0):
        return _ZeroPaddingRows.apply(value, mask)
    return value.masked_fill(mask[..., None], float(0))


def mha_self_attention(mha, tgt, query_pos, query_mask, carried=None):
    """The decoder's query self-attention, batch first:
    ``mha((tgt + pos)^T, (tgt + pos)^T, tgt^T, key_padding_mask=~query_mask)[0]^T`` (reference
    unimodal_deformable_transformer.py:352-353 and the multimodal / sparse decoders) with the
    module's own parameters (``in_proj_weight`` / ``in_proj_bias`` / ``out_proj``, so state_dicts
    are unchanged).  The reference discards the attention weights it asks for, so the product runs
    as one ``F.scaled_dot_product_attention`` (dropout on the attention probabilities as the
    module's) instead of bmm / softmax / dropout / bmm and the sequence-first transposes.
    tgt, query_pos (B, L, E); query_mask (B, L) bool, True = a real query.  ``carried``: optional
    ``(bf16(tgt), bf16(tgt + query_pos))`` written by the previous layer's fused add + LayerNorm (the
    same values this function would cast; their gradients flow back into that kernel)."""
    if (mha.batch_first or not mha._qkv_same_embed_dim or mha.bias_k is not None or mha.add_zero_attn
            or mha.in_proj_bias is None or (query_pos is not None and query_pos.shape != tgt.shape)):
        qk = (tgt if query_pos is None else tgt + query_pos).transpose(0, 1)
        return mha(qk, qk, tgt.transpose(0, 1), key_padding_mask=~query_mask)[0].transpose(0, 1)
    B, L, E = tgt.shape
    H = mha.num_heads
    hd = E // H
    w, b = mha.in_proj_weight, mha.in_proj_bias
    with_pos = (lambda: tgt if query_pos is None else tgt + query_pos)  # noqa: E731 (not built when carried)
    if (tgt.is_cuda and torch.is_autocast_enabled("cuda") and torch.get_autocast_dtype("cuda") == torch.bfloat16
            and w.dtype == torch.float32 and mha.out_proj.bias is not None and w.device == tgt.device):
        # the projections as the autocast Linear's: bf16 weights from the trainer's shadow, fp32
        # weight / bias gradients straight from the GEMMs (no per-use casts, no slice-gradient adds)
        sh = getattr(mha, "_mfl_shadow", None)
        ok = sh is not None and sh[4] == w._version and sh[5] == mha.out_proj.weight._version
        if (carried is not None and carried[0] is not None and carried[1] is not None
                and carried[0].dtype == carried[1].dtype == torch.bfloat16):
            v16, qk16 = carried
        else:
            qk16, v16 = with_pos().to(torch.bfloat16), tgt.to(torch.bfloat16)
        with torch.autocast("cuda", enabled=False):
            qk, v = _InProjection.apply(qk16, v16, w, b, sh[0] if ok else None, sh[1] if ok else None)
            q, k = qk.view(B, L, 2, H, hd).permute(2, 0, 3, 1, 4).unbind(0)
            v = v.view(B, L, H, hd).transpose(1, 2)
            out = F.scaled_dot_product_attention(q, k, v, attn_mask=query_mask[:, None, None, :],
                                                 dropout_p=mha.dropout if mha.training else 0.0)
            return _AutocastLinear.apply(out.transpose(1, 2).reshape(B, L, E), mha.out_proj.weight,
                                         mha.out_proj.bias, sh[2] if ok else None, sh[3] if ok else None)
    qk = F.linear(with_pos(), w[:2 * E], b[:2 * E])
    v = F.linear(tgt, w[2 * E:], b[2 * E:])
    q, k = qk.view(B, L, 2, H, hd).permute(2, 0, 3, 1, 4).unbind(0)
    v = v.view(B, L, H, hd).transpose(1, 2)
    out = F.scaled_dot_product_attention(q, k, v, attn_mask=query_mask[:, None, None, :],
                                         dropout_p=mha.dropout if mha.training else 0.0)
    return F.linear(out.transpose(1, 2).reshape(B, L, E), mha.out_proj.weight, mha.out_proj.bias)


class _InProjection(torch.autograd.Function):
    """(x_qk W_qk^T + b_qk, x_v W_v^T + b_v) with W = in_proj_weight (3E, E) split [q; k | v]: two
    bf16 GEMMs forward; backward two dgrad GEMMs and ONE fp32 (3E, E) weight gradient / (3E,)
    bias gradient (no slice gradients to add)."""

    @staticmethod
    def forward(ctx, x_qk, x_v, w, b, wc, bc):
        from ... import _trace
        _trace.hit("sdpa_self_attn_shadow" if wc is not None else "sdpa_self_attn_cast")
        dt = x_qk.dtype
        wc = w.to(dt) if wc is None else wc
        bc = b.to(dt) if bc is None else bc
        e = w.shape[1]
        a2, v2 = x_qk.reshape(-1, e), x_v.reshape(-1, e)
        qk = _addmm(bc[:2 * e], a2, wc[:2 * e])
        v = _addmm(bc[2 * e:], v2, wc[2 * e:])
        ctx.save_for_backward(a2, v2, wc)
        ctx.shape = x_qk.shape
        ctx.params = (w, b)
        lead = x_qk.shape[:-1]
        return (torch.ops.aten._unsafe_view(qk, (*lead, 2 * e)), torch.ops.aten._unsafe_view(v, (*lead, e)))

    @staticmethod
    def backward(ctx, gqk, gv):
        a2, v2, wc = ctx.saved_tensors
        e = wc.shape[1]
        gqk = gqk.reshape(-1, 2 * e).to(wc.dtype)
        gv = gv.reshape(-1, e).to(wc.dtype)
        nig = ctx.needs_input_grad
        dqk = _mm_nn(gqk, wc[:2 * e]).view(ctx.shape) if nig[0] else None
        dv = _mm_nn(gv, wc[2 * e:]).view(ctx.shape) if nig[1] else None
        w, b = ctx.params  # weight / bias gradients batched with the other short-K layers' (linear.py)
        if nig[2] and nig[3] and _defer((gqk, a2, w, 0, b), (gv, v2, w, 2 * e, b)):
            return dqk, dv, None, None, None, None
        dw = db = None
        if nig[2]:
            dw = torch.cat((_weight_grad(gqk, a2), _weight_grad(gv, v2)), 0)
        if nig[3]:
            db = torch.cat((_bias_grad(gqk), _bias_grad(gv)), 0)
        return dqk, dv, dw, db, None, None


def masked_scores_softmax(scores, masked, scale, neg_fill=-1e20):
    """softmax(scale * scores.masked_fill(masked, neg_fill)) over the last dim — the order of the
    reference's CrossAttention (attention.py:288-294: fill with -1e20, then scale): a fully
    masked row is uniform there, not NaN.  ``neg_fill=-inf`` gives nn.MultiheadAttention's."""
    if masked is not None:
        scores = scores.masked_fill(masked, neg_fill)
    return (scores * scale).softmax(dim=-1)


class CrossAttention(nn.Module):
    """Multi-head attention of the caption decoder, reference attention.py:213-306: separate
    ``q_linear`` / ``k_linear`` / ``v_linear`` (bias = qkv_bias), ``projection_layer``; masks are
    boolean (True = masked) — ``attn_mask`` broadcast against (B, H, Lq, Lk), ``key_padding_mask``
    (B, Lk) — filled with -1e20 before the 1/sqrt(hd) scale.

    The weighted sum runs as one ``F.scaled_dot_product_attention`` (a fused attention kernel on
    the GPU) with the masks folded into an additive bias of -1e20*scale: scores are O(1), so
    ``s*scale + (-1e20*scale)`` rounds to exactly the reference's ``(-1e20)*scale`` and softmax
    sees the same values, including uniform rows where everything is masked."""

    def __init__(self, d_model, num_heads=12, qkv_bias=False, attention_dropout=0., projection_dropout=0.):
        super().__init__()
        self.d_model = d_model
        self.num_heads = num_heads
        self.head_dim = d_model // num_heads
        assert d_model == self.head_dim * num_heads, "The model dimension must be divisible by the number of heads."
        self.scale = self.head_dim ** -0.5
        self.q_linear = Linear(d_model, d_model, bias=qkv_bias)
        self.k_linear = Linear(d_model, d_model, bias=qkv_bias)
        self.v_linear = Linear(d_model, d_model, bias=qkv_bias)
        self.attention_dropout = nn.Dropout(attention_dropout)
        self.projection_layer = Linear(d_model, d_model)

    def _mask(self, attn_mask, key_padding_mask):
        """attn_mask | key_padding_mask (broadcast), built once per pair of mask tensors: the caption
        decoder's layers all pass the step's same two masks, so its later layers reuse the first
        one's (the key holds both tensors' identities and versions)."""
        if key_padding_mask is None:
            return attn_mask
        key = (None if attn_mask is None else attn_mask._version, key_padding_mask._version)
        cached = getattr(key_padding_mask, "_mfl_mask", None)
        if cached is not None and cached[0] == key and cached[2] is attn_mask:  # (the entry holds attn_mask)
            return cached[1]
        kpm = key_padding_mask.unsqueeze(1).unsqueeze(1)
        m = kpm if attn_mask is None else (attn_mask | kpm)
        key_padding_mask._mfl_mask = (key, m, attn_mask)
        return m

    def _sdpa_bias(self, masked, dtype):
        """The additive -1e20*scale bias of a boolean mask for SDPA, once per mask tensor (the caption
        decoder's layers share the step's mask, _mask), its last dimension padded to a multiple of 16
        elements and handed over as a view: the fused kernel's alignment rule then needs no padded
        copy per call."""
        key = (dtype, self.scale, masked._version)
        cached = getattr(masked, "_mfl_sdpa_bias", None)
        if cached is not None and cached[0] == key:
            return cached[1]
        lk = masked.shape[-1]
        full = torch.zeros(masked.shape[:-1] + ((lk + 15) // 16 * 16,), dtype=dtype, device=masked.device)
        bias = full[..., :lk]
        bias.masked_fill_(masked, -1e20 * self.scale)
        masked._mfl_sdpa_bias = (key, bias)
        return bias

    def forward(self, q, k, v, attn_mask=None, key_padding_mask=None, need_weights=False):
        assert k.shape == v.shape, (f"The keys and values inputted to the cross attention module should have the same "
                                    f"shape. However, key has {k.shape} and value has {v.shape}.")
        B, Lq, _ = q.shape
        Lk = k.shape[1]
        H, hd = self.num_heads, self.head_dim
        segments = isinstance(k, SegmentMemory)
        key_mask = segment_key_mask(q, k, attn_mask, key_padding_mask, H) if segments and v is k else False
        if key_mask is not False and not need_weights:
            # the DVC caption decoder's cross-attention into the matched segments: HIP kernels that
            # read each segment's projected rows in place (models/modules/seg_attention.py)
            out = segment_attention(self.q_linear(q), k, v, self.k_linear, self.v_linear, key_mask, H, self.scale,
                                    self.attention_dropout)
            return self.projection_layer(out), None
        if q is k and k is v and not segments and linear_group_supported(
                (self.q_linear, self.k_linear, self.v_linear), q):
            # self-attention: the three projections of the same rows as one GEMM each way
            q, k, v = (t.reshape(B, Lq, H, hd).transpose(1, 2)
                       for t in linear_group((self.q_linear, self.k_linear, self.v_linear), q))
            masked = self._mask(attn_mask, key_padding_mask)
            return self._attend(q, k, v, masked, need_weights, segments, Lq)
        q = self.q_linear(q).reshape(B, Lq, H, hd).transpose(1, 2)
        if segments:  # the DVC's cropped memory: projections of the clips' rows, gathered
            k = k.project(self.k_linear).reshape(B, Lk, H, hd).transpose(1, 2)
            v = v.project(self.v_linear).reshape(B, Lk, H, hd).transpose(1, 2)
        else:
            k = self.k_linear(k).reshape(B, Lk, H, hd).transpose(1, 2)
            v = self.v_linear(v).reshape(B, Lk, H, hd).transpose(1, 2)
        masked = self._mask(attn_mask, key_padding_mask)
        return self._attend(q, k, v, masked, need_weights, segments, Lq)

    def _attend(self, q, k, v, masked, need_weights, segments, Lq):
        """(projection_layer(softmax(scale q k^T masked) v), weights or None) of head-split q / k / v."""
        # the explicit form (the reference's own, attention.py:288-299) also for the caption
        # decoder's segment cross-attention: ~20 queries over ~2,000 keys, where the fused kernel's
        # backward took 148 us a call against tens for two small batched GEMMs and a softmax
        if need_weights or (segments and Lq <= 64):
            att = self.attention_dropout(masked_scores_softmax(q @ k.transpose(-2, -1), masked, self.scale))
            out = att @ v
        else:
            bias = None
            if masked is not None:
                bias = self._sdpa_bias(masked, q.dtype)
            out = F.scaled_dot_product_attention(q, k, v, attn_mask=bias, scale=self.scale,
                                                 dropout_p=self.attention_dropout.p if self.training else 0.0)
            att = None
        x = self.projection_layer(out.transpose(1, 2).flatten(2))
        return x, att


def _shape_tensor(input_spatial_shapes, shapes, device):
    """The int64 (L,) T_l tensor the reference divides offsets by (attention.py:474-476).

    Dividing by the integer tensor keeps the reference's dtype promotion (bf16 offsets
    under autocast stay bf16)."""
    if isinstance(input_spatial_shapes, torch.Tensor) and input_spatial_shapes.device == device:
        return input_spatial_shapes.reshape(-1)
    return torch.as_tensor(shapes, dtype=torch.long, device=device)
