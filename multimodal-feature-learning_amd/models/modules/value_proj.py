"""The value projections of every decoder layer as ONE batched GEMM each way.

Reference: each decoder layer's cross-attention projects the same encoder memory,
``value = self.value_proj(input_flatten)`` then ``masked_fill(input_padding_mask[..., None], 0)``
(models/modules/attention.py:461-463, called from unimodal_deformable_transformer.py:365 by all
``num_decoder_layers`` layers).  Under bf16 autocast that is, per layer and step: a cast of the
fp32 memory, a (B*S x d) x (d x d) GEMM and a masked fill; in the backward a dgrad GEMM, a cast of
its bf16 result to fp32, an fp32 add into the memory gradient, a weight-gradient GEMM and a bias
column sum.  With d = 512 and B*S = 15,360 tokens each of those GEMMs is too small for 256 CUs.

``layer_values`` computes all n layers' values at once (same numbers, one bf16 rounding of the
fp32-accumulated product + bias, as the reference's addmm):
  forward:  Y = [x | 1] @ [W_l^T ; b_l] as one strided-batched GEMM whose A operand (the memory,
            the encoder's carried bf16 copy when there is one) is shared by all n batches, then the
            padding rows zeroed in place (only padding rows written);
  backward: G = [g_1 | ... | g_n] (tokens x n*d, padding rows zeroed), then
            dx = G @ [W_1; ...; W_n]      (one GEMM: the sum over layers inside its K loop),
            dW = G^T @ x                  (one split-K GEMM, fp32), db = column sums of G (fp32).
"""
import torch
from torch.autograd import Function

from .linear import Linear, _accum_group, _bias_grad, _claim_group, _weight_grad

__all__ = ["layer_values", "layer_values_supported", "linear_group", "linear_group_supported"]

_PAD = 16  # [x | 1 | 0 ...]: K padded to a multiple of 16 elements


def _zero_rows(y, nbatch, rows, mask):
    from ... import _native
    lib = _native.load_library()
    rc = lib.mfl_zero_masked_rows_batched(y.data_ptr(), nbatch, rows, y.numel() * y.element_size() // (nbatch * rows),
                                          mask.data_ptr(), _native.stream_handle(y.device))
    if rc != 0:
        raise RuntimeError("mfl_zero_masked_rows_batched failed: " + lib.mfl_relu_dropout_last_error().decode())


class _LayerValues(Function):
    @staticmethod
    def forward(ctx, x, mask, n, *params):
        from ... import _trace
        w, b, wc, bc = params[:n], params[n:2 * n], params[2 * n:3 * n], params[3 * n:4 * n]
        _trace.hit("layer_values_shadow" if all(t is not None for t in wc) else "layer_values")
        dt = torch.bfloat16
        lead = x.shape[:-1]
        c = x.shape[-1]
        x16 = x.reshape(-1, c)
        x16 = x16 if x16.dtype == dt else x16.to(dt)
        k = x16.shape[0]
        wcs = [wc[i] if wc[i] is not None else w[i].to(dt) for i in range(n)]
        bcs = [bc[i] if bc[i] is not None else b[i].to(dt) for i in range(n)]
        c_out = wcs[0].shape[0]
        wcat = torch.cat(wcs, 0)
        if x16.is_cuda and c % 8 == 0 and x16.is_contiguous():
            # [x | 1 | 0 ...] and [W_i^T ; b_i ; 0 ...] in one pass each (include/ffn_glue.h)
            from ... import _native
            lib = _native.load_library()
            x16 = x16.contiguous()
            bcat = torch.cat(bcs, 0)
            x_aug = torch.empty(k, c + _PAD, dtype=dt, device=x.device)
            w_aug = torch.empty(n, c + _PAD, c_out, dtype=dt, device=x.device)
            st = _native.stream_handle(x.device)
            rc = lib.mfl_augment_rows(x16.data_ptr(), k, c, c + _PAD, x_aug.data_ptr(), st)
            rc = rc or lib.mfl_augment_weights(wcat.data_ptr(), bcat.data_ptr(), n, c, c + _PAD, c_out,
                                               w_aug.data_ptr(), st)
            if rc != 0:
                raise RuntimeError("mfl_augment_rows / weights failed: " + lib.mfl_relu_dropout_last_error().decode())
        else:
            x_aug = torch.zeros(k, c + _PAD, dtype=dt, device=x.device)
            x_aug[:, :c] = x16
            x_aug[:, c] = 1
            w_aug = torch.zeros(n, c + _PAD, c_out, dtype=dt, device=x.device)
            w_aug[:, :c] = torch.stack(wcs).transpose(1, 2)
            w_aug[:, c] = torch.stack(bcs)
        y = torch.bmm(x_aug.expand(n, k, c + _PAD), w_aug)  # (n, k, c_out); A shared (batch stride 0)
        if mask is not None:
            _zero_rows(y, n, k, mask)
        ctx.save_for_backward(x16, wcat, mask)
        ctx.n, ctx.x_shape, ctx.x_dtype, ctx.c_out = n, x.shape, x.dtype, c_out
        ctx.params = (w, b)  # (the parameters whose flat gradient views the backward may claim)
        outs = tuple(torch.ops.aten._unsafe_view(y[i], (*lead, c_out)) for i in range(n))
        if x.is_cuda:
            # the backward's G = [g_1 | ... | g_n]: each layer's value gradient may be written straight
            # into its column block (the MSDA backward's strided grad_value, msda_hip_backward_ex)
            # instead of stacked afterwards (a (tokens x n d) copy)
            G = torch.empty(k, n * c_out, dtype=dt, device=x.device)
            slots = G.view(k, n, c_out)
            for i, o in enumerate(outs):
                o._mfl_grad_dest = slots[:, i].view(*lead, c_out)
            ctx.G = G
        else:
            ctx.G = None
        return outs

    @staticmethod
    def backward(ctx, *gs):
        x16, wcat, mask = ctx.saved_tensors
        n, c_out = ctx.n, ctx.c_out
        k = x16.shape[0]
        G, ctx.G = ctx.G, None
        if G is not None and all(gi is not None and gi.dtype == G.dtype and gi.data_ptr() == G.data_ptr() + i * c_out *
                                 G.element_size() and gi.reshape(k, c_out).stride() == (n * c_out, 1)
                                 for i, gi in enumerate(gs)):
            from ... import _trace
            _trace.hit("layer_values_slots")
            g = G  # every layer's gradient already in its column block
        else:
            g = torch.stack([gi.reshape(k, c_out).to(wcat.dtype) if gi is not None
                             else x16.new_zeros(k, c_out) for gi in gs], dim=1).view(k, n * c_out)
        if mask is not None:
            _zero_rows(g, 1, k, mask)
        nig = ctx.needs_input_grad
        dx = torch.mm(g, wcat).view(ctx.x_shape).to(ctx.x_dtype) if nig[0] else None
        dws = dbs = (None,) * n
        ws, bs = ctx.params
        # the n layers' weights (biases) back to back in the trainer's flat gradient buffer
        # (flat_groups): the split-K sum (column sums) written straight into that one view
        # (the same layers used again in this backward: added into the view an earlier call claimed)
        if any(nig[3:3 + n]):
            acc = _accum_group(ws) if all(nig[3:3 + n]) else None
            if acc is not None:
                _weight_grad(g, x16, acc, accumulate=True)
            else:
                dw = _weight_grad(g, x16, _claim_group(ws) if all(nig[3:3 + n]) else None)
                dws = tuple(dw[i * c_out:(i + 1) * c_out] for i in range(n))
        if any(nig[3 + n:3 + 2 * n]):
            acc = _accum_group(bs) if all(nig[3 + n:3 + 2 * n]) else None
            if acc is not None:
                _bias_grad(g, acc, accumulate=True)
            else:
                db = _bias_grad(g, _claim_group(bs) if all(nig[3 + n:3 + 2 * n]) else None)
                dbs = tuple(db[i * c_out:(i + 1) * c_out] for i in range(n))
        return (dx, None, None) + dws + dbs + (None,) * (2 * n)


def layer_values_supported(attns, src, mask):
    """Whether ``layer_values`` takes these MSDeformAttn modules' value projections of ``src``."""
    if len(attns) < 2 or not (src.is_cuda and torch.is_autocast_enabled("cuda")
                              and torch.get_autocast_dtype("cuda") == torch.bfloat16):
        return False
    p0 = attns[0].value_proj
    for a in attns:
        vp = getattr(a, "value_proj", None)
        if (not isinstance(vp, Linear) or vp.bias is None or vp.weight.dtype != torch.float32
                or vp.weight.device != src.device
                or vp.weight.shape != p0.weight.shape):
            return False
    if src.shape[-1] != p0.weight.shape[1] or src.numel() == 0 or src.dtype not in (torch.float32, torch.bfloat16):
        return False
    if (p0.weight.shape[0] * 2) % 16:
        return False
    if mask is not None and (mask.dtype != torch.bool or mask.shape != src.shape[:-1] or not mask.is_contiguous()):
        return False
    return True


def layer_values(attns, src, mask=None):
    """``[a.value_proj(src).masked_fill(mask[..., None], 0) for a in attns]`` under bf16 autocast,
    as one batched GEMM each way (see the module docstring).  ``src`` may carry its bf16 copy as
    ``src._mfl_bf16`` (the encoder's last fused add + LayerNorm writes it); the projection then
    reads that copy and its gradient flows to it."""
    n = len(attns)
    x = getattr(src, "_mfl_bf16", None)
    if x is None or x.shape != src.shape or x.dtype != torch.bfloat16:
        x = src
    ws = [a.value_proj.weight for a in attns]
    bs = [a.value_proj.bias for a in attns]
    low = [a.value_proj._low(torch.bfloat16) for a in attns]
    with torch.autocast("cuda", enabled=False):
        return _LayerValues.apply(x.contiguous(), mask, n, *ws, *bs, *[lw[0] for lw in low], *[lw[1] for lw in low])


class _Holder:
    """Presents a Linear as an object with ``value_proj`` (the interface layer_values reads)."""

    def __init__(self, linear):
        self.value_proj = linear


def linear_group_supported(linears, x):
    """Whether ``linear_group`` takes these Linear layers (same shape, biases) on input x
    (MFL_LINEAR_GROUP=0: never, for A/B runs)."""
    import os
    if os.environ.get("MFL_LINEAR_GROUP", "1") == "0":
        return False
    return len(linears) >= 2 and layer_values_supported([_Holder(lin) for lin in linears], x, None)


def linear_group(linears, x):
    """``[lin(x) for lin in linears]`` under bf16 autocast as one batched GEMM each way (the
    _LayerValues GEMMs without a mask): the caption decoder's 2 x depth cross-attention key / value
    projections of the clip memory, and each self-attention's q / k / v projections of the same
    rows.  The input gradient is one K-concatenated GEMM (the sum over the layers inside its K
    loop: no fp32 gradient adds), the weight gradients one split-K GEMM."""
    return layer_values([_Holder(lin) for lin in linears], x, None)
