"""``dropout(relu(h))`` of the deformable transformer FFNs as one HIP kernel each way.

Reference pattern: ``self.dropout2(self.activation(self.linear1(src)))`` of the encoder FFN and
``self.dropout3(self.activation(self.linear1(tgt)))`` of the decoder's
(unimodal_deformable_transformer.py:233-236, 360-362; the multimodal and sparse layers repeat it).
Under bf16 autocast ATen runs a relu, a dropout that also writes a byte mask, and in the backward
a masked scale and relu's threshold_backward, each a full pass over the (tokens x d_ffn) hidden
tensor.  ``relu_dropout`` runs csrc/ffn_glue.hip (include/ffn_glue.h): one pass forward (keep bits
from a device-side seed, as the fused add + LayerNorm's dropout), one pass backward from the
output alone (out > 0 exactly where x > 0 and the element was kept).  Outside autocast, on the
CPU, for non-relu activations or other dtypes it is exactly ``dropout(activation(h))``.
"""
import torch
import torch.nn.functional as F
from torch import nn
from torch.autograd import Function

from .add_norm import _attach_colsum, _drop_args, _ptr

__all__ = ["relu_dropout", "gelu_dropout"]


class _ReluDropout(Function):
    @staticmethod
    def forward(ctx, h, p_drop, seed):
        from ... import _native, _trace
        _trace.hit("relu_dropout")
        lib = _native.load_library()
        out = torch.empty_like(h)
        rc = lib.mfl_relu_dropout_forward(h.data_ptr(), h.numel(), p_drop, _ptr(seed), out.data_ptr(),
                                          _native.stream_handle(h.device))
        if rc != 0:
            raise RuntimeError(lib.mfl_relu_dropout_last_error().decode())
        ctx.p_drop, ctx.dropped = p_drop, seed is not None
        ctx.save_for_backward(out)
        return out

    @staticmethod
    def backward(ctx, dy):
        from ... import _native
        lib = _native.load_library()
        (out,) = ctx.saved_tensors
        dy = dy.to(out.dtype).contiguous()
        dx = torch.empty_like(out)
        cols = out.shape[-1]
        rows = out.numel() // cols if cols else 0
        if cols % 8 == 0 and rows > 0:
            # dx and its column sums in one pass: linear1's bias gradient, handed to it with dx
            # (add_norm._attach_colsum; linear._given_colsum) instead of a column-sum pass over dx
            colsum = torch.empty(cols, dtype=torch.float32, device=out.device)
            ws = torch.empty(lib.mfl_relu_dropout_colsum_workspace_bytes(rows, cols), dtype=torch.uint8,
                             device=out.device)
            rc = lib.mfl_relu_dropout_backward_colsum(dy.data_ptr(), out.data_ptr(), rows, cols, ctx.p_drop,
                                                      int(ctx.dropped), dx.data_ptr(), colsum.data_ptr(), ws.data_ptr(),
                                                      _native.stream_handle(out.device))
        else:
            colsum = None
            rc = lib.mfl_relu_dropout_backward(dy.data_ptr(), out.data_ptr(), out.numel(), ctx.p_drop,
                                               int(ctx.dropped), dx.data_ptr(), _native.stream_handle(out.device))
        if rc != 0:
            raise RuntimeError(lib.mfl_relu_dropout_last_error().decode())
        _attach_colsum(dx, colsum)
        return dx, None, None


def relu_dropout(h, activation, dropout: nn.Dropout):
    """``dropout(activation(h))``; one HIP kernel each way for a bf16 ``h`` on the GPU with
    ``activation`` = ``F.relu`` (see the module docstring)."""
    if (activation is F.relu and h.is_cuda and h.dtype == torch.bfloat16 and h.is_contiguous()
            and h.numel() % 8 == 0 and h.data_ptr() % 16 == 0 and isinstance(dropout, nn.Dropout)):
        p_drop, seed = _drop_args(dropout, h.device)
        return _ReluDropout.apply(h, p_drop, seed)
    return dropout(activation(h))


class _GeluDropout(Function):
    """dropout(gelu(h)) of the caption decoder's MLP (include/ffn_glue.h mfl_gelu_dropout_*): saves h
    and the dropout seed; the backward regenerates the keep bits."""

    @staticmethod
    def forward(ctx, h, p_drop, seed):
        from ... import _native, _trace
        _trace.hit("gelu_dropout")
        lib = _native.load_library()
        out = torch.empty_like(h)
        rc = lib.mfl_gelu_dropout_forward(h.data_ptr(), h.numel(), p_drop, _ptr(seed), out.data_ptr(),
                                          _native.stream_handle(h.device))
        if rc != 0:
            raise RuntimeError(lib.mfl_relu_dropout_last_error().decode())
        ctx.p_drop = p_drop
        ctx.save_for_backward(h, seed)
        return out

    @staticmethod
    def backward(ctx, dy):
        from ... import _native
        lib = _native.load_library()
        h, seed = ctx.saved_tensors
        dy = dy.to(h.dtype).contiguous()
        dx = torch.empty_like(h)
        rc = lib.mfl_gelu_dropout_backward(dy.data_ptr(), h.data_ptr(), h.numel(), ctx.p_drop, _ptr(seed),
                                           dx.data_ptr(), _native.stream_handle(h.device))
        if rc != 0:
            raise RuntimeError(lib.mfl_relu_dropout_last_error().decode())
        return dx, None, None


def gelu_dropout(h, activation, dropout: nn.Dropout):
    """``dropout(activation(h))`` for ``activation`` an exact-erf ``nn.GELU``: one HIP kernel each way
    for a bf16 ``h`` on the GPU (ATen's roundings, keep bits from a device seed); the modules as they
    are elsewhere."""
    if (isinstance(activation, nn.GELU) and activation.approximate == "none" and h.is_cuda
            and h.dtype == torch.bfloat16 and h.is_contiguous() and h.numel() % 8 == 0 and h.data_ptr() % 16 == 0
            and isinstance(dropout, nn.Dropout)):
        p_drop, seed = _drop_args(dropout, h.device)
        return _GeluDropout.apply(h, p_drop, seed)
    return dropout(activation(h))
