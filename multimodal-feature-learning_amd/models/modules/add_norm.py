"""``norm(x + dropout(y))`` of the deformable transformer layers as one HIP kernel each way.

Reference pattern: ``src = self.norm1(src + self.dropout1(src2))`` and the FFN's
``self.norm2(src + self.dropout3(src2))`` (unimodal_deformable_transformer.py:238-249,
362-373; the multimodal and sparse layers repeat it).  Under bf16 autocast that is an fp32 add
of the residual stream and the 16-bit branch, an fp32 LayerNorm, and in the backward
LayerNorm's input and gamma/beta kernels plus a cast of the branch gradient back to 16 bits.
``add_layer_norm`` runs it as csrc/add_layernorm.hip (include/add_layernorm.h): the same fp32
arithmetic (z = r + y in fp32, fp32 statistics), with the branch gradient written directly in
its own dtype.  Outside autocast, on the CPU, or for shapes the kernel does not take
(d % 256 != 0, d > 1024, other dtypes) it is exactly ``norm(r + y)``.
"""
import torch
from torch import nn
from torch.autograd import Function

__all__ = ["add_layer_norm"]

_TAGS = {torch.float32: 0, torch.bfloat16: 2}


class _AddLayerNorm(Function):
    @staticmethod
    def forward(ctx, r, y, weight, bias, eps):
        from ... import _native
        lib = _native.load_library()
        d = r.shape[-1]
        rows = r.numel() // d
        out = torch.empty(r.shape, dtype=torch.float32, device=r.device)
        mean = torch.empty(rows, dtype=torch.float32, device=r.device)
        rstd = torch.empty(rows, dtype=torch.float32, device=r.device)
        rc = lib.mfl_add_layernorm_forward(r.data_ptr(), _TAGS[r.dtype], y.data_ptr(), _TAGS[y.dtype],
                                           weight.data_ptr(), bias.data_ptr(), rows, d, float(eps), out.data_ptr(),
                                           mean.data_ptr(), rstd.data_ptr(), _native.stream_handle(r.device))
        if rc != 0:
            raise RuntimeError(lib.mfl_add_layernorm_last_error().decode())
        ctx.save_for_backward(r, y, weight, mean, rstd)
        return out

    @staticmethod
    def backward(ctx, dout):
        from ... import _native
        lib = _native.load_library()
        r, y, weight, mean, rstd = ctx.saved_tensors
        dout = dout.to(torch.float32).contiguous()
        d = r.shape[-1]
        rows = r.numel() // d
        dr = torch.empty_like(r)
        dy = torch.empty_like(y)
        dw = torch.empty(d, dtype=torch.float32, device=r.device)
        db = torch.empty(d, dtype=torch.float32, device=r.device)
        ws = torch.empty(max(lib.mfl_add_layernorm_workspace_bytes(rows, d), 4), dtype=torch.uint8, device=r.device)
        rc = lib.mfl_add_layernorm_backward(dout.data_ptr(), r.data_ptr(), _TAGS[r.dtype], y.data_ptr(),
                                            _TAGS[y.dtype], weight.data_ptr(), mean.data_ptr(), rstd.data_ptr(), rows,
                                            d, dr.data_ptr(), dy.data_ptr(), dw.data_ptr(), db.data_ptr(),
                                            ws.data_ptr(), _native.stream_handle(r.device))
        if rc != 0:
            raise RuntimeError(lib.mfl_add_layernorm_last_error().decode())
        return dr, dy, dw, db, None


def add_layer_norm(r, y, norm: nn.LayerNorm):
    """``norm(r + y)``; fused on the GPU under autocast (see the module docstring)."""
    d = r.shape[-1]
    if (r.is_cuda and torch.is_autocast_enabled("cuda") and isinstance(norm, nn.LayerNorm)
            and norm.elementwise_affine and norm.bias is not None and tuple(norm.normalized_shape) == (d,)
            and norm.weight.dtype == torch.float32 and r.shape == y.shape and r.dtype in _TAGS
            and y.dtype in _TAGS and d % 256 == 0 and d <= 1024 and r.numel() > 0):
        with torch.autocast("cuda", enabled=False):
            return _AddLayerNorm.apply(r.contiguous(), y.contiguous(), norm.weight, norm.bias, norm.eps)
    return norm(r + y)
