"""``norm(x + dropout(y))`` of the deformable transformer layers as one HIP kernel each way.

Reference pattern: ``src = self.norm1(src + self.dropout1(src2))`` and the FFN's
``self.norm2(src + self.dropout3(src2))`` (unimodal_deformable_transformer.py:238-249,
362-373; the multimodal and sparse layers repeat it).  Under bf16 autocast that is an fp32 add
of the residual stream and the 16-bit branch, an fp32 LayerNorm, and in the backward
LayerNorm's input and gamma/beta kernels plus a cast of the branch gradient back to 16 bits.
``add_layer_norm`` runs it as csrc/add_layernorm.hip (include/add_layernorm.h): the same
arithmetic (z = r + y in fp32 — rounded to bf16 when both operands are bf16, as autocast's bf16
add is, e.g. the multimodal FFN — and fp32 statistics), with the branch gradient written
directly in its own dtype.  Outside autocast, on the CPU, or for shapes the kernel does not take
(d % 256 != 0, d > 1024, other dtypes) it is exactly ``norm(r + y)``.
"""
import torch
from torch import nn
from torch.autograd import Function

__all__ = ["add_layer_norm", "add_layer_norm_carry", "seed_pool", "pos_sink", "PosGradAcc", "carry_entry"]

_TAGS = {torch.float32: 0, torch.bfloat16: 2}


def _ptr(t):
    return t.data_ptr() if t is not None else None


def _attach_colsum(dy, colsum):
    """Hand the column sums of ``dy`` (as stored) to the Linear layer whose output gradient it is
    (linear.py: its bias gradient, no column-sum pass).  Tagged with dy's version counter: autograd
    adding another gradient into dy in place would make them stale, and the consumer then ignores them."""
    if colsum is not None:
        dy._mfl_colsum = (colsum, dy._version)


class PosGradAcc:
    """The summed gradient of a pos read by several fused add + LayerNorms (the encoder's level
    position embedding, the decoder's query_pos): each backward adds its dq16 into ``buf`` in its
    own kernel (mfl_add_layernorm_backward_ex2, dpos_accumulate), and ``pos_sink``'s node hands the
    sum to autograd once, after all of them (autograd runs a node after every consumer of its output)."""

    def __init__(self):
        self.buf = None


class _PosSink(Function):
    @staticmethod
    def forward(ctx, pos, acc):
        ctx.set_materialize_grads(False)
        ctx.acc = acc
        return pos.view_as(pos)

    @staticmethod
    def backward(ctx, g):
        buf, ctx.acc.buf = ctx.acc.buf, None
        if buf is None:
            return g, None
        if g is not None:  # the other (autograd) consumers' gradient
            buf = buf.add_(g)
        return buf, None


def pos_sink(pos):
    """``(pos', acc)``: give the layers ``pos'`` as their pos and ``acc`` as ``add_layer_norm_carry``'s
    ``pos_acc``; the fused backwards then sum pos's gradient in place instead of autograd adding one
    fp32 tensor per layer (reference: the gradient of ``tensor + pos`` summed over the layers).
    ``(pos, None)`` where the fused path does not run."""
    if (pos is None or not pos.requires_grad or not pos.is_cuda or pos.dtype != torch.float32
            or not torch.is_autocast_enabled("cuda") or torch.get_autocast_dtype("cuda") != torch.bfloat16):
        return pos, None
    acc = PosGradAcc()
    return _PosSink.apply(pos, acc), acc


class _SeedPool:
    """Dropout seeds for one step drawn in blocks: inside ``seed_pool(device)`` (the training step
    opens it around its forward) the fused kernels' seeds are consecutive elements of device
    tensors of ``block`` seeds, each drawn by ONE kernel, instead of one random kernel per dropout
    site (42 a step in the bench's 6 + 6 layers).  The pool starts empty on entry, so every
    seed used inside a captured graph is drawn inside it (fresh on every replay)."""
    active = None

    def __init__(self, device, block=64):
        self.device, self.block, self.buf, self.i = device, block, None, 0

    def take(self):
        if self.buf is None or self.i >= self.block:
            self.buf = torch.randint(0, 2 ** 62, (self.block,), device=self.device, dtype=torch.int64)
            self.i = 0
        self.i += 1
        return self.buf[self.i - 1:self.i]


class seed_pool:  # noqa: N801  (a context manager, used like a function)
    def __init__(self, device, block=64):
        self.pool = _SeedPool(torch.device(device), block)

    def __enter__(self):
        self.prev, _SeedPool.active = _SeedPool.active, self.pool
        return self.pool

    def __exit__(self, *exc):
        _SeedPool.active = self.prev
        return False


def _drop_args(dropout, device):
    """(p, seed tensor) of an active nn.Dropout, else (0.0, None).  The seed is drawn on the device
    from torch's generator (graph-capture safe: a fresh value on every replay; from the step's
    seed pool when one is open) and kept for the backward, which regenerates the keep bits
    from it."""
    if isinstance(dropout, nn.Dropout) and dropout.training and dropout.p > 0:
        pool = _SeedPool.active
        if pool is not None and pool.device == device:
            return float(dropout.p), pool.take()
        return float(dropout.p), torch.randint(0, 2 ** 62, (1,), device=device, dtype=torch.int64)
    return 0.0, None


class _AddLayerNorm(Function):
    @staticmethod
    def forward(ctx, r, y, weight, bias, eps, p_drop, seed):
        from ... import _native, _trace
        _trace.hit("add_ln")
        lib = _native.load_library()
        d = r.shape[-1]
        rows = r.numel() // d
        out = torch.empty(r.shape, dtype=torch.float32, device=r.device)
        mean = torch.empty(rows, dtype=torch.float32, device=r.device)
        rstd = torch.empty(rows, dtype=torch.float32, device=r.device)
        rc = lib.mfl_add_layernorm_forward_ex(r.data_ptr(), _TAGS[r.dtype], y.data_ptr(), _TAGS[y.dtype],
                                              weight.data_ptr(), bias.data_ptr(), rows, d, float(eps), out.data_ptr(),
                                              mean.data_ptr(), rstd.data_ptr(), None, None, None, p_drop, _ptr(seed),
                                              _native.stream_handle(r.device))
        if rc != 0:
            raise RuntimeError(lib.mfl_add_layernorm_last_error().decode())
        ctx.p_drop = p_drop
        ctx.save_for_backward(r, y, weight, mean, rstd, seed)
        return out

    @staticmethod
    def backward(ctx, dout):
        from ... import _native
        lib = _native.load_library()
        r, y, weight, mean, rstd, seed = ctx.saved_tensors
        dout = dout.to(torch.float32).contiguous()
        d = r.shape[-1]
        rows = r.numel() // d
        dr = torch.empty_like(r)
        dy = torch.empty_like(y)
        dw = torch.empty(d, dtype=torch.float32, device=r.device)
        db = torch.empty(d, dtype=torch.float32, device=r.device)
        ws = torch.empty(max(lib.mfl_add_layernorm_workspace_bytes(rows, d), 4), dtype=torch.uint8, device=r.device)
        ysum = torch.empty(d, dtype=torch.float32, device=r.device) if y.dtype != torch.float32 else None
        rc = lib.mfl_add_layernorm_backward_ex2(dout.data_ptr(), None, None, r.data_ptr(), _TAGS[r.dtype], y.data_ptr(),
                                                _TAGS[y.dtype], weight.data_ptr(), mean.data_ptr(), rstd.data_ptr(),
                                                rows, d, dr.data_ptr(), dy.data_ptr(), dw.data_ptr(), db.data_ptr(),
                                                None, 0, _ptr(ysum), ctx.p_drop, _ptr(seed), ws.data_ptr(),
                                                _native.stream_handle(r.device))
        if rc != 0:
            raise RuntimeError(lib.mfl_add_layernorm_last_error().decode())
        _attach_colsum(dy, ysum)
        return dr, dy, dw, db, None, None, None


def add_layer_norm(r, y, norm: nn.LayerNorm, dropout=None):
    """``norm(r + dropout(y))`` (``norm(r + y)`` without ``dropout``); fused on the GPU under autocast,
    dropout included (see the module docstring)."""
    d = r.shape[-1]
    if (r.is_cuda and torch.is_autocast_enabled("cuda") and isinstance(norm, nn.LayerNorm)
            and norm.elementwise_affine and norm.bias is not None and tuple(norm.normalized_shape) == (d,)
            and norm.weight.dtype == torch.float32 and r.shape == y.shape and r.dtype in _TAGS
            and y.dtype in _TAGS and d % 256 == 0 and d <= 1024 and r.numel() > 0
            and y.device == r.device and norm.weight.device == r.device):
        p_drop, seed = _drop_args(dropout, r.device)
        with torch.autocast("cuda", enabled=False):
            return _AddLayerNorm.apply(r.contiguous(), y.contiguous(), norm.weight, norm.bias, norm.eps, p_drop, seed)
    return norm(r + (dropout(y) if dropout is not None else y))


def _gsum_tagged(r):
    return bool(getattr(r, "_mfl_gsum", False))


class _AddLayerNormCarry(Function):
    @staticmethod
    def forward(ctx, r, y, weight, bias, pos, eps, p_drop, seed, pos_acc=None):
        from ... import _native, _trace
        _trace.hit("add_ln_carry")
        lib = _native.load_library()
        ctx.set_materialize_grads(False)
        d = r.shape[-1]
        rows = r.numel() // d
        out = torch.empty(r.shape, dtype=torch.float32, device=r.device)
        out16 = torch.empty(r.shape, dtype=torch.bfloat16, device=r.device)
        q16 = torch.empty(r.shape, dtype=torch.bfloat16, device=r.device) if pos is not None else None
        mean = torch.empty(rows, dtype=torch.float32, device=r.device)
        rstd = torch.empty(rows, dtype=torch.float32, device=r.device)
        rc = lib.mfl_add_layernorm_forward_ex(
            r.data_ptr(), _TAGS[r.dtype], y.data_ptr(), _TAGS[y.dtype], weight.data_ptr(), bias.data_ptr(), rows, d,
            float(eps), out.data_ptr(), mean.data_ptr(), rstd.data_ptr(), out16.data_ptr(),
            _ptr(pos), _ptr(q16), p_drop, _ptr(seed), _native.stream_handle(r.device))
        if rc != 0:
            raise RuntimeError(lib.mfl_add_layernorm_last_error().decode())
        ctx.has_pos = pos is not None
        ctx.pos_needs_grad = pos is not None and pos.requires_grad
        ctx.pos_acc = pos_acc if ctx.pos_needs_grad else None
        ctx.n_grads = 9 if pos_acc is not None else 8  # (apply called without pos_acc: 8 inputs)
        ctx.p_drop = p_drop
        ctx.gsum = _gsum_tagged(r)
        ctx.save_for_backward(r, y, weight, mean, rstd, seed)
        return out, out16, q16

    @staticmethod
    def backward(ctx, dout, dout16, dq16):
        from ... import _native
        lib = _native.load_library()
        r, y, weight, mean, rstd, seed = ctx.saved_tensors
        d = r.shape[-1]
        rows = r.numel() // d
        if dout is None and dout16 is None and dq16 is None:
            return (None,) * ctx.n_grads
        dout = dout.to(torch.float32).contiguous() if dout is not None else None
        dout16 = dout16.to(torch.bfloat16).contiguous() if dout16 is not None else None
        dq16 = dq16.to(torch.bfloat16).contiguous() if dq16 is not None else None
        dr = torch.empty_like(r)
        dy = torch.empty_like(y)
        dw = torch.empty(d, dtype=torch.float32, device=r.device)
        db = torch.empty(d, dtype=torch.float32, device=r.device)
        dpos, acc, accumulate = None, ctx.pos_acc, 0
        if acc is not None:
            # the shared pos's summed gradient (PosGradAcc): the first backward writes it, the others add
            if dq16 is not None:
                accumulate = 1 if acc.buf is not None else 0
                if acc.buf is None:
                    acc.buf = torch.empty(r.shape, dtype=torch.float32, device=r.device)
                dpos = acc.buf
        elif ctx.pos_needs_grad:
            dpos = (torch.empty(r.shape, dtype=torch.float32, device=r.device) if dq16 is not None
                    else torch.zeros(r.shape, dtype=torch.float32, device=r.device))
        ysum = torch.empty(d, dtype=torch.float32, device=r.device) if y.dtype != torch.float32 else None
        ws = torch.empty(max(lib.mfl_add_layernorm_workspace_bytes(rows, d), 4), dtype=torch.uint8, device=r.device)
        rc = lib.mfl_add_layernorm_backward_ex2(
            _ptr(dout), _ptr(dout16), _ptr(dq16), r.data_ptr(), _TAGS[r.dtype], y.data_ptr(), _TAGS[y.dtype],
            weight.data_ptr(), mean.data_ptr(), rstd.data_ptr(), rows, d, dr.data_ptr(), dy.data_ptr(),
            dw.data_ptr(), db.data_ptr(), _ptr(dpos) if dq16 is not None else None, accumulate, _ptr(ysum),
            ctx.p_drop, _ptr(seed), ws.data_ptr(), _native.stream_handle(r.device))
        if rc != 0:
            raise RuntimeError(lib.mfl_add_layernorm_last_error().decode())
        _attach_colsum(dy, ysum)
        if ctx.gsum:
            from .linear import grad_sum_give
            grad_sum_give(True, r, dr)
        return (dr, dy, dw, db, (None if acc is not None else dpos), None, None, None, None)[:ctx.n_grads]


def carry_supported(r, norm) -> bool:
    """Whether ``add_layer_norm_carry`` runs fused for residual ``r`` and ``norm``."""
    d = r.shape[-1]
    return (r.is_cuda and torch.is_autocast_enabled("cuda")
            and torch.get_autocast_dtype("cuda") == torch.bfloat16 and isinstance(norm, nn.LayerNorm)
            and norm.elementwise_affine and norm.bias is not None and tuple(norm.normalized_shape) == (d,)
            and norm.weight.dtype == torch.float32 and r.dtype in _TAGS and d % 256 == 0 and d <= 1024
            and r.numel() > 0 and norm.weight.device == r.device)


def add_layer_norm_carry(r, y, norm: nn.LayerNorm, pos=None, dropout=None, pos_acc=None):
    """``(out, out16, q16)`` with ``out = norm(r + dropout(y))`` (fp32 under autocast), ``out16`` its bf16
    copy and ``q16 = bf16(out + pos)`` (None without ``pos``).  Fused on the GPU under bf16
    autocast; elsewhere ``(out, out, out + pos)``, which every consumer treats exactly as before.
    ``pos_acc``: pos came from ``pos_sink`` and its gradient is summed there (see PosGradAcc)."""
    if (carry_supported(r, norm) and r.shape == y.shape and y.dtype in _TAGS
            and (pos is None or (pos.shape == r.shape and pos.dtype == torch.float32))):
        p_drop, seed = _drop_args(dropout, r.device)
        args = (r.contiguous(), y.contiguous(), norm.weight, norm.bias, pos.contiguous() if pos is not None else None,
                norm.eps, p_drop, seed)
        if pos is not None and pos_acc is not None:
            args += (pos_acc,)
        with torch.autocast("cuda", enabled=False):
            return _AddLayerNormCarry.apply(*args)
    out = add_layer_norm(r, y, norm, dropout)
    return out, out, (out + pos if pos is not None else None)


class _CarryEntry(Function):
    """(src, bf16(src), bf16(src + pos)): an encoder's first-layer operands in one pass, and one pass
    back summing src's three gradients (csrc/add_layernorm.hip carry_entry_*)."""

    @staticmethod
    def forward(ctx, src, pos, acc):
        from ... import _native, _trace
        _trace.hit("carry_entry")
        lib = _native.load_library()
        v16 = torch.empty(src.shape, dtype=torch.bfloat16, device=src.device)
        q16 = torch.empty(src.shape, dtype=torch.bfloat16, device=src.device)
        rc = lib.mfl_carry_entry_forward(src.data_ptr(), _ptr(pos), src.numel(), v16.data_ptr(), q16.data_ptr(),
                                         _native.stream_handle(src.device))
        if rc != 0:
            raise RuntimeError("mfl_carry_entry_forward failed: " + lib.mfl_add_layernorm_last_error().decode())
        ctx.set_materialize_grads(False)
        ctx.acc, ctx.has_pos, ctx.shape = acc, pos is not None, src.shape
        return src.view_as(src), v16, q16

    @staticmethod
    def backward(ctx, dr, dv16, dq16):
        from ... import _native
        lib = _native.load_library()
        nig = ctx.needs_input_grad
        ref = next(t for t in (dr, dv16, dq16) if t is not None) if any(
            t is not None for t in (dr, dv16, dq16)) else None
        if ref is None:
            return None, None, None
        dev = ref.device
        n = 1
        for k in ctx.shape:
            n *= k
        dr = dr.contiguous() if dr is not None and dr.dtype == torch.float32 else (None if dr is None else dr.float())
        dv16 = None if dv16 is None else dv16.to(torch.bfloat16).contiguous()
        dq16 = None if dq16 is None else dq16.to(torch.bfloat16).contiguous()
        dsrc = torch.empty(ctx.shape, dtype=torch.float32, device=dev) if nig[0] else None
        dpos, acc_flag, out_pos = None, 0, None
        if ctx.has_pos and nig[1] and dq16 is not None:
            if ctx.acc is not None:
                if ctx.acc.buf is None:
                    ctx.acc.buf = torch.empty(ctx.shape, dtype=torch.float32, device=dev)
                else:
                    acc_flag = 1
                dpos = ctx.acc.buf
            else:
                dpos = out_pos = torch.empty(ctx.shape, dtype=torch.float32, device=dev)
        if dsrc is None:  # (the kernel always writes dsrc: a scratch buffer when src needs no gradient)
            dsrc_buf = torch.empty(ctx.shape, dtype=torch.float32, device=dev)
        else:
            dsrc_buf = dsrc
        rc = lib.mfl_carry_entry_backward(_ptr(dr), _ptr(dv16), _ptr(dq16), n, dsrc_buf.data_ptr(), _ptr(dpos),
                                          acc_flag, _native.stream_handle(dev))
        if rc != 0:
            raise RuntimeError("mfl_carry_entry_backward failed: " + lib.mfl_add_layernorm_last_error().decode())
        return dsrc, out_pos, None


def carry_entry(src, pos=None, pos_acc=None):
    """``(src, bf16(src), bf16(src + pos))`` — the first carried layer's residual, value and query
    operands (reference ``with_pos_embed(src, pos)``, unimodal_deformable_transformer.py:241, cast by
    autocast at each Linear) — from one fused kernel each way under bf16 autocast on the GPU;
    None where it does not apply (the caller keeps the composition).  ``pos_acc``: pos came from
    ``pos_sink`` and its gradient is summed there."""
    if not (src.is_cuda and src.dtype == torch.float32 and src.is_contiguous() and src.numel() % 8 == 0
            and torch.is_autocast_enabled("cuda") and torch.get_autocast_dtype("cuda") == torch.bfloat16
            and src.data_ptr() % 16 == 0):
        return None
    if pos is not None and not (pos.is_cuda and pos.dtype == torch.float32 and pos.is_contiguous()
                                and pos.shape == src.shape and pos.data_ptr() % 16 == 0):
        return None
    return _CarryEntry.apply(src, pos, pos_acc)

