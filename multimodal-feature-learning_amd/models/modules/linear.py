"""``nn.Linear`` with an MI355X-shaped backward under bf16/fp16 autocast.

Same parameters, state_dict keys, init and forward math as ``torch.nn.Linear`` (every Linear
of the reference's deformable stack, e.g. ``models/modules/attention.py:417-420`` and the
FFNs of ``unimodal_deformable_transformer.py:174-177``).  Only the autocast backward differs:

* autograd computes ``dW = dY^T X`` as ONE hipBLASLt GEMM with a bf16 output.  At the bench
  step's shapes (K = 15,360 tokens, 512x512 or 128x512 outputs) that GEMM has 16-64 output
  tiles for 256 CUs and no split-K: ~100-125 us each (tools/gemm_probe.py).  Then it casts
  the bf16 result to fp32 and adds it into ``p.grad`` (two more kernels, bf16 rounding
  of the whole gradient).
* here the K dimension is split into ``s`` chunks, one strided-batched GEMM writes the fp32
  partial products (fp32 accumulate and output, ``out_dtype``), and their sum is the fp32
  gradient: 30-55 us at the same shapes and ~1000x less rounding error; short K (decoder
  queries) uses a single GEMM with fp32 output.  The bias gradient is one fp32-output
  reduction.

Outside autocast on a GPU (fp32 / fp64 parity runs) and on the CPU it is exactly
``F.linear``.

Deferred weight gradients.  Inside ``deferred_weight_grads(deliver)`` (the training step's
backward, train_step.py) a short-K layer (at most ``DEFER_MAX_ROWS`` input rows: the decoder's
800 query rows, the caption decoder's words) does not compute dW and db in its backward: it
queues (dY, X) and returns no weight gradient; ``flush()`` then computes every queued product
of one shape as ONE strided-batched GEMM (fp32 output) and every bias gradient of one shape as
one reduction, and hands each parameter its gradient through ``deliver(param, grad)``.  The
decoder's 48 weight-gradient GEMMs of a step (800-row, 10-15 us each at 25-140 TF/s: each is
too small to fill 256 CUs) become five batched GEMMs.  dX stays in the backward (the chain
needs it).  ``flush_point(t)`` marks a tensor whose gradient completes a group of layers (the
decoder's memory): the queue is flushed there inside the backward, so a data-parallel step
all-reduces those gradients while the encoder's backward runs.
"""
import contextlib

import torch
import torch.nn.functional as F
from torch import nn

__all__ = ["Linear", "split_k_chunks", "linear_pair", "deferred_weight_grads", "flush_point",
           "flat_grad_destinations", "small_addmm", "small_mm_nn"]

# GEMM K (input rows) up to which weight gradients are queued and batched: the decoder's 800 query
# rows (each GEMM too small for the chip).  Not the caption decoder's ~3,200 word tokens (DVC step):
# their GEMMs fill the chip alone, and batching them stacked every dY and X (~300 MB of copies a
# step, tools/op_census.py --config dvc) and handed the gradients over as fresh tensors to copy.
DEFER_MAX_ROWS = 1024


class _WgradQueue:
    """Queued weight / bias gradient products of one backward (see the module docstring)."""

    def __init__(self, deliver):
        self.deliver = deliver
        # (dY (K, N), X (K, C), weight param, row offset, bias param or None, dY's column sums or None)
        self.entries = []

    def push(self, g2, x2, weight, row, bias, colsum=None):
        self.entries.append((g2, x2, weight, row, bias, colsum))

    @torch.no_grad()
    def flush(self):
        entries, self.entries = self.entries, []
        if not entries:
            return
        groups = {}
        for e in entries:
            g2, x2 = e[0], e[1]
            groups.setdefault((g2.shape[0], g2.shape[1], x2.shape[1], g2.dtype), []).append(e)
        from ... import _trace
        _trace.hit("wgrad_batched", len(entries))
        parts = {}  # param -> [(row offset, fp32 grad rows)]
        for (_, n_out, _, _), es in groups.items():
            # whole weights of one shape laid out back to back in the trainer's flat gradient buffer
            # (flat_groups, e.g. the decoder layers' linear1): the batched GEMM writes their gradients
            # straight into that one view (no fresh tensors to copy into the buffer afterwards)
            dest = None
            if len(es) > 1 and es[0][0].is_cuda and all(e[3] == 0 and e[0].shape[1] == e[2].shape[0] for e in es):
                es = sorted(es, key=lambda e: _dest_offset(e[2]))
                dest = _claim_group([e[2] for e in es])
            gs = es[0][0][None] if len(es) == 1 else torch.stack([e[0] for e in es])
            xs = es[0][1][None] if len(es) == 1 else torch.stack([e[1] for e in es])
            if dest is not None:
                dw = torch.bmm(gs.transpose(1, 2), xs, out_dtype=torch.float32,
                               out=dest.view(len(es), gs.shape[2], xs.shape[2]))
            elif gs.is_cuda:  # fp32 accumulate and output
                dw = torch.bmm(gs.transpose(1, 2), xs, out_dtype=torch.float32)
            else:  # (CPU unit tests of the queue: no 16-bit-in / fp32-out GEMM there)
                dw = torch.bmm(gs.transpose(1, 2).float(), xs.float())
            # bias gradients: the column sums handed over with dY (add_norm: the add + LayerNorm
            # backward that produced dY summed them), else one reduction for the group
            need = any(e[4] is not None and e[5] is None for e in es)
            db = gs.sum(1, dtype=torch.float32) if need else None
            for k, (_, _, w, row, b, cs) in enumerate(es):
                parts.setdefault(w, []).append((row, dw[k]))
                if b is not None:
                    parts.setdefault(b, []).append((row, cs if cs is not None else db[k]))
        for prm, ps in parts.items():
            ps.sort(key=lambda rp: rp[0])
            rows = [r for r, _ in ps]
            ends = [r + g.shape[0] for r, g in ps]
            if len(ps) == 1 and ps[0][0] == 0 and ps[0][1].shape == prm.shape:
                grad = ps[0][1]
            elif rows[0] == 0 and ends[-1] == prm.shape[0] and all(e == r for e, r in zip(ends[:-1], rows[1:])):
                grad = torch.cat([g for _, g in ps])  # row blocks tiling the weight (in_proj q / k | v)
            else:  # a weight used several times
                grad = torch.zeros(prm.shape, dtype=torch.float32, device=prm.device)
                for row, g in ps:
                    grad[row:row + g.shape[0]] += g
            self.deliver(prm, grad)


_queue = None


@contextlib.contextmanager
def deferred_weight_grads(deliver):
    """Queue the short-K layers' weight / bias gradients of the backward run inside; the caller
    calls ``flush()`` on the yielded queue after the backward (flush points flush earlier)."""
    global _queue
    prev, _queue = _queue, _WgradQueue(deliver)
    try:
        yield _queue
    finally:
        _queue = prev


def _defer(*entries):
    """Queue the (dY, X, weight, row offset, bias[, dY column sums]) products of one backward when a
    queue is active and every K is short — all of them or none; True if queued."""
    q = _queue
    if q is None or any(e[0].shape[0] > DEFER_MAX_ROWS or e[2].dtype != torch.float32 for e in entries):
        return False
    for e in entries:
        q.push(*e)
    return True


class _FlushPoint(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        if _queue is not None:
            _queue.flush()
        return g


def flush_point(t):
    """Identity; in a deferred backward the queued weight gradients are computed once t's gradient
    is (see the module docstring)."""
    if _queue is None and not torch.is_grad_enabled():
        return t
    return _FlushPoint.apply(t) if t.requires_grad else t


SMALL_GEMM_MAX_ROWS = 1024  # GEMM rows (tokens) up to which small_addmm runs the HIP kernel


def small_addmm(bias, x2, w):
    """``bias + x2 @ w.T`` (bias may be None) for bf16 x2 (M, K) with M <= SMALL_GEMM_MAX_ROWS and
    w (N, K), on the short-M HIP GEMM (include/gemm_small.h: a workgroup a 32 x 32 tile, its waves
    splitting K): the decoder's 800-token Linear layers take 9-15 us in the library GEMM, latency
    bound.  None where it does not apply (the caller keeps torch.addmm).  MFL_SMALL_GEMM=0 turns it
    off."""
    M, K = x2.shape
    N = w.shape[0]
    # (graph-timed against hipBLASLt, tools/small_gemm_ab.py: ahead for N, K <= 512 — 800 x 256 x 512
    # 4.3 vs 5.4 us, 800 x 512 x 512 6.2 vs 6.5 — behind from N or K = 1024 on)
    # (operands on another device than x2 — a module left on the host — go to torch.addmm, which
    # raises; their pointers must never reach the kernel)
    if not (x2.is_cuda and x2.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and 0 < M <= SMALL_GEMM_MAX_ROWS
            and w.device == x2.device and (bias is None or bias.device == x2.device)
            and N <= 512 and K <= 512
            and N % 32 == 0 and K % 32 == 0 and x2.stride(1) == 1 and w.stride(1) == 1
            and x2.stride(0) % 8 == 0 and w.stride(0) % 8 == 0 and x2.stride(0) >= K and w.stride(0) >= K
            and (bias is None or (bias.dtype == torch.bfloat16 and bias.is_contiguous() and bias.numel() == N))
            and x2.data_ptr() % 16 == 0 and w.data_ptr() % 16 == 0):
        return None
    import os
    if os.environ.get("MFL_SMALL_GEMM", "1") == "0":
        return None
    from ... import _native, _trace
    lib = _native.load_library()
    out = torch.empty(M, N, dtype=torch.bfloat16, device=x2.device)
    rc = lib.mfl_gemm_nt_bf16(x2.data_ptr(), w.data_ptr(), None if bias is None else bias.data_ptr(), out.data_ptr(),
                              M, N, K, x2.stride(0), w.stride(0), N, _native.stream_handle(x2.device))
    if rc == 2:  # MFL_GEMM_UNSUPPORTED
        return None
    if rc != 0:
        raise RuntimeError("mfl_gemm_nt_bf16 failed: " + lib.mfl_gemm_last_error().decode())
    _trace.hit("small_gemm")
    return out


def small_mm_nn(g2, w):
    """``g2 @ w`` for bf16 g2 (M, N) with M <= SMALL_GEMM_MAX_ROWS and w (N, K) row-major — a Linear
    layer's input gradient — on the short-M HIP GEMM (mfl_gemm_nn_bf16); None where it does not apply."""
    M, N = g2.shape
    K = w.shape[1]
    # (ahead of hipBLASLt for N, K <= 512: 800 x 512 x 512 5.4 vs 7.4 us; behind from 1024 on)
    if not (g2.is_cuda and g2.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and 0 < M <= SMALL_GEMM_MAX_ROWS
            and w.device == g2.device
            and N <= 512 and K <= 512
            and K % 32 == 0 and N % 32 == 0 and g2.stride(1) == 1 and w.stride(1) == 1
            and g2.stride(0) % 8 == 0 and w.stride(0) % 8 == 0 and g2.stride(0) >= N and w.stride(0) >= K
            and g2.data_ptr() % 16 == 0 and w.data_ptr() % 16 == 0):
        return None
    import os
    if os.environ.get("MFL_SMALL_GEMM", "1") == "0":
        return None
    from ... import _native, _trace
    lib = _native.load_library()
    out = torch.empty(M, K, dtype=torch.bfloat16, device=g2.device)
    rc = lib.mfl_gemm_nn_bf16(g2.data_ptr(), w.data_ptr(), None, out.data_ptr(), M, K, N, g2.stride(0), w.stride(0), K,
                              _native.stream_handle(g2.device))
    if rc == 2:  # MFL_GEMM_UNSUPPORTED
        return None
    if rc != 0:
        raise RuntimeError("mfl_gemm_nn_bf16 failed: " + lib.mfl_gemm_last_error().decode())
    _trace.hit("small_gemm_nn")
    return out


def _mm_nn(g2, w):
    """``g2 @ w`` (a Linear layer's input gradient): the short-M HIP GEMM where it applies."""
    y = small_mm_nn(g2, w)
    return torch.mm(g2, w) if y is None else y


def _addmm(bias, x2, w):
    """``bias + x2 @ w.T`` (``x2 @ w.T`` without bias): the short-M HIP GEMM where it applies."""
    y = small_addmm(bias, x2, w)
    if y is not None:
        return y
    return torch.mm(x2, w.t()) if bias is None else torch.addmm(bias, x2, w.t())


def split_k_chunks(k, min_chunk=1024, max_split=8):
    """Number of K chunks for the weight-gradient GEMM: the largest s <= max_split dividing K
    with K / s >= min_chunk (1 = no split)."""
    s = max_split
    while s > 1:
        if k % s == 0 and k // s >= min_chunk:
            return s
        s //= 2
    return 1


_dest = None  # flat_grad_destinations: {"views": {id(param): flat view}, "claimed": set()}


@contextlib.contextmanager
def flat_grad_destinations(views, may_claim=None):
    """Inside (the trainer's backward): the first gradient produced for a parameter in ``views``
    ({id(param): its fp32 view of the flat gradient buffer}) is written straight into that view,
    which autograd then hands to the parameter as its .grad — instead of a fresh tensor copied
    into the flat buffer afterwards (one 171 MB copy pass per step at the bench shape).
    ``may_claim(param)``, when given, vetoes a view at the time it would be handed out (the
    trainer refuses the views of gradient buckets it has already all-reduced or is reducing)."""
    global _dest
    prev, _dest = _dest, {"views": views, "claimed": set(), "may_claim": may_claim}
    try:
        yield
    finally:
        _dest = prev


def _claim(param):
    """The flat view ``param``'s gradient may be written into, or None: once per backward and
    only while the parameter has no gradient yet (a later producer's result is added by autograd,
    into that view or a copy of it)."""
    d = _dest
    if d is None or param is None or param.grad is not None:
        return None
    v = d["views"].get(id(param))
    if v is None or id(param) in d["claimed"]:
        return None
    if d["may_claim"] is not None and not d["may_claim"](param):
        return None
    d["claimed"].add(id(param))
    return v.view_as(v)  # a fresh view object: autograd adopts it as .grad instead of cloning


def _given_colsum(gy, n):
    """The fp32 column sums handed over with the output gradient ``gy`` (add_norm._attach_colsum:
    the fused add + LayerNorm backward that produced it summed them), or None — also when gy was
    modified in place since (its version counter moved) or the shape does not match."""
    t = getattr(gy, "_mfl_colsum", None)
    if t is None:
        return None
    cs, ver = t
    if ver != gy._version or tuple(cs.shape) != (n,):
        return None
    return cs


def _dest_offset(param):
    """Offset of param's flat gradient view (for ordering a group), or -1."""
    d = _dest
    v = None if d is None else d["views"].get(id(param))
    return -1 if v is None else v.storage_offset()


def _claim_group(params):
    """One view of the flat gradient buffer covering the given parameters' gradient views, when they
    lie back to back in this order (the trainer's flat_groups layout; stacked along dim 0), claimed for
    all of them — or None, and nothing claimed (see _claim)."""
    d = _dest
    if d is None or len(params) < 2:
        return None
    views = [d["views"].get(id(p)) for p in params]
    if any(v is None for v in views) or len({id(p) for p in params}) != len(params):
        return None
    if any(p.grad is not None or id(p) in d["claimed"] for p in params):
        return None
    if d["may_claim"] is not None and not all(d["may_claim"](p) for p in params):
        return None
    base, off = views[0], views[0].storage_offset()
    for v in views:
        if (v.storage_offset() != off or not v.is_contiguous() or v.shape[1:] != base.shape[1:]
                or v.untyped_storage().data_ptr() != base.untyped_storage().data_ptr()):
            return None
        off += v.numel()
    for p in params:
        d["claimed"].add(id(p))
    rows = sum(v.shape[0] for v in views)
    return base.new_empty(0).set_(base.untyped_storage(), base.storage_offset(), (rows,) + tuple(base.shape[1:]))


def _bias_grad(g2, out=None):
    """fp32 column sum of dY (K, N) through mfl_colsum (one streaming pass, fixed order);
    torch's column reduction where the kernel's layout conditions do not hold.  ``out``: an fp32
    (N,) destination (a flat-buffer view)."""
    if g2.dtype not in (torch.bfloat16, torch.float16) or (g2.shape[1] * 2) % 16 or not g2.is_contiguous():
        r = g2.sum(0, dtype=torch.float32)
        return r if out is None else out.copy_(r)
    from ... import _native
    lib = _native.load_library()
    K, N = g2.shape
    if out is None:
        out = torch.empty(N, dtype=torch.float32, device=g2.device)
    ws = torch.empty(lib.mfl_colsum_workspace_bytes(K, N), dtype=torch.uint8, device=g2.device)
    rc = lib.mfl_colsum(g2.data_ptr(), _native.DTYPE_TAGS[g2.dtype], K, N, out.data_ptr(), ws.data_ptr(),
                        _native.stream_handle(g2.device))
    if rc != 0:
        raise RuntimeError("mfl_colsum failed: " + lib.flat_adamw_last_error().decode())
    return out


def _sum_slabs(part, out=None):
    """part.sum(0) of the fp32 split-K partials (s, n_out, n_in) through mfl_sum_slabs (one pass,
    chunk order), into ``out`` if given."""
    n = part[0].numel()
    if n % 4 or not part.is_contiguous():
        return part.sum(0) if out is None else torch.sum(part, 0, out=out)
    from ... import _native
    lib = _native.load_library()
    if out is None:
        out = torch.empty(part.shape[1:], dtype=torch.float32, device=part.device)
    rc = lib.mfl_sum_slabs(part.data_ptr(), part.shape[0], n, out.data_ptr(), _native.stream_handle(part.device))
    if rc != 0:
        raise RuntimeError("mfl_sum_slabs failed: " + lib.flat_adamw_last_error().decode())
    return out


def _weight_grad(g2, x2, out=None):
    """fp32 dW = dY^T X of 16-bit dY (K, N) and X (K, C): K split into chunks, one strided-batched
    GEMM with fp32 partial outputs, then their sum (into ``out`` if given)."""
    k, n_out, n_in = x2.shape[0], g2.shape[1], x2.shape[1]
    s = split_k_chunks(k)
    if s > 1:
        # (bmm, not baddbmm(out=part, beta=0): that form first copies `part` into the output — an
        # extra 8-32 MB pass per call, ~0.3 ms per step, tools/op_census.py)
        part = torch.bmm(g2.view(s, k // s, n_out).transpose(1, 2), x2.view(s, k // s, n_in),
                         out_dtype=torch.float32)
        return _sum_slabs(part, out)
    r = torch.mm(g2.t(), x2, out_dtype=torch.float32)
    return r if out is None else out.copy_(r)


class _AutocastLinear(torch.autograd.Function):
    """y = x W^T + b with x already in the autocast dtype; W, b fp32 masters; wc / bc optional
    low-precision copies of W / b (the trainer's shadow) used instead of casting."""

    @staticmethod
    def forward(ctx, x, weight, bias, wc, bc):
        from ... import _trace
        _trace.hit("linear_shadow" if wc is not None else "linear_cast")
        dt = x.dtype
        if wc is None:
            wc = weight.to(dt)
        x2 = x.reshape(-1, x.shape[-1])
        y = _addmm((bias.to(dt) if bc is None else bc) if bias is not None else None, x2, wc)
        ctx.save_for_backward(x2, wc)
        ctx.has_bias = bias is not None
        ctx.x_shape = x.shape
        ctx.weight, ctx.bias = weight, bias  # the parameters a deferred gradient is delivered to
        # not an autograd view of the 2-D GEMM output (as F.linear's 3-D result): callers may
        # modify it in place (MSDeformAttn zeroes the padding rows of value_proj's output)
        return torch.ops.aten._unsafe_view(y, (*x.shape[:-1], wc.shape[0]))

    @staticmethod
    def backward(ctx, gy):
        x2, wc = ctx.saved_tensors
        cs = _given_colsum(gy, wc.shape[0]) if ctx.has_bias else None
        g2 = gy.reshape(-1, gy.shape[-1]).to(wc.dtype)
        gx = gw = gb = None
        nig = ctx.needs_input_grad
        if nig[0]:
            gx = _mm_nn(g2, wc).view(ctx.x_shape)
        if nig[1] and (not ctx.has_bias or nig[2]) and _defer((g2, x2, ctx.weight, 0, ctx.bias if ctx.has_bias else None,
                                                                cs)):
            return gx, None, None, None, None
        if nig[1]:
            gw = _weight_grad(g2, x2, _claim(ctx.weight))
        if ctx.has_bias and nig[2]:
            gb = cs if cs is not None else _bias_grad(g2, _claim(ctx.bias))
        return gx, gw, gb, None, None


class _AutocastLinearPair(torch.autograd.Function):
    """(x A^T + a, x B^T + b) of ONE 16-bit input: two forward GEMMs on the shared cast, and a
    backward on the concatenated output gradient — one dgrad GEMM (no second input-gradient
    cast and add), one split-K weight-gradient GEMM and one column sum for both layers."""

    @staticmethod
    def forward(ctx, x, wa, ba, wb, bb, wca, bca, wcb, bcb):
        from ... import _trace
        _trace.hit("linear_pair_shadow" if wca is not None and wcb is not None else "linear_pair_cast")
        dt = x.dtype
        wca = wa.to(dt) if wca is None else wca
        wcb = wb.to(dt) if wcb is None else wcb
        x2 = x.reshape(-1, x.shape[-1])
        ya = _addmm(ba.to(dt) if bca is None else bca, x2, wca)
        yb = _addmm(bb.to(dt) if bcb is None else bcb, x2, wcb)
        ctx.save_for_backward(x2, wca, wcb)
        ctx.x_shape = x.shape
        ctx.params = (wa, ba, wb, bb)
        lead = x.shape[:-1]
        return ya.view(*lead, wca.shape[0]), yb.view(*lead, wcb.shape[0])

    @staticmethod
    def backward(ctx, gya, gyb):
        x2, wca, wcb = ctx.saved_tensors
        na, nb = wca.shape[0], wcb.shape[0]
        k = x2.shape[0]
        ga = gya.reshape(k, na).to(wca.dtype) if gya is not None else x2.new_zeros(k, na)
        gb_ = gyb.reshape(k, nb).to(wca.dtype) if gyb is not None else x2.new_zeros(k, nb)
        g2 = torch.cat((ga, gb_), 1)
        nig = ctx.needs_input_grad
        gx = torch.mm(g2, torch.cat((wca, wcb), 0)).view(ctx.x_shape) if nig[0] else None
        wa, ba, wb, bb = ctx.params
        if all(nig[1:5]) and _defer((ga, x2, wa, 0, ba), (gb_, x2, wb, 0, bb)):
            return gx, None, None, None, None, None, None, None, None
        gwa = gwb = gba = gbb = None
        if nig[1] or nig[3]:
            gw = _weight_grad(g2, x2)
            gwa, gwb = gw[:na], gw[na:]
        if nig[2] or nig[4]:
            gbias = _bias_grad(g2)
            gba, gbb = gbias[:na], gbias[na:]
        return gx, gwa, gba, gwb, gbb, None, None, None, None


def linear_pair(x, a, b):
    """``(a(x), b(x))`` for two Linear layers with biases that read the same input (the
    ``sampling_offsets`` / ``attention_weights`` projections of MSDeformAttn,
    attention.py:468-470).  Under 16-bit autocast on the GPU: one input cast and a fused
    backward (_AutocastLinearPair); elsewhere the two layers as they are."""
    if not (isinstance(a, Linear) and isinstance(b, Linear) and a.bias is not None and b.bias is not None
            and a._autocast_dtype(x) is not None):
        return a(x), b(x)
    dt = a._autocast_dtype(x)
    wca, bca = a._low(dt)
    wcb, bcb = b._low(dt)
    with torch.autocast("cuda", enabled=False):
        return _AutocastLinearPair.apply(x.to(dt), a.weight, a.bias, b.weight, b.bias, wca, bca, wcb, bcb)


class Linear(nn.Linear):
    _shadow = None  # (weight copy, bias copy, weight version) set by set_bf16_shadow

    def _autocast_dtype(self, x):
        """The 16-bit autocast dtype this layer computes in for input x, or None (F.linear)."""
        if (x.is_cuda and torch.is_autocast_enabled("cuda") and self.weight.dtype == torch.float32
                and self.weight.device == x.device
                and torch.get_autocast_dtype("cuda") in (torch.bfloat16, torch.float16)):
            return torch.get_autocast_dtype("cuda")
        return None

    def _low(self, dt):
        """(weight, bias) 16-bit copies from the trainer's shadow while it is current, else None."""
        sh = self._shadow
        if sh is not None and dt == torch.bfloat16 and sh[2] == self.weight._version:
            return sh[0], sh[1]
        return None, None

    def set_bf16_shadow(self, weight_bf16, bias_bf16):
        """Use these bf16 copies of weight / bias under bf16 autocast for as long as the fp32
        weight is not modified in place (its version counter is recorded now).  The training
        step refreshes them after every optimizer step (train_step.FlatGradTrainer)."""
        self._shadow = (weight_bf16, bias_bf16, self.weight._version)

    def forward(self, x):
        if self._autocast_dtype(x) is not None:
            dt = torch.get_autocast_dtype("cuda")
            wc = bc = None
            sh = self._shadow
            if sh is not None and dt == torch.bfloat16 and sh[2] == self.weight._version:
                wc, bc = sh[0], sh[1]
            with torch.autocast("cuda", enabled=False):
                return _AutocastLinear.apply(x.to(dt), self.weight, self.bias, wc, bc)
        return F.linear(x, self.weight, self.bias)
