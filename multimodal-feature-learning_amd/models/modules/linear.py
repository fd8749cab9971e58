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
import os

import torch
import torch.nn.functional as F
from torch import nn

__all__ = ["Linear", "split_k_chunks", "linear_pair", "deferred_weight_grads", "flush_point",
           "flat_grad_destinations", "small_addmm", "small_mm_nn", "mark_grad_sum"]

# GEMM K (input rows) up to which weight gradients are queued and batched: the decoder's 800 query
# rows (each GEMM too small for the chip).  Not the caption decoder's ~3,200 word tokens (DVC step):
# their GEMMs fill the chip alone, and batching them stacked every dY and X (~300 MB of copies a
# step, tools/op_census.py --config dvc) and handed the gradients over as fresh tensors to copy.
DEFER_MAX_ROWS = 1024


class _WgradQueue:
    """Queued weight / bias gradient products of one backward (see the module docstring)."""

    def __init__(self, deliver, target=None):
        self.deliver = deliver
        # target(param): the tensor a finished gradient for param may be added into in place (the
        # trainer: param.grad while its bucket is not reduced), or None.  deliver(param, None) then
        # means "added into target(param)"
        self.target = target
        # (dY (K, N), X (K, C), weight param, row offset, bias param or None, dY's column sums or None)
        self.entries = []

    def push(self, g2, x2, weight, row, bias, colsum=None):
        self.entries.append((g2, x2, weight, row, bias, colsum))

    def _finish(self, prm, ts, dest=None):
        """Hand parameter prm the sum of its full-shape gradient products ts: added in place into
        target(prm) when there is one (one kernel, no fresh tensor), else summed into dest (its
        claimed flat view) or a fresh tensor — a single product is handed over as it is."""
        tgt = self.target(prm) if self.target is not None and ACCUMULATE_IN_PLACE else None
        if tgt is not None:
            from ... import _trace
            _trace.hit("wgrad_into_grad")
            _sum_into(ts, tgt, accumulate=True)
            self.deliver(prm, None)
            return
        if len(ts) == 1 and dest is None:
            self.deliver(prm, ts[0])
            return
        out = dest if dest is not None else torch.empty(prm.shape, dtype=torch.float32, device=ts[0].device)
        if len(ts) == 1:
            out.copy_(ts[0])
        else:
            _sum_into(ts, out, accumulate=False)
        self.deliver(prm, out)

    def _runs(self, groups):
        """The batches of one flush: each shape group's entries sorted so one parameter's products
        sit next to each other and the parameters follow the flat gradient buffer.  Split further
        only where that lets a batch's GEMM write a claimed view of the flat gradient buffer: the
        whole-weight products of parameters with no gradient yet are cut where their flat views stop
        lying back to back (the decoder's self_attn.out_proj and cross_attn.output_proj share a shape
        but are two runs) — unless that gives more than 3 batches (each costs a stacking copy, a GEMM
        and possibly a bias reduction).  Row-block products (in_proj's q / k | v) and products added
        into an existing .grad stay one batch each.  Off by default (MFL_QUEUE_RUNS=1 turns it on): one
        batch per shape measured the same (888.9 vs 885.5 clips/s headline, 529.9 vs 529.8 configs[2])."""
        import os
        split = os.environ.get("MFL_QUEUE_RUNS", "0") == "1"
        whole = lambda e: e[3] == 0 and e[0].shape[1] == e[2].shape[0]  # noqa: E731
        has_t = lambda w: (self.target is not None and ACCUMULATE_IN_PLACE  # noqa: E731
                           and self.target(w) is not None)
        for es in groups.values():
            es = sorted(es, key=lambda e: (_dest_offset(e[2]), id(e[2]), e[3]))
            if not split:
                yield es
                continue
            rows = [e for e in es if not whole(e)]
            accs = [e for e in es if whole(e) and has_t(e[2])]
            rest = [e for e in es if whole(e) and not has_t(e[2])]
            runs, run, prev = [], [], None
            for e in rest:
                w = e[2]
                off = _dest_offset(w)
                if prev is not None and w is not prev[0]:
                    if not (off >= 0 and prev[1] >= 0 and off == prev[1] + prev[0].numel()):
                        runs.append(run)
                        run = []
                run.append(e)
                prev = (w, off)
            if run:
                runs.append(run)
            if len(runs) > 3:
                runs = [rest]
            for r in [rows, accs] + runs:
                if r:
                    yield r

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
        parts = {}  # param -> [(row offset, fp32 grad rows)] (weights of several row blocks)
        for es in self._runs(groups):
            uniq = list({id(e[2]): e[2] for e in es}.values())
            uses = [sum(1 for e in es if e[2] is w) for w in uniq]
            full = all(e[3] == 0 and e[0].shape[1] == e[2].shape[0] for e in es)
            # whole weights of one shape laid out back to back in the trainer's flat gradient buffer
            # (flat_groups, e.g. the decoder layers' linear1): the batched GEMM (or the sum of a
            # shared weight's products) writes their gradients straight into that one view
            dest = None
            if (es[0][0].is_cuda and full and len(set(uses)) == 1 and (ACCUMULATE_IN_PLACE or uses[0] == 1)
                    and not any(self.target is not None and self.target(w) is not None for w in uniq)):
                dest = _claim_group(uniq, returned=False) if len(uniq) > 1 else _claim(uniq[0], returned=False)
            gs = es[0][0][None] if len(es) == 1 else torch.stack([e[0] for e in es])
            xs = es[0][1][None] if len(es) == 1 else torch.stack([e[1] for e in es])
            if dest is not None and uses[0] == 1:
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
            bias_parts = {}
            for k, (_, _, w, row, b, cs) in enumerate(es):
                if not full:
                    parts.setdefault(w, []).append((row, dw[k]))
                if b is not None:
                    if full:
                        bias_parts.setdefault(b, []).append(cs if cs is not None else db[k])
                    else:
                        parts.setdefault(b, []).append((row, cs if cs is not None else db[k]))
            if full:
                if dest is not None and uses[0] == 1:
                    for k, w in enumerate(uniq):
                        self.deliver(w, dw[k])
                elif dest is not None:  # every weight's u products summed into its view, one kernel
                    _sum_slabs(dw, dest.view(len(uniq), -1), groups=len(uniq))
                    for k, w in enumerate(uniq):
                        self.deliver(w, dest[k * w.shape[0]:(k + 1) * w.shape[0]].view_as(w))
                else:
                    k0 = 0
                    for w, u in zip(uniq, uses):
                        self._finish(w, [dw[k] for k in range(k0, k0 + u)])
                        k0 += u
            for b, ts in bias_parts.items():
                self._finish(b, ts)
        for prm, ps in parts.items():
            ps.sort(key=lambda rp: rp[0])
            rows = [r for r, _ in ps]
            ends = [r + g.shape[0] for r, g in ps]
            if len(ps) == 1 and ps[0][0] == 0 and ps[0][1].shape == prm.shape:
                grad = ps[0][1]
            elif rows[0] == 0 and ends[-1] == prm.shape[0] and all(e == r for e, r in zip(ends[:-1], rows[1:])):
                # row blocks tiling the weight (in_proj q / k | v): concatenated straight into its flat view
                v = _claim(prm, returned=False) if ps[0][1].is_cuda else None
                grad = torch.cat([g for _, g in ps]) if v is None else torch.cat([g for _, g in ps], out=v)
            elif all(r == 0 and g.shape == prm.shape for r, g in ps):
                # a whole weight used several times (the multimodal decoder's cross-attention over both
                # memories): its products summed into its flat view in list order (one slab-sum kernel
                # when they are slabs of one batched GEMM's output)
                v = _claim(prm, returned=False) if ps[0][1].is_cuda else None
                out = v.view_as(prm) if v is not None else torch.empty(prm.shape, dtype=torch.float32,
                                                                         device=prm.device)
                grad = _sum_into([g for _, g in ps], out, accumulate=False)
            else:  # row blocks of a weight used several times
                grad = torch.zeros(prm.shape, dtype=torch.float32, device=prm.device)
                for row, g in ps:
                    grad[row:row + g.shape[0]].add_(g)  # (in place: no write-back copy of the slice)
            self.deliver(prm, grad)


def _sum_into(ts, out, accumulate):
    """out (+)= the sum of the equal-shape fp32 tensors ts (formed first, in list order): one slab-sum
    kernel when they are consecutive slabs of one buffer (a batched GEMM's outputs), else adds."""
    n = ts[0].numel()
    base = ts[0]
    adjacent = (out.is_cuda and all(t.is_contiguous() and t.dtype == torch.float32 for t in ts)
                and all(t.untyped_storage().data_ptr() == base.untyped_storage().data_ptr()
                        and t.storage_offset() == base.storage_offset() + i * n for i, t in enumerate(ts)))
    if adjacent and out.is_contiguous():
        part = base.new_empty(0).set_(base.untyped_storage(), base.storage_offset(), (len(ts), n))
        _sum_slabs(part, out.view(-1), accumulate=accumulate)
        return out
    acc = ts[0] if len(ts) == 1 else torch.stack(ts).sum(0)
    if accumulate:
        out.add_(acc.view_as(out))
    else:
        out.copy_(acc.view_as(out))
    return out


_queue = None


@contextlib.contextmanager
def deferred_weight_grads(deliver, target=None):
    """Queue the short-K layers' weight / bias gradients of the backward run inside; the caller
    calls ``flush()`` on the yielded queue after the backward (flush points flush earlier).
    ``deliver(param, grad)`` receives each parameter's gradient; with ``target(param)`` given (a
    tensor to add a finished gradient into, or None) a gradient may instead be added into that
    tensor in place, announced as ``deliver(param, None)``."""
    global _queue
    prev, _queue = _queue, _WgradQueue(deliver, target)
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


# (min_chunk, max_split) for weight gradients of at most _SPLITK_SMALL elements (e.g. 512 x 512: 8
# chunks of a 15,360-token K give only 8 x 32 output tiles; 16 chunks of 960: 889 vs 885 clips/s on
# the headline, two A/B pairs); MFL_SPLITK_SMALL="min,max" for A/B runs ("1024,8": the general rule)
_SPLITK = tuple(int(v) for v in os.environ.get("MFL_SPLITK_SMALL", "512,16").split(","))
_SPLITK_SMALL = 512 * 512


def split_k_chunks(k, min_chunk=1024, max_split=8):
    """Number of K chunks for the weight-gradient GEMM: the largest s <= max_split dividing K
    with K / s >= min_chunk (1 = no split)."""
    s = max_split
    while s > 1:
        if k % s == 0 and k // s >= min_chunk:
            return s
        s //= 2
    return 1


def _split_k_ragged(k, out_elems):
    """(s, r): s chunks of K // s rows (a power of two, the chunk sizes split_k_chunks asks for) and r
    leftover rows, for a K that split_k_chunks cannot divide; (1, 0) when not worth it."""
    min_chunk, max_split = _SPLITK if out_elems <= _SPLITK_SMALL else (1024, 8)
    s = max_split
    while s > 1 and k // s < min_chunk:
        s //= 2
    return (s, k - s * (k // s)) if s > 1 else (1, 0)


_dest = None  # flat_grad_destinations: {"views": {id(param): flat view}, "claimed": set(), ...}
# later products of a parameter added into the view / .grad in place (False: autograd's accumulation,
# for A/B tests)
ACCUMULATE_IN_PLACE = True
# a tagged activation's later consumer adds its input gradient into an earlier one's in its dgrad GEMM
# (mark_grad_sum; False: autograd's bf16 add, for A/B tests)
GRAD_SUM_IN_GEMM = True


@contextlib.contextmanager
def flat_grad_destinations(views, may_claim=None):
    """Inside (the trainer's backward): the first gradient produced for a parameter in ``views``
    ({id(param): its fp32 view of the flat gradient buffer}) is written straight into that view,
    which autograd then hands to the parameter as its .grad — instead of a fresh tensor copied
    into the flat buffer afterwards (one 171 MB copy pass per step at the bench shape).
    ``may_claim(param)``, when given, vetoes a view at the time it would be handed out (the
    trainer refuses the views of gradient buckets it has already all-reduced or is reducing).
    A parameter used several times in the backward (a module shared by several calls: the
    multimodal encoder's self-attention, the decoder's cross-attention over two memories): the
    later producers add their products into the view the first one handed to autograd
    (``_accum_target``) and return no gradient — autograd's accumulation into .grad happens only
    once all of them have run, so the view then holds the whole sum (the same sum, added in the
    same order: the products are formed first, then added)."""
    global _dest
    prev, _dest = _dest, {"views": views, "claimed": set(), "may_claim": may_claim, "returned": {}, "groups": {}}
    try:
        yield
    finally:
        _dest = prev


def _claim(param, returned=True):
    """The flat view ``param``'s gradient may be written into, or None: once per backward and
    only while the parameter has no gradient yet (a later producer's result is added by autograd,
    into that view or a copy of it, or added into the view itself: _accum_target).  ``returned``:
    the caller hands the view to autograd as the parameter's gradient (later producers may add
    into it until autograd has accumulated it)."""
    d = _dest
    if d is None or param is None or param.grad is not None:
        return None
    v = d["views"].get(id(param))
    if v is None or id(param) in d["claimed"]:
        return None
    if d["may_claim"] is not None and not d["may_claim"](param):
        return None
    d["claimed"].add(id(param))
    if returned:
        d["returned"][id(param)] = v
    return v.view_as(v)  # a fresh view object: autograd adopts it as .grad instead of cloning


def _accum_target(param):
    """The flat view an earlier producer of this backward wrote ``param``'s gradient into and handed
    to autograd, while autograd has not accumulated it yet (param.grad is None): a later producer
    adds its product into it in place and returns no gradient.  None otherwise."""
    d = _dest
    if d is None or param is None or param.grad is not None or not ACCUMULATE_IN_PLACE:
        return None
    v = d["returned"].get(id(param))
    if v is not None:
        from ... import _trace
        _trace.hit("grad_accum_view")
    return v


def _accum_group(params):
    """_accum_target for parameters claimed together (_claim_group): their one view, or None."""
    d = _dest
    if d is None or any(p.grad is not None for p in params) or not ACCUMULATE_IN_PLACE:
        return None
    v = d["groups"].get(tuple(id(p) for p in params))
    if v is not None:
        from ... import _trace
        _trace.hit("grad_accum_view")
    return v


def mark_grad_sum(x):
    """Declare that EVERY consumer of the 16-bit activation x hands its input gradient through
    grad_sum_mm / grad_sum_give (the multimodal encoder's bf16 streams: v16 is the value of one
    cross-modal call and the query of the other; an FFN input is linear1's input and the add +
    LayerNorm's residual).  In the trainer's backward a later consumer's dgrad GEMM then adds its
    product into the gradient an earlier consumer produced (C += dY W, one rounding of the fp32 sum)
    instead of autograd's separate bf16 add of the two (a read of both and a write per pair).
    Returns x."""
    if x is not None and x.is_cuda and x.is_contiguous() and x.dtype in (torch.bfloat16, torch.float16):
        x._mfl_gsum = True
    return x


def grad_sum_tagged(x):
    return bool(getattr(x, "_mfl_gsum", False))


_GSUM_DEBUG = os.environ.get("MFL_GSUM_DEBUG", "0") == "1"


def _gsum_registry():
    d = _dest
    if d is None or not GRAD_SUM_IN_GEMM:
        return None
    return d.setdefault("gsum", {})


def _gsum_key(x):
    return x if isinstance(x, tuple) else (x.data_ptr(), x.numel(), x.dtype)


def grad_sum_mm(tagged, x2, g2, w, x_shape):
    """A tagged (mark_grad_sum) input's gradient ``g2 @ w``: added in place into the gradient an
    earlier consumer of the same input produced and still holds pending in autograd (then None is
    returned: autograd gets no second gradient to add), else computed, registered for the later
    consumers and returned."""
    reg = _gsum_registry() if tagged else None
    if reg is None:
        return _mm_nn(g2, w).view(x_shape)
    k = _gsum_key(x2)
    t = reg.get(k)
    if _GSUM_DEBUG:
        print("grad_sum_mm", k[0] % 100000, k[1], "target" if t is not None else "none", flush=True)
    if t is not None and t.dtype == g2.dtype:
        from ... import _trace
        _trace.hit("grad_sum_into")
        t.view(-1, w.shape[1]).addmm_(g2, w)
        return None
    gx = _mm_nn(g2, w).view(x_shape)
    reg[k] = gx
    return gx


def grad_sum_give(tagged, x, g):
    """A consumer of tagged input x returning its gradient ``g`` to autograd as usual: g becomes the
    gradient later consumers add into — or, when an earlier consumer's is registered (autograd now
    adds the two out of place, leaving that tensor behind), the registration is dropped."""
    reg = _gsum_registry() if tagged else None
    if reg is None or g is None:
        return
    k = _gsum_key(x)  # (x: the input, or its key taken in the forward)
    if _GSUM_DEBUG:
        print("grad_sum_give", k[0] % 100000, k[1], "drop" if k in reg else "register", flush=True)
    if k in reg:
        del reg[k]
    elif g.is_contiguous() and g.dtype == k[2] and g.numel() == k[1]:
        reg[k] = g


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


def _claim_group(params, returned=True):
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
    g = base.new_empty(0).set_(base.untyped_storage(), base.storage_offset(), (rows,) + tuple(base.shape[1:]))
    if returned:
        for p, v in zip(params, views):
            d["returned"][id(p)] = v
        d["groups"][tuple(id(p) for p in params)] = g
    return g


def _bias_grad(g2, out=None, accumulate=False):
    """fp32 column sum of dY (K, N) through mfl_colsum (one streaming pass, fixed order);
    torch's column reduction where the kernel's layout conditions do not hold.  ``out``: an fp32
    (N,) destination (a flat-buffer view); ``accumulate``: added into it."""
    if g2.dtype not in (torch.bfloat16, torch.float16) or (g2.shape[1] * 2) % 16 or not g2.is_contiguous():
        r = g2.sum(0, dtype=torch.float32)
        if out is None:
            return r
        return out.add_(r) if accumulate else out.copy_(r)
    from ... import _native
    lib = _native.load_library()
    K, N = g2.shape
    if out is None:
        out = torch.empty(N, dtype=torch.float32, device=g2.device)
    ws = torch.empty(lib.mfl_colsum_workspace_bytes(K, N), dtype=torch.uint8, device=g2.device)
    rc = lib.mfl_colsum_ex(g2.data_ptr(), _native.DTYPE_TAGS[g2.dtype], K, N, out.data_ptr(), 1 if accumulate else 0,
                           ws.data_ptr(), _native.stream_handle(g2.device))
    if rc != 0:
        raise RuntimeError("mfl_colsum failed: " + lib.flat_adamw_last_error().decode())
    return out


def _sum_slabs(part, out=None, accumulate=False, groups=1):
    """part.sum(0) of the fp32 split-K partials (s, n_out, n_in) through mfl_sum_slabs (one pass,
    chunk order), into ``out`` if given (added into it with ``accumulate``).  ``groups`` > 1: part's
    groups * s slabs are ``groups`` consecutive runs of s, each summed into its own part of out
    (groups, n_out, n_in)."""
    s = part.shape[0] // groups
    n = part[0].numel()
    if n % 4 or not part.is_contiguous() or not part.is_cuda or (out is not None and not out.is_contiguous()):
        r = part.reshape(groups, s, -1).sum(1)
        r = r.view(part.shape[1:]) if groups == 1 else r.view((groups,) + tuple(part.shape[1:]))
        if out is None:
            return r
        return out.add_(r.view_as(out)) if accumulate else out.copy_(r.view_as(out))
    from ... import _native
    lib = _native.load_library()
    if out is None:
        out = torch.empty(((groups,) if groups > 1 else ()) + tuple(part.shape[1:]), dtype=torch.float32,
                          device=part.device)
    rc = lib.mfl_sum_slabs_ex(part.data_ptr(), groups, s, n, out.data_ptr(), 1 if accumulate else 0,
                              _native.stream_handle(part.device))
    if rc != 0:
        raise RuntimeError("mfl_sum_slabs failed: " + lib.flat_adamw_last_error().decode())
    return out


def _weight_grad(g2, x2, out=None, accumulate=False):
    """fp32 dW = dY^T X of 16-bit dY (K, N) and X (K, C): K split into chunks, one strided-batched
    GEMM with fp32 partial outputs, then their sum (into ``out`` if given; added into it with
    ``accumulate``)."""
    k, n_out, n_in = x2.shape[0], g2.shape[1], x2.shape[1]
    s = split_k_chunks(k, *_SPLITK) if n_out * n_in <= _SPLITK_SMALL else split_k_chunks(k)
    s2, r = _split_k_ragged(k, n_out * n_in)
    # an exact split at least half as wide as the ragged one is taken as it is: the ragged form's
    # leftover rows cost a GEMM launch of their own (the multimodal joint rows, K = 16,120 = 16 x 1,007
    # + 8: a (512 x 8) . (8 x 512) product at ~6 us, 36 a step; tools/splitk_probe.py)
    if s > 1 and not (s2 > 2 * s and g2.is_cuda):
        # (bmm, not baddbmm(out=part, beta=0): that form first copies `part` into the output — an
        # extra 8-32 MB pass per call, ~0.3 ms per step, tools/op_census.py)
        part = torch.bmm(g2.view(s, k // s, n_out).transpose(1, 2), x2.view(s, k // s, n_in),
                         out_dtype=torch.float32)
        return _sum_slabs(part, out, accumulate)
    s = s2
    if s > 1 and g2.is_cuda:
        # K not divisible by a useful chunk count (the multimodal encoder's joint rows: 16,120): s equal
        # chunks in one strided-batched GEMM plus the last r rows as one more slab, summed together
        c = k // s
        part = torch.empty((s + 1, n_out, n_in), dtype=torch.float32, device=g2.device)
        torch.bmm(g2[:s * c].view(s, c, n_out).transpose(1, 2), x2[:s * c].view(s, c, n_in), out_dtype=torch.float32,
                  out=part[:s])
        torch.mm(g2[s * c:].t(), x2[s * c:], out_dtype=torch.float32, out=part[s])
        return _sum_slabs(part, out, accumulate)
    r = torch.mm(g2.t(), x2, out_dtype=torch.float32)
    if out is None:
        return r
    return out.add_(r) if accumulate else out.copy_(r)


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
        ctx.gsum = grad_sum_tagged(x)
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
            gx = grad_sum_mm(ctx.gsum, x2, g2, wc, ctx.x_shape)
        if nig[1] and (not ctx.has_bias or nig[2]) and _defer((g2, x2, ctx.weight, 0, ctx.bias if ctx.has_bias else None,
                                                                cs)):
            return gx, None, None, None, None
        if nig[1]:
            acc = _accum_target(ctx.weight)  # (a shared layer: added into an earlier call's view)
            if acc is not None:
                _weight_grad(g2, x2, acc, accumulate=True)
            else:
                gw = _weight_grad(g2, x2, _claim(ctx.weight))
        if ctx.has_bias and nig[2]:
            acc = _accum_target(ctx.bias)
            if acc is not None:
                if cs is not None:
                    acc.add_(cs)
                else:
                    _bias_grad(g2, acc, accumulate=True)
            else:
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
        ctx.gsum = grad_sum_tagged(x)
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
        grad_sum_give(ctx.gsum, x2, gx)
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
