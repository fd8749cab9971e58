"""One data-parallel training step of the DVC core, MI355X-first.

The reference trains one process per GPU under DDP (main.py:55,98; engine.py:86-134):
forward, ``loss.backward()`` with the bucketed NCCL all-reduce overlapped, then
``clip_grad_norm_(max_norm)`` and the optimizer step.  Here the step is restructured for
the MI355X the way the hardware wants it:

* parameters and gradients each live in ONE flat fp32 buffer (``p`` and ``p.grad`` are views
  into them).  The backward starts with ``p.grad = None``, so autograd hands each parameter
  its freshly computed gradient without an accumulate kernel, and one multi-tensor copy
  moves them into the flat gradient buffer (instead of ~260 per-parameter add kernels);
* under bf16 autocast a bf16 shadow of the flat parameters is refreshed after every optimizer
  step, and the Linear layers read their bf16 weights from it (instead of ~200 per-use weight /
  bias casts, models/modules/linear.py);
* on the GPU, clip_grad_norm_ + AdamW + the shadow refresh are ONE pass over the flat buffers
  (csrc/flat_adamw.hip, three kernels) instead of torch's foreach AdamW over 260 tensors, whose
  capturable path also launches ~520 per-tensor division kernels (~3.5 ms of a 21 ms step);
* the forward+backward and the clip+AdamW halves are each captured once into a HIP graph
  and replayed — the ~1500 kernels of a step are launched by two ``hipGraphLaunch`` calls
  instead of ~1500 Python-driven launches (the eager step is launch-bound: its GPU is idle
  for about a quarter of the step, profiles/);
* with several ranks the flat gradient is all-reduced in a few large buckets (contiguous ranges
  of the flat buffer in reverse parameter order, ``bucket_mb`` each: 7 point-to-point xGMI
  links per GPU favour few large transfers over DDP's 25 MB) overlapped with the backward: a
  parameter's post-accumulate-grad hook hands its gradient to the bucket, and a bucket whose
  gradients are all final is copied into the flat buffer and all-reduced on a side stream while
  autograd computes the earlier layers (the reference's DDP overlap, main.py:85).  Under graphs
  the bucket collectives are captured with the backward (``capture_collectives``; otherwise one
  all-reduce runs between the two graphs).  The all-reduce is the only data-path collective:
  every MSDA call reads only its own clip, so the path shards by clip.

``graph=False`` runs the same three phases eagerly (CPU tests, world_size-2 gloo).
"""
import os
import time

import torch
import torch.distributed as dist

from .models.modules.add_norm import seed_pool
from .models.modules.linear import Linear, deferred_weight_grads, flat_grad_destinations

__all__ = ["FlatGradTrainer"]


def _flat_order(model, params):
    """``params`` in model order, except that the groups modules ask to be adjacent
    (``flat_groups()``, e.g. MSDeformAttn's two query projections) are laid out back to back where
    the group's first member stands: their views into the flat buffers (fp32 values / gradients,
    bf16 shadow) are then consecutive, and a fused kernel reads them as one tensor."""
    follow = {}
    for mod in model.modules():
        groups = getattr(mod, "flat_groups", None)
        if callable(groups):
            for g in groups():
                if all(p.requires_grad for p in g) and all(id(p) not in follow for p in g):
                    follow[id(g[0])] = list(g)
                    for p in g[1:]:
                        follow[id(p)] = None
    out, seen = [], set()
    for p in params:
        if id(p) in seen:
            continue
        grp = follow.get(id(p), [p]) if id(p) in follow else [p]
        if grp is None:  # placed with its group's first member
            continue
        for q in grp:
            if id(q) not in seen:
                seen.add(id(q))
                out.append(q)
    for p in params:  # a member whose group leader is absent (frozen) keeps its place at the end
        if id(p) not in seen:
            seen.add(id(p))
            out.append(p)
    return out


_CAPTURE_GROUPS = {}


def _capture_group(pg, device):
    """The process group the captured bucket all-reduces run on: the trainer's group's ranks again, as a
    group that runs nothing eagerly but its first collective (one per (group, device) for the process).

    The RCCL process group's watchdog thread polls the end event of every eager collective
    (WorkNCCL::isCompleted -> hipEventQuery) until it retires it, ~100 ms later.  HIP refuses that query
    (hipErrorCapturedEvent, and invalidates the capture) whenever the stream the event was recorded on
    is capturing at the time of the query — even for an event recorded and completed before the capture
    began (tools/probes/event_capture_probe.py) — and the watchdog takes the refusal as fatal.  A
    blocking collective runs on, and records its end event on, the CURRENT stream; so no stream that
    carries an eager collective may ever capture: the trainer's warm-up, its captures, its
    eager and its captured bucket collectives each run on a stream of their own (``_native.own_stream``),
    and the captured collectives on this group, whose NCCL stream (high-priority pool) no eager
    collective of the trainer's group uses.  Its first collective, which connects the communicator, runs
    eagerly on the caller's current stream, which never captures."""
    key = (id(pg), device.index)
    grp = _CAPTURE_GROUPS.get(key)
    if grp is None:
        ranks = dist.get_process_group_ranks(pg if pg is not None else dist.group.WORLD)
        opts = dist.ProcessGroupNCCL.Options()
        opts.is_high_priority_stream = True
        grp = dist.new_group(ranks, backend="nccl", pg_options=opts, device_id=device)
        dist.all_reduce(torch.zeros(64, dtype=torch.float32, device=device), group=grp)  # (connects it)
        torch.cuda.synchronize(device)
        _CAPTURE_GROUPS[key] = grp
    return grp


def _record(events):
    e = torch.cuda.Event(enable_timing=True)
    e.record()
    return e


class FlatGradTrainer:
    def __init__(self, model, loss_fn, lr=1e-4, weight_decay=1e-4, max_norm=0.1, use_bf16=True, graph=True,
                 process_group=None, fused_optimizer=None, betas=(0.9, 0.999), eps=1e-8, handover=True,
                 shadow=True, bucket_mb=32.0, overlap=True, capture_collectives=None):
        self.model = model
        self.loss_fn = loss_fn
        self.max_norm = max_norm
        self.use_bf16 = use_bf16
        self.graph = graph
        self.pg = process_group
        self.world = dist.get_world_size(process_group) if dist.is_available() and dist.is_initialized() else 1
        self.params = _flat_order(model, [p for p in model.parameters() if p.requires_grad])
        dev = self.params[0].device
        self.device = dev
        for p in self.params:
            if p.dtype != torch.float32:
                raise TypeError("FlatGradTrainer keeps fp32 master parameters; got " + str(p.dtype))
        # every parameter starts on a 16-byte boundary (the 16-byte vector kernels that write weight
        # gradients straight into their views, linear.py _claim); the pad elements stay zero
        self._offs, n = [], 0
        for p in self.params:
            self._offs.append(n)
            n += (p.numel() + 3) // 4 * 4
        self.flat_param = torch.zeros(n, dtype=torch.float32, device=dev)
        self.flat_grad = torch.zeros(n, dtype=torch.float32, device=dev)
        self.grad_views = []
        for p, off in zip(self.params, self._offs):
            k = p.numel()
            self.flat_param[off:off + k].copy_(p.detach().reshape(-1))
            p.data = self.flat_param[off:off + k].view_as(p)
            self.grad_views.append(self.flat_grad[off:off + k].view_as(p))
        self._attach_grads()
        # the flat views the large weight-gradient GEMMs write into directly (linear.py, _claim)
        self._grad_dest = {id(p): v for p, v in zip(self.params, self.grad_views)}
        # bf16 weight shadow for the autocast Linear layers (one cast per step, _refresh_shadow)
        self.flat_bf16 = None
        self._linears = []
        self._mhas = []
        self.handover = handover
        if use_bf16 and dev.type == "cuda" and shadow:
            self.flat_bf16 = self.flat_param.to(torch.bfloat16)
            index = {id(p): v for p, v in zip(self.params, self._views(self.flat_bf16))}
            for mod in model.modules():
                if isinstance(mod, Linear) and id(mod.weight) in index:
                    b = index.get(id(mod.bias)) if mod.bias is not None else None
                    if mod.bias is not None and b is None:
                        continue
                    self._linears.append((mod, index[id(mod.weight)], b))
                elif (isinstance(mod, torch.nn.MultiheadAttention) and mod.in_proj_weight is not None
                      and id(mod.in_proj_weight) in index and mod.in_proj_bias is not None
                      and id(mod.in_proj_bias) in index and id(mod.out_proj.weight) in index
                      and mod.out_proj.bias is not None and id(mod.out_proj.bias) in index):
                    # the decoder's query self-attention (attention.py::mha_self_attention) reads these
                    self._mhas.append((mod, index[id(mod.in_proj_weight)], index[id(mod.in_proj_bias)],
                                       index[id(mod.out_proj.weight)], index[id(mod.out_proj.bias)]))
            self._refresh_shadow()
        self.betas, self.eps = betas, eps
        self.fused = (dev.type == "cuda") if fused_optimizer is None else bool(fused_optimizer)
        # lr / weight_decay live in device memory read by the update kernels, so a replayed graph
        # uses the current values (setting trainer.lr between replays is a schedule step)
        self._lr_wd = torch.tensor([lr, weight_decay], dtype=torch.float32, device=dev)
        self._lr, self._wd = float(lr), float(weight_decay)
        if self.fused:
            from . import _native
            self._lib = _native.load_library()
            self.exp_avg = torch.zeros_like(self.flat_param)
            self.exp_avg_sq = torch.zeros_like(self.flat_param)
            self.opt_step = torch.zeros(1, dtype=torch.float32, device=dev)
            self._opt_ws = torch.empty(self._lib.flat_adamw_workspace_bytes(), dtype=torch.uint8, device=dev)
            self.opt = None
        else:
            # a tensor lr under graphs: the captured step reads it (schedules fill it in place)
            lr0 = torch.tensor(float(lr), device=dev) if graph else lr
            self.opt = torch.optim.AdamW(self.params, lr=lr0, betas=betas, eps=eps, weight_decay=weight_decay,
                                         capturable=graph, foreach=True)
        # a loss with a host step inside the forward (the DVC step's Hungarian matching): an object
        # with stage_a(model, batch) -> state, request(state) -> device tensor for the host,
        # host(state, cpu_tensor), upload() (stream-ordered H2D copies into its static device
        # buffers) and stage_b(model, batch, state) -> loss.  Captured as two graphs around the
        # host step (capture()).
        self.staged = all(hasattr(loss_fn, a) for a in ("stage_a", "request", "host", "upload", "stage_b"))
        self._g_a = None
        self._stage_state = None
        self._request_like = None
        self._request_host = None
        self.phase_events = None  # a list: step() appends (name, start, end) HIP events per phase
        self._g_fb = None
        self._g_up = None
        self._loss = None
        # gradient buckets: contiguous flat ranges, reverse parameter order (the backward's order)
        self.buckets = self._make_buckets(int(bucket_mb * 2 ** 20 / 4))
        # overlap="force": the bucket collectives also at world size 1 (a one-rank RCCL smoke)
        self.overlap = handover and (overlap == "force" or (bool(overlap) and self.world > 1))
        backend = dist.get_backend(process_group) if dist.is_available() and dist.is_initialized() else None
        self.capture_collectives = (backend == "nccl") if capture_collectives is None else bool(capture_collectives)
        self._comm_stream = None
        self._pending = None
        self._overlap_now = self.overlap  # eager steps; capture() decides for the graph
        self._fb_reduces = False          # the captured fwd+bwd graph all-reduces the buckets
        self._capturing_now = False       # inside capture()'s fwd+bwd graph capture
        self._capture_pg = None           # the group of the captured bucket all-reduces (_capture_group)
        # parameters that no rank gave a gradient are left untouched, as torch AdamW leaves a
        # parameter whose grad is None (reference DDP find_unused_parameters=True, main.py:85):
        # found again after every eager step; the captured graphs keep the set of their capture
        # (a replay runs the captured kernels, so which parameters get gradients cannot change)
        self._got = [False] * len(self.params)
        self._unused = None
        self._frozen = None       # (views of their values / moments / shadow, scratch copies)
        self._frozen_keep = []    # earlier scratch sets, alive while a captured graph may read them
        self._late = False
        self._late_parts = {}       # param index -> local gradient that arrived after its bucket's reduce
        self._late_global = False   # some rank had a late gradient on the last eager step
        self._bucket_of = {}
        for bi, (_, _, idx) in enumerate(self.buckets):
            for i in idx:
                self._bucket_of[i] = bi
        self._index = {id(p): i for i, p in enumerate(self.params)}
        self._hooks = {}
        if self.overlap:
            for i, p in enumerate(self.params):
                self._hooks[i] = self._make_hook(i)
                p.register_post_accumulate_grad_hook(self._hooks[i])

    # --- gradient buckets ----------------------------------------------------------------
    def _make_buckets(self, cap_elems):
        """[(start, end, [param index, ...]), ...]: consecutive parameters from the last one
        backwards, each bucket a contiguous range of the flat buffer of at most cap_elems elements
        (or one parameter larger than that)."""
        offs = self._offs
        buckets, cur, cur_n = [], [], 0
        for i in reversed(range(len(self.params))):
            n = (self.params[i].numel() + 3) // 4 * 4  # its span in the flat buffer (16-B aligned)
            if cur and cur_n + n > cap_elems:
                buckets.append(cur)
                cur, cur_n = [], 0
            cur.append(i)
            cur_n += n
        if cur:
            buckets.append(cur)
        out = []
        for idx in buckets:
            lo, hi = min(idx), max(idx)
            end = offs[hi + 1] if hi + 1 < len(offs) else self.flat_grad.numel()  # (with the 16-B pad)
            out.append((offs[lo], end, sorted(idx)))
        return out

    def _make_hook(self, i):
        def hook(p):
            if self._pending is None:  # backward outside _forward_backward (user code): nothing to do
                return
            if p.grad is None:
                # autograd runs the hook for an input whose backward returned no gradient (a deferred
                # weight gradient, delivered later by _deliver): nothing arrived yet
                return
            if not self._overlap_now:  # every bucket is copied once after the backward
                self._got[i] = True
                return
            b = self._bucket_of[i]
            if b < self._next_flush:
                # a gradient for a parameter whose bucket is reduced already (one found unused last
                # step): kept aside and reduced after the backward (_find_unused).  It is a local
                # tensor: the reduced bucket's views are never handed out (_may_claim)
                if p.grad.data_ptr() == self.grad_views[i].data_ptr():
                    raise RuntimeError("FlatGradTrainer: a reduced bucket's gradient view was written")
                # p.grad holds only what arrived since the flush (_flush_bucket released the copied
                # part): keep it aside and release it too, so a further late gradient is again
                # just its own increment
                self._late_add(i, p.grad)
                p.grad = None
                return
            first = not self._got[i]
            self._got[i] = True
            if not first or i in self._known_unused:
                # a second gradient (added into p.grad before the flush), or a parameter the bucket
                # does not wait for: either way the bucket's copy takes p.grad as it stands
                return
            self._pending[b] -= 1
            if self._pending[b] == 0:
                self._ready[b] = True
                self._flush_ready()
        return hook

    def _flush_ready(self):
        """Reduce the complete buckets in index order: every rank issues the same collectives in
        the same order and sizes, whatever order its backward completes them in (DDP's bucket
        order; a bucket waiting on a late parameter holds back the ones after it)."""
        while self._next_flush < len(self.buckets) and self._ready[self._next_flush]:
            self._flush_bucket(self._next_flush)
            self._next_flush += 1

    def _flush_bucket(self, b):
        start, end, idx = self.buckets[b]
        for i in idx:
            if self.params[i].grad is not None:
                self._got[i] = True
        got = [(self.grad_views[i], self.params[i].grad) for i in idx if self.params[i].grad is not None
               and self.params[i].grad.data_ptr() != self.grad_views[i].data_ptr()]  # (written in place)
        missing = [self.grad_views[i] for i in idx if self.params[i].grad is None]
        if got:
            torch._foreach_copy_([v for v, _ in got], [g for _, g in got])
        if missing:
            torch._foreach_zero_(missing)
        if self._pending is not None:
            # inside the backward: the copied gradients are released, so a gradient that arrives
            # for one of these parameters after the reduce (autograd's accumulation after a deferred
            # delivery, or a parameter found unused last step) reaches the hook as its increment
            # alone, never as a running total whose copied part would be reduced twice.
            # (_attach_grads hands the flat views back after the backward.)
            for i in idx:
                self.params[i].grad = None
        if self._overlap_now:
            cur = torch.cuda.current_stream(self.device) if self.device.type == "cuda" else None
            if cur is not None:
                from . import _native
                # eager and captured collectives on streams of their own, the captured ones on the
                # capture-only group: no stream that carries an eager collective ever captures
                # (_capture_group)
                captured = self._capturing_now and self._capture_pg is not None
                self._comm_stream = _native.own_stream(self.device, "comm_capture" if captured else "comm")
                self._comm_stream.wait_stream(cur)
                with torch.cuda.stream(self._comm_stream):
                    dist.all_reduce(self.flat_grad[start:end], group=self._capture_pg if captured else self.pg)
            else:
                self._works.append(dist.all_reduce(self.flat_grad[start:end], group=self.pg, async_op=True))

    @property
    def lr(self):
        return self._lr

    @lr.setter
    def lr(self, value):
        self._lr = float(value)
        self._lr_wd[0] = self._lr  # in place: the captured update graph reads it
        if self.opt is not None:
            for group in self.opt.param_groups:
                if torch.is_tensor(group["lr"]):
                    group["lr"].fill_(self._lr)
                else:
                    group["lr"] = self._lr

    @property
    def weight_decay(self):
        return self._wd

    @weight_decay.setter
    def weight_decay(self, value):
        if self.opt is not None and self._g_up is not None and float(value) != self._wd:
            # torch AdamW reads weight_decay as a Python float: the captured update graph has the
            # capture's value baked in (the fused update reads it from device memory instead)
            raise RuntimeError("FlatGradTrainer: weight_decay cannot change after capture() with the torch AdamW "
                               "update (fused_optimizer=False); capture again or use the fused update")
        self._wd = float(value)
        self._lr_wd[1] = self._wd
        if self.opt is not None:
            for group in self.opt.param_groups:
                group["weight_decay"] = self._wd

    # --- the three phases ------------------------------------------------------------
    def _views(self, flat):
        return [flat[off:off + p.numel()].view_as(p) for p, off in zip(self.params, self._offs)]

    def _attach_grads(self):
        for p, g in zip(self.params, self.grad_views):
            p.grad = g

    def _refresh_shadow(self, copy=True):
        """bf16 copy of every parameter (one kernel, or already written by the fused optimizer);
        Linear layers use it while their fp32 weight's version counter still matches (any other
        in-place change disables it)."""
        if self.flat_bf16 is None:
            return
        if copy:
            self.flat_bf16.copy_(self.flat_param)
        for mod, w, b in self._linears:
            mod.set_bf16_shadow(w, b)
        for mod, w, b, ow, ob in self._mhas:
            mod._mfl_shadow = (w, b, ow, ob, mod.in_proj_weight._version, mod.out_proj.weight._version)

    def _forward_backward(self, batch, cache_casts=True, stage_state=None):
        if not self.handover and self.staged:
            raise ValueError("FlatGradTrainer: a staged loss needs handover=True")
        if not self.handover:  # accumulate into the zeroed flat buffer (one add kernel per parameter)
            self.flat_grad.zero_()
            with torch.autocast(self.device.type, dtype=torch.bfloat16, enabled=self.use_bf16,
                                cache_enabled=cache_casts):
                loss = self.loss_fn(self.model(*batch))
            loss.backward()
            return loss.detach()
        for p in self.params:  # autograd then hands over fresh gradients (no accumulate kernels)
            p.grad = None
        with torch.autocast(self.device.type, dtype=torch.bfloat16, enabled=self.use_bf16,
                            cache_enabled=cache_casts), seed_pool(self.device):
            if not self.staged:
                out = self.model(*batch)
                loss = self.loss_fn(out)
            else:  # a host step inside the forward (staged loss, see capture())
                if stage_state is None:
                    stage_state = self.loss_fn.stage_a(self.model, batch)
                    req = self.loss_fn.request(stage_state)
                    self._request_like = (tuple(req.shape), req.dtype)
                    self.loss_fn.host(stage_state, req.cpu())  # the step's host synchronisation
                    self.loss_fn.upload()
                loss = self.loss_fn.stage_b(self.model, batch, stage_state)
        capturing = self.device.type == "cuda" and torch.cuda.is_current_stream_capturing()
        # parameters found unused (by every rank, last step) do not hold their buckets back
        self._known_unused = frozenset(self._unused or ())
        self._got = [False] * len(self.params)
        self._pending = [sum(1 for i in idx if i not in self._known_unused) for _, _, idx in self.buckets]
        self._ready = [n == 0 for n in self._pending]
        self._next_flush = 0
        self._late = False
        self._late_parts = {}
        self._works = []
        try:
            # the short-K layers' weight gradients are batched (models/modules/linear.py) and
            # handed over by _deliver, at the model's flush points or after the backward
            with deferred_weight_grads(self._deliver, self._accum_target) as queue, \
                    flat_grad_destinations(self._grad_dest, self._may_claim):
                self._flush_ready()
                loss.backward()  # overlap: complete buckets are copied and all-reduced from the hooks, in order
                queue.flush()
        finally:
            self._pending = None
        self._ready = [True] * len(self.buckets)  # buckets with parameters that got no gradient
        self._flush_ready()
        if self._overlap_now:
            if self._comm_stream is not None:
                torch.cuda.current_stream(self.device).wait_stream(self._comm_stream)
            for w in self._works:
                w.wait()
            self._works = []
        if not capturing:
            self._find_unused()  # also reduces again if any rank had a late gradient
        if self._overlap_now:
            self.flat_grad.div_(self.world)
        self._attach_grads()
        if self._unused and self.opt is not None:
            for i in self._unused:  # torch AdamW skips a parameter whose grad is None
                self.params[i].grad = None
        return loss.detach()

    def _may_claim(self, p):
        """Whether the backward may write p's gradient straight into its flat view (linear._claim):
        not once p's bucket is reduced (or being reduced on the comm stream), and not for a
        parameter found unused, which its bucket does not wait for (the bucket could be copied and
        reduced, the view zeroed, while the producing kernel is still queued)."""
        if not self._overlap_now or self._pending is None:
            return True
        i = self._index.get(id(p))
        return i is None or (i not in self._known_unused and self._bucket_of[i] >= self._next_flush)

    def _late_add(self, i, grad):
        self._late = True
        self._got[i] = True
        prev = self._late_parts.get(i)
        self._late_parts[i] = grad if prev is None else prev + grad

    def _reduced(self, p):
        """Whether p's bucket is reduced (or being reduced) already in this backward."""
        i = self._index.get(id(p))
        return (i is not None and self._pending is not None and self._overlap_now
                and self._bucket_of[i] < self._next_flush)

    def _accum_target(self, p):
        """Where a batched gradient for p may be added in place (linear._WgradQueue): p.grad while
        p's bucket is not reduced, else None."""
        g = p.grad
        if g is None or self._reduced(p) or g.dtype != torch.float32 or g.shape != p.shape or not g.is_contiguous():
            return None
        return g

    def _deliver(self, p, grad):
        """A batched weight / bias gradient for parameter p: set (or added to) p.grad, then the
        parameter's post-accumulate step (bucket hand-over) as autograd's hook would run it.  Once
        p's bucket is reduced, the gradient is kept aside instead (never added into the reduced
        view, which the comm stream may still be reading).  grad None: the queue already added it
        into p.grad (_accum_target)."""
        i = self._index.get(id(p))
        if grad is not None and self._reduced(p):
            self._late_add(i, grad)
            return
        if grad is None:
            pass
        elif p.grad is None:
            p.grad = grad
        else:
            p.grad.add_(grad)
        if i is not None and i in self._hooks:
            self._hooks[i](p)

    def _find_unused(self):
        """After an eager backward: the parameters no rank gave a gradient (one small MAX all-reduce
        of the per-parameter flags at world size > 1, which also carries the late-gradient flag).
        The fused update leaves their values, moments and bf16 shadow as they were before it (saved
        and restored around the update kernels, captured with the update graph), so weight decay
        never touches them.  A step on which some rank gave a gradient to a parameter found unused
        before, or a gradient delivered after its bucket was reduced, has those late gradients
        (kept aside by _late_add) summed over ranks in one more all-reduce, which every rank joins,
        and added to the reduced buffer."""
        flags = [1 if g else 0 for g in self._got] + [1 if self._late else 0]
        if self.world > 1:
            t = torch.tensor(flags, dtype=torch.int32, device=self.device)
            dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.pg)
            flags = t.tolist()
        self._late_global = bool(flags[-1])
        if flags[-1] and self._overlap_now:
            late = torch.zeros_like(self.flat_grad)
            for i, g in self._late_parts.items():
                off = self._offs[i]
                late[off:off + g.numel()].copy_(g.reshape(-1))
            dist.all_reduce(late, group=self.pg)
            self.flat_grad.add_(late)
        self._late_parts = {}
        unused = [i for i, g in enumerate(flags[:-1]) if g == 0]
        if unused == self._unused:
            return
        self._unused = unused
        if self._frozen is not None:
            self._frozen_keep.append(self._frozen)
        self._frozen = None
        if not unused or self.opt is not None:
            return
        views = []
        flats = [self.flat_param, self.exp_avg, self.exp_avg_sq] + ([self.flat_bf16] if self.flat_bf16 is not None
                                                                     else [])
        offs = self._offs
        for i in unused:
            n = self.params[i].numel()
            views.extend(f[offs[i]:offs[i] + n] for f in flats)
        self._frozen = (views, [torch.empty_like(v) for v in views])

    def _allreduce(self):
        if self.world > 1 and not self._overlap_now:
            dist.all_reduce(self.flat_grad, group=self.pg)  # SUM: gloo has no AVG
            self.flat_grad.div_(self.world)

    def _update(self):
        if not self.fused:
            torch.nn.utils.clip_grad_norm_(self.params, self.max_norm, foreach=True)
            self.opt.step()
            self._refresh_shadow()
            return
        from . import _native
        shadow = self.flat_bf16.data_ptr() if self.flat_bf16 is not None else None
        if self._frozen is not None:  # parameters without gradients: saved before, restored after
            torch._foreach_copy_(self._frozen[1], self._frozen[0])
        rc = self._lib.flat_adamw_step(
            self.flat_param.data_ptr(), self.flat_grad.data_ptr(), self.exp_avg.data_ptr(), self.exp_avg_sq.data_ptr(),
            shadow, self.flat_param.numel(), self.opt_step.data_ptr(), self._opt_ws.data_ptr(), self._lr,
            self.betas[0], self.betas[1], self.eps, self._wd, self.max_norm, self._lr_wd.data_ptr(),
            _native.stream_handle(self.device))
        if rc != 0:
            raise RuntimeError("flat_adamw_step failed: " + self._lib.flat_adamw_last_error().decode())
        if self._frozen is not None:  # values, moments and shadow as before the update
            torch._foreach_copy_(self._frozen[0], self._frozen[1])
        self._refresh_shadow(copy=False)

    # --- public -------------------------------------------------------------------------
    def eager_step(self, batch):
        loss = self._forward_backward(batch)
        self._allreduce()
        self._update()
        return loss

    def capture(self, batch, warmup=3):
        """Warm up on a side stream (lazy optimizer state, BLAS / MIOpen plans, the MSDA
        library's LDS attributes), then capture fwd+bwd and clip+AdamW as two graphs.
        ``batch`` tensors are the graph's static inputs: refill them in place to change data."""
        if not self.graph:
            return
        if warmup < 1:  # the eager warm-up finds the unused parameters the graphs keep (_find_unused)
            raise ValueError("FlatGradTrainer.capture: warmup must be >= 1")
        import importlib
        pkg = importlib.import_module(__name__.rsplit(".", 1)[0])
        if not pkg.graph_packet_capture_off():
            raise RuntimeError(
                "FlatGradTrainer.capture: the HIP runtime's graph packet capture is on "
                "(DEBUG_CLR_GRAPH_PACKET_CAPTURE must be '0' before HIP initialises: import the package "
                "before any device call, or export the variable); with it on, replays after allocating "
                "eager work produced corrupted gradients (DESIGN.md §6)")
        from . import _native
        # the warm-up and the captures run on the package's own stream: never a pool stream that the
        # RCCL process group's NCCL stream can be; the warm-up's eager collectives on another stream than
        # the captures (_capture_group)
        side = _native.own_stream(self.device, "capture")
        warm = _native.own_stream(self.device, "warmup")
        warm.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(warm):
            for _ in range(warmup):
                self.eager_step(batch)
        torch.cuda.current_stream(self.device).wait_stream(warm)
        torch.cuda.synchronize(self.device)
        side.wait_stream(torch.cuda.current_stream(self.device))
        # capture_error_mode "thread_local": the RCCL process group's watchdog thread polls the
        # events of the warm-up collectives (hipEventQuery) while this thread captures; under the
        # default global mode that poll is refused.  Those events sit on streams that never capture,
        # and the captured collectives run on a group of their own (_capture_group)
        pool = None
        if (self.overlap and self.capture_collectives and not self._late_global and dist.is_available()
                and dist.is_initialized() and dist.get_backend(self.pg) == "nccl"):
            self._capture_pg = _capture_group(self.pg, self.device)
        if self.staged:
            # graph A: the forward up to the host step and the copy of its request into pinned
            # host memory; graph B (same memory pool) runs the rest of the forward and the whole
            # backward, through graph A's autograd nodes, whose saved tensors A refreshes in place
            shape, dtype = self._request_like  # from the eager warm-up
            self._request_host = torch.empty(shape, dtype=dtype, device="cpu").pin_memory()
            self._g_a = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self._g_a, stream=side, capture_error_mode="thread_local"):
                with torch.autocast(self.device.type, dtype=torch.bfloat16, enabled=self.use_bf16,
                                    cache_enabled=False), seed_pool(self.device):
                    self._stage_state = self.loss_fn.stage_a(self.model, batch)
                self._request_host.copy_(self.loss_fn.request(self._stage_state), non_blocking=True)
            pool = self._g_a.pool()
        self._g_fb = torch.cuda.CUDAGraph()
        # a step with late gradients (the last warm-up step had one on some rank) needs the extra
        # reduce decided on the host after the backward: such a step is captured with one
        # all-reduce between the two graphs instead of the overlapped bucket collectives
        self._overlap_now = self.overlap and self.capture_collectives and not self._late_global
        try:
            self._capturing_now = True
            with torch.cuda.graph(self._g_fb, pool=pool, stream=side, capture_error_mode="thread_local"):
                self._loss = self._forward_backward(batch, cache_casts=False, stage_state=self._stage_state)
        finally:
            self._capturing_now = False
            self._fb_reduces, self._overlap_now = self._overlap_now, self.overlap
        if self._fb_reduces and self._late:
            # (the captured bucket reduces would replay without this rank's late gradients)
            raise RuntimeError("FlatGradTrainer.capture: a gradient arrived after its bucket was reduced inside the "
                               "captured backward; capture with capture_collectives=False")
        self._g_up = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self._g_up, pool=self._g_fb.pool(), stream=side, capture_error_mode="thread_local"):
            self._update()
        torch.cuda.synchronize(self.device)

    def step(self, batch=None):
        """One training step; with graphs, replays on the current stream (batch is the
        static input given to capture())."""
        if not self.graph:
            return self.eager_step(batch)
        if self._g_fb is None:
            raise RuntimeError("FlatGradTrainer.capture(batch) must run before step()")
        ev = self.phase_events
        mark = (lambda: None) if ev is None else (lambda: _record(ev))
        t0 = mark()
        if self.staged:
            self._g_a.replay()
            t1 = mark()
            c0 = time.perf_counter()
            torch.cuda.current_stream(self.device).synchronize()  # the request is in pinned memory
            c1 = time.perf_counter()
            self.loss_fn.host(self._stage_state, self._request_host)
            c2 = time.perf_counter()
            self.loss_fn.upload()
            t2 = mark()
            if ev is not None:
                ev.append(("graph A: forward to the host step", t0, t1))
                ev.append(("host step (device->host wait, host work, upload)", t1, t2))
                # host clock: the wait for graph A (its launch returns before the GPU finishes it) and
                # the host work alone
                ev.append(("host: synchronize (ms, host clock)", c0, c1))
                ev.append(("host: matching + index lists (ms, host clock)", c1, c2))
            t0 = t2
        self._g_fb.replay()
        t1 = mark()
        if not self._fb_reduces:
            self._overlap_now = False
            self._allreduce()  # one all-reduce between the two graphs
            self._overlap_now = self.overlap
        self._g_up.replay()
        if ev is not None:
            ev.append(("graph B: rest of forward + backward" if self.staged else "forward + backward", t0, t1))
            ev.append(("all-reduce + clip + AdamW", t1, mark()))
        return self._loss
