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
* between the two graphs the flat buffer is all-reduced with ONE RCCL call over xGMI
  (a single large collective instead of DDP's 25 MB buckets; 7 point-to-point xGMI links
  per GPU favour few large transfers).  The all-reduce is the only data-path collective:
  every MSDA call reads only its own clip, so the path shards by clip.

``graph=False`` runs the same three phases eagerly (CPU tests, world_size-2 gloo).
"""
import torch
import torch.distributed as dist

from .models.modules.linear import Linear

__all__ = ["FlatGradTrainer"]


class FlatGradTrainer:
    def __init__(self, model, loss_fn, lr=1e-4, weight_decay=1e-4, max_norm=0.1, use_bf16=True, graph=True,
                 process_group=None, fused_optimizer=None, betas=(0.9, 0.999), eps=1e-8, handover=True,
                 shadow=True):
        self.model = model
        self.loss_fn = loss_fn
        self.max_norm = max_norm
        self.use_bf16 = use_bf16
        self.graph = graph
        self.pg = process_group
        self.world = dist.get_world_size(process_group) if dist.is_available() and dist.is_initialized() else 1
        self.params = [p for p in model.parameters() if p.requires_grad]
        dev = self.params[0].device
        self.device = dev
        for p in self.params:
            if p.dtype != torch.float32:
                raise TypeError("FlatGradTrainer keeps fp32 master parameters; got " + str(p.dtype))
        n = sum(p.numel() for p in self.params)
        self.flat_param = torch.empty(n, dtype=torch.float32, device=dev)
        self.flat_grad = torch.zeros(n, dtype=torch.float32, device=dev)
        self.grad_views = []
        off = 0
        for p in self.params:
            k = p.numel()
            self.flat_param[off:off + k].copy_(p.detach().reshape(-1))
            p.data = self.flat_param[off:off + k].view_as(p)
            self.grad_views.append(self.flat_grad[off:off + k].view_as(p))
            off += k
        self._attach_grads()
        # bf16 weight shadow for the autocast Linear layers (one cast per step, _refresh_shadow)
        self.flat_bf16 = None
        self._linears = []
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
            self._refresh_shadow()
        self.lr, self.weight_decay, self.betas, self.eps = lr, weight_decay, betas, eps
        self.fused = (dev.type == "cuda") if fused_optimizer is None else bool(fused_optimizer)
        if self.fused:
            from . import _native
            self._lib = _native.load_library()
            self.exp_avg = torch.zeros_like(self.flat_param)
            self.exp_avg_sq = torch.zeros_like(self.flat_param)
            self.opt_step = torch.zeros(1, dtype=torch.float32, device=dev)
            self._opt_ws = torch.empty(self._lib.flat_adamw_workspace_bytes(), dtype=torch.uint8, device=dev)
            self.opt = None
        else:
            self.opt = torch.optim.AdamW(self.params, lr=lr, betas=betas, eps=eps, weight_decay=weight_decay,
                                         capturable=graph, foreach=True)
        self._g_fb = None
        self._g_up = None
        self._loss = None

    # --- the three phases ------------------------------------------------------------
    def _views(self, flat):
        out, off = [], 0
        for p in self.params:
            out.append(flat[off:off + p.numel()].view_as(p))
            off += p.numel()
        return out

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

    def _forward_backward(self, batch, cache_casts=True):
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
                            cache_enabled=cache_casts):
            out = self.model(*batch)
            loss = self.loss_fn(out)
        loss.backward()
        got = [(v, p.grad) for p, v in zip(self.params, self.grad_views) if p.grad is not None]
        missing = [v for p, v in zip(self.params, self.grad_views) if p.grad is None]
        if got:
            torch._foreach_copy_([v for v, _ in got], [g for _, g in got])
        if missing:
            torch._foreach_zero_(missing)
        self._attach_grads()
        return loss.detach()

    def _allreduce(self):
        if self.world > 1:
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
        rc = self._lib.flat_adamw_step(
            self.flat_param.data_ptr(), self.flat_grad.data_ptr(), self.exp_avg.data_ptr(), self.exp_avg_sq.data_ptr(),
            shadow, self.flat_param.numel(), self.opt_step.data_ptr(), self._opt_ws.data_ptr(), self.lr,
            self.betas[0], self.betas[1], self.eps, self.weight_decay, self.max_norm,
            _native.stream_handle(self.device))
        if rc != 0:
            raise RuntimeError("flat_adamw_step failed: " + self._lib.flat_adamw_last_error().decode())
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
        side = torch.cuda.Stream(self.device)
        side.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(side):
            for _ in range(warmup):
                self.eager_step(batch)
        torch.cuda.current_stream(self.device).wait_stream(side)
        torch.cuda.synchronize(self.device)
        self._g_fb = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self._g_fb):
            self._loss = self._forward_backward(batch, cache_casts=False)
        self._g_up = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self._g_up, pool=self._g_fb.pool()):
            self._update()
        torch.cuda.synchronize(self.device)

    def step(self, batch=None):
        """One training step; with graphs, replays on the current stream (batch is the
        static input given to capture())."""
        if not self.graph:
            return self.eager_step(batch)
        if self._g_fb is None:
            raise RuntimeError("FlatGradTrainer.capture(batch) must run before step()")
        self._g_fb.replay()
        self._allreduce()
        self._g_up.replay()
        return self._loss
