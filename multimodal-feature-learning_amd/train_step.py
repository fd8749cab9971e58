"""One data-parallel training step of the DVC core, MI355X-first.

The reference trains one process per GPU under DDP (main.py:55,98; engine.py:86-134):
forward, ``loss.backward()`` with the bucketed NCCL all-reduce overlapped, then
``clip_grad_norm_(max_norm)`` and the optimizer step.  Here the step is restructured for
the MI355X the way the hardware wants it:

* every gradient lives in ONE flat fp32 buffer (``p.grad`` are views into it, so autograd
  accumulates in place and there is nothing to copy in or out of buckets);
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

__all__ = ["FlatGradTrainer"]


class FlatGradTrainer:
    def __init__(self, model, loss_fn, lr=1e-4, weight_decay=1e-4, max_norm=0.1, use_bf16=True, graph=True,
                 process_group=None):
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
        n = sum(p.numel() for p in self.params)
        self.flat_grad = torch.zeros(n, dtype=torch.float32, device=dev)
        off = 0
        for p in self.params:
            if p.dtype != torch.float32:
                raise TypeError("FlatGradTrainer keeps fp32 master parameters; got " + str(p.dtype))
            p.grad = self.flat_grad[off:off + p.numel()].view_as(p)
            off += p.numel()
        self.opt = torch.optim.AdamW(self.params, lr=lr, weight_decay=weight_decay, capturable=graph,
                                     foreach=True)
        self._g_fb = None
        self._g_up = None
        self._loss = None

    # --- the three phases ------------------------------------------------------------
    def _forward_backward(self, batch, cache_casts=True):
        self.flat_grad.zero_()
        with torch.autocast(self.device.type, dtype=torch.bfloat16, enabled=self.use_bf16,
                            cache_enabled=cache_casts):
            out = self.model(*batch)
            loss = self.loss_fn(out)
        loss.backward()
        return loss.detach()

    def _allreduce(self):
        if self.world > 1:
            dist.all_reduce(self.flat_grad, group=self.pg)  # SUM: gloo has no AVG
            self.flat_grad.div_(self.world)

    def _update(self):
        torch.nn.utils.clip_grad_norm_(self.params, self.max_norm, foreach=True)
        self.opt.step()

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
