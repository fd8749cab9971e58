"""Host side of the MSDA hot path: tensor checks, layout normalisation, the C-ABI calls
and the autograd.Function.

Semantics follow the reference's live core ``ms_deform_attn_core_pytorch``
(models/modules/attention.py:331-383, padding "border") or its dormant CUDA extension
(models/ops/src/cuda/ms_deform_im2col_cuda.cuh, padding "zeros").  There is no CPU
path: a non-ROCm tensor raises, like the reference extension's CPU stub
(models/ops/src/cpu/ms_deform_attn_cpu.cpp:17-41).
"""
import functools

import torch
from torch.autograd import Function
from torch.autograd.function import once_differentiable

from . import _native

__all__ = [
    "host_levels", "msda_forward", "msda_backward", "MSDAFunction", "msda_apply", "KernelTimer",
    "algorithmic_bytes", "gathered_bytes", "prologue_supported", "prologue_forward", "prologue_backward", "MSDAPrologueFunction",
    "msda_prologue_apply", "level_major_ok", "LEVEL_MAJOR",
]

LEVEL_MAJOR = 1  # coordinate layout tag (include/msda_hip.h MSDA_COORD_LEVEL_MAJOR): loc / aw (B, M, L, Lq, P)

_timer = None  # KernelTimer while bench.py measures; None otherwise


def gathered_bytes(B, M, D, Lq, L, P, value_bytes):
    """Row-fragment bytes one forward or fused-backward launch gathers: two taps of D values per
    sample (value rows in the forward, grad_out rows in the backward's pull)."""
    return B * Lq * M * L * P * 2 * D * value_bytes


def algorithmic_bytes(kind, B, S, M, D, Lq, L, P, value_bytes):
    """Algorithmic HBM bytes of one launch: every value / loc / aw / out
    element once; backward adds grad_out, the fp32 grad_value and grad_loc / grad_aw."""
    vals = B * S * M * D
    coords = 2 * B * Lq * M * L * P * 4
    rows = B * Lq * M * D
    if kind == "fwd":
        return vals * value_bytes + coords + rows * value_bytes
    return vals * value_bytes + rows * value_bytes + coords + vals * 4 + coords


class KernelTimer:
    """Brackets every MSDA C-ABI call with HIP events on the stream the kernel runs on
    (torch's current stream, which is what the C-ABI is given).  Records
    (kind, Lq, algorithmic bytes, start, end); read after a synchronize."""

    def __init__(self):
        self.records = []
        self.calls = {}

    def __enter__(self):
        global _timer
        _timer = self
        return self

    def __exit__(self, *exc):
        global _timer
        _timer = None
        return False

    # Eager steps are host-bound: an idle GPU would take the start event as soon as it is
    # queued and then wait for the host to issue the launch (the ctypes call), which inflates
    # the kernel time.  A short device spin queued first keeps the GPU busy until both the
    # event and the launch are queued, so the events bracket the kernel alone.
    SPIN_CYCLES = 200_000

    def _begin(self):
        try:
            torch.cuda._sleep(self.SPIN_CYCLES)
        except (AttributeError, RuntimeError):
            pass
        ev = torch.cuda.Event(enable_timing=True)
        ev.record()
        return ev

    def _end(self, kind, key, nbytes, ev0, gathered=0, call=None, keep=()):
        ev1 = torch.cuda.Event(enable_timing=True)
        ev1.record()
        self.records.append((kind, key, nbytes, gathered, ev0, ev1))
        if call is not None:
            self.calls[(kind, key)] = (call, keep)  # the last call of each shape, for burst()

    BURST = 20

    def burst(self, n=BURST):
        """Re-issue the last recorded C-ABI call of every (kind, shape) n times back to back between
        two events on the same stream: {(kind, key): average ms a launch}.  One pair of events around a
        single launch also holds the ~6 us between the start event and the kernel's dispatch (rocprof
        shows the gap); n launches in a row amortise it, so this average is the kernel's own duration
        (the outputs are rewritten with the same values)."""
        out = {}
        for k, (call, _keep) in self.calls.items():
            call()  # (warm)
            ev0 = self._begin()
            for _ in range(n):
                call()
            ev1 = torch.cuda.Event(enable_timing=True)
            ev1.record()
            out[k] = (ev0, ev1, n)
        torch.cuda.synchronize()
        return {k: ev0.elapsed_time(ev1) / n for k, (ev0, ev1, n) in out.items()}

    def summary(self):
        """{(kind, key): {"launches", "total_ms", "avg_ms", "bytes_per_launch", "gather_bytes_per_launch"}}"""
        out = {}
        for kind, key, nbytes, gathered, e0, e1 in self.records:
            d = out.setdefault((kind, key), {"launches": 0, "total_ms": 0.0, "bytes_per_launch": nbytes,
                                             "gather_bytes_per_launch": gathered})
            d["launches"] += 1
            d["total_ms"] += e0.elapsed_time(e1)
        for d in out.values():
            d["avg_ms"] = d["total_ms"] / d["launches"]
        return out


def _as_int_list(x):
    if isinstance(x, torch.Tensor):
        return [int(v) for v in x.reshape(-1).tolist()]  # device tensor => one host sync
    return [int(v) for v in x]


def host_levels(spatial_shapes, level_start_index=None):
    """Normalise level metadata to host tuples ``(T_l...), (start_l...)``.

    Accepts the forms the reference passes around: a (L,) tensor of T_l
    (unimodal_deformable_transformer.py:129), the (L,1) form of attention.py:495, the
    (L,2) ``[H, W]`` form of the 2-D extension API with H == 1
    (models/ops/modules/ms_deform_attn.py:117), or plain Python sequences.  A tensor
    carrying a ``_mfl_host`` attribute (set by this package's transformer) is read
    without touching the device.
    """
    cached = getattr(spatial_shapes, "_mfl_host", None)
    if cached is not None:
        shapes = tuple(cached)
    elif isinstance(spatial_shapes, torch.Tensor) and spatial_shapes.dim() == 2:
        if spatial_shapes.shape[1] == 1:
            shapes = tuple(_as_int_list(spatial_shapes[:, 0]))
        elif spatial_shapes.shape[1] == 2:
            hw = spatial_shapes.tolist()
            if any(int(h) != 1 for h, _ in hw):
                raise NotImplementedError(
                    "MSDA HIP kernel is temporal (1-D): 2-D spatial_shapes must have H == 1, got "
                    f"{hw}")
            shapes = tuple(int(w) for _, w in hw)
        else:
            raise ValueError(f"spatial_shapes must be (L,), (L,1) or (L,2); got {tuple(spatial_shapes.shape)}")
    else:
        shapes = tuple(_as_int_list(spatial_shapes))
    if level_start_index is None:
        starts, acc = [], 0
        for t in shapes:
            starts.append(acc)
            acc += t
        starts = tuple(starts)
    else:
        cached = getattr(level_start_index, "_mfl_host", None)
        starts = tuple(cached) if cached is not None else tuple(_as_int_list(level_start_index))
    if len(starts) != len(shapes):
        raise ValueError(f"level_start_index has {len(starts)} levels, spatial_shapes {len(shapes)}")
    return shapes, starts


def _coord_dtype(value):
    return torch.float64 if value.dtype == torch.float64 else torch.float32


def _coord_dims(loc, layout):
    """(Lq, M, L, P) of a coordinate tensor in the reference layout (B, Lq, M, L, P) or level-major
    (B, M, L, Lq, P)."""
    if layout == LEVEL_MAJOR:
        _, M, L, Lq, P = loc.shape
    else:
        _, Lq, M, L, P = loc.shape
    return Lq, M, L, P


def level_major_ok(value, shapes, Lq, P):
    """Whether an MSDA call on ``value`` (B, S, M, D) with Lq queries and P points may keep its
    coordinates level-major (msda_hip_level_major_ok: its backward takes the row-block path fed by
    the forward's tile intervals, and the prologue's level-major kernel covers it)."""
    import os
    if os.environ.get("MSDA_HIP_LEVEL_MAJOR", "1") == "0":  # A/B switch: the reference layout throughout
        return False
    if not value.is_cuda or value.dtype not in _native.DTYPE_TAGS or value.dim() != 4:
        return False
    B, S, M, D = value.shape
    lib = _native.load_library()
    return bool(lib.msda_hip_level_major_ok(_native.DTYPE_TAGS[value.dtype], _native.host_i64_array(shapes),
                                            len(shapes), B, S, M, D, Lq, P))


def _check_inputs(value, loc, aw, shapes, starts, layout=0):
    if value.dtype not in _native.DTYPE_TAGS:
        raise TypeError(f"MSDA: unsupported value dtype {value.dtype}")
    for name, t in (("value", value), ("sampling_loc", loc), ("attn_weight", aw)):
        if not t.is_cuda:
            raise RuntimeError(f"MSDA HIP kernel: {name} must be a ROCm device tensor (got {t.device}); "
                               "there is no CPU implementation")
        if not t.is_contiguous():
            raise ValueError(f"MSDA: {name} must be contiguous")
    if value.dim() != 4:
        raise ValueError(f"value must be (B, S, M, D); got {tuple(value.shape)}")
    B, S, M, D = value.shape
    if loc.dim() != 5 or aw.dim() != 5:
        raise ValueError(f"sampling_loc / attn_weight must be (B, Lq, M, L, P); got "
                         f"{tuple(loc.shape)} / {tuple(aw.shape)}")
    if tuple(loc.shape) != tuple(aw.shape):
        raise ValueError(f"sampling_loc {tuple(loc.shape)} and attn_weight {tuple(aw.shape)} differ")
    _, lm, ll, _ = _coord_dims(loc, layout)
    if loc.shape[0] != B or lm != M or ll != len(shapes):
        raise ValueError(f"shape mismatch: value {tuple(value.shape)}, loc {tuple(loc.shape)}, "
                         f"{len(shapes)} levels")
    if len(shapes) > _native.MAX_LEVELS:
        raise ValueError(f"at most {_native.MAX_LEVELS} levels supported")
    cd = _coord_dtype(value)
    if loc.dtype != cd or aw.dtype != cd:
        raise TypeError(f"MSDA: sampling_loc / attn_weight must be {cd} for {value.dtype} values")
    if len(shapes) and max(s + t for s, t in zip(starts, shapes)) > S:
        raise ValueError(f"levels {shapes} starting at {starts} exceed spatial size {S}")


def msda_forward(value, shapes, starts, loc, aw, padding_mode="border", want_tiles=False, layout=0, out=None):
    """out (B, Lq, M*D) = MSDA(value (B,S,M,D), loc/aw (B,Lq,M,L,P)) on the HIP kernel.

    ``want_tiles``: also return the backward's row intervals when the call's backward takes the
    row-block path (``msda_hip_forward_tiles``; None otherwise): ``(out, tiles)``.
    ``layout=LEVEL_MAJOR``: loc / aw are (B, M, L, Lq, P) (``msda_hip_forward_tiles_layout``; the
    call must satisfy ``level_major_ok``; tiles are always written).  ``out``: a contiguous
    (B, Lq, M*D) tensor of value's dtype to write into (a row range of a joint output)."""
    _check_inputs(value, loc, aw, shapes, starts, layout)
    lib = _native.load_library()
    B, S, M, D = value.shape
    Lq, _, L, P = _coord_dims(loc, layout)
    if out is None:
        out = torch.empty((B, Lq, M * D), dtype=value.dtype, device=value.device)
    elif (tuple(out.shape) != (B, Lq, M * D) or out.dtype != value.dtype or not out.is_contiguous()
          or out.device != value.device):
        raise ValueError(f"MSDA: out must be a contiguous {(B, Lq, M * D)} {value.dtype} tensor")
    tiles = None
    if want_tiles or layout == LEVEL_MAJOR:
        nb = lib.msda_hip_forward_tiles_bytes(_native.DTYPE_TAGS[value.dtype], _native.host_i64_array(shapes), L,
                                              B, S, M, D, Lq, P)
        if nb:
            tiles = torch.empty(nb, dtype=torch.uint8, device=value.device)
    timer = _timer
    if timer is not None:
        ev0 = timer._begin()
    args = (value.data_ptr(), _native.DTYPE_TAGS[value.dtype],
            _native.host_i64_array(shapes), _native.host_i64_array(starts), L,
            loc.data_ptr(), aw.data_ptr(), out.data_ptr())
    tail = (B, S, M, D, Lq, P, _native.PAD_TAGS[padding_mode], _native.stream_handle(value.device))
    if layout == LEVEL_MAJOR:
        if tiles is None:
            raise RuntimeError("MSDA: the level-major coordinate layout needs a row-block call (level_major_ok)")
        call = functools.partial(lib.msda_hip_forward_tiles_layout, *args, tiles.data_ptr(), *tail[:-1], layout,
                                 tail[-1])
    elif tiles is None:
        call = functools.partial(lib.msda_hip_forward, *args, *tail)
    else:
        call = functools.partial(lib.msda_hip_forward_tiles, *args, tiles.data_ptr(), *tail)
    rc = call()
    _native.check(rc, "msda_hip_forward")
    if timer is not None:
        timer._end("fwd", (S, Lq), algorithmic_bytes("fwd", B, S, M, D, Lq, L, P, value.element_size()), ev0,
                   gathered_bytes(B, M, D, Lq, L, P, value.element_size()), call, (value, loc, aw, out, tiles))
    return (out, tiles) if want_tiles else out


def _strided_slot(dest, value):
    """dest's row stride when it is a (B, S, M, D) view with value's shape and dtype whose rows are
    whole (h, c) blocks a fixed stride apart (msda_hip_backward_ex), else 0."""
    if dest is None or dest.shape != value.shape or dest.dtype != value.dtype or dest.device != value.device:
        return 0
    B, S, M, D = value.shape
    st = dest.stride()
    rs = st[1]
    if st[3] != 1 or st[2] != D or st[0] != S * rs or rs < M * D or rs % 8 or dest.data_ptr() % 16:
        return 0
    return rs


def msda_backward(value, shapes, starts, loc, aw, grad_output, padding_mode="border",
                  need_value=True, need_loc=True, need_aw=True, tiles=None, layout=0, grad_value_out=None,
                  gv_out=None):
    """(grad_value, grad_loc, grad_aw) of msda_forward; unneeded ones come back None.
    ``tiles``: the row intervals ``msda_forward(..., want_tiles=True)`` returned for these inputs
    (required with ``layout=LEVEL_MAJOR``; grad_loc / grad_aw then come back level-major too).
    ``grad_value_out``: a strided (B, S, M, D) slot to write grad_value into (msda_hip_backward_ex;
    the decoder layers' stacked value gradients): returned as grad_value when the call's kernel path
    writes it, else ignored (a fresh grad_value comes back).  ``gv_out``: a contiguous tensor of value's
    shape and dtype the other paths write grad_value into (a row range of a joint value's gradient)."""
    rs = _strided_slot(grad_value_out, value) if need_value and layout == 0 and tiles is None else 0
    if rs:
        rc_ex = _backward_ex(value, shapes, starts, loc, aw, grad_output, padding_mode, need_loc, need_aw,
                             grad_value_out, rs)
        if rc_ex is not None:
            return rc_ex
    return _backward(value, shapes, starts, loc, aw, grad_output, padding_mode, need_value, need_loc, need_aw,
                     tiles, layout, gv_out)


def _backward_ex(value, shapes, starts, loc, aw, grad_output, padding_mode, need_loc, need_aw, gv, rs):
    """msda_hip_backward_ex into the strided slot gv; None when the call's path does not take it."""
    _check_inputs(value, loc, aw, shapes, starts, 0)
    grad_output = grad_output.to(value.dtype).contiguous()
    B, S, M, D = value.shape
    Lq, _, L, P = _coord_dims(loc, 0)
    if tuple(grad_output.shape) != (B, Lq, M * D):
        raise ValueError(f"grad_output must be {(B, Lq, M * D)}, got {tuple(grad_output.shape)}")
    lib = _native.load_library()
    gl = torch.empty_like(loc) if need_loc else None
    ga = torch.empty_like(aw) if need_aw else None
    ws = None
    nbytes = lib.msda_hip_backward_workspace_bytes(_native.DTYPE_TAGS[value.dtype], B, S, M, D, Lq, L, P)
    if nbytes:
        ws = torch.empty(nbytes, dtype=torch.uint8, device=value.device)
    ptr = lambda t: None if t is None else t.data_ptr()  # noqa: E731
    timer = _timer
    if timer is not None:
        ev0 = timer._begin()
    call = functools.partial(lib.msda_hip_backward_ex, value.data_ptr(), _native.DTYPE_TAGS[value.dtype],
                             _native.host_i64_array(shapes), _native.host_i64_array(starts), L, loc.data_ptr(),
                             aw.data_ptr(), grad_output.data_ptr(), gv.data_ptr(), ptr(gl), ptr(ga), ptr(ws), B, S, M,
                             D, Lq, P, _native.PAD_TAGS[padding_mode], rs, _native.stream_handle(value.device))
    rc = call()
    if rc == _native.MSDA_ERR_UNSUPPORTED:
        return None
    _native.check(rc, "msda_hip_backward_ex")
    if timer is not None:
        timer._end("bwd", (S, Lq), algorithmic_bytes("bwd", B, S, M, D, Lq, L, P, value.element_size()), ev0,
                   gathered_bytes(B, M, D, Lq, L, P, value.element_size()), call,
                   (value, loc, aw, grad_output, gv, gl, ga, ws))
    from . import _trace
    _trace.hit("msda_grad_value_slot")
    return gv, gl, ga


def _backward(value, shapes, starts, loc, aw, grad_output, padding_mode, need_value, need_loc, need_aw, tiles,
              layout, gv_out=None):
    _check_inputs(value, loc, aw, shapes, starts, layout)
    grad_output = grad_output.to(value.dtype).contiguous()
    B, S, M, D = value.shape
    Lq, _, L, P = _coord_dims(loc, layout)
    if tuple(grad_output.shape) != (B, Lq, M * D):
        raise ValueError(f"grad_output must be {(B, Lq, M * D)}, got {tuple(grad_output.shape)}")
    lib = _native.load_library()
    if need_value and gv_out is not None:
        if gv_out.shape != value.shape or gv_out.dtype != value.dtype or not gv_out.is_contiguous():
            raise ValueError(f"MSDA: gv_out must be a contiguous {tuple(value.shape)} {value.dtype} tensor")
        gv = gv_out
    else:
        gv = torch.empty_like(value) if need_value else None
    gl = torch.empty_like(loc) if need_loc else None
    ga = torch.empty_like(aw) if need_aw else None
    ws = None
    nbytes = lib.msda_hip_backward_workspace_bytes(_native.DTYPE_TAGS[value.dtype], B, S, M, D, Lq, L, P)
    if nbytes and (tiles is None or nbytes != tiles.numel()):
        # through the caching allocator: no hipMalloc on the hot path, graph-capturable (the
        # row-block path needs nothing beyond the forward's tiles)
        ws = torch.empty(nbytes, dtype=torch.uint8, device=value.device)
    ptr = lambda t: None if t is None else t.data_ptr()  # noqa: E731
    timer = _timer
    if timer is not None:
        ev0 = timer._begin()
    args = (value.data_ptr(), _native.DTYPE_TAGS[value.dtype],
            _native.host_i64_array(shapes), _native.host_i64_array(starts), L,
            loc.data_ptr(), aw.data_ptr(), grad_output.data_ptr(),
            ptr(gv), ptr(gl), ptr(ga), ptr(ws))
    tail = (B, S, M, D, Lq, P, _native.PAD_TAGS[padding_mode], _native.stream_handle(value.device))
    if layout == LEVEL_MAJOR:
        if tiles is None:
            raise RuntimeError("MSDA: a level-major backward needs the forward's tile intervals")
        call = functools.partial(lib.msda_hip_backward_tiles_layout, *args, tiles.data_ptr(), *tail[:-1], layout,
                                 tail[-1])
    elif tiles is None:
        call = functools.partial(lib.msda_hip_backward, *args, *tail)
    else:
        call = functools.partial(lib.msda_hip_backward_tiles, *args, tiles.data_ptr(), *tail)
    rc = call()
    _native.check(rc, "msda_hip_backward")
    if timer is not None:
        timer._end("bwd", (S, Lq), algorithmic_bytes("bwd", B, S, M, D, Lq, L, P, value.element_size()), ev0,
                   gathered_bytes(B, M, D, Lq, L, P, value.element_size()), call,
                   (value, loc, aw, grad_output, gv, gl, ga, ws, tiles))
    return gv, gl, ga


class MSDAFunction(Function):
    """autograd wrapper (shape of the reference's MSDeformAttnFunction,
    models/modules/attention.py:310-328): saves the inputs, backward returns
    grads for value / loc / aw, ``once_differentiable`` like the reference."""

    @staticmethod
    def forward(ctx, value, loc, aw, shapes, starts, padding_mode, layout=0):
        from . import _trace
        _trace.hit("msda_" + str(value.dtype).replace("torch.", ""))
        if layout == LEVEL_MAJOR:
            _trace.hit("msda_level_major")
        ctx.meta = (shapes, starts, padding_mode, layout)
        ctx.save_for_backward(value, loc, aw)
        # a strided slot for grad_value offered by value's producer (value_proj.layer_values)
        ctx.gdest = getattr(value, "_mfl_grad_dest", None)
        if ctx.gdest is not None:
            if getattr(value, "_mfl_grad_dest_taken", False):  # (one consumer per slot)
                ctx.gdest = None
            else:
                value._mfl_grad_dest_taken = True
        # the row intervals of the row-block backward come with the forward (it reads loc anyway)
        if any(ctx.needs_input_grad[:3]) or layout == LEVEL_MAJOR:
            out, ctx.tiles = msda_forward(value, shapes, starts, loc, aw, padding_mode, want_tiles=True,
                                          layout=layout)
        else:
            out, ctx.tiles = msda_forward(value, shapes, starts, loc, aw, padding_mode), None
        return out

    @staticmethod
    @once_differentiable
    def backward(ctx, grad_output):
        value, loc, aw = ctx.saved_tensors
        shapes, starts, padding_mode, layout = ctx.meta
        nv, nl, na = ctx.needs_input_grad[:3]
        gdest, ctx.gdest = ctx.gdest, None
        gv, gl, ga = msda_backward(value, shapes, starts, loc, aw, grad_output, padding_mode,
                                   need_value=nv, need_loc=nl, need_aw=na, tiles=ctx.tiles, layout=layout,
                                   grad_value_out=gdest)
        ctx.tiles = None
        if gv is not None and gv is not gdest:
            gv._mfl_private = True  # fresh, referenced by nothing else: consumers may write it in place
        return gv, gl, ga, None, None, None, None


def msda_apply(value, shapes, starts, loc, aw, padding_mode="border", layout=0):
    """Differentiable MSDA on normalised inputs: value (B,S,M,D); loc, aw (B,Lq,M,L,P) — or
    (B,M,L,Lq,P) with ``layout=LEVEL_MAJOR`` (the fused MSDeformAttn path's internal layout).

    Casts loc / aw to the coordinate dtype (fp32, or fp64 for fp64 values) and makes
    everything contiguous outside the Function, so autograd tracks those copies."""
    cd = _coord_dtype(value)
    value = value.contiguous()
    loc = loc.to(cd).contiguous()
    aw = aw.to(cd).contiguous()
    return MSDAFunction.apply(value, loc, aw, tuple(shapes), tuple(starts), padding_mode, layout)


# --- MSDA prologue -------------------------------------------------------

def prologue_supported(n_heads, n_levels, n_points):
    """The fused prologue kernel's shape limits (include/msda_hip.h)."""
    return n_heads * n_levels * n_points <= 1024


def prologue_forward(offsets, logits, ref, shapes):
    """(sampling_loc, attn_weight) of the reference's MSDeformAttn prologue
    (models/modules/attention.py:468-483) in one HIP kernel.

    offsets (B, Lq, M, L, P) and logits (B, Lq, M, L*P) in one dtype (bf16 under autocast);
    ref (B, Lq, L, 1 or 2) in the coordinate dtype; outputs (B, Lq, M, L, P) coord dtype."""
    if not (offsets.is_cuda and logits.is_cuda and ref.is_cuda):
        raise RuntimeError("MSDA prologue: ROCm device tensors required (no CPU implementation)")
    if offsets.dtype not in _native.DTYPE_TAGS or logits.dtype != offsets.dtype:
        raise TypeError(f"MSDA prologue: offsets / logits dtypes {offsets.dtype} / {logits.dtype}")
    B, Lq, M, L, P = offsets.shape
    cd = torch.float64 if offsets.dtype == torch.float64 else torch.float32
    if ref.dtype != cd or ref.dim() != 4 or tuple(ref.shape[:3]) != (B, Lq, L) or ref.shape[3] not in (1, 2):
        raise ValueError(f"MSDA prologue: reference_points {tuple(ref.shape)} {ref.dtype} does not match "
                         f"offsets {tuple(offsets.shape)}")
    if len(shapes) != L:
        raise ValueError(f"MSDA prologue: {len(shapes)} level shapes for {L} levels")
    for name, t in (("offsets", offsets), ("logits", logits), ("reference_points", ref)):
        if not t.is_contiguous():
            raise ValueError(f"MSDA prologue: {name} must be contiguous")
    lib = _native.load_library()
    loc = torch.empty((B, Lq, M, L, P), dtype=cd, device=offsets.device)
    aw = torch.empty_like(loc)
    rc = lib.msda_hip_prologue_forward(
        offsets.data_ptr(), logits.data_ptr(), _native.DTYPE_TAGS[offsets.dtype], ref.data_ptr(), ref.shape[3],
        _native.host_i64_array(shapes), L, B, Lq, M, P, loc.data_ptr(), aw.data_ptr(),
        _native.stream_handle(offsets.device))
    _native.check(rc, "msda_hip_prologue_forward")
    return loc, aw


def prologue_backward(grad_loc, grad_aw, aw, offsets, ref, shapes, need_off=True, need_logits=True,
                      need_ref=True):
    """(grad_offsets, grad_logits, grad_ref) of prologue_forward; unneeded ones are None."""
    B, Lq, M, L, P = offsets.shape
    cd = aw.dtype
    lib = _native.load_library()
    if grad_loc is None:
        grad_loc = torch.zeros_like(aw)
    if grad_aw is None:
        grad_aw = torch.zeros_like(aw)
    grad_loc = grad_loc.to(cd).contiguous()
    grad_aw = grad_aw.to(cd).contiguous()
    g_off = torch.empty_like(offsets) if need_off else None
    g_log = torch.empty((B, Lq, M, L * P), dtype=offsets.dtype, device=offsets.device) if need_logits else None
    g_ref = torch.empty_like(ref) if need_ref else None
    ptr = lambda t: None if t is None else t.data_ptr()  # noqa: E731
    rc = lib.msda_hip_prologue_backward(
        grad_loc.data_ptr(), grad_aw.data_ptr(), aw.data_ptr(), offsets.data_ptr(),
        _native.DTYPE_TAGS[offsets.dtype], ref.data_ptr(), ref.shape[3], _native.host_i64_array(shapes), L,
        B, Lq, M, P, ptr(g_off), ptr(g_log), ptr(g_ref), _native.stream_handle(offsets.device))
    _native.check(rc, "msda_hip_prologue_backward")
    return g_off, g_log, g_ref


def prologue_forward_rows(y, B, Lq, M, L, P, ref, shapes, layout=0):
    """``prologue_forward`` on the output of ONE query-projection GEMM: y (B*Lq, 2*M*L*P), each
    row [sampling offsets | attention logits] (``msda_hip_prologue_forward_ex``, read in place).
    ``layout=LEVEL_MAJOR``: loc / aw written (B, M, L, Lq, P) (``msda_hip_prologue_forward_layout``)."""
    n = M * L * P
    if y.dim() != 2 or tuple(y.shape) != (B * Lq, 2 * n) or not y.is_contiguous() or not y.is_cuda:
        raise ValueError(f"MSDA prologue rows: y must be a contiguous device (B*Lq, 2*M*L*P) tensor, got "
                         f"{tuple(y.shape)}")
    cd = torch.float64 if y.dtype == torch.float64 else torch.float32
    if ref.dtype != cd or tuple(ref.shape[:3]) != (B, Lq, L) or not ref.is_contiguous():
        raise ValueError(f"MSDA prologue rows: reference_points {tuple(ref.shape)} {ref.dtype}")
    lib = _native.load_library()
    loc = torch.empty((B, M, L, Lq, P) if layout == LEVEL_MAJOR else (B, Lq, M, L, P), dtype=cd, device=y.device)
    aw = torch.empty_like(loc)
    base = y.data_ptr()
    rc = lib.msda_hip_prologue_forward_layout(
        base, base + n * y.element_size(), _native.DTYPE_TAGS[y.dtype], ref.data_ptr(), ref.shape[3],
        _native.host_i64_array(shapes), L, B, Lq, M, P, 2 * n, layout, loc.data_ptr(), aw.data_ptr(),
        _native.stream_handle(y.device))
    _native.check(rc, "msda_hip_prologue_forward_layout")
    return loc, aw


def prologue_backward_rows(grad_loc, grad_aw, aw, y, ref, shapes, need_ref=True, layout=0, g2_out=None):
    """``prologue_backward`` into ONE (B*Lq, 2*M*L*P) buffer of [grad offsets | grad logits] rows
    (the dgrad GEMM's input) -> (g2, grad_ref or None); grad_loc / grad_aw / aw in ``layout``.
    ``g2_out``: a contiguous tensor like y to write into (a row range of a joint buffer)."""
    B = aw.shape[0]
    Lq, M, L, P = _coord_dims(aw, layout)
    n = M * L * P
    cd = aw.dtype
    lib = _native.load_library()
    grad_loc = torch.zeros_like(aw) if grad_loc is None else grad_loc.to(cd).contiguous()
    grad_aw = torch.zeros_like(aw) if grad_aw is None else grad_aw.to(cd).contiguous()
    if g2_out is not None:
        if g2_out.shape != y.shape or g2_out.dtype != y.dtype or not g2_out.is_contiguous():
            raise ValueError(f"MSDA prologue rows: g2_out must be a contiguous {tuple(y.shape)} {y.dtype} tensor")
        g2 = g2_out
    else:
        g2 = torch.empty_like(y)
    g_ref = torch.empty_like(ref) if need_ref else None
    base, ybase = g2.data_ptr(), y.data_ptr()
    rc = lib.msda_hip_prologue_backward_layout(
        grad_loc.data_ptr(), grad_aw.data_ptr(), aw.data_ptr(), ybase, _native.DTYPE_TAGS[y.dtype], ref.data_ptr(),
        ref.shape[3], _native.host_i64_array(shapes), L, B, Lq, M, P, 2 * n, layout, base,
        base + n * g2.element_size(), None if g_ref is None else g_ref.data_ptr(), _native.stream_handle(y.device))
    _native.check(rc, "msda_hip_prologue_backward_layout")
    return g2, g_ref


class MSDAPrologueFunction(Function):
    @staticmethod
    def forward(ctx, offsets, logits, ref, shapes):
        from . import _trace
        _trace.hit("msda_prologue")
        loc, aw = prologue_forward(offsets, logits, ref, shapes)
        ctx.shapes = shapes
        ctx.save_for_backward(aw, offsets, ref)
        return loc, aw

    @staticmethod
    @once_differentiable
    def backward(ctx, grad_loc, grad_aw):
        aw, offsets, ref = ctx.saved_tensors
        n_off, n_log, n_ref = ctx.needs_input_grad[:3]
        g_off, g_log, g_ref = prologue_backward(grad_loc, grad_aw, aw, offsets, ref, ctx.shapes, n_off, n_log,
                                                n_ref)
        return g_off, g_log, g_ref, None


def msda_prologue_apply(offsets, logits, ref, shapes):
    """Differentiable fused prologue: offsets (B,Lq,M,L,P), logits (B,Lq,M,L*P) (same dtype),
    ref (B,Lq,L,1|2) -> (sampling_loc, attn_weight) (B,Lq,M,L,P) in the coordinate dtype."""
    cd = torch.float64 if offsets.dtype == torch.float64 else torch.float32
    return MSDAPrologueFunction.apply(offsets.contiguous(), logits.to(offsets.dtype).contiguous(),
                                      ref.to(cd).contiguous(), tuple(int(t) for t in shapes))
