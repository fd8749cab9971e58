"""ORACLE — test infrastructure, never product code.

CPU restatement (numpy) of the reference's live MSDA core and its gradient, used ONLY by
tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg as the checker.

Follows:
  * forward  — reference models/modules/attention.py:331-383: per level, a 1-D bilinear
    ``F.grid_sample(mode='bilinear', padding_mode='border', align_corners=False)`` of the
    (B*M, D, T_l, 1) value image at grid (x=-1, y=2*loc-1) (:349,:363,:367-368), times the
    attention weights, summed over levels and points (:374,:381).
  * grid_sample arithmetic — ATen's CPU grid sampler (torch 2.10, the version the reference
    runs on here; third-party code, not in /root/reference): unnormalize
    y = fma(g + 1, T/2, -0.5) (ONE rounding: measured in tests/test_oracle.py, where the
    unfused (g+1)*(T/2)-0.5 picks the other tap segment for ~1% of near-integer fp32
    locations at T = 50/75/300/1000), border clip to [0, T-1], taps floor(y) / floor(y)+1 with
    weights (1-n, n), n = y - floor(y), out-of-map taps read 0; backward
    ``clip_coordinates_get_grad`` treats the border itself as out of bounds (zero
    y-gradient when y <= 0 or y >= T-1), d y / d g = T/2.
  * backward — autograd of the above: grad_value scatter of aw*w*grad_out,
    grad_aw = <grad_out, sample>, grad_loc = 2 * (T/2) * aw * <grad_out, v1 - v0>.
  * padding "zeros" — the dormant CUDA extension on the 1-D (H=1) lift:
    models/ops/src/cuda/ms_deform_im2col_cuda.cuh:34-85 (im2col_bilinear), :238-300
    (forward, sample skipped unless -1 < w_im < W) and :88-160 (col2im_bilinear:
    grad_w = W * aw * <grad_out, v_high - v_low>).  The kernel itself is CUDA-only and
    unbuildable here; the mode is pinned against the comparator of the reference's own kernel
    test (models/ops/test.py:38-39, the 2-D core of ops/functions/ms_deform_attn_func.py:44-71)
    run with grid_sample's padding set to the kernel's zeros (tests/golden/ops_api_f64.pt).
  * msda_h1 — the extension API's (..., 2) [x, y] form on H = 1 maps (row weight of y folded
    into the attention weight, cuh:34-160).

Pinned: border mode against golden vectors produced by the real reference
(tests/golden/make_golden.py imports /root/reference on CPU), zeros mode and the 2-D form
against ops_api_f64 — see tests/test_oracle.py.

All arithmetic happens in the dtype of ``value`` (float32 or float64) in the reference's
operation order for the coordinates, so tap indices are bit-identical to ATen's.
"""
import numpy as np

__all__ = ["taps", "msda_forward", "msda_backward", "level_starts", "row_weight_h1", "msda_h1"]


def level_starts(shapes):
    out, acc = [], 0
    for t in shapes:
        out.append(acc)
        acc += int(t)
    return out


def _fma(a, b, c):
    """a*b + c with one rounding.  fp32: the fp64 product of two fp32 numbers is exact and
    adding c is exact at these magnitudes, so one cast back rounds once.  fp64: numpy has
    no fma; the separate operations differ from it only at exact ties (never hit by the
    fp64 fixtures)."""
    if a.dtype == np.float32:
        return (a.astype(np.float64) * np.float64(b) + np.float64(c)).astype(np.float32)
    return a * b + c


def taps(loc, T, padding="border"):
    """Tap rows / weights for locations ``loc`` (any shape) on a T-long level.

    Returns (i0, i1, w0, w1, ok0, ok1, gmul): tap rows (always valid indices), their
    weights (0 where a tap is outside the map), validity masks, and d(y)/d(loc) with the
    clamp folded in (0 where the reference's location gradient is 0)."""
    dt = loc.dtype.type
    if padding == "border":
        g = loc * dt(2) - dt(1)                                  # attention.py:349
        y = _fma(g + dt(1), dt(T * 0.5), dt(-0.5))               # ATen unnormalize, align_corners=False
        ymax = dt(T - 1)
        inb = (y > 0) & (y < ymax)                               # clip_coordinates_get_grad
        yc = np.clip(y, dt(0), ymax)
        y0 = np.floor(yc)
        n = (yc - y0).astype(loc.dtype)
        i0 = y0.astype(np.int64)
        ok0 = np.ones_like(inb)
        ok1 = (i0 + 1) <= T - 1
        i1 = np.where(ok1, i0 + 1, i0)
        w0 = (dt(1) - n).astype(loc.dtype)
        w1 = n
        gmul = np.where(inb, dt(T), dt(0)).astype(loc.dtype)     # 2 * T/2
        return i0, i1, w0, w1, ok0, ok1, gmul
    if padding == "zeros":
        x = loc * dt(T) - dt(0.5)                                # cuh:276-279 (w_im), H=1 lift
        live = (x > dt(-1)) & (x < dt(T))                        # cuh:289
        xs = np.where(live, x, dt(0))
        x0 = np.floor(xs)
        lw = (xs - x0).astype(loc.dtype)
        lo = x0.astype(np.int64)
        ok0 = live & (lo >= 0)
        ok1 = live & (lo + 1 <= T - 1)
        i0 = np.where(ok0, lo, 0)
        i1 = np.where(ok1, lo + 1, 0)
        w0 = np.where(ok0, dt(1) - lw, dt(0)).astype(loc.dtype)
        w1 = np.where(ok1, lw, dt(0)).astype(loc.dtype)
        gmul = np.where(live, dt(T), dt(0)).astype(loc.dtype)
        return i0, i1, w0, w1, ok0, ok1, gmul
    raise ValueError(padding)


def _gather(Vl, idx):
    """Vl (B, T, M, D), idx (B, Lq, M, P) -> (B, Lq, M, P, D)"""
    B, _, M, _ = Vl.shape
    b = np.arange(B)[:, None, None, None]
    m = np.arange(M)[None, None, :, None]
    return Vl[b, idx, m]


def msda_forward(value, shapes, loc, aw, starts=None, padding="border"):
    """value (B,S,M,D); loc, aw (B,Lq,M,L,P) -> out (B, Lq, M*D), dtype of value."""
    value = np.asarray(value)
    loc = np.asarray(loc, dtype=value.dtype)
    aw = np.asarray(aw, dtype=value.dtype)
    B, S, M, D = value.shape
    Lq = loc.shape[1]
    starts = level_starts(shapes) if starts is None else list(starts)
    out = np.zeros((B, Lq, M, D), dtype=value.dtype)
    for l, T in enumerate(shapes):
        T = int(T)
        Vl = value[:, starts[l]:starts[l] + T]
        i0, i1, w0, w1, ok0, ok1, _ = taps(loc[:, :, :, l, :], T, padding)
        v0 = _gather(Vl, i0) * ok0[..., None]
        v1 = _gather(Vl, i1) * ok1[..., None]
        samp = v0 * w0[..., None] + v1 * w1[..., None]
        out += (samp * aw[:, :, :, l, :, None]).sum(3)
    return out.reshape(B, Lq, M * D)


def msda_backward(value, shapes, loc, aw, grad_out, starts=None, padding="border"):
    """-> (grad_value (B,S,M,D), grad_loc (B,Lq,M,L,P), grad_aw (B,Lq,M,L,P))"""
    value = np.asarray(value)
    dt = value.dtype
    loc = np.asarray(loc, dtype=dt)
    aw = np.asarray(aw, dtype=dt)
    B, S, M, D = value.shape
    Lq, L, P = loc.shape[1], loc.shape[3], loc.shape[4]
    g = np.asarray(grad_out, dtype=dt).reshape(B, Lq, M, 1, D)
    starts = level_starts(shapes) if starts is None else list(starts)
    gv = np.zeros_like(value)
    gl = np.zeros_like(loc)
    ga = np.zeros_like(aw)
    b = np.broadcast_to(np.arange(B)[:, None, None, None], (B, Lq, M, P))
    m = np.broadcast_to(np.arange(M)[None, None, :, None], (B, Lq, M, P))
    for l, T in enumerate(shapes):
        T = int(T)
        Vl = value[:, starts[l]:starts[l] + T]
        i0, i1, w0, w1, ok0, ok1, gmul = taps(loc[:, :, :, l, :], T, padding)
        v0 = _gather(Vl, i0) * ok0[..., None]
        v1 = _gather(Vl, i1) * ok1[..., None]
        samp = v0 * w0[..., None] + v1 * w1[..., None]
        a = aw[:, :, :, l, :]
        ga[:, :, :, l, :] = (g * samp).sum(-1)
        gl[:, :, :, l, :] = a * gmul * (g * (v1 - v0)).sum(-1)
        gvl = np.zeros((B, T, M, D), dtype=dt)
        c0 = (a * w0)[..., None] * g * ok0[..., None]
        c1 = (a * w1)[..., None] * g * ok1[..., None]
        np.add.at(gvl, (b, i0, m), c0)
        np.add.at(gvl, (b, i1, m), c1)
        gv[:, starts[l]:starts[l] + T] += gvl
    return gv, gl, ga


def row_weight_h1(y, padding):
    """Weight of the single row of an H = 1 map and its y-derivative, for the 2-D extension API
    ((L, 2) [H, W] shapes, (..., 2) [x, y] locations; models/ops/modules/ms_deform_attn.py:114-117).

    zeros — cuh:34-85 / 88-160: h = y*H - 0.5, the sample lives iff -1 < h < H; h_low = floor(h);
    row 0 is h_low (weight 1 - (h - h_low)) when h >= 0, else h_high (weight h - h_low); the y
    gradient is H * (+-1) * aw * <grad, x-sample>.
    border — grid_sample border on one row: y clamps to row 0, weight 1, zero y-gradient."""
    y = np.asarray(y)
    dt = y.dtype.type
    if padding == "border":
        return np.ones_like(y), np.zeros_like(y)
    h = y - dt(0.5)
    live = (h > dt(-1)) & (h < dt(1))
    upper = h >= 0
    rw = np.where(live, np.where(upper, dt(1) - h, h + dt(1)), dt(0)).astype(y.dtype)
    drw = np.where(live, np.where(upper, dt(-1), dt(1)), dt(0)).astype(y.dtype)
    return rw, drw


def msda_h1(value, shapes, loc2, aw, grad_out, padding="zeros"):
    """The extension API's 2-D form on H = 1 maps: (out, grad_value, grad_loc2 (...,2), grad_aw).
    The row weight folds into the attention weight; the x part is msda_forward / msda_backward."""
    loc2 = np.asarray(loc2)
    x, y = loc2[..., 0], loc2[..., 1]
    rw, drw = row_weight_h1(y, padding)
    aw = np.asarray(aw)
    out = msda_forward(value, shapes, x, aw * rw, padding=padding)
    gv, gx, ga_eff = msda_backward(value, shapes, x, aw * rw, grad_out, padding=padding)
    gy = aw * drw * ga_eff
    return out, gv, np.stack([gx, gy], -1), ga_eff * rw
