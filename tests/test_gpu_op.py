"""HIP kernel parity (``-m gpu``): libmsda_hip.so through the C-ABI vs the reference's golden
vectors and vs the oracle restatement, over dtypes, channel counts, level layouts, both
padding modes and the edge cases (clamp borders, near-integer positions, empty inputs).

Tolerances: fp64 1e-12 (only the grad_value atomic-add order differs); fp32 outputs /
grads within 1e-5 / 1e-4 relative of the fp32 reference (north_star asks 1e-3);
bf16 / fp16 values against the oracle on the same rounded inputs in fp32.
"""
import numpy as np
import pytest
import torch

from conftest import PKG
from oracle import msda_oracle as O
from test_oracle import near_integer_locations, regenerate_enc_inputs

pytestmark = pytest.mark.gpu
msda = PKG.msda


def _np(t):
    return t.detach().float().cpu().numpy() if t.dtype in (torch.bfloat16, torch.float16) else t.detach().cpu().numpy()


def run_hip(value, shapes, loc, aw, gout, padding="border", dev="cuda"):
    starts = O.level_starts(shapes)
    v, lc, a, g = (t.to(dev) for t in (value, loc, aw, gout))
    out = msda.msda_forward(v, shapes, starts, lc, a, padding)
    gv, gl, ga = msda.msda_backward(v, shapes, starts, lc, a, g, padding)
    torch.cuda.synchronize()
    return out.cpu(), gv.cpu(), gl.cpu(), ga.cpu()


def rand_case(shapes, B, M, D, Lq, P, dtype, seed, lo=-0.2, hi=1.2):
    gen = torch.Generator().manual_seed(seed)
    S = sum(shapes)
    value = torch.randn((B, S, M, D), generator=gen).to(dtype)
    cd = torch.float64 if dtype == torch.float64 else torch.float32
    loc = (torch.rand((B, Lq, M, len(shapes), P), generator=gen, dtype=torch.float64) * (hi - lo) + lo).to(cd)
    aw = torch.rand((B, Lq, M, len(shapes), P), generator=gen, dtype=torch.float64).to(cd)
    gout = torch.randn((B, Lq, M * D), generator=gen).to(dtype)
    return value, loc, aw, gout


@pytest.mark.parametrize("name,rtol,atol", [("op_border_f64", 1e-12, 1e-12), ("op_border_f32", 1e-5, 1e-6)])
def test_kernel_matches_reference_golden(golden, dev, name, rtol, atol):
    g = golden(name)
    shapes = g["shapes"].tolist()
    out, gv, gl, ga = run_hip(g["value"], shapes, g["loc"], g["aw"], g["grad_out"])
    torch.testing.assert_close(out, g["out"], rtol=rtol, atol=atol)
    torch.testing.assert_close(gv, g["grad_value"], rtol=rtol * 10, atol=atol * 10)
    torch.testing.assert_close(ga, g["grad_aw"], rtol=rtol * 10, atol=atol * 10)
    torch.testing.assert_close(gl, g["grad_loc"], rtol=rtol * 10, atol=atol * 64)


def test_kernel_matches_reference_golden_enc_shape(golden, dev):
    g = golden("op_border_f32_enc")
    shapes, value, loc, aw, gout = regenerate_enc_inputs(g)
    out, gv, gl, ga = run_hip(value, shapes, loc, aw, gout)
    torch.testing.assert_close(out, g["out"], rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(ga, g["grad_aw"], rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(gl, g["grad_loc"], rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(gv.sum(-1), g["grad_value_rowsum"], rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(gv[:, g["grad_value_rows"]], g["grad_value_at_rows"], rtol=1e-4, atol=1e-5)


CASES = [
    # shapes,               B, M, D,    Lq, P
    ([32, 16, 8, 4],        2, 4, 8,    20, 4),
    ([1024, 512, 256, 128], 1, 8, 64,   64, 4),
    ([50, 25, 13, 7],       3, 8, 64,   95, 4),    # audio pyramid of config 3
    ([300, 150, 75, 38],    2, 8, 32,   40, 2),    # video_rescale_len = 300
    ([17],                  2, 2, 30,   9, 3),
    ([1, 1, 1],             1, 1, 16,   5, 1),     # T = 1 levels
    ([64, 32],              1, 2, 71,   7, 4),     # odd channel count (scalar path)
    ([40, 20, 10],          1, 1, 1025, 3, 2),     # D > 64 lanes: chunked lanes
    ([40, 20, 10],          1, 2, 256,  6, 2),
    # >= 256 (b, m, level) workgroups: fused sort+pull backward (entry lists in LDS)
    ([32, 16, 8, 4],        8, 8, 64,   60, 4),
    ([32, 16, 8, 4],        4, 16, 32,  30, 4),    # 8 rows per wave (fp32 D=32)
    ([16, 8, 4, 2],         8, 8, 30,   20, 2),    # odd channel count: lane-per-channel pull
    ([8, 4, 2, 1],          8, 8, 16,   200, 4),   # 800 taps on one row
    ([64, 32, 16, 8],       8, 8, 16,   4000, 2),  # 16000 entries: near the LDS budget
    ([50, 25, 13, 7],       4, 8, 64,   1920, 4),  # video queries over the audio pyramid: ~1100 taps a row
]


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
@pytest.mark.parametrize("padding", ["border", "zeros"])
@pytest.mark.parametrize("case", range(len(CASES)))
def test_kernel_matches_oracle(dev, case, padding, dtype):
    shapes, B, M, D, Lq, P = CASES[case]
    value, loc, aw, gout = rand_case(shapes, B, M, D, Lq, P, dtype, seed=100 + case)
    out, gv, gl, ga = run_hip(value, shapes, loc, aw, gout, padding)
    r_out = O.msda_forward(_np(value), shapes, _np(loc), _np(aw), padding=padding)
    r_gv, r_gl, r_ga = O.msda_backward(_np(value), shapes, _np(loc), _np(aw), _np(gout), padding=padding)
    tol = dict(rtol=1e-11, atol=1e-11) if dtype == torch.float64 else dict(rtol=2e-5, atol=2e-5)
    np.testing.assert_allclose(_np(out), r_out, **tol)
    np.testing.assert_allclose(_np(ga), r_ga, **tol)
    np.testing.assert_allclose(_np(gv), r_gv, rtol=tol["rtol"] * 10, atol=tol["atol"] * 10)
    scale = max(shapes)
    np.testing.assert_allclose(_np(gl), r_gl, rtol=tol["rtol"] * 10, atol=tol["atol"] * scale)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("D", [64, 30])
@pytest.mark.parametrize("B", [2, 8])  # 8: fused sort+pull backward
def test_half_values_match_oracle_on_rounded_inputs(dev, dtype, D, B):
    shapes, M, Lq, P = [256, 128, 64, 32], 8, 96, 4
    value, loc, aw, gout = rand_case(shapes, B, M, D, Lq, P, dtype, seed=7)
    out, gv, gl, ga = run_hip(value, shapes, loc, aw, gout)
    assert out.dtype == dtype and gv.dtype == dtype and gl.dtype == torch.float32
    v32, g32 = value.float(), gout.float()
    r_out = O.msda_forward(_np(v32), shapes, _np(loc), _np(aw))
    r_gv, r_gl, r_ga = O.msda_backward(_np(v32), shapes, _np(loc), _np(aw), _np(g32))
    eps = 2 ** -8 if dtype == torch.bfloat16 else 2 ** -11        # output rounding of the storage type
    np.testing.assert_allclose(_np(out), r_out, rtol=eps, atol=eps * np.abs(r_out).max())
    np.testing.assert_allclose(_np(ga), r_ga, rtol=1e-4, atol=1e-4)   # fp32 math on exact inputs
    np.testing.assert_allclose(_np(gl), r_gl, rtol=1e-4, atol=1e-2)
    np.testing.assert_allclose(_np(gv), r_gv, rtol=eps, atol=eps * np.abs(r_gv).max())


@pytest.mark.parametrize("T", [1024, 1000, 300, 75, 50])
def test_tap_segment_bit_identical_near_integers(dev, T):
    """Same construction as the oracle's pin: the fp32 kernel picks ATen's segment."""
    loc = torch.from_numpy(near_integer_locations(T)).view(1, -1, 1, 1, 1)
    value = (torch.arange(T, dtype=torch.float32) ** 2).view(1, T, 1, 1)
    aw = torch.ones_like(loc)
    gout = torch.ones(1, loc.shape[1], 1)
    _, _, gl, _ = run_hip(value, [T], loc, aw, gout)
    _, r_gl, _ = O.msda_backward(value.numpy(), [T], loc.numpy(), aw.numpy(), gout.numpy())
    np.testing.assert_allclose(gl.numpy(), r_gl, rtol=1e-6)


def test_border_gradient_exactly_zero_at_clamp(golden, dev):
    g = golden("op_border_f32")
    shapes = g["shapes"].tolist()
    _, _, gl, _ = run_hip(g["value"], shapes, g["loc"], g["aw"], g["grad_out"])
    ref = g["grad_loc"]
    assert torch.equal(gl == 0, ref == 0)


@pytest.mark.parametrize("B,Lq", [(0, 5), (2, 0)])
def test_empty_inputs(dev, B, Lq):
    shapes = [8, 4]
    value, loc, aw, gout = rand_case(shapes, max(B, 1), 2, 16, max(Lq, 1), 2, torch.float32, seed=1)
    value, loc, aw, gout = value[:B], loc[:B, :Lq], aw[:B, :Lq], gout[:B, :Lq]
    out, gv, gl, ga = run_hip(value.contiguous(), shapes, loc.contiguous(), aw.contiguous(), gout.contiguous())
    assert out.shape == (B, Lq, 32) and gv.shape == value.shape
    assert gv.abs().sum() == 0


def test_needs_input_grad_subsets(dev):
    shapes = [32, 16]
    value, loc, aw, gout = rand_case(shapes, 2, 4, 16, 10, 2, torch.float64, seed=5)
    v, lc, a = value.cuda().requires_grad_(True), loc.cuda(), aw.cuda().requires_grad_(True)
    out = msda.msda_apply(v, shapes, O.level_starts(shapes), lc, a)
    out.backward(gout.cuda())
    _, r_gl, r_ga = O.msda_backward(_np(value), shapes, _np(loc), _np(aw), _np(gout))
    assert lc.grad is None
    np.testing.assert_allclose(a.grad.cpu().numpy(), r_ga, rtol=1e-12, atol=1e-12)


@pytest.mark.parametrize("channels", [30, 32, 64, 71, 1025, 2048, 3096])
def test_gradcheck_fp64(dev, channels):
    """torch.autograd.gradcheck in fp64 over the channel counts of the reference's own
    test (models/ops/test.py:85-86), locations kept off the interpolation kinks."""
    N, M, Lq, L, P = 1, 2, 2, 2, 2
    shapes = [6, 3]
    gen = torch.Generator().manual_seed(3)
    value = (torch.rand(N, sum(shapes), M, channels, generator=gen, dtype=torch.float64) * 0.01)
    loc = torch.rand(N, Lq, M, L, P, generator=gen, dtype=torch.float64) * 0.8 + 0.1
    for l, T in enumerate(shapes):
        y = loc[:, :, :, l] * T - 0.5
        frac = y - y.floor()
        loc[:, :, :, l] += torch.where((frac < 1e-3) | (frac > 1 - 1e-3), 5e-3 / T, 0.0)
    aw = torch.rand(N, Lq, M, L, P, generator=gen, dtype=torch.float64) + 1e-5
    aw = aw / aw.sum(-1, keepdim=True).sum(-2, keepdim=True)
    starts = O.level_starts(shapes)
    for padding in ("border", "zeros"):
        f = lambda v, lc, a: msda.MSDAFunction.apply(v, lc, a, tuple(shapes), tuple(starts), padding)  # noqa: E731
        inputs = tuple(t.cuda().requires_grad_(True) for t in (value, loc, aw))
        assert torch.autograd.gradcheck(f, inputs, eps=1e-6, atol=1e-5, rtol=1e-4)


@pytest.mark.parametrize("shapes,B", [([1024, 512, 256, 128], 8),     # configs[1] encoder call (fp32: pair backward)
                                      ([4096, 2048, 1024, 512], 2)])  # configs[3]: S = 7680 (fp32: workspace-staged pair)
def test_full_size_properties(dev, shapes, B):
    """At full encoder-call sizes (the bench's B=8, T=1024; and T=4096, S=7680) where the oracle
    is too slow to run whole: linearity in value and in aw, the adjoint identity
    <g, fwd(v)> = <bwd_value(g), v>, and the grad_value checksum
    sum_s grad_value[b,s,m,:] = sum_q (sum_{l,p} aw[b,q,m,l,p]) grad_out[b,q,m,:] (border
    weights of a sample sum to 1); plus oracle parity on one clip."""
    M, D, P = 8, 64, 4
    Lq = sum(shapes)
    v1, loc, aw, gout = rand_case(shapes, B, M, D, Lq, P, torch.float32, seed=11, lo=0.0, hi=1.0)
    v2 = torch.randn_like(v1)
    starts = O.level_starts(shapes)
    c = lambda t: t.cuda()  # noqa: E731
    o1 = msda.msda_forward(c(v1), shapes, starts, c(loc), c(aw))
    o2 = msda.msda_forward(c(v2), shapes, starts, c(loc), c(aw))
    o12 = msda.msda_forward(c(2 * v1 - 3 * v2), shapes, starts, c(loc), c(aw))
    torch.testing.assert_close(o12, 2 * o1 - 3 * o2, rtol=1e-4, atol=1e-4)
    gv, _, _ = msda.msda_backward(c(v1), shapes, starts, c(loc), c(aw), c(gout))
    lhs = gv.double().sum(1)                                               # (B, M, D)
    rhs = (aw.double().sum((-1, -2))[..., None] * gout.double().view(B, Lq, M, D)).sum(1)
    torch.testing.assert_close(lhs.cpu(), rhs, rtol=1e-4, atol=1e-3)
    # adjoint: grad_value is the transpose of the forward's linear map in value
    dot_fwd = (o1.double() * c(gout).double()).sum().item()
    dot_bwd = (gv.double() * c(v1).double()).sum().item()
    assert abs(dot_fwd - dot_bwd) <= 1e-4 * abs(dot_fwd) + 1e-3, (dot_fwd, dot_bwd)
    # linearity in the attention weights
    aw2 = torch.rand_like(aw)
    oa = msda.msda_forward(c(v1), shapes, starts, c(loc), c(aw2))
    oab = msda.msda_forward(c(v1), shapes, starts, c(loc), c(aw + 0.5 * aw2))
    torch.testing.assert_close(oab, o1 + 0.5 * oa, rtol=1e-4, atol=1e-4)
    r_out = O.msda_forward(_np(v1[:1]), shapes, _np(loc[:1]), _np(aw[:1]))
    np.testing.assert_allclose(o1[:1].cpu().numpy(), r_out, rtol=2e-5, atol=2e-5)
    # the whole backward of one clip against the oracle (clips are independent)
    gv, gl, ga = msda.msda_backward(c(v1), shapes, starts, c(loc), c(aw), c(gout))
    r_gv, r_gl, r_ga = O.msda_backward(_np(v1[:1]), shapes, _np(loc[:1]), _np(aw[:1]), _np(gout[:1]))
    np.testing.assert_allclose(ga[:1].cpu().numpy(), r_ga, rtol=2e-5, atol=2e-5)
    np.testing.assert_allclose(gv[:1].cpu().numpy(), r_gv, rtol=2e-4, atol=2e-4)
    np.testing.assert_allclose(gl[:1].cpu().numpy(), r_gl, rtol=2e-4, atol=2e-5 * max(shapes))


@pytest.mark.parametrize("path", ["rows", "pair"])
def test_bf16_T4096_bench_instantiation_matches_oracle(dev, path, monkeypatch):
    """The configs[3] per-rank call exactly as the T=4096 bench runs it: bf16 values, B=8, T=4096
    (S = Lq = 7680), M=8, D=64, P=4 — by default the row-block MFMA backward (csrc/msda_win.hip:
    a level's 30,720 samples do not fit the pair kernel's LDS lists); "pair": the pair backward
    with 8 slots a wave, one workgroup per (b, m, level) and (c0, c1) / positions staged in the
    workspace.  Clips 0 and 7 against the oracle on the same bf16-rounded inputs in fp32
    (reference semantics attention.py:331-383)."""
    if path == "pair":
        monkeypatch.setenv("MSDA_HIP_BWD_WIN", "0")
    else:
        monkeypatch.delenv("MSDA_HIP_BWD_WIN", raising=False)
    shapes, B, M, D, P = [4096, 2048, 1024, 512], 8, 8, 64, 4
    Lq = sum(shapes)
    lib = PKG._native.load_library()
    ws = lib.msda_hip_backward_workspace_bytes(PKG._native.DTYPE_TAGS[torch.bfloat16], B, Lq, M, D, Lq, 4, P)
    if path == "pair":
        assert ws >= B * M * 4 * Lq * P * 12  # the workspace-staged pair path (12 B per sample)
    else:
        assert ws == B * M * 4 * ((Lq + 31) // 32) * 8 + 128  # the row-block path's tile intervals + tail only
    value, loc, aw, gout = rand_case(shapes, B, M, D, Lq, P, torch.bfloat16, seed=41, lo=0.0, hi=1.0)
    out, gv, gl, ga = run_hip(value, shapes, loc, aw, gout)
    assert gv.dtype == torch.bfloat16
    eps = 2 ** -8
    for b in (0, B - 1):
        v32, g32 = value[b:b + 1].float(), gout[b:b + 1].float()
        r_out = O.msda_forward(_np(v32), shapes, _np(loc[b:b + 1]), _np(aw[b:b + 1]))
        r_gv, r_gl, r_ga = O.msda_backward(_np(v32), shapes, _np(loc[b:b + 1]), _np(aw[b:b + 1]), _np(g32))
        np.testing.assert_allclose(_np(out[b:b + 1]), r_out, rtol=eps, atol=eps * np.abs(r_out).max())
        np.testing.assert_allclose(_np(gv[b:b + 1]), r_gv, rtol=eps, atol=eps * np.abs(r_gv).max())
        np.testing.assert_allclose(_np(ga[b:b + 1]), r_ga, rtol=1e-4, atol=1e-4)
        np.testing.assert_allclose(_np(gl[b:b + 1]), r_gl, rtol=1e-4, atol=2e-5 * max(shapes))


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_striped_levels_near_lds_budget_take_workspace(dev, dtype):
    """Short (striped) levels with ~9.7K samples each and few (b, m, level) workgroups: the plan
    needs the striped levels' wave-partial rows beside keys / (c0, c1) / positions, which does not
    fit LDS, so the call takes the workspace-staged plan — the workspace query must ask for it
    (the query once left the partial rows out, returned 0 bytes, and the call then ran
    the sort / pull path without its workspace)."""
    shapes, B, M, D, Lq, P = [100, 50, 25, 13], 1, 8, 64, 2425, 4
    lib = PKG._native.load_library()
    ws = lib.msda_hip_backward_workspace_bytes(PKG._native.DTYPE_TAGS[dtype], B, sum(shapes), M, D, Lq, 4, P)
    assert ws > 0
    value, loc, aw, gout = rand_case(shapes, B, M, D, Lq, P, dtype, seed=43)
    out, gv, gl, ga = run_hip(value, shapes, loc, aw, gout)
    v32, g32 = value.float(), gout.float()
    r_gv, r_gl, r_ga = O.msda_backward(_np(v32), shapes, _np(loc), _np(aw), _np(g32))
    eps = 2 ** -8 if dtype == torch.bfloat16 else 2e-5
    np.testing.assert_allclose(_np(gv), r_gv, rtol=eps, atol=eps * np.abs(r_gv).max())
    np.testing.assert_allclose(_np(ga), r_ga, rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(_np(gl), r_gl, rtol=1e-4, atol=2e-5 * max(shapes))


def test_backward_without_required_workspace_is_refused(dev):
    """A call that needs a workspace and gets none returns an error (no device fault)."""
    shapes, B, M, D, Lq, P = [100, 50, 25, 13], 1, 8, 64, 2425, 4
    value, loc, aw, gout = (t.cuda() for t in rand_case(shapes, B, M, D, Lq, P, torch.float32, seed=44))
    lib = PKG._native.load_library()
    gv = torch.empty_like(value)
    rc = lib.msda_hip_backward(value.data_ptr(), PKG._native.DTYPE_TAGS[torch.float32],
                               PKG._native.host_i64_array(shapes), PKG._native.host_i64_array(O.level_starts(shapes)),
                               4, loc.data_ptr(), aw.data_ptr(), gout.data_ptr(), gv.data_ptr(), None, None, None,
                               B, sum(shapes), M, D, Lq, P, 0, PKG._native.stream_handle(value.device))
    torch.cuda.synchronize()
    assert rc != 0
    assert b"workspace" in lib.msda_hip_last_error()


WIN_CASES = [
    # shapes,                 B, M, Lq,   P, locations
    ([1024, 512, 256, 128],  2, 8, 1920, 4, "uniform"),    # encoder call
    ([256, 128, 64, 32],     2, 8, 300,  4, "clustered"),
    ([1000, 500, 250],       1, 4, 1750, 4, "uniform"),    # T not a multiple of the 64-row block
    ([50, 25, 13, 7],        3, 8, 200,  4, "uniform"),    # audio pyramid: levels shorter than a block
    ([64, 32],               2, 2, 77,   8, "clustered"),  # P = 8, a partial last query tile
    ([4096, 2048, 1024, 512], 1, 8, 7680, 4, "local"),     # configs[3] per-clip shape, encoder-like samples
    ([50, 25, 13, 7],        2, 8, 1920, 4, "uniform"),    # configs[2]: video queries on the audio pyramid
]


def local_locations(B, Lq, M, shapes, P, seed):
    """Encoder-like sampling: every query samples near its own position (within +-6 rows of a
    reference point spread over [0, 1]), as the deformable encoder does at and after init."""
    gen = torch.Generator().manual_seed(seed)
    ref = (torch.arange(Lq, dtype=torch.float64) % shapes[0] + 0.5) / shapes[0]
    loc = torch.empty(B, Lq, M, len(shapes), P, dtype=torch.float64)
    for l, T in enumerate(shapes):
        off = (torch.rand(B, Lq, M, P, generator=gen, dtype=torch.float64) * 12 - 6) / T
        loc[:, :, :, l] = ref[None, :, None, None] + off
    return loc.float()


@pytest.mark.parametrize("split", ["", "1", "8"])
@pytest.mark.parametrize("padding", ["border", "zeros"])
@pytest.mark.parametrize("case", range(len(WIN_CASES)))
def test_row_block_mfma_backward_matches_oracle(dev, monkeypatch, case, padding, split):
    """The row-block MFMA backward (csrc/msda_win.hip; MSDA_HIP_BWD_WIN=1 forces it where it
    applies: bf16 values, D = 64, P <= 8, > 512 samples a level) against the oracle on the same
    bf16-rounded inputs in fp32 (reference semantics attention.py:331-383), with the default and
    forced waves per row block (MSDA_HIP_WIN_SPLIT: visits dealt over 1 or 8 waves, partial sums
    added through LDS)."""
    monkeypatch.setenv("MSDA_HIP_BWD_WIN", "1")
    if split:
        monkeypatch.setenv("MSDA_HIP_WIN_SPLIT", split)
    else:
        monkeypatch.delenv("MSDA_HIP_WIN_SPLIT", raising=False)
    shapes, B, M, Lq, P, kind = WIN_CASES[case]
    D = 64
    value, loc, aw, gout = rand_case(shapes, B, M, D, Lq, P, torch.bfloat16, seed=60 + case)
    if kind == "clustered":
        loc = clustered_locations(B, Lq, M, shapes, P, seed=61 + case)
    elif kind == "local":
        loc = local_locations(B, Lq, M, shapes, P, seed=61 + case)
    out, gv, gl, ga = run_hip(value, shapes, loc, aw, gout, padding)
    v32, g32 = value.float(), gout.float()
    r_gv, r_gl, r_ga = O.msda_backward(_np(v32), shapes, _np(loc), _np(aw), _np(g32), padding=padding)
    eps = 2 ** -8
    np.testing.assert_allclose(_np(gv), r_gv, rtol=eps, atol=eps * np.abs(r_gv).max())
    np.testing.assert_allclose(_np(ga), r_ga, rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(_np(gl), r_gl, rtol=1e-4, atol=2e-5 * max(shapes))


@pytest.mark.parametrize("padding", ["border", "zeros"])
@pytest.mark.parametrize("case", range(len(WIN_CASES)))
def test_forward_tiles_equal_backward_prepass(dev, monkeypatch, case, padding):
    """The tiles forward (msda_hip_forward_tiles: (b, m, q)-ordered items, the row-block
    backward's tile intervals reduced in the workgroup) gives the plain forward's output bit for
    bit, and the backward fed those intervals (msda_hip_backward_tiles) gives the gradients of
    the backward that computes them in its own prepass bit for bit — both see the same rows
    (msda_win.h win_sample_rows), so every row block visits the same tiles in the same order.
    (The row-block protocol: the audio-pyramid cases would otherwise take the dense small-pyramid
    kernels, which neither write nor read tile intervals — tests/test_gpu_dense.py.)"""
    monkeypatch.setenv("MSDA_HIP_BWD_WIN", "1")
    monkeypatch.setenv("MSDA_HIP_DENSE", "0")
    shapes, B, M, Lq, P, kind = WIN_CASES[case]
    D = 64
    value, loc, aw, gout = rand_case(shapes, B, M, D, Lq, P, torch.bfloat16, seed=70 + case)
    if kind == "clustered":
        loc = clustered_locations(B, Lq, M, shapes, P, seed=71 + case)
    elif kind == "local":
        loc = local_locations(B, Lq, M, shapes, P, seed=71 + case)
    starts = O.level_starts(shapes)
    v, lc, a, g = (t.cuda() for t in (value, loc, aw, gout))
    out = msda.msda_forward(v, shapes, starts, lc, a, padding)
    out_t, tiles = msda.msda_forward(v, shapes, starts, lc, a, padding, want_tiles=True)
    n_iv = B * M * len(shapes) * ((Lq + 31) // 32) * 8  # the intervals, then the 128-B tail (msda_win.h)
    assert tiles is not None and tiles.numel() == n_iv + 128
    tail = tiles[n_iv:].view(torch.int32).cpu()
    assert torch.all(tail[:16] == 0)  # the persistent backward's queue words, zeroed by the forward
    assert torch.equal(out, out_t)
    ref = msda.msda_backward(v, shapes, starts, lc, a, g, padding)
    got = msda.msda_backward(v, shapes, starts, lc, a, g, padding, tiles=tiles)
    for r, x in zip(ref, got):
        assert torch.equal(r, x)
    # intervals: every (b, m, level, tile) interval holds each of its samples' base rows (up to
    # one row of slack: this float64 restatement may floor differently at exact row boundaries)
    iv = tiles[:n_iv].view(torch.int32).view(B, M, len(shapes), -1, 2).cpu()
    x = loc.double()
    for l, T in enumerate(shapes):
        if padding == "border":
            y = ((x[..., l, :] * 2 - 1 + 1) * (T * 0.5) - 0.5).clamp(0, T - 1).floor()
            lo_r = y
        else:
            y = x[..., l, :] * T - 0.5
            live = (y > -1) & (y < T)
            lo_r = torch.where(live, y.floor().clamp(min=0), torch.zeros_like(y))
        q_tile = torch.arange(Lq) // 32
        for t in (0, (Lq - 1) // 32):
            sel = q_tile == t
            rows = lo_r[:, sel].permute(0, 2, 1, 3).reshape(B, M, -1)  # (B, M, samples)
            assert (iv[:, :, l, t, 0] <= rows.min(-1).values.long() + 1).all()
            assert (iv[:, :, l, t, 1] >= rows.max(-1).values.long()).all()


def test_row_block_dispatch_orders_agree(dev, monkeypatch):
    """The position-chunk dispatch order (default) and the coarsest-level-first order
    (MSDA_HIP_WIN_ORDER=0) compute every row block the same way: bitwise equal gradients."""
    monkeypatch.setenv("MSDA_HIP_BWD_WIN", "1")
    shapes, B, M, Lq, P = [1024, 512, 256, 128], 3, 8, 1920, 4   # B * M = 24: pairs over 8 XCDs, 3 each
    value, loc, aw, gout = rand_case(shapes, B, M, 64, Lq, P, torch.bfloat16, seed=80)
    loc = local_locations(B, Lq, M, shapes, P, seed=81)
    runs = []
    for order in ("0", "1"):
        monkeypatch.setenv("MSDA_HIP_WIN_ORDER", order)
        runs.append(run_hip(value, shapes, loc, aw, gout))
    for a, b in zip(runs[0][1:], runs[1][1:]):
        assert torch.equal(a, b)


def clustered_locations(B, Lq, M, shapes, P, seed):
    """Half the samples scattered, half piled onto a few positions per level: long lists on a few
    rows (split between slots in table mode, walked by one slot in run mode) beside short ones."""
    gen = torch.Generator().manual_seed(seed)
    L = len(shapes)
    loc = torch.rand(B, Lq, M, L, P, generator=gen)
    hot = torch.tensor([0.1, 0.5, 0.73, 0.999]).view(1, 1, 1, 1, 4)
    pick = torch.randint(0, 4, (B, Lq, M, L, P), generator=gen)
    piled = hot.expand(B, Lq, M, L, 4).gather(-1, pick) + torch.randn(B, Lq, M, L, P, generator=gen) * 1e-3
    mask = torch.rand(B, Lq, M, L, P, generator=gen) < 0.5
    return torch.where(mask, piled, loc).clamp(-0.1, 1.1)


@pytest.mark.parametrize("rs", ["", "1", "3", "8"])
@pytest.mark.parametrize("striped_rows", ["0", ""])
@pytest.mark.parametrize("padding", ["border", "zeros"])
@pytest.mark.parametrize("shapes", [[256, 128, 64, 32], [1024, 512, 64, 32]])
def test_pair_backward_work_splits_match_oracle(dev, monkeypatch, rs, striped_rows, padding, shapes):
    """The pair-pull backward under each of its work splits: workgroups per (b, m, level)
    (MSDA_HIP_PAIR_RS; "" = the default choice), run vs striped mode per level
    (MSDA_HIP_STRIPED_ROWS: 0 = run mode everywhere, "" = striped where T + 1 < 2 x slots) and
    row mode (levels with at most 4 samples a row: T = 1024, 512 in the second pyramid)."""
    monkeypatch.setenv("MSDA_HIP_PAIR_RS", rs)
    monkeypatch.setenv("MSDA_HIP_STRIPED_ROWS", striped_rows)
    B, M, D, Lq, P = 2, 8, 64, 300, 4
    value, _, aw, gout = rand_case(shapes, B, M, D, Lq, P, torch.float32, seed=21)
    loc = clustered_locations(B, Lq, M, shapes, P, seed=22)
    out, gv, gl, ga = run_hip(value, shapes, loc, aw, gout, padding)
    r_gv, r_gl, r_ga = O.msda_backward(_np(value), shapes, _np(loc), _np(aw), _np(gout), padding=padding)
    np.testing.assert_allclose(_np(ga), r_ga, rtol=2e-5, atol=2e-5)
    np.testing.assert_allclose(_np(gv), r_gv, rtol=2e-4, atol=2e-4)
    np.testing.assert_allclose(_np(gl), r_gl, rtol=2e-4, atol=2e-5 * max(shapes))


def test_deterministic_backward_is_bitwise_reproducible(dev, tmp_path):
    """MSDA_HIP_DETERMINISTIC=1 (read once per process, so in a child process): lists sorted,
    run mode only — two calls give bitwise equal gradients, equal to the default path within
    fp32 summation-order error."""
    import subprocess
    import sys
    import os
    code = f"""
import sys, torch
sys.path.insert(0, {repr(str(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))})
sys.path.insert(0, {repr(os.path.dirname(os.path.abspath(__file__)))})
from test_gpu_op import rand_case, clustered_locations
from conftest import PKG
from oracle import msda_oracle as O
shapes = [256, 128, 64, 32]
value, _, aw, gout = rand_case(shapes, 2, 8, 64, 300, 4, torch.bfloat16, seed=31)
loc = clustered_locations(2, 300, 8, shapes, 4, seed=32)
args = [t.cuda() for t in (value, loc, aw, gout)]
starts = O.level_starts(shapes)
r1 = PKG.msda.msda_backward(args[0], shapes, starts, args[1], args[2], args[3])
r2 = PKG.msda.msda_backward(args[0], shapes, starts, args[1], args[2], args[3])
torch.save([t.cpu() for t in r1] + [t.cpu() for t in r2], sys.argv[1])
"""
    outs = {}
    for det in ("1", "0"):
        f = tmp_path / f"det{det}.pt"
        env = dict(os.environ, MSDA_HIP_DETERMINISTIC=det)
        subprocess.run([sys.executable, "-c", code, str(f)], check=True, env=env, timeout=300)
        outs[det] = torch.load(f, weights_only=True)
    d = outs["1"]
    for a, b in zip(d[:3], d[3:]):
        assert torch.equal(a, b)
    for a, b in zip(d[:3], outs["0"][:3]):
        torch.testing.assert_close(a.float(), b.float(), rtol=2e-2, atol=2e-2)


def _to_level_major(t):
    """(B, Lq, M, L, P) -> the level-major coordinate layout (B, M, L, Lq, P), contiguous."""
    return t.permute(0, 2, 3, 1, 4).contiguous()


def _from_level_major(t):
    return t.permute(0, 3, 1, 2, 4).contiguous()


@pytest.mark.parametrize("padding", ["border", "zeros"])
@pytest.mark.parametrize("case", [0, 5, 6])
def test_level_major_layout_equals_reference_layout(dev, monkeypatch, case, padding):
    """Coordinates kept level-major (MSDA_COORD_LEVEL_MAJOR, (B, M, L, Lq, P): the fused module
    path's layout) give the reference layout's forward and backward bit for bit: every row block
    visits the same samples in the same order, only the coordinate addresses differ."""
    monkeypatch.delenv("MSDA_HIP_BWD_WIN", raising=False)
    shapes, B, M, Lq, P, kind = WIN_CASES[case]
    D = 64
    value, loc, aw, gout = rand_case(shapes, B, M, D, Lq, P, torch.bfloat16, seed=90 + case)
    if kind == "local":
        loc = local_locations(B, Lq, M, shapes, P, seed=91 + case)
    starts = O.level_starts(shapes)
    v, lc, a, g = (t.cuda() for t in (value, loc, aw, gout))
    assert msda.level_major_ok(v, shapes, Lq, P)
    out, tiles = msda.msda_forward(v, shapes, starts, lc, a, padding, want_tiles=True)
    ref = msda.msda_backward(v, shapes, starts, lc, a, g, padding, tiles=tiles)
    lcm, am = _to_level_major(lc), _to_level_major(a)
    out_m, tiles_m = msda.msda_forward(v, shapes, starts, lcm, am, padding, want_tiles=True, layout=msda.LEVEL_MAJOR)
    assert torch.equal(out, out_m) and torch.equal(tiles, tiles_m)
    gv, gl, ga = msda.msda_backward(v, shapes, starts, lcm, am, g, padding, tiles=tiles_m, layout=msda.LEVEL_MAJOR)
    assert torch.equal(ref[0], gv)
    assert torch.equal(ref[1], _from_level_major(gl))
    assert torch.equal(ref[2], _from_level_major(ga))


def test_level_major_refused_without_row_block_path(dev):
    """A call whose backward does not take the row-block path (decoder-like: 100 queries) is not
    level-major capable, and the layout entry points refuse it (no silent misread)."""
    shapes, B, M, D, Lq, P = [1024, 512, 256, 128], 2, 8, 64, 100, 4
    value, loc, aw, gout = (t.cuda() for t in rand_case(shapes, B, M, D, Lq, P, torch.bfloat16, seed=95))
    assert not msda.level_major_ok(value, shapes, Lq, P)
    with pytest.raises(RuntimeError, match="level-major"):
        msda.msda_forward(value, shapes, O.level_starts(shapes), _to_level_major(loc), _to_level_major(aw),
                          layout=msda.LEVEL_MAJOR)


LM_CASES = [
    # shapes,                  B, M, P: every case has > 4096 row blocks (the persistent kernel's calls)
    ([1024, 512, 256, 128],    8, 8, 4),   # the bench's encoder call
    ([1000, 500, 250, 125],    8, 8, 4),   # ragged: T not a multiple of 16, Lq not of 32
    ([1000, 500, 250, 125],    8, 8, 2),
    ([2048, 1024, 512, 256],   2, 16, 1),
]


@pytest.mark.parametrize("padding", ["border", "zeros"])
@pytest.mark.parametrize("case", range(len(LM_CASES)))
def test_level_major_row_kernel_equals_per_block_kernel(dev, monkeypatch, case, padding):
    """win_lm_kernel (the level-major row-block backward: swizzled LDS rows, reordered phases, the
    tile order read from the tiles tail) gives win_bwd_kernel's gradients bit for bit (same visits in
    the same order, same MFMA products); three backwards on one forward's tiles agree, and the
    tail's reserved words stay zero."""
    for k in ("MSDA_HIP_BWD_WIN", "MSDA_HIP_WIN_SPLIT", "MSDA_HIP_WIN_ORDER", "MSDA_HIP_BWD_PATH", "MSDA_HIP_QORDER",
              "MSDA_HIP_WIN_LM"):
        monkeypatch.delenv(k, raising=False)
    monkeypatch.setenv("MSDA_HIP_WIN_LM_SPLIT", "0")  # (one wave a block: the per-block kernel's sum order)
    shapes, B, M, P = LM_CASES[case]
    D, Lq = 64, sum(shapes)
    value, _, aw, gout = rand_case(shapes, B, M, D, Lq, P, torch.bfloat16, seed=120 + case, lo=0.0, hi=1.0)
    loc = local_locations(B, Lq, M, shapes, P, seed=121 + case)
    starts = O.level_starts(shapes)
    v, g = value.cuda(), gout.cuda()
    lcm, am = _to_level_major(loc).cuda(), _to_level_major(aw).cuda()
    _, tiles = msda.msda_forward(v, shapes, starts, lcm, am, padding, want_tiles=True, layout=msda.LEVEL_MAJOR)
    assert tiles is not None
    runs = [msda.msda_backward(v, shapes, starts, lcm, am, g, padding, tiles=tiles, layout=msda.LEVEL_MAJOR)
            for _ in range(3)]
    n_iv = B * M * len(shapes) * ((Lq + 31) // 32) * 8
    torch.cuda.synchronize()
    assert torch.all(tiles[n_iv:].view(torch.int32)[:16].cpu() == 0)
    monkeypatch.setenv("MSDA_HIP_WIN_LM", "0")
    ref = msda.msda_backward(v, shapes, starts, lcm, am, g, padding, tiles=tiles, layout=msda.LEVEL_MAJOR)
    for run in runs:
        for r, x in zip(ref, run):
            assert torch.equal(r, x)


@pytest.mark.parametrize("padding", ["border", "zeros"])
@pytest.mark.parametrize("case", range(len(LM_CASES)))
def test_level_major_split_blocks_equal_single_wave_blocks(dev, monkeypatch, case, padding):
    """win_lm_kernel's split mode (round 6, opt-in MSDA_HIP_WIN_LM_SPLIT=1: 4-wave workgroups, the coarse
    levels' blocks shared by 2 / 4 waves that take the block's visits round-robin and add their
    grad_value partials in wave order) against one wave a block (the default): the coordinate gradients bit for bit (each
    visit's arithmetic is unchanged), grad_value within one bf16 rounding (fp32 partial sums added in
    another order); the split backward is reproducible bit for bit."""
    for k in ("MSDA_HIP_BWD_WIN", "MSDA_HIP_WIN_SPLIT", "MSDA_HIP_WIN_ORDER", "MSDA_HIP_BWD_PATH", "MSDA_HIP_QORDER",
              "MSDA_HIP_WIN_LM", "MSDA_HIP_WIN_LM_SPLIT"):
        monkeypatch.delenv(k, raising=False)
    shapes, B, M, P = LM_CASES[case]
    D, Lq = 64, sum(shapes)
    value, _, aw, gout = rand_case(shapes, B, M, D, Lq, P, torch.bfloat16, seed=140 + case, lo=0.0, hi=1.0)
    loc = local_locations(B, Lq, M, shapes, P, seed=141 + case)
    starts = O.level_starts(shapes)
    v, g = value.cuda(), gout.cuda()
    lcm, am = _to_level_major(loc).cuda(), _to_level_major(aw).cuda()
    _, tiles = msda.msda_forward(v, shapes, starts, lcm, am, padding, want_tiles=True, layout=msda.LEVEL_MAJOR)
    monkeypatch.setenv("MSDA_HIP_WIN_LM_SPLIT", "1")
    split = [msda.msda_backward(v, shapes, starts, lcm, am, g, padding, tiles=tiles, layout=msda.LEVEL_MAJOR)
             for _ in range(2)]
    monkeypatch.setenv("MSDA_HIP_WIN_LM_SPLIT", "0")
    one = msda.msda_backward(v, shapes, starts, lcm, am, g, padding, tiles=tiles, layout=msda.LEVEL_MAJOR)
    torch.cuda.synchronize()
    for x, y in zip(split[0], split[1]):
        assert torch.equal(x, y)
    assert torch.equal(split[0][1], one[1]) and torch.equal(split[0][2], one[2])
    a, b = split[0][0].float(), one[0].float()
    torch.testing.assert_close(a, b, rtol=2 ** -8, atol=2 ** -8 * b.abs().max().item())


@pytest.mark.parametrize("padding", ["border", "zeros"])
@pytest.mark.parametrize("case", range(len(WIN_CASES)))
@pytest.mark.parametrize("stage", ["1", "2"])
def test_staged_forward_equals_gathering_forward(dev, monkeypatch, case, padding, stage):
    """msda_fwd16_stage_kernel (each wave's rows of a level staged in its LDS slice when the window
    fits, 48 / 32 rows; global gathers otherwise) gives the gathering tiles forward's output and tile
    intervals bit for bit, in both coordinate layouts — on encoder-like local sampling (windows
    staged) and on uniform / clustered sampling (windows over the cap: the fallback)."""
    monkeypatch.setenv("MSDA_HIP_DENSE", "0")  # (the gathering forwards' tile protocol; tests/test_gpu_dense.py)
    for k in ("MSDA_HIP_FWD_LDS", "MSDA_HIP_QORDER", "MSDA_HIP_BWD_WIN"):
        monkeypatch.delenv(k, raising=False)
    monkeypatch.setenv("MSDA_HIP_BWD_WIN", "1")
    shapes, B, M, Lq, P, kind = WIN_CASES[case]
    D = 64
    value, loc, aw, gout = rand_case(shapes, B, M, D, Lq, P, torch.bfloat16, seed=140 + case)
    if kind == "clustered":
        loc = clustered_locations(B, Lq, M, shapes, P, seed=141 + case)
    elif kind == "local" or (kind == "uniform" and Lq == sum(shapes)):
        loc = local_locations(B, Lq, M, shapes, P, seed=141 + case)
    starts = O.level_starts(shapes)
    v, lc, a = value.cuda(), loc.cuda(), aw.cuda()
    for layout in (0, msda.LEVEL_MAJOR):
        if layout and not msda.level_major_ok(v, shapes, Lq, P):
            continue
        lcx, ax = (_to_level_major(lc), _to_level_major(a)) if layout else (lc, a)
        monkeypatch.setenv("MSDA_HIP_FWD_STAGE", "0")
        ref = msda.msda_forward(v, shapes, starts, lcx, ax, padding, want_tiles=True, layout=layout)
        monkeypatch.setenv("MSDA_HIP_FWD_STAGE", stage)
        got = msda.msda_forward(v, shapes, starts, lcx, ax, padding, want_tiles=True, layout=layout)
        assert torch.equal(ref[0], got[0]) and torch.equal(ref[1], got[1])


def test_profiling_switch_refused_in_training(dev, monkeypatch):
    """MSDA_HIP_WIN_EXP skips parts of the row-block kernel (wrong gradients, profiling only): set
    without MSDA_HIP_PROFILING=1 the backward raises instead of silently returning them."""
    shapes, B, M, D, P = [256, 128, 64, 32], 2, 8, 64, 4
    Lq = sum(shapes)
    value, loc, aw, gout = (t.cuda() for t in rand_case(shapes, B, M, D, Lq, P, torch.bfloat16, seed=130))
    starts = O.level_starts(shapes)
    monkeypatch.setenv("MSDA_HIP_BWD_WIN", "1")
    monkeypatch.delenv("MSDA_HIP_PROFILING", raising=False)
    monkeypatch.setenv("MSDA_HIP_WIN_EXP", "1")
    with pytest.raises(RuntimeError, match="MSDA_HIP_WIN_EXP"):
        msda.msda_backward(value, shapes, starts, loc, aw, gout, "border", tiles=None)


@pytest.mark.parametrize("layout", ["reference", "level_major"])
def test_bf16_T1024_bench_instantiation_matches_oracle(dev, monkeypatch, layout):
    """The configs[1] encoder call exactly as the bench step runs it: bf16 values, B=8, T=1024
    (S = Lq = 1920), M=8, D=64, P=4, no environment forcing, through the autograd Function — the
    forward writes the tile intervals (msda_fwd16_tiles_kernel) and the backward takes the
    row-block MFMA kernel fed by them; "level_major": with the module path's level-major
    coordinates.  Clips 0 and 7 against the oracle on the same bf16-rounded inputs in fp32
    (reference semantics attention.py:331-383)."""
    for k in ("MSDA_HIP_BWD_WIN", "MSDA_HIP_WIN_SPLIT", "MSDA_HIP_WIN_ORDER", "MSDA_HIP_BWD_PATH",
              "MSDA_HIP_LEVEL_MAJOR", "MSDA_HIP_QORDER"):
        monkeypatch.delenv(k, raising=False)
    shapes, B, M, D, P = [1024, 512, 256, 128], 8, 8, 64, 4
    Lq = sum(shapes)
    value, _, aw, gout = rand_case(shapes, B, M, D, Lq, P, torch.bfloat16, seed=97, lo=0.0, hi=1.0)
    loc = local_locations(B, Lq, M, shapes, P, seed=98)
    starts = O.level_starts(shapes)
    lm = layout == "level_major"
    v = value.cuda().requires_grad_(True)
    lc = (_to_level_major(loc) if lm else loc).cuda().requires_grad_(True)
    a = (_to_level_major(aw) if lm else aw).cuda().requires_grad_(True)
    assert msda.level_major_ok(v, shapes, Lq, P)
    PKG._trace.clear()
    out = msda.msda_apply(v, shapes, starts, lc, a, "border", layout=msda.LEVEL_MAJOR if lm else 0)
    out.backward(gout.cuda())
    torch.cuda.synchronize()
    assert PKG._trace.hits.get("msda_bfloat16", 0) == 1
    assert (PKG._trace.hits.get("msda_level_major", 0) == 1) == lm
    gl, ga = (_from_level_major(t.grad) if lm else t.grad for t in (lc, a))
    eps = 2 ** -8
    for b in (0, B - 1):
        v32, g32 = value[b:b + 1].float(), gout[b:b + 1].float()
        r_out = O.msda_forward(_np(v32), shapes, _np(loc[b:b + 1]), _np(aw[b:b + 1]))
        r_gv, r_gl, r_ga = O.msda_backward(_np(v32), shapes, _np(loc[b:b + 1]), _np(aw[b:b + 1]), _np(g32))
        np.testing.assert_allclose(_np(out[b:b + 1]), r_out, rtol=eps, atol=eps * np.abs(r_out).max())
        np.testing.assert_allclose(_np(v.grad[b:b + 1]), r_gv, rtol=eps, atol=eps * np.abs(r_gv).max())
        np.testing.assert_allclose(_np(ga[b:b + 1]), r_ga, rtol=1e-4, atol=1e-4)
        np.testing.assert_allclose(_np(gl[b:b + 1]), r_gl, rtol=1e-4, atol=2e-5 * max(shapes))


@pytest.mark.parametrize("layout", ["reference", "level_major"])
@pytest.mark.parametrize("padding", ["border", "zeros"])
@pytest.mark.parametrize("shapes", [[128, 64, 32, 16], [1024, 512, 256, 128], [96, 48, 24]])
def test_position_order_tiles_equal_consecutive_tiles(dev, monkeypatch, shapes, padding, layout):
    """Encoder-shaped calls (Lq == S) group the row-block backward's query tiles in position order
    (msda_win.h QOrder: every level's tokens of one stretch of the sequence together); grouping
    only, so the output and the coordinate gradients equal those of tiles of consecutive queries
    (MSDA_HIP_QORDER=0) bit for bit, and grad_value (the same terms added in another visit order,
    fp32 accumulation) within one bf16 rounding — ragged last tile (S = 240), 3 levels, both
    paddings and coordinate layouts.  Spread around each query's position."""
    for k in ("MSDA_HIP_WIN_SPLIT", "MSDA_HIP_WIN_ORDER", "MSDA_HIP_BWD_PATH"):
        monkeypatch.delenv(k, raising=False)
    monkeypatch.setenv("MSDA_HIP_BWD_WIN", "1")  # (the row-block path on the short pyramids too)
    B, M, D, P = 2, 8, 64, 4
    Lq = sum(shapes)
    value, _, aw, gout = rand_case(shapes, B, M, D, Lq, P, torch.bfloat16, seed=31, lo=0.0, hi=1.0)
    loc = local_locations(B, Lq, M, shapes, P, seed=32)
    starts = O.level_starts(shapes)
    lm = layout == "level_major"
    res = []
    for qorder in ("1", "0"):
        monkeypatch.setenv("MSDA_HIP_QORDER", qorder)
        v = value.cuda().requires_grad_(True)
        lc = (_to_level_major(loc) if lm else loc).cuda().requires_grad_(True)
        a = (_to_level_major(aw) if lm else aw).cuda().requires_grad_(True)
        PKG._trace.clear()
        out = msda.msda_apply(v, shapes, starts, lc, a, padding, layout=msda.LEVEL_MAJOR if lm else 0)
        out.backward(gout.cuda())
        torch.cuda.synchronize()
        assert PKG._trace.hits.get("msda_bfloat16", 0) == 1
        res.append([out.detach(), v.grad, lc.grad, a.grad])
    (o1, gv1, gl1, ga1), (o0, gv0, gl0, ga0) = res
    assert torch.equal(o1, o0) and torch.equal(gl1, gl0) and torch.equal(ga1, ga0)
    eps = 2 ** -8
    torch.testing.assert_close(gv1.float(), gv0.float(), rtol=eps, atol=eps * gv0.float().abs().max().item())


def test_bf16_sparse_bench_instantiation_matches_oracle(dev, monkeypatch):
    """The Sparse-DETR encoder call of the sparse bench line (rho = 0.3: 577 of the 1920 tokens of
    the T = 1024 pyramid, B = 8, bf16, reference coordinate layout), default path with no
    environment forcing, through the autograd Function: the top-k tokens in position order as
    models/sparse/unimodal_sparse_deformable_transformer.py hands them over (reference points of
    every level interleaved), each sampling around its own position, so the backward takes the
    row-block kernel (win_applies: Lq P >= 2048 on >= 64-row levels).  Clips 0 and 7 against the
    oracle on the same bf16-rounded inputs in fp32 (reference attention.py:331-383, sparse
    transformer :210-218, 425-450)."""
    for k in ("MSDA_HIP_BWD_WIN", "MSDA_HIP_WIN_SPLIT", "MSDA_HIP_WIN_ORDER", "MSDA_HIP_BWD_PATH",
              "MSDA_HIP_QORDER"):
        monkeypatch.delenv(k, raising=False)
    shapes, B, M, D, P, Lq = [1024, 512, 256, 128], 8, 8, 64, 4, 577
    S = sum(shapes)
    value, _, aw, gout = rand_case(shapes, B, M, D, Lq, P, torch.bfloat16, seed=113, lo=0.0, hi=1.0)
    pos = torch.cat([(torch.arange(T, dtype=torch.float64) + 0.5) / T for T in shapes])
    gen = torch.Generator().manual_seed(114)
    loc = torch.empty(B, Lq, M, len(shapes), P, dtype=torch.float64)
    for b in range(B):
        tok = torch.randperm(S, generator=gen)[:Lq]
        tok = tok[pos[tok].sort(stable=True)[1]]
        for l, T in enumerate(shapes):
            off = (torch.rand(Lq, M, P, generator=gen, dtype=torch.float64) * 8 - 4) / T
            loc[b, :, :, l] = pos[tok][:, None, None] + off
    loc = loc.float()
    starts = O.level_starts(shapes)
    v = value.cuda().requires_grad_(True)
    lc, a = loc.cuda().requires_grad_(True), aw.cuda().requires_grad_(True)
    out = msda.msda_apply(v, shapes, starts, lc, a, "border")
    out.backward(gout.cuda())
    torch.cuda.synchronize()
    lib = PKG._native.load_library()
    nb = lib.msda_hip_forward_tiles_bytes(PKG._native.DTYPE_TAGS[torch.bfloat16], PKG._native.host_i64_array(shapes),
                                          len(shapes), B, S, M, D, Lq, P)
    assert nb > 0  # the tiles forward + row-block backward take this call
    eps = 2 ** -8
    for b in (0, B - 1):
        v32, g32 = value[b:b + 1].float(), gout[b:b + 1].float()
        r_out = O.msda_forward(_np(v32), shapes, _np(loc[b:b + 1]), _np(aw[b:b + 1]))
        r_gv, r_gl, r_ga = O.msda_backward(_np(v32), shapes, _np(loc[b:b + 1]), _np(aw[b:b + 1]), _np(g32))
        np.testing.assert_allclose(_np(out[b:b + 1]), r_out, rtol=eps, atol=eps * np.abs(r_out).max())
        np.testing.assert_allclose(_np(v.grad[b:b + 1]), r_gv, rtol=eps, atol=eps * np.abs(r_gv).max())
        np.testing.assert_allclose(_np(a.grad[b:b + 1]), r_ga, rtol=1e-4, atol=1e-4)
        np.testing.assert_allclose(_np(lc.grad[b:b + 1]), r_gl, rtol=1e-4, atol=2e-5 * max(shapes))


@pytest.mark.parametrize("padding", ["border", "zeros"])
@pytest.mark.parametrize("case", range(len(WIN_CASES)))
def test_lds_staged_forward_equals_gather_forward(dev, monkeypatch, case, padding):
    """The LDS-staged tiles forward (msda_fwd16_lds_kernel: each workgroup's per-level row
    intervals staged in LDS, taps read there; levels over the row budget gathered from global)
    gives the gathering tiles forward's output and tile intervals bit for bit."""
    monkeypatch.setenv("MSDA_HIP_DENSE", "0")  # (the gathering forwards' tile protocol; tests/test_gpu_dense.py)
    monkeypatch.setenv("MSDA_HIP_BWD_WIN", "1")
    shapes, B, M, Lq, P, kind = WIN_CASES[case]
    value, loc, aw, _ = rand_case(shapes, B, M, 64, Lq, P, torch.bfloat16, seed=100 + case)
    if kind == "clustered":
        loc = clustered_locations(B, Lq, M, shapes, P, seed=101 + case)
    elif kind == "local":
        loc = local_locations(B, Lq, M, shapes, P, seed=101 + case)
    starts = O.level_starts(shapes)
    v, lc, a = (t.cuda() for t in (value, loc, aw))
    runs = []
    for flag in ("0", "1"):
        monkeypatch.setenv("MSDA_HIP_FWD_LDS", flag)
        runs.append(msda.msda_forward(v, shapes, starts, lc, a, padding, want_tiles=True))
    assert torch.equal(runs[0][0], runs[1][0]) and torch.equal(runs[0][1], runs[1][1])


@pytest.mark.gpu
def test_strided_grad_value_slot_matches_contiguous(dev):
    """msda_hip_backward_ex (ABI v8): a decoder-like call (the per-tap fused backward) writes
    grad_value into a strided column block of a wider buffer — the decoder layers' stacked value
    gradients (value_proj.layer_values) — with the values of the contiguous backward and nothing
    outside the block touched; an encoder-like call, whose path cannot write the slot, reports it and
    the wrapper returns a fresh grad_value instead."""
    B, M, D, P, n = 8, 8, 64, 4, 3  # (B M L >= 256: the fused path's own condition)
    for shapes, Lq, slot_expected in (([64, 32, 16, 8], 50, True), ([256, 128, 64, 32], 480, False)):
        starts = O.level_starts(shapes)
        S = sum(shapes)
        value, loc, aw, gout = (t.to(dev) for t in rand_case(shapes, B, M, D, Lq, P, torch.bfloat16, 41))
        G = torch.full((B * S, n * M * D), float("nan"), dtype=torch.bfloat16, device=dev)
        slot = G.view(B * S, n, M * D)[:, 1].view(B, S, M, D)
        PKG._trace.clear()
        gv, gl, ga = msda.msda_backward(value, shapes, starts, loc, aw, gout, grad_value_out=slot)
        want_v, want_l, want_a = msda.msda_backward(value, shapes, starts, loc, aw, gout)
        torch.cuda.synchronize()
        took = PKG._trace.hits.get("msda_grad_value_slot", 0) == 1
        assert took == slot_expected and (gv is slot) == slot_expected
        # (per-row fp32 sums in list order: the fused kernel's order may differ run to run)
        torch.testing.assert_close(gv.float(), want_v.float(), rtol=1e-2, atol=1e-2)
        torch.testing.assert_close(gl, want_l, rtol=1e-4, atol=1e-4)
        torch.testing.assert_close(ga, want_a, rtol=1e-4, atol=1e-4)
        others = G.view(B * S, n, M * D)[:, [0, 2]]
        assert torch.isnan(others.float()).all()
        if not slot_expected:
            assert torch.isnan(slot.float()).all()


@pytest.mark.gpu
def test_bf16_unsorted_topk_call_takes_row_block_correctly(dev, monkeypatch):
    """win_applies' clause for Lq P >= 2048 on >= 64-row levels also takes query sets that
    are NOT position-ordered (each tile's intervals then span a whole level).  The same 577-of-1920
    top-k call as the sparse bench line with the tokens in random (score) order: the row-block backward
    still matches the oracle, and its time is reported against the pair kernel's on the same inputs
    (MSDA_HIP_BWD_WIN=0) — allowed to be slower, not pathologically (<= 4x)."""
    for k in ("MSDA_HIP_BWD_WIN", "MSDA_HIP_WIN_SPLIT", "MSDA_HIP_WIN_ORDER", "MSDA_HIP_BWD_PATH",
              "MSDA_HIP_QORDER"):
        monkeypatch.delenv(k, raising=False)
    shapes, B, M, D, P, Lq = [1024, 512, 256, 128], 8, 8, 64, 4, 577
    S = sum(shapes)
    value, _, aw, gout = rand_case(shapes, B, M, D, Lq, P, torch.bfloat16, seed=115, lo=0.0, hi=1.0)
    pos = torch.cat([(torch.arange(T, dtype=torch.float64) + 0.5) / T for T in shapes])
    gen = torch.Generator().manual_seed(116)
    loc = torch.empty(B, Lq, M, len(shapes), P, dtype=torch.float64)
    for b in range(B):
        tok = torch.randperm(S, generator=gen)[:Lq]  # score order: no sort by position
        for l, T in enumerate(shapes):
            off = (torch.rand(Lq, M, P, generator=gen, dtype=torch.float64) * 8 - 4) / T
            loc[b, :, :, l] = pos[tok][:, None, None] + off
    loc = loc.float()
    starts = O.level_starts(shapes)
    vd, ld, ad, gd = value.cuda(), loc.cuda(), aw.cuda(), gout.cuda()
    lib = PKG._native.load_library()
    nb = lib.msda_hip_forward_tiles_bytes(PKG._native.DTYPE_TAGS[torch.bfloat16], PKG._native.host_i64_array(shapes),
                                          len(shapes), B, S, M, D, Lq, P)
    assert nb > 0  # the row-block path takes it

    def timed(env):
        if env is None:
            monkeypatch.delenv("MSDA_HIP_BWD_WIN", raising=False)
        else:
            monkeypatch.setenv("MSDA_HIP_BWD_WIN", env)
        _, tiles = msda.msda_forward(vd, shapes, starts, ld, ad, want_tiles=True)
        res = msda.msda_backward(vd, shapes, starts, ld, ad, gd, tiles=tiles)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            msda.msda_backward(vd, shapes, starts, ld, ad, gd, tiles=tiles)
        e1.record()
        torch.cuda.synchronize()
        return res, e0.elapsed_time(e1) / 10 * 1e3

    (gv, gl, ga), t_win = timed(None)
    _, t_pair = timed("0")
    print(f"unsorted top-k backward: row-block {t_win:.1f} us, pair {t_pair:.1f} us")
    assert t_win <= 4 * t_pair, (t_win, t_pair)
    eps = 2 ** -8
    v32, g32 = value[:1].float(), gout[:1].float()
    r_gv, r_gl, r_ga = O.msda_backward(_np(v32), shapes, _np(loc[:1]), _np(aw[:1]), _np(g32))
    np.testing.assert_allclose(_np(gv[:1]), r_gv, rtol=eps, atol=eps * np.abs(r_gv).max())
    np.testing.assert_allclose(_np(ga[:1]), r_ga, rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(_np(gl[:1]), r_gl, rtol=1e-4, atol=2e-5 * max(shapes))
