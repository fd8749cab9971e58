"""The reference's extension API on the GPU (``-m gpu``), called with the reference's own signatures
and checked against fixtures the reference produced (tests/golden/make_golden.py):

* ``MultiScaleDeformableAttention.ms_deform_attn_forward / _backward`` (vision.cpp:14-15) on (L,2)
  [H=1, W] shapes and (...,2) [x, y] locations — zeros padding of the extension kernel, y-gradient
  included — against ``ops_api_f64[zeros]`` (the reference's 2-D core with zero padding: the
  comparator of its own models/ops/test.py:38-39);
* ``MSDeformAttnFunction.apply(value, shapes, lsi, loc, aw, im2col_step)`` from both reference
  locations (ops/functions/ms_deform_attn_func.py:23-41, modules/attention.py:310-328) through autograd;
* the 2-D border core (ops/functions/ms_deform_attn_func.py:44-71) and both ``return_value`` stacks
  (there :67-68 and attention.py:376-378);
* the ops modules ``MSDeformAttn`` (zero-padding kernel on the GPU, :119-122) and ``MSDeformAttnCap``;
* the im2col_step divisibility check of ms_deform_attn_cuda.cu:50-52;
* the bench precision: the transformer under bf16 autocast vs the reference's own bf16-autocast run.

Tolerances: fp64 paths 1e-10 relative (only accumulation order differs); bf16 in its test."""
import pytest
import torch

from conftest import PKG

pytestmark = pytest.mark.gpu
MSDA = PKG.MultiScaleDeformableAttention
OPS = PKG.models.ops


def _close(a, b, rtol=1e-10, atol=1e-11):
    torch.testing.assert_close(a.detach().cpu().to(b.dtype), b, rtol=rtol, atol=atol)


def _inputs(g, dev):
    shapes2d = g["shapes2d"].to(dev)
    lsi = torch.cat((shapes2d.new_zeros(1), shapes2d.prod(1).cumsum(0)[:-1]))
    return (g["value"].to(dev), shapes2d, lsi, g["loc2"].to(dev), g["aw"].to(dev), g["grad_out"].to(dev))


def test_extension_forward_backward_zeros_2d(golden, dev):
    g = golden("ops_api_f64")
    value, shapes2d, lsi, loc2, aw, gout = _inputs(g, dev)
    r = g["zeros"]
    out = MSDA.ms_deform_attn_forward(value, shapes2d, lsi, loc2, aw, 2)
    gv, gl, ga = MSDA.ms_deform_attn_backward(value, shapes2d, lsi, loc2, aw, gout, 2)
    _close(out, r["out"])
    _close(gv, r["grad_value"])
    _close(ga, r["grad_aw"])
    _close(gl, r["grad_loc"], rtol=1e-10, atol=1e-9)
    assert gl.shape == loc2.shape and (r["grad_loc"][..., 1] != 0).any()


@pytest.mark.parametrize("where", ["ops.functions", "modules.attention"])
@pytest.mark.parametrize("im2col_step", [2, 64])
def test_msdeformattnfunction_apply_reference_signature(golden, dev, where, im2col_step):
    g = golden("ops_api_f64")
    value, shapes2d, lsi, loc2, aw, gout = _inputs(g, dev)
    fn = (OPS.functions.MSDeformAttnFunction if where == "ops.functions"
          else PKG.models.modules.attention.MSDeformAttnFunction)
    v, lc, a = (t.clone().requires_grad_(True) for t in (value, loc2, aw))
    out = fn.apply(v, shapes2d, lsi, lc, a, im2col_step)
    out.backward(gout)
    r = g["zeros"]
    _close(out, r["out"])
    _close(v.grad, r["grad_value"])
    _close(a.grad, r["grad_aw"])
    _close(lc.grad, r["grad_loc"], rtol=1e-10, atol=1e-9)


def test_im2col_step_must_divide_batch(golden, dev):
    g = golden("ops_api_f64")
    value, shapes2d, lsi, loc2, aw, _ = _inputs(g, dev)
    v3, l3, a3 = (torch.cat([t, t[:1]]) for t in (value, loc2, aw))
    with pytest.raises(RuntimeError, match="must divide im2col_step"):
        MSDA.ms_deform_attn_forward(v3.contiguous(), shapes2d, lsi, l3.contiguous(), a3.contiguous(), 2)
    MSDA.ms_deform_attn_forward(v3.contiguous(), shapes2d, lsi, l3.contiguous(), a3.contiguous(), 64)  # min(B, step)
    with pytest.raises(RuntimeError, match="contiguous"):
        MSDA.ms_deform_attn_forward(value.transpose(2, 3), shapes2d, lsi, loc2, aw, 2)


def test_ops_core_border_2d(golden, dev):
    g = golden("ops_api_f64")
    value, shapes2d, _, loc2, aw, gout = _inputs(g, dev)
    v, lc, a = (t.clone().requires_grad_(True) for t in (value, loc2, aw))
    out = OPS.functions.ms_deform_attn_core_pytorch(v, shapes2d, lc, a)
    out.backward(gout)
    r = g["border"]
    _close(out, r["out"])
    _close(v.grad, r["grad_value"])
    _close(a.grad, r["grad_aw"])
    _close(lc.grad, r["grad_loc"], rtol=1e-10, atol=1e-9)
    assert (lc.grad[..., 1] == 0).all()


@pytest.mark.parametrize("which", ["ops_border", "live"])
def test_return_value_stacks(golden, dev, which):
    g = golden("ops_api_f64")
    value, shapes2d, _, loc2, aw, _ = _inputs(g, dev)
    v, lc, a = (t.clone().requires_grad_(True) for t in (value, loc2, aw))
    if which == "live":
        shapes = torch.tensor([int(w) for _, w in g["shapes2d"].tolist()], device=dev).unsqueeze(-1)
        st = PKG.models.modules.attention.ms_deform_attn_core_pytorch(v, shapes, lc[..., :1], a, return_value=True)
    else:
        st = OPS.functions.ms_deform_attn_core_pytorch(v, shapes2d, lc, a, return_value=True)
    (st * g["w_stack"].to(dev)).sum().backward()
    r = g["stack_" + which]
    assert st.shape == r["stack"].shape
    _close(st, r["stack"])
    _close(v.grad, r["grad_value"])
    _close(lc.grad, r["grad_loc"], rtol=1e-10, atol=1e-9)


@pytest.mark.parametrize("name", ["attn", "cap"])
@pytest.mark.parametrize("case", ["enc", "dec"])
def test_ops_modules_match_reference(golden, dev, name, case):
    g = golden("ops_module_f64")
    e = g[name]
    d_model = e["state_dict"]["value_proj.weight"].shape[0]
    cls = OPS.modules.MSDeformAttn if name == "attn" else OPS.modules.MSDeformAttnCap
    m = cls(d_model, 4, 4, 4).double()
    m.load_state_dict({k: v.double() for k, v in e["state_dict"].items()})
    m = m.to(dev)
    shp = g["shapes"].to(dev)
    start = torch.cat((shp.new_zeros(1), shp.cumsum(0)[:-1]))
    d = e[case]
    q = d["query"].to(dev).requires_grad_(True)
    x = d["input_flatten"].to(dev).requires_grad_(True)
    y = m(q, d["reference_points"].to(dev), x, shp, start, e["padding_mask"].to(dev))
    y.backward(d["grad_out"].to(dev))
    _close(y, d["output"], 1e-9, 1e-10)
    _close(q.grad, d["grad_query"], 1e-8, 1e-10)
    _close(x.grad, d["grad_input_flatten"], 1e-8, 1e-10)
    for k, p in m.named_parameters():
        if k in d["param_grads"]:
            _close(p.grad, d["param_grads"][k], 1e-8, 1e-10)
        else:
            assert p.grad is None


def test_transformer_bf16_autocast_matches_reference_bf16(golden, dev):
    """The bench precision pinned against the reference: the same 2+2 transformer, weights and
    inputs as transformer_f64, under bf16 autocast here (cuda) and in the reference (cpu).  Our bf16
    result must be as close to the fp64 truth as the reference's own bf16 run (within 1.5x + 2e-3)
    and close to that run itself."""
    from test_host_modules import build_transformer_stack, run_transformer_stack
    g64 = golden("transformer_f64")
    gb = golden("transformer_bf16")
    mods = build_transformer_stack(g64, device=dev)
    for m in mods.values():
        m.float()
    video = g64["video"].to(dev, torch.float32).requires_grad_(True)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        memory, hs, _ = run_transformer_stack(mods, video, g64["mask"].to(dev), g64["durations"].to(dev, torch.float32))
    loss = (hs.float() * g64["w_hs"].to(dev).float()).sum() + (memory.float() * g64["w_mem"].to(dev).float()).sum()
    loss.backward()

    def rel(a, b):
        a, b = a.detach().cpu().double(), b.double()
        return ((a - b).norm() / b.norm()).item()

    for ours, key, ref64 in ((memory, "memory", g64["memory"]), (hs, "hs", g64["hs"]),
                             (video.grad, "grad_video", g64["grad_video"])):
        ref16 = gb[key]
        ours_err, ref_err = rel(ours, ref64), rel(ref16, ref64)
        assert ours_err <= 1.5 * ref_err + 2e-3, (key, ours_err, ref_err)
        assert rel(ours, ref16) <= 2.5 * ref_err + 2e-3, (key, rel(ours, ref16), ref_err)
