"""Diagnose the caption head weight-gradient error (bf16 autocast vs the fixture's fp64 truth)."""
import importlib.util, os, sys
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
from conftest import PKG
spec = importlib.util.spec_from_file_location("_mg", os.path.join(ROOT, "tests", "golden", "make_golden.py"))
MG = importlib.util.module_from_spec(spec); spec.loader.exec_module(MG)
dev = torch.device("cuda", 0)
g = torch.load(os.path.join(ROOT, "tests/golden/caption_bf16.pt"), weights_only=True)
c = {k: (float(v) if k == "head_scale" else int(v)) for k, v in g["config"].items()}
dec = PKG.models.unimodal_caption_decoder.UnimodalCaptionDecoder(c["vocab"], seq_len=c["seq_len"], d_model=c["d_model"], depth=c["depth"], num_heads=c["heads"], mlp_ratio=4, qkv_bias=True, pre_norm=False, return_intermediate=True)
MG.regen_parameters(dec, c["seed"], scale={"head.weight": c["head_scale"]})
dec = dec.to(dev)
tgt, memory, kmask = (t.to(dev) for t in MG.caption_inputs())
padding, tgt_mask = MG.caption_masks(tgt, c["pad"])
nxt = torch.cat([tgt[:, 1:], torch.full((c["N"], 1), c["eos"], device=dev)], 1)
live = nxt != c["pad"]
cap = {}
real_fwd = PKG.models.modules.linear._AutocastLinear.forward
def _hook(m, i, o):
    cap["x"] = i[0]
    o.register_hook(lambda gr: cap.__setitem__("gy", gr))


h = dec.head.register_forward_hook(_hook)
with torch.autocast("cuda", dtype=torch.bfloat16):
    out = dec(tgt, memory, tgt_mask=tgt_mask, memory_mask=kmask[:, None, None, :], tgt_padding_mask=padding)
print("out dtype", out.dtype, "logits dtype", cap["x"].dtype)
out = out.float()
p_t = out.gather(-1, nxt[None, :, :, None].expand(out.shape[0], -1, -1, 1))[..., 0]
(-(torch.log(p_t + 1e-9) * live).sum()).backward()
idx = MG.grad_sample_index("decoder.head.weight", dec.head.weight.numel()).to(dev)
truth = g["truth"]["grads"]["decoder"]["head.weight"]["sample"].double()
ref = g["bf16"]["grads"]["decoder"]["head.weight"]["sample"].double()
rel = lambda a: ((a.double().cpu() - truth).norm() / truth.norm()).item()
ours = dec.head.weight.grad.reshape(-1)[idx]
gy, x = cap["gy"], cap["x"]
print("gy dtype", gy.dtype, gy.shape, "x", x.dtype, x.shape)
x2 = x.reshape(-1, x.shape[-1]); g2 = gy.reshape(-1, gy.shape[-1])
w32 = (g2.float().t() @ x2.float()).reshape(-1)[idx]
w16 = torch.mm(g2.to(torch.bfloat16).t(), x2.to(torch.bfloat16), out_dtype=torch.float32).reshape(-1)[idx]
w16f = (g2.to(torch.bfloat16).float().t() @ x2.to(torch.bfloat16).float()).reshape(-1)[idx]
print("ours", rel(ours), "ref", rel(ref), "fp32 of captured gy/x", rel(w32), "mm out_dtype", rel(w16), "bf16-rounded fp32 mm", rel(w16f))
print("truth sample norm", truth.norm().item(), "ours norm", ours.norm().item())
big = truth.abs().topk(10).indices
print("largest truth", truth[big].tolist()); print("ours", ours.cpu()[big].tolist()); print("ref", ref[big].tolist())
