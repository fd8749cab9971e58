import torch, torch.nn.functional as F
torch.manual_seed(0)
m = torch.nn.MultiheadAttention(64, 4, batch_first=True).double()
x = torch.randn(3, 8, 64, dtype=torch.float64); mem = torch.randn(3, 20, 64, dtype=torch.float64)
kpm = torch.zeros(3, 20, dtype=torch.bool); kpm[1, 11:] = True
a = m(x, mem, mem, key_padding_mask=kpm, need_weights=False)[0]
b = m.cuda()(x.cuda(), mem.cuda(), mem.cuda(), key_padding_mask=kpm.cuda(), need_weights=False)[0].cpu()
print("mha fp64 gpu-cpu max abs", (a - b).abs().max().item())
q = torch.randn(3, 4, 8, 16, dtype=torch.float64); k = torch.randn(3, 4, 20, 16, dtype=torch.float64)
s1 = F.scaled_dot_product_attention(q, k, k); s2 = F.scaled_dot_product_attention(q.cuda(), k.cuda(), k.cuda()).cpu()
print("sdpa fp64 gpu-cpu", (s1 - s2).abs().max().item())
g = torch.randn(1000, dtype=torch.float64)
print("gelu fp64", (F.gelu(g) - F.gelu(g.cuda()).cpu()).abs().max().item())
ln = torch.nn.LayerNorm(64, eps=1e-6).double(); y = torch.randn(10, 64, dtype=torch.float64)
print("ln fp64", (ln(y) - ln.cuda()(y.cuda()).cpu()).abs().max().item())
w = torch.randn(64, 30, dtype=torch.float64)
print("mm fp64", (y @ w - (y.cuda() @ w.cuda()).cpu()).abs().max().item())
