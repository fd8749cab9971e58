"""Segment cross-attention kernels (csrc/seg_attention.hip) against the explicit form of the
reference's CrossAttention (models/modules/attention.py:278-300) over the materialised crop, in
fp32 on the same bf16 inputs — forward, and every gradient (q, both projections, both biases).

Tolerance: the kernels round the probabilities and dS to bf16 before their MFMA products (the
reference under autocast rounds the scores and the probabilities), so outputs and gradients are
compared as max|a - b| <= 2e-2 * max|b|."""
import numpy as np
import pytest
import torch

from conftest import PKG

pytestmark = pytest.mark.gpu


def _drop_keep(seed, n, H, Lq, K, p):
    """The kernels' keep bits (seg_attention.hip drop_pair / pair_keep): one 32-bit draw per key pair
    (2i, 2i + 1) of query row r = (s*H + h)*Lq + q, at index r * ceil(K / 2) + i; its low 16 bits
    decide key 2i, its high 16 bits key 2i + 1 (kept iff >= p * 2^16)."""
    key = np.uint32((seed & 0xffffffff) ^ (seed >> 32))
    k2 = (K + 1) // 2
    with np.errstate(over="ignore"):
        x = np.arange(n * H * Lq * k2, dtype=np.uint32) * np.uint32(0x9E3779B1) + key
        x ^= x >> np.uint32(16)
        x *= np.uint32(0x85EBCA6B)
        x ^= x >> np.uint32(13)
        x *= np.uint32(0xC2B2AE35)
        x ^= x >> np.uint32(16)
    half = np.stack([x & np.uint32(0xffff), x >> np.uint32(16)], axis=-1).reshape(n * H * Lq, 2 * k2)[:, :K]
    thresh = np.uint32(min(p * 65536.0, 65536.0))
    return torch.from_numpy((half >= thresh).reshape(n, H, Lq, K))


def _reference(q, pk, pv, bk, bv, index, keep, masked, H, scale, drop=None, p=0.0):
    n, Lq, d = q.shape
    K, hd = pk.shape[1], d // H
    k = torch.where(keep[..., None], pk[index], bk)
    v = torch.where(keep[..., None], pv[index], bv)
    qh = q.view(n, Lq, H, hd).transpose(1, 2)
    kh = k.view(n, K, H, hd).transpose(1, 2)
    vh = v.view(n, K, H, hd).transpose(1, 2)
    s = qh @ kh.transpose(-2, -1)
    if masked is not None:
        s = s.masked_fill(masked[:, None, None, :], -1e20)
    att = (s * scale).softmax(-1)
    if drop is not None:
        att = att * drop.to(att) / (1 - p)
    return (att @ vh).transpose(1, 2).reshape(n, Lq, d)


def _case(n, B, K, Lq, H, seed, dead=(), bias_rows=True):
    g = torch.Generator().manual_seed(seed)
    d = 64 * H
    q = torch.randn(n, Lq, d, generator=g)
    pk = torch.randn(B, K, d, generator=g) * 0.5
    pv = torch.randn(B, K, d, generator=g)
    bk = torch.randn(d, generator=g) * 0.1
    bv = torch.randn(d, generator=g)
    index = torch.randint(0, B, (n,), generator=g)
    # key windows like crop_segments': a few ranges per segment; the memory keep a subset of the
    # unmasked keys (a crop of a crop) so that some unmasked keys read the bias rows
    live = torch.zeros(n, K, dtype=torch.bool)
    for s in range(n):
        for _ in range(3):
            a = int(torch.randint(0, K, (1,), generator=g))
            live[s, a:a + int(torch.randint(1, max(2, K // 4), (1,), generator=g))] = True
    for s in dead:
        live[s] = False
    keep = live & (torch.rand(n, K, generator=g) < (0.8 if bias_rows else 1.1))
    return q, pk, pv, bk, bv, index, keep, ~live


CASES = [
    # (n, B, K, Lq, H, dead segments)
    (28, 8, 1920, 19, 8, (3, 17)),  # the DVC step's shape (ActivityNet T=1024 pyramid)
    (5, 2, 1000, 32, 8, ()),         # K not a multiple of 32, full 32-query tile
    (3, 3, 64, 1, 2, (1,)),          # one query, two heads
    (7, 1, 333, 11, 4, (0, 6)),
    (4, 2, 240, 19, 8, (2,)),        # K a multiple of 16, not of 32 (16-byte mask rows, half last block)
]


def _run(case, p=0.0, with_bias=True, with_mask=True):
    dev = torch.device("cuda")
    n, B, K, Lq, H, dead = case
    q, pk, pv, bk, bv, index, keep, masked = _case(n, B, K, Lq, H, seed=n * 131 + K, dead=dead)
    if not with_mask:
        masked = None
    scale = 64 ** -0.5
    bf = [t.to(dev, torch.bfloat16) for t in (q, pk, pv, bk, bv)]
    leaves = [t.clone().requires_grad_(True) for t in bf]
    seed_t = torch.tensor([987654321], dtype=torch.int64, device=dev) if p > 0 else None
    out = PKG.models.modules.seg_attention._SegmentAttention.apply(
        leaves[0], leaves[1], leaves[2], leaves[3] if with_bias else None, leaves[4] if with_bias else None,
        index.to(dev), keep.to(dev), None if masked is None else masked.to(dev), H, scale, p, seed_t)
    gout = torch.randn(out.shape, generator=torch.Generator().manual_seed(5)).to(dev, torch.bfloat16)
    out.backward(gout)
    torch.cuda.synchronize()
    ref_leaves = [t.detach().float().cpu().requires_grad_(True) for t in bf]
    zb = torch.zeros(64 * H)
    drop = _drop_keep(987654321, n, H, Lq, K, p) if p > 0 else None
    ref = _reference(ref_leaves[0], ref_leaves[1], ref_leaves[2], ref_leaves[3] if with_bias else zb,
                     ref_leaves[4] if with_bias else zb, index, keep, masked, H, scale, drop, p)
    ref.backward(gout.float().cpu())
    pairs = [("out", out, ref)] + [(nm, a.grad, b.grad) for nm, a, b in
                                   zip(("dq", "dpk", "dpv", "dbk", "dbv"), leaves, ref_leaves)
                                   if with_bias or nm in ("dq", "dpk", "dpv")]
    for name, a, b in pairs:
        a, b = a.detach().float().cpu(), b.detach().float()
        err = (a - b).abs().max().item()
        assert err <= 2e-2 * b.abs().max().item() + 1e-6, (name, err, b.abs().max().item())


@pytest.mark.parametrize("case", CASES, ids=lambda c: f"n{c[0]}_B{c[1]}_K{c[2]}_Lq{c[3]}_H{c[4]}")
def test_segment_attention_matches_explicit(case):
    _run(case)


def test_segment_attention_dropout_bits():
    _run(CASES[0], p=0.1)


@pytest.mark.parametrize("ci", [0, 1, 3, 4])
def test_segment_attention_recorded_drop_bits_equal_redrawn(ci, monkeypatch):
    """The backward reading the forward's recorded keep bits (mfl_seg_attention_forward_ex /
    backward_ex2, the default) gives the same output and gradients, bit for bit, as re-drawing them
    from the seed (MFL_SEG_DROP_BITS=0) — dead segments, ragged K and one-query tiles included."""
    dev = torch.device("cuda")
    n, B, K, Lq, H, dead = CASES[ci]
    q, pk, pv, bk, bv, index, keep, masked = _case(n, B, K, Lq, H, seed=n * 131 + K, dead=dead)
    bf = [t.to(dev, torch.bfloat16) for t in (q, pk, pv, bk, bv)]
    seed_t = torch.tensor([24681357], dtype=torch.int64, device=dev)
    gout = torch.randn(n, Lq, 64 * H, generator=torch.Generator().manual_seed(9)).to(dev, torch.bfloat16)
    res = {}
    for mode in ("1", "0"):
        monkeypatch.setenv("MFL_SEG_DROP_BITS", mode)
        leaves = [t.clone().requires_grad_(True) for t in bf]
        out = PKG.models.modules.seg_attention._SegmentAttention.apply(
            *leaves, index.to(dev), keep.to(dev), masked.to(dev), H, 64 ** -0.5, 0.1, seed_t)
        out.backward(gout)
        torch.cuda.synchronize()
        res[mode] = [out.detach()] + [t.grad for t in leaves]
    for name, a, b in zip(("out", "dq", "dpk", "dpv", "dbk", "dbv"), res["1"], res["0"]):
        assert torch.equal(a, b), name


def test_segment_attention_no_bias_no_mask():
    _run(CASES[1], with_bias=False, with_mask=False)


@pytest.mark.parametrize("kind", ["key_padding_mask", "attn_mask"])
def test_cross_attention_module_paths_agree(monkeypatch, kind):
    """CrossAttention over a SegmentMemory under autocast: kernel path vs the explicit form, with
    the mask as key_padding_mask (n, K) or as the DVC's broadcast attn_mask (n, 1, 1, K)."""
    dev = torch.device("cuda")
    torch.manual_seed(0)
    n, B, K, Lq, H = 12, 4, 480, 19, 8
    ca = PKG.models.modules.attention.CrossAttention(512, H, qkv_bias=True).to(dev)
    q, _, _, _, _, index, keep, masked = _case(n, B, K, Lq, H, seed=3)
    src = torch.randn(B, K, 512, device=dev)
    x = torch.randn(n, Lq, 512, device=dev)
    SM = PKG.utils.preds_postprocess.SegmentMemory
    results = []
    for flag in ("1", "0"):
        monkeypatch.setenv("MFL_SEG_ATTENTION", flag)
        ca.zero_grad()
        xi = x.clone().requires_grad_(True)
        mem = SM(src, index.to(dev), keep.to(dev))
        with torch.autocast("cuda", dtype=torch.bfloat16):
            m = masked.to(dev)
            y, _ = (ca(xi, mem, mem, key_padding_mask=m) if kind == "key_padding_mask"
                    else ca(xi, mem, mem, attn_mask=m[:, None, None, :]))
        y.float().square().sum().backward()
        results.append({"out": y.float(), "x": xi.grad, **{nm: p.grad.clone() for nm, p in ca.named_parameters()}})
    for name, b in results[1].items():
        a = results[0][name]
        # k_linear's bias shifts every key's score of a query by the same amount (softmax-invariant):
        # its gradient is rounding noise in both forms, measured against the weight gradient's scale
        ref = results[1]["k_linear.weight"] if name == "k_linear.bias" else b
        err = (a - b).abs().max().item()
        assert err <= 3e-2 * ref.abs().max().item() + 1e-6, (name, err, ref.abs().max().item())
