"""Layers of the reference's ``models/modules/layers.py`` on the DVC path: the head MLPs
(``FFN`` :871-906, ``ContextMaskModel`` :909-944), the caption-decoder ``MLP`` (:827-869) and
the two caption-decoder layers (:509-823), with the reference's parameter names.

The caption-decoder layers also run one decode step incrementally (``step``): the reference's
greedy decode (models/deformable/unimodal_deformable_dvc.py:318-354) re-runs the whole decoder
over the full prefix for every word; ``step`` processes only the new rows against cached keys /
values (``CaptionKVCache``), which is the same arithmetic for the rows it produces."""
import math

import torch
import torch.nn.functional as F
from torch import nn

from .add_norm import add_layer_norm, add_layer_norm_carry, carry_supported
from .attention import CrossAttention, masked_scores_softmax
from .ffn import gelu_dropout
from .linear import Linear

__all__ = ["MLP", "FFN", "ContextMaskModel", "UnimodalCaptionDecoderLayer", "MultimodalCaptionDecoderLayer",
           "CaptionKVCache"]


class MLP(nn.Module):
    """fc1 -> GELU -> dropout -> fc2 -> dropout (reference layers.py:827-869)."""

    def __init__(self, in_dim, hidden_dim, out_dim, dropout_1=0., dropout_2=0.):
        super().__init__()
        self.fully_connected_1 = Linear(in_dim, hidden_dim)
        self.activation_layer = nn.GELU()
        self.dropout_1 = nn.Dropout(dropout_1)
        self.fully_connected_2 = Linear(hidden_dim, out_dim)
        self.dropout_2 = nn.Dropout(dropout_2)

    def forward(self, x):
        x = self.dropout_1(self.activation_layer(self.fully_connected_1(x)))
        return self.dropout_2(self.fully_connected_2(x))


class FFN(nn.Module):
    """n-layer MLP with ReLU between layers (reference layers.py:871-906)."""

    def __init__(self, in_dim, hidden_dim, out_dim, num_layers, dropout=0.):
        super().__init__()
        self.num_layers = num_layers
        h = [hidden_dim] * (num_layers - 1)
        self.layers = nn.ModuleList(Linear(n, k) for n, k in zip([in_dim] + h, h + [out_dim]))
        self.relu = nn.ReLU()

    def forward(self, x):
        for i, layer in enumerate(self.layers):
            x = self.relu(layer(x)) if i < self.num_layers - 1 else layer(x)
        return x


class ContextMaskModel(nn.Module):
    """Predicted context mask over memory tokens (reference layers.py:909-944)."""

    def __init__(self, in_dim, out_dim):
        super().__init__()
        self.layer_1 = Linear(in_dim, in_dim // 2)
        self.layer_2 = Linear(in_dim // 2, in_dim // 2)
        self.layer_3 = Linear(in_dim // 2, out_dim)
        self.relu = nn.ReLU()

    def forward(self, x):
        x = self.relu(self.layer_1(x))
        x = self.relu(self.layer_2(x))
        return self.layer_3(x)


class CaptionKVCache:
    """Per-layer keys / values of the committed caption positions (self-attention) and of the
    memory (cross-attention), for ``step``.

    self_k / self_v[layer]: (N, H, L_max, hd); key_valid: (N, L_max) bool (token != <pad>, the
    reference's key padding mask); cross[layer][name]: (k, v, key_mask) of one memory."""

    def __init__(self, n, l_max, device):
        self.n = n
        self.l_max = l_max
        self.self_k, self.self_v = {}, {}
        self.key_valid = torch.zeros(n, l_max, dtype=torch.bool, device=device)
        self.cross = {}

    def self_buffers(self, layer_idx, heads, head_dim, like):
        if layer_idx not in self.self_k:
            shape = (self.n, heads, self.l_max, head_dim)
            self.self_k[layer_idx] = like.new_zeros(shape)
            self.self_v[layer_idx] = like.new_zeros(shape)
        return self.self_k[layer_idx], self.self_v[layer_idx]


def _heads(x, h):
    n, r, d = x.shape
    return x.view(n, r, h, d // h).transpose(1, 2)


def _cached_self_attention(q, k_new, v_new, cache, layer_idx, pos, scale, neg_fill):
    """Rows ``q`` (N, H, R, hd) at positions pos..pos+R-1; row 0 is committed at ``pos`` (its k / v
    enter the cache), the others are probes that see keys 0..pos (causal, <pad> keys masked)."""
    K, V = cache.self_buffers(layer_idx, q.shape[1], q.shape[3], k_new)
    K[:, :, pos] = k_new[:, :, 0]
    V[:, :, pos] = v_new[:, :, 0]
    keys_k, keys_v = K[:, :, :pos + 1], V[:, :, :pos + 1]
    masked = ~cache.key_valid[:, None, None, :pos + 1]
    p = masked_scores_softmax(q @ keys_k.transpose(-2, -1), masked, scale, neg_fill)
    return p @ keys_v


class UnimodalCaptionDecoderLayer(nn.Module):
    """Self-attention over the caption, cross-attention into the (cropped) memory, GELU MLP; three
    LayerNorms (eps 1e-6), pre- or post-norm (reference layers.py:509-644)."""

    def __init__(self, d_model, num_heads, mlp_ratio=4., qkv_bias=False, attention_dropout=0.,
                 projection_dropout=0., bridge_dropout=0., mlp_dropout_1=0., mlp_dropout_2=0., pre_norm=True):
        super().__init__()
        self.pre_norm = pre_norm
        self.self_attention = CrossAttention(d_model=d_model, num_heads=num_heads, qkv_bias=qkv_bias,
                                             attention_dropout=attention_dropout,
                                             projection_dropout=projection_dropout)
        self.cross_attention = CrossAttention(d_model=d_model, num_heads=num_heads, qkv_bias=qkv_bias,
                                              attention_dropout=attention_dropout,
                                              projection_dropout=projection_dropout)
        self.projection_dropout_1 = nn.Dropout(projection_dropout)
        self.projection_dropout_2 = nn.Dropout(projection_dropout)
        self.layer_norm_1 = nn.LayerNorm(d_model, eps=1e-6)
        self.layer_norm_2 = nn.LayerNorm(d_model, eps=1e-6)
        self.layer_norm_3 = nn.LayerNorm(d_model, eps=1e-6)
        self.mlp = MLP(in_dim=d_model, hidden_dim=int(d_model * mlp_ratio), out_dim=d_model,
                       dropout_1=mlp_dropout_1, dropout_2=mlp_dropout_2)

    def forward(self, target, memory, tgt_mask=None, memory_mask=None, tgt_padding_mask=None,
                memory_padding_mask=None):
        x = target
        if self.pre_norm:
            x = x + self._sa_block(self.layer_norm_1(x), tgt_mask, tgt_padding_mask)
            x = x + self._ca_block(self.layer_norm_2(x), memory, memory_mask, memory_padding_mask)
            return x + self.mlp(self.layer_norm_3(x))
        # post-norm: norm(x + dropout(branch)) as one fused kernel each way under autocast (the
        # residual add of the fp32 stream and the 16-bit branch alone took ~60 us a call in ATen's
        # mixed-dtype elementwise kernel); exactly the three modules' composition otherwise
        sa = self.self_attention(x, x, x, attn_mask=tgt_mask, key_padding_mask=tgt_padding_mask)[0]
        m = self.mlp
        if carry_supported(x, self.layer_norm_1) and x.dtype == torch.float32:
            # each fused add + LayerNorm also writes bf16(out): the cross-attention's query projection,
            # the MLP's first Linear and the next layer's q / k / v projections (value_proj.layer_values
            # reads ``_mfl_bf16``) take it instead of casting the fp32 stream, and its gradient is summed
            # into the fp32 one inside the fused backward (no cast-backward and add kernels)
            x, x16, _ = add_layer_norm_carry(x, sa, self.layer_norm_1, dropout=self.projection_dropout_1)
            ca = self.cross_attention(x16, memory, memory, attn_mask=memory_mask,
                                      key_padding_mask=memory_padding_mask)[0]
            x, x16, _ = add_layer_norm_carry(x, ca, self.layer_norm_2, dropout=self.projection_dropout_2)
            h = gelu_dropout(m.fully_connected_1(x16), m.activation_layer, m.dropout_1)
            out, out16, _ = add_layer_norm_carry(x, m.fully_connected_2(h), self.layer_norm_3, dropout=m.dropout_2)
            out._mfl_bf16 = out16
            return out
        x = add_layer_norm(x, sa, self.layer_norm_1, self.projection_dropout_1)
        x = add_layer_norm(x, self.cross_attention(x, memory, memory, attn_mask=memory_mask,
                                                   key_padding_mask=memory_padding_mask)[0],
                           self.layer_norm_2, self.projection_dropout_2)
        h = m.dropout_1(m.activation_layer(m.fully_connected_1(x)))
        return add_layer_norm(x, m.fully_connected_2(h), self.layer_norm_3, m.dropout_2)

    def _sa_block(self, x, attn_mask, key_padding_mask):
        x = self.self_attention(x, x, x, attn_mask=attn_mask, key_padding_mask=key_padding_mask,
                                need_weights=False)[0]
        return self.projection_dropout_1(x)

    def _ca_block(self, x, mem, attn_mask, key_padding_mask):
        x = self.cross_attention(x, mem, mem, attn_mask=attn_mask, key_padding_mask=key_padding_mask,
                                 need_weights=False)[0]
        return self.projection_dropout_2(x)

    # --- incremental decode -------------------------------------------------------------------
    def prime(self, cache, layer_idx, memory, memory_key_mask):
        """Project the memory once (cross-attention keys / values) for this layer."""
        ca = self.cross_attention
        cache.cross[layer_idx] = (_heads(ca.k_linear(memory), ca.num_heads), _heads(ca.v_linear(memory), ca.num_heads),
                                  memory_key_mask)

    def _sa_step(self, x, cache, layer_idx, pos):
        sa = self.self_attention
        q, k, v = (_heads(f(x), sa.num_heads) for f in (sa.q_linear, sa.k_linear, sa.v_linear))
        o = _cached_self_attention(q, k, v, cache, layer_idx, pos, sa.scale, -1e20)
        return self.projection_dropout_1(sa.projection_layer(o.transpose(1, 2).flatten(2)))

    def _ca_step(self, x, cache, layer_idx):
        ca = self.cross_attention
        k, v, key_mask = cache.cross[layer_idx]
        q = _heads(ca.q_linear(x), ca.num_heads)
        p = masked_scores_softmax(q @ k.transpose(-2, -1), key_mask, ca.scale, -1e20)
        return self.projection_dropout_2(ca.projection_layer((p @ v).transpose(1, 2).flatten(2)))

    def step(self, x, cache, layer_idx, pos):
        """x (N, R, d): row 0 committed at ``pos``, rows 1.. probes; same math as ``forward``."""
        if self.pre_norm:
            x = x + self._sa_step(self.layer_norm_1(x), cache, layer_idx, pos)
            x = x + self._ca_step(self.layer_norm_2(x), cache, layer_idx)
            return x + self.mlp(self.layer_norm_3(x))
        x = self.layer_norm_1(x + self._sa_step(x, cache, layer_idx, pos))
        x = self.layer_norm_2(x + self._ca_step(x, cache, layer_idx))
        return self.layer_norm_3(x + self.mlp(x))


def _mha_project(mha, x, which):
    """q / k / v projection (which = 0 / 1 / 2) of an ``nn.MultiheadAttention`` (packed in_proj)."""
    d = mha.embed_dim
    w = mha.in_proj_weight[which * d:(which + 1) * d]
    b = None if mha.in_proj_bias is None else mha.in_proj_bias[which * d:(which + 1) * d]
    return F.linear(x, w, b)


class MultimodalCaptionDecoderLayer(nn.Module):
    """Caption self-attention, video and audio cross-attentions (``nn.MultiheadAttention``,
    batch_first) fused by the bridge (concat -> LayerNorm(2d) in pre-norm -> Linear(2d -> d) ->
    dropout -> GELU), then the MLP (reference layers.py:648-823).

    The reference class cannot run at HEAD: its ``super()`` names UnimodalCaptionDecoderLayer
    (:667) and its forward reads undefined ``self.activation`` (:760/798), ``self.cross_attention``
    (:819) and ``self.audio_projection_dropout_3`` (:823).  Restated intent: ``activation_layer``,
    ``audio_cross_attention`` and ``projection_dropout_3`` — the modules it constructs for those
    roles (:674-692).  Pre-norm applies layer_norm_3 to the 2d concat as written; post-norm, as
    written, normalises after the bridge Linear (d features).  The reference's pre-norm
    ``LayerNorm(d)`` on a 2d concat cannot run either; pre-norm here uses the written order with
    layer_norm_3 sized for what it normalises (2d, a parameter-shape deviation noted in DESIGN)."""

    def __init__(self, d_model, num_heads, mlp_ratio=4., qkv_bias=False, attention_dropout=0.,
                 projection_dropout=0., bridge_dropout=0., mlp_dropout_1=0., mlp_dropout_2=0., pre_norm=True):
        super().__init__()
        self.pre_norm = pre_norm
        self.self_attention = nn.MultiheadAttention(embed_dim=d_model, num_heads=num_heads, dropout=attention_dropout,
                                                    bias=qkv_bias, batch_first=True)
        self.video_cross_attention = nn.MultiheadAttention(embed_dim=d_model, num_heads=num_heads,
                                                           dropout=attention_dropout, bias=qkv_bias, batch_first=True)
        self.audio_cross_attention = nn.MultiheadAttention(embed_dim=d_model, num_heads=num_heads,
                                                           dropout=attention_dropout, bias=qkv_bias, batch_first=True)
        self.projection_dropout_1 = nn.Dropout(projection_dropout)
        self.projection_dropout_2 = nn.Dropout(projection_dropout)
        self.projection_dropout_3 = nn.Dropout(projection_dropout)
        self.linear_layer = Linear(2 * d_model, d_model)
        self.activation_layer = nn.GELU()
        self.dropout = nn.Dropout(bridge_dropout)
        self.layer_norm_1 = nn.LayerNorm(d_model, eps=1e-6)
        self.layer_norm_2 = nn.LayerNorm(d_model, eps=1e-6)
        self.layer_norm_3 = nn.LayerNorm(2 * d_model if pre_norm else d_model, eps=1e-6)
        self.layer_norm_4 = nn.LayerNorm(d_model, eps=1e-6)
        self.mlp = MLP(in_dim=d_model, hidden_dim=int(d_model * mlp_ratio), out_dim=d_model,
                       dropout_1=mlp_dropout_1, dropout_2=mlp_dropout_2)

    def forward(self, target, video_memory, audio_memory, tgt_mask=None, video_memory_mask=None,
                audio_memory_mask=None, tgt_padding_mask=None, video_memory_padding_mask=None,
                audio_memory_padding_mask=None):
        x = target
        sa = lambda h: self.projection_dropout_1(self.self_attention(  # noqa: E731
            h, h, h, attn_mask=tgt_mask, key_padding_mask=tgt_padding_mask, need_weights=False)[0])
        ca_v = lambda h: self.projection_dropout_2(self.video_cross_attention(  # noqa: E731
            h, video_memory, video_memory, attn_mask=video_memory_mask, key_padding_mask=video_memory_padding_mask,
            need_weights=False)[0])
        ca_a = lambda h: self.projection_dropout_3(self.audio_cross_attention(  # noqa: E731
            h, audio_memory, audio_memory, attn_mask=audio_memory_mask, key_padding_mask=audio_memory_padding_mask,
            need_weights=False)[0])
        return self._combine(x, sa, ca_v, ca_a)

    def _combine(self, x, sa, ca_v, ca_a):
        if self.pre_norm:
            x = x + sa(self.layer_norm_1(x))
            x = self.layer_norm_2(x)
            x = torch.cat([x + ca_v(x), x + ca_a(x)], dim=-1)
            x = self.activation_layer(self.dropout(self.linear_layer(self.layer_norm_3(x))))
            return x + self.mlp(self.layer_norm_4(x))
        x = self.layer_norm_1(x + sa(x))
        vid_x = self.layer_norm_2(x + ca_v(x))
        aud_x = self.layer_norm_2(x + ca_a(x))
        x = self.dropout(self.linear_layer(torch.cat([vid_x, aud_x], dim=-1)))
        x = self.activation_layer(self.layer_norm_3(x))
        return self.layer_norm_4(x + self.mlp(x))

    # --- incremental decode -------------------------------------------------------------------
    def prime(self, cache, layer_idx, memories):
        """memories: {"video": (memory, key_padding_mask), "audio": (...)}."""
        ent = {}
        for name, mha in (("video", self.video_cross_attention), ("audio", self.audio_cross_attention)):
            mem, kpm = memories[name]
            h = mha.num_heads
            ent[name] = (_heads(_mha_project(mha, mem, 1), h), _heads(_mha_project(mha, mem, 2), h),
                         None if kpm is None else kpm[:, None, None, :])
        cache.cross[layer_idx] = ent

    def step(self, x, cache, layer_idx, pos):
        def sa(h):
            mha = self.self_attention
            q, k, v = (_heads(_mha_project(mha, h, i), mha.num_heads) for i in range(3))
            o = _cached_self_attention(q, k, v, cache, layer_idx, pos, 1.0 / math.sqrt(q.shape[-1]), float("-inf"))
            return self.projection_dropout_1(mha.out_proj(o.transpose(1, 2).flatten(2)))

        def ca(name, mha, drop):
            def f(h):
                k, v, key_mask = cache.cross[layer_idx][name]
                q = _heads(_mha_project(mha, h, 0), mha.num_heads)
                p = masked_scores_softmax(q @ k.transpose(-2, -1), key_mask, 1.0 / math.sqrt(q.shape[-1]),
                                          float("-inf"))
                return drop(mha.out_proj((p @ v).transpose(1, 2).flatten(2)))
            return f

        return self._combine(x, sa, ca("video", self.video_cross_attention, self.projection_dropout_2),
                             ca("audio", self.audio_cross_attention, self.projection_dropout_3))
