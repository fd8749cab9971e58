"""Video-only deformable encoder/decoder, same interface as the reference's
``models/deformable/unimodal_deformable_transformer.py`` (DVC callers:
unimodal_deformable_dvc.py:152-178).

The MSDA calls (encoder self-attention :241, decoder cross-attention :365) go to the
HIP kernel through ``MSDeformAttn``.  The level metadata is produced once per forward
as device tensors (for API compatibility) that also carry their host values
(``_mfl_host``), so no layer needs a device->host sync to read T_l.
Dense projections / FFN / LayerNorm / ``nn.MultiheadAttention`` stay stock PyTorch-ROCm.
"""
import copy
import math

import torch
import torch.nn.functional as F
from torch import nn
from torch.nn.init import constant_, normal_, xavier_uniform_

from ..modules.pyramid import flatten_levels, level_pos_flatten
from ..modules.attention import MSDeformAttn, mha_self_attention
from ..modules.misc_modules import inverse_sigmoid
from ..modules.linear import Linear, flush_point
from ..modules.add_norm import add_layer_norm, add_layer_norm_carry, carry_entry, carry_supported, pos_sink
from ..modules.ffn import relu_dropout
from ..modules.value_proj import layer_values, layer_values_supported

__all__ = [
    "DeformableTransformer", "DeformableTransformerEncoderLayer", "DeformableTransformerEncoder",
    "DeformableTransformerDecoderLayer", "DeformableTransformerDecoder",
    "build_unimodal_deformable_transformer", "level_metadata", "encoder_reference_points",
]


_LEVEL_CACHE = {}


def level_metadata(lengths, device):
    """(temporal_shapes, level_start_index) as int64 device tensors tagged with host tuples
    (reference unimodal_deformable_transformer.py:129-130 builds the same two tensors).
    Cached per (lengths, device): read-only, and no host->device copy inside a step (so the
    step can be captured in a HIP graph)."""
    lengths = tuple(int(t) for t in lengths)
    key = (lengths, str(torch.device(device)))
    hit = _LEVEL_CACHE.get(key)
    if hit is not None:
        return hit
    starts, run = [], 0
    for t in lengths:
        starts.append(run)
        run += t
    shapes_t = torch.tensor(lengths, dtype=torch.long, device=device)
    starts_t = torch.tensor(starts, dtype=torch.long, device=device)
    shapes_t._mfl_host = lengths
    starts_t._mfl_host = tuple(starts)
    _LEVEL_CACHE[key] = (shapes_t, starts_t)
    return shapes_t, starts_t


def encoder_reference_points(temporal_shapes, valid_ratios, device):
    """Reference point of every encoder token on every level, (B, S, L, 1).

    Token i of level l sits at (i + 0.5) / T_l of the valid part of its own level, then
    is re-expressed in each level's coordinates by the valid ratios — reference
    DeformableTransformerEncoder.get_reference_points (:259-276)."""
    lengths = getattr(temporal_shapes, "_mfl_host", None)
    if lengths is None:
        lengths = [int(t) for t in temporal_shapes]
    per_level = []
    for lvl, t in enumerate(lengths):
        centres = torch.linspace(0.5, t - 0.5, t, dtype=torch.float32, device=device)
        per_level.append(centres.reshape(-1)[None] / (valid_ratios[:, None, lvl] * t))
    ref = torch.cat(per_level, 1)
    return (ref[:, :, None] * valid_ratios[:, None])[..., None]


class DeformableTransformer(nn.Module):
    """Encoder (MSDA self-attention + FFN) and decoder (query self-attention + MSDA
    cross-attention + FFN) over a flattened multi-level temporal pyramid.

    Constructor arguments, submodule names and initialisation follow reference
    unimodal_deformable_transformer.py:13-67, so its state_dicts load unchanged."""

    def __init__(self, d_model=256, num_head=8, num_encoder_layers=6, num_decoder_layers=6,
                 dim_feedforward=1024, dropout=0.1, activation="relu", return_intermediate_dec=False,
                 num_feature_levels=4, dec_n_points=4, enc_n_points=4):
        super().__init__()
        self.d_model = d_model
        self.num_head = num_head
        self.no_encoder = num_encoder_layers == 0
        self.num_feature_levels = num_feature_levels
        self.encoder = DeformableTransformerEncoder(
            DeformableTransformerEncoderLayer(d_model, dim_feedforward, dropout, activation,
                                              num_feature_levels, num_head, enc_n_points),
            num_encoder_layers)
        self.decoder = DeformableTransformerDecoder(
            DeformableTransformerDecoderLayer(d_model, dim_feedforward, dropout, activation,
                                              num_feature_levels, num_head, dec_n_points),
            num_decoder_layers, return_intermediate_dec)
        self.level_embed = nn.Parameter(torch.Tensor(num_feature_levels, d_model))
        self.reference_points = Linear(d_model, 1)
        self._reset_parameters()

    def _reset_parameters(self):
        for p in self.parameters():
            if p.dim() > 1:
                nn.init.xavier_uniform_(p)
        for m in self.modules():
            if isinstance(m, MSDeformAttn):
                m._reset_parameters()
        xavier_uniform_(self.reference_points.weight.data, gain=1.0)
        constant_(self.reference_points.bias.data, 0.)
        normal_(self.level_embed)

    def get_proposal_pos_embed(self, proposals):
        """sine embedding of (sigmoid) proposals, reference :70-83"""
        num_pos_feats, temperature, scale = 256, 10000, 2 * math.pi
        dim_t = torch.arange(num_pos_feats, dtype=torch.float32, device=proposals.device)
        dim_t = temperature ** (2 * (dim_t // 2) / num_pos_feats)
        pos = (proposals.sigmoid() * scale)[:, :, :, None] / dim_t
        return torch.stack((pos[:, :, :, 0::2].sin(), pos[:, :, :, 1::2].cos()), dim=4).flatten(2)

    def get_valid_ratio(self, mask):
        return torch.sum(~mask, 1).float() / mask.shape[1]

    def prepare_encoder_inputs(self, srcs, masks, pos_embeds):
        """Flatten the (B, d_model, T_l) pyramid to (B, S, d_model), S = sum_l T_l.

        :return src_flatten, temporal_shapes (L,), level_start_index (L,), valid_ratios (B, L),
                lvl_pos_embed_flatten (B, S, d_model), mask_flatten (B, S)
        (reference :90-134)"""
        src_flatten = flatten_levels(srcs)
        lvl_pos_embed_flatten = level_pos_flatten(pos_embeds, self.level_embed)
        mask_flatten = torch.cat(list(masks), 1)
        temporal_shapes, level_start_index = level_metadata([s.shape[-1] for s in srcs], src_flatten.device)
        valid_ratios = torch.stack([self.get_valid_ratio(m) for m in masks], 1)
        return src_flatten, temporal_shapes, level_start_index, valid_ratios, lvl_pos_embed_flatten, mask_flatten

    def forward_encoder(self, src_flatten, temporal_shapes, level_start_index, valid_ratios,
                        lvl_pos_embed_flatten, mask_flatten):
        """:return memory (B, S, d_model) (reference :136-155)"""
        if self.no_encoder:
            return src_flatten
        return self.encoder(src_flatten, temporal_shapes, level_start_index, valid_ratios,
                            lvl_pos_embed_flatten, mask_flatten)

    def prepare_decoder_input_query(self, batch_size, query_embed):
        """Split the (num_queries, 2*d_model) query embedding into position / content halves
        and predict initial reference points (reference :157-174).
        :return init_reference_out (B,Q,1), tgt (B,Q,d), reference_points (B,Q,1), query_embed (B,Q,d)"""
        query_embed, tgt = torch.chunk(query_embed, 2, dim=1)
        query_embed = query_embed.unsqueeze(0).expand(batch_size, -1, -1)
        tgt = tgt.unsqueeze(0).expand(batch_size, -1, -1)
        reference_points = self.reference_points(query_embed).sigmoid()
        return reference_points, tgt, reference_points, query_embed

    def prepare_decoder_input_proposal(self, gt_reference_points):
        """reference :176-182 (needs pos_trans / pos_trans_norm, which the reference's
        unimodal transformer does not create either)."""
        topk_coords_unact = inverse_sigmoid(gt_reference_points)
        pos_trans_out = self.pos_trans_norm(self.pos_trans(self.get_proposal_pos_embed(topk_coords_unact)))
        query_embed, tgt = torch.chunk(pos_trans_out, 2, dim=2)
        return gt_reference_points, tgt, gt_reference_points, query_embed

    def forward_decoder(self, *kargs):
        return self.decoder(*kargs)


class DeformableTransformerEncoderLayer(nn.Module):
    """MSDA self-attention (query = src + pos, value = src) -> residual + LayerNorm ->
    FFN(ReLU) -> residual + LayerNorm (reference :189-249)."""

    def __init__(self, d_model=256, d_ffn=1024, dropout=0.1, activation="relu",
                 n_levels=4, n_heads=8, n_points=4):
        super().__init__()
        self.self_attn = MSDeformAttn(d_model, n_levels, n_heads, n_points)
        self.dropout1 = nn.Dropout(dropout)
        self.norm1 = nn.LayerNorm(d_model)
        self.linear1 = Linear(d_model, d_ffn)
        self.activation = _get_activation_fn(activation)
        self.dropout2 = nn.Dropout(dropout)
        self.linear2 = Linear(d_ffn, d_model)
        self.dropout3 = nn.Dropout(dropout)
        self.norm2 = nn.LayerNorm(d_model)

    @staticmethod
    def with_pos_embed(tensor, pos):
        return tensor if pos is None else tensor + pos

    def forward_ffn(self, src):
        hidden = relu_dropout(self.linear1(src), self.activation, self.dropout2)
        return add_layer_norm(src, self.linear2(hidden), self.norm2, dropout=self.dropout3)

    def forward(self, src, pos, reference_points, temporal_shapes, level_start_index, padding_mask=None):
        attn = self.self_attn(self.with_pos_embed(src, pos), reference_points, src, temporal_shapes,
                              level_start_index, padding_mask)
        src = add_layer_norm(src, attn, self.norm1, dropout=self.dropout1)
        return self.forward_ffn(src)

    def forward_carry(self, src, value, query, next_pos, reference_points, temporal_shapes, level_start_index,
                      padding_mask=None, pos_acc=None):
        """``forward`` with the 16-bit operands carried between layers (bf16 autocast on the GPU):
        ``value`` / ``query`` are this layer's MSDA inputs (``src`` and ``src + pos`` in bf16, or
        the fp32 tensors themselves), and the fused add + LayerNorms hand back the next layer's
        ``(src, value, query)`` (query = bf16(out + next_pos); None when next_pos is None).
        ``pos_acc``: next_pos came from ``pos_sink`` (its gradient summed in place)."""
        attn = self.self_attn(query, reference_points, value, temporal_shapes, level_start_index, padding_mask)
        src, src16, _ = add_layer_norm_carry(src, attn, self.norm1, dropout=self.dropout1)
        hidden = relu_dropout(self.linear1(src16), self.activation, self.dropout2)
        return add_layer_norm_carry(src, self.linear2(hidden), self.norm2, next_pos, self.dropout3, pos_acc=pos_acc)


class DeformableTransformerEncoder(nn.Module):
    """Stack of encoder layers sharing one set of reference points (reference :252-295)."""

    def __init__(self, encoder_layer, num_layers):
        super().__init__()
        self.layers = _get_clones(encoder_layer, num_layers)
        self.num_layers = num_layers

    @staticmethod
    def get_reference_points(temporal_shapes, valid_ratios, device):
        return encoder_reference_points(temporal_shapes, valid_ratios, device)

    def forward(self, src, temporal_shapes, level_start_index, valid_ratios, pos=None, padding_mask=None):
        reference_points = self.get_reference_points(temporal_shapes, valid_ratios, device=src.device)
        out = src
        if (self.layers and all(type(layer) is DeformableTransformerEncoderLayer for layer in self.layers)
                and carry_supported(src, self.layers[0].norm1)):
            # bf16 operands carried from each fused add + LayerNorm to the next layer (no casts,
            # no pos add, no gradient accumulation kernels between layers; pos's gradient summed in
            # place by the fused backwards: add_norm.pos_sink)
            pos, pos_acc = pos_sink(pos)
            entry = carry_entry(src, pos, pos_acc)  # (src, bf16(src), bf16(src + pos)) in one pass
            if entry is not None:
                out, value, query = entry
            else:
                value, query = src, DeformableTransformerEncoderLayer.with_pos_embed(src, pos)
            for i, layer in enumerate(self.layers):
                next_pos = pos if i + 1 < len(self.layers) else None
                out, value, query = layer.forward_carry(out, value, query, next_pos, reference_points,
                                                        temporal_shapes, level_start_index, padding_mask,
                                                        pos_acc=pos_acc)
                if query is None:
                    query = value
            out._mfl_bf16 = value  # the last layer's bf16(out): the decoder's value projections read it
            return out
        for layer in self.layers:
            out = layer(out, pos, reference_points, temporal_shapes, level_start_index, padding_mask)
        return out


class DeformableTransformerDecoderLayer(nn.Module):
    """Query self-attention (``nn.MultiheadAttention``, sequence-first) -> MSDA
    cross-attention into the encoder memory -> FFN, each with residual + LayerNorm
    (reference :298-373)."""

    def __init__(self, d_model=256, d_ffn=1024, dropout=0.1, activation="relu",
                 n_levels=4, n_heads=8, n_points=4):
        super().__init__()
        self.cross_attn = MSDeformAttn(d_model, n_levels, n_heads, n_points)
        self.dropout1 = nn.Dropout(dropout)
        self.norm1 = nn.LayerNorm(d_model)
        self.self_attn = nn.MultiheadAttention(d_model, n_heads, dropout=dropout)
        self.dropout2 = nn.Dropout(dropout)
        self.norm2 = nn.LayerNorm(d_model)
        self.linear1 = Linear(d_model, d_ffn)
        self.activation = _get_activation_fn(activation)
        self.dropout3 = nn.Dropout(dropout)
        self.linear2 = Linear(d_ffn, d_model)
        self.dropout4 = nn.Dropout(dropout)
        self.norm3 = nn.LayerNorm(d_model)

    @staticmethod
    def with_pos_embed(tensor, pos):
        return tensor if pos is None else tensor + pos

    def forward_ffn(self, tgt):
        hidden = relu_dropout(self.linear1(tgt), self.activation, self.dropout3)
        return add_layer_norm(tgt, self.linear2(hidden), self.norm3, dropout=self.dropout4)

    def forward(self, tgt, query_pos, reference_points, src, src_temporal_shapes, level_start_index,
                src_padding_mask=None, query_mask=None, value=None):
        """``value``: this layer's cross-attention value, when the decoder computed it (value_proj.py)."""
        return self.forward_carry(tgt, query_pos, reference_points, src, src_temporal_shapes, level_start_index,
                                  src_padding_mask, query_mask, value)[0]

    def forward_carry(self, tgt, query_pos, reference_points, src, src_temporal_shapes, level_start_index,
                      src_padding_mask=None, query_mask=None, value=None, carried=None, pos_acc=None):
        """``forward`` returning ``(out, out16, q16)``: under bf16 autocast on the GPU the last fused add +
        LayerNorm also writes bf16(out) and bf16(out + query_pos), the next layer's self-attention
        inputs (``carried``); (out, None, None) otherwise."""
        sa = mha_self_attention(self.self_attn, tgt, query_pos, query_mask, carried)
        if carry_supported(tgt, self.norm2) and (query_pos is None or query_pos.shape == tgt.shape):
            # bf16(tgt + query_pos) for the cross-attention query and bf16(tgt) for linear1 straight
            # from the fused add + LayerNorms (no pos add, no casts, no gradient accumulation)
            tgt, tgt16, q16 = add_layer_norm_carry(tgt, sa, self.norm2, query_pos, self.dropout2, pos_acc=pos_acc)
            ca = self.cross_attn(q16 if q16 is not None else tgt16, reference_points, src, src_temporal_shapes,
                                 level_start_index, src_padding_mask, value=value)
            tgt, tgt16, _ = add_layer_norm_carry(tgt, ca, self.norm1, dropout=self.dropout1)
            hidden = relu_dropout(self.linear1(tgt16), self.activation, self.dropout3)
            out, out16, q16 = add_layer_norm_carry(tgt, self.linear2(hidden), self.norm3, query_pos, self.dropout4,
                                                   pos_acc=pos_acc)
            return out, out16, q16
        tgt = add_layer_norm(tgt, sa, self.norm2, dropout=self.dropout2)
        ca = self.cross_attn(self.with_pos_embed(tgt, query_pos), reference_points, src, src_temporal_shapes,
                             level_start_index, src_padding_mask, value=value)
        tgt = add_layer_norm(tgt, ca, self.norm1, dropout=self.dropout1)
        return self.forward_ffn(tgt), None, None


class DeformableTransformerDecoder(nn.Module):
    """Decoder stack; reference points scaled into every level by the valid ratios,
    optional iterative refinement through ``bbox_head`` (reference :376-441).
    :return (hs, references): stacked over layers when ``return_intermediate``."""

    def __init__(self, decoder_layer, num_layers, return_intermediate=False):
        super().__init__()
        self.layers = _get_clones(decoder_layer, num_layers)
        self.num_layers = num_layers
        self.return_intermediate = return_intermediate
        self.bbox_head = None

    def flat_groups(self):
        """Parameters a flat-buffer trainer should lay out back to back (train_step._flat_order): each
        same-shape weight / bias of the layers, so that the layers' batched gradient GEMMs (the
        deferred short-K queue, value_proj.layer_values) write one view of the flat gradient buffer."""
        layers = [layer for layer in self.layers if type(layer) is DeformableTransformerDecoderLayer]
        if len(layers) < 2:
            return []
        names = ("linear1.weight", "linear2.weight", "self_attn.out_proj.weight", "cross_attn.value_proj.weight",
                 "cross_attn.value_proj.bias", "cross_attn.output_proj.weight")
        groups = [tuple(layer.get_parameter(n) for layer in layers) for n in names]
        # the query prologue's [W_off; W_aw] pairs of every layer interleaved: each pair stays back to
        # back (MSDeformAttn.flat_groups, read as one tensor) and the 2 x layers weights (biases) form
        # one run of the deferred queue's (800 x 128 x 512) batch
        for kind in ("weight", "bias"):
            groups.append(tuple(layer.get_parameter(f"cross_attn.{n}.{kind}") for layer in layers
                                for n in ("sampling_offsets", "attention_weights")))
        return groups

    def forward(self, tgt, reference_points, src, src_temporal_shapes, src_level_start_index, src_valid_ratios,
                query_pos=None, src_padding_mask=None, query_padding_mask=None, disable_iterative_refine=False):
        # the decoder's batched weight gradients are computed once the query's gradient is (the
        # first layer's backward done), so a data-parallel step reduces them while the encoder's
        # backward runs (linear.py); not on src: its carried bf16 copy must stay attached
        output = flush_point(tgt)
        hs, refs = [], []
        if query_pos is not None and not query_pos.is_contiguous():
            query_pos = query_pos.contiguous()  # once, not per layer (the fused layers read it flat)
        values = None
        attns = [getattr(layer, "cross_attn", None) for layer in self.layers]
        if (all(type(layer) is DeformableTransformerDecoderLayer for layer in self.layers)
                and layer_values_supported(attns, src, src_padding_mask)):
            # every layer projects the same memory: one batched GEMM each way (value_proj.py)
            values = layer_values(attns, src, src_padding_mask)
        carried = None
        pos_acc = None
        if all(type(layer) is DeformableTransformerDecoderLayer for layer in self.layers):
            query_pos, pos_acc = pos_sink(query_pos)  # its gradient summed in place (add_norm.pos_sink)
        for lid, layer in enumerate(self.layers):
            if reference_points.shape[-1] == 2:
                scale = torch.stack([src_valid_ratios, src_valid_ratios], -1)[:, None]
                reference_points_input = reference_points[:, :, None] * scale
            else:
                assert reference_points.shape[-1] == 1
                reference_points_input = reference_points[:, :, None] * src_valid_ratios[:, None, :, None]
            if type(layer) is DeformableTransformerDecoderLayer:
                # bf16 self-attention inputs carried from the previous layer's last add + LayerNorm
                output, out16, q16 = layer.forward_carry(
                    output, query_pos, reference_points_input, src, src_temporal_shapes, src_level_start_index,
                    src_padding_mask, query_padding_mask, values[lid] if values is not None else None, carried,
                    pos_acc=pos_acc)
                carried = (out16, q16)
            elif values is not None:
                output = layer(output, query_pos, reference_points_input, src, src_temporal_shapes,
                               src_level_start_index, src_padding_mask, query_padding_mask, value=values[lid])
            else:
                output = layer(output, query_pos, reference_points_input, src, src_temporal_shapes,
                               src_level_start_index, src_padding_mask, query_padding_mask)
            if not disable_iterative_refine and self.bbox_head is not None:
                delta = self.bbox_head[lid](output)
                if reference_points.shape[-1] == 2:
                    refined = (delta + inverse_sigmoid(reference_points)).sigmoid()
                else:
                    assert reference_points.shape[-1] == 1
                    refined = delta
                    refined[..., :1] = delta[..., :1] + inverse_sigmoid(reference_points)
                    refined = refined.sigmoid()
                reference_points = refined.detach()
            if self.return_intermediate:
                hs.append(output)
                refs.append(reference_points)
        if self.return_intermediate:
            return torch.stack(hs), torch.stack(refs)
        return output, reference_points


def _get_clones(module, N):
    return nn.ModuleList([copy.deepcopy(module) for _ in range(N)])


def _get_activation_fn(activation):
    if activation == "relu":
        return F.relu
    if activation == "gelu":
        return F.gelu
    if activation == "glu":
        return F.glu
    raise RuntimeError(f"activation should be relu/gelu, not {activation}.")


def build_unimodal_deformable_transformer(args):
    """reference :460-471 (args = the ``cfg.dvc.detr`` ConfigDict or any namespace)."""
    return DeformableTransformer(
        d_model=args.d_model, num_head=args.num_heads, num_encoder_layers=args.enc_layers,
        num_decoder_layers=args.dec_layers, dim_feedforward=args.transformer_ff_dim,
        dropout=args.transformer_dropout_prob, activation="relu",
        return_intermediate_dec=args.return_intermediate, num_feature_levels=args.num_feature_levels,
        dec_n_points=args.dec_n_points, enc_n_points=args.enc_n_points)
