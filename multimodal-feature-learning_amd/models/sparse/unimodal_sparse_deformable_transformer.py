"""Sparse-DETR deformable encoder/decoder, same interface as the
reference's ``models/sparse/unimodal_sparse_deformable_transformer.py`` — the model family
``UnimodalSparseDVC`` (models/sparse/unimodal_sparse_dvc.py:83,162-185) trains.

What differs from the dense transformer:
  * a MaskPredictor scores every encoder token (prepare_encoder_inputs, reference :199-218) and
    only the top rho*valid tokens are refined by the encoder: their queries sample the FULL
    pyramid (MSDA with Lq = top-k, value = all S tokens — the same HIP kernel, any Lq);
  * the refined tokens are scattered back into the full memory after every layer
    (reference :441-448, a per-clip Python loop there, one scatter here);
  * every MSDA call returns its sampling locations / attention weights (``is_sparse=True``),
    stacked per layer for the criterion's decoder attention map (utils/dam.py, HIP kernel).
Submodule names, constructor arguments and initialisation follow the reference so its
state_dicts load unchanged.
"""
import copy
import math
import os

import torch
import torch.nn.functional as F
from torch import nn
from torch.autograd import Function
from torch.nn.init import constant_, normal_, xavier_uniform_

from ..deformable.unimodal_deformable_transformer import encoder_reference_points, level_metadata
from ..modules.pyramid import flatten_levels, level_pos_flatten
from ..modules.attention import MSDeformAttn, mha_self_attention
from ..modules.linear import Linear, grad_sum_give, grad_sum_tagged, mark_grad_sum
from ..modules.add_norm import add_layer_norm, add_layer_norm_carry, carry_supported, pos_sink
from ..modules.value_proj import layer_values, layer_values_supported
from ..modules.ffn import relu_dropout
from ..modules.misc_modules import inverse_sigmoid

__all__ = [
    "SparseDeformableTransformer", "DeformableTransformerEncoderLayer", "DeformableTransformerEncoder",
    "DeformableTransformerDecoderLayer", "DeformableTransformerDecoder", "MaskPredictor",
    "build_sparse_deforamble_transformer",
]


class _GatherRows(Function):
    """``src.gather(1, topk[..., None].expand(-1, -1, C))`` for src (B, S, C) by flat row index
    (``rows`` = b * S + topk, unique per clip): index_select over rows instead of an expanded
    (B, k, C) int64 index (18.9 MB at the bench shape, read by the gather and again by its
    scatter_add backward); the backward copies the gradient rows into a zeroed (B, S, C)."""

    @staticmethod
    def forward(ctx, src, rows, k):
        B, S, C = src.shape
        ctx.save_for_backward(rows)
        ctx.shape = (B, S, C)
        return src.reshape(B * S, C).index_select(0, rows).view(B, k, C)

    @staticmethod
    def backward(ctx, g):
        (rows,) = ctx.saved_tensors
        B, S, C = ctx.shape
        gs = g.new_zeros(B * S, C)
        gs.index_copy_(0, rows, g.reshape(-1, C))
        return gs.view(B, S, C), None, None


class _ScatterRows(Function):
    """``prev.scatter(1, topk[..., None].expand(-1, -1, C), new)`` by flat row index (as _GatherRows):
    a copy of prev with those rows replaced.  Backward: prev's gradient is a copy with the rows
    zeroed — handed through ``grad_sum_give`` when prev is tagged (``mark_grad_sum``: the MSDA value
    projection of the next layer then adds its input gradient into it in its GEMM) — and new's the
    gathered rows."""

    @staticmethod
    def forward(ctx, prev, rows, new):
        B, S, C = prev.shape
        out = prev.contiguous().clone()
        out.view(B * S, C).index_copy_(0, rows, new.reshape(-1, C).to(out.dtype))
        ctx.save_for_backward(rows)
        ctx.gsum = grad_sum_tagged(prev)
        ctx.key = (prev.data_ptr(), prev.numel(), prev.dtype)
        ctx.new_shape, ctx.new_dtype = new.shape, new.dtype
        return out

    @staticmethod
    def backward(ctx, g):
        (rows,) = ctx.saved_tensors
        C = g.shape[-1]
        g = g.contiguous()
        g_new = g.view(-1, C).index_select(0, rows).view(ctx.new_shape).to(ctx.new_dtype)
        g_prev = g.clone()
        g_prev.view(-1, C).index_fill_(0, rows, 0)
        grad_sum_give(ctx.gsum, ctx.key, g_prev)
        return g_prev, None, g_new


class SparseDeformableTransformer(nn.Module):
    """reference :10-282 (two-stage / eff_query_init paths are inert there as well)."""

    def __init__(self, d_model=256, num_head=8, num_encoder_layers=6, num_decoder_layers=6, dim_feedforward=1024,
                 dropout=0.1, activation="relu", return_intermediate_dec=False, num_feature_levels=4,
                 dec_n_points=4, enc_n_points=4, rho=0.3, use_enc_aux_loss=False, eff_query_init=False,
                 eff_specific_head=False):
        super().__init__()
        self.d_model = d_model
        self.num_head = num_head
        self.num_feature_levels = num_feature_levels
        self.eff_query_init = eff_query_init
        self.eff_specific_head = eff_specific_head
        self.rho = rho
        # True: the top-k width is the host-known bound min(S, int(S * rho) + 1) of every clip's
        # sparse_token_nums instead of their maximum (a device -> host read, :212); the per-clip
        # ``keep`` masks select the same tokens, so outputs are unchanged, and the step can be
        # captured in a HIP graph.  Equal widths when no clip is padded.
        self.static_topk = False
        self.two_stage = False
        self.use_enc_aux_loss = use_enc_aux_loss
        self.sparse_enc_head = 1 if self.two_stage and self.rho else 0
        self.enc_mask_predictor = MaskPredictor(d_model, d_model) if rho else None
        self.encoder = DeformableTransformerEncoder(
            DeformableTransformerEncoderLayer(d_model, dim_feedforward, dropout, activation, num_feature_levels,
                                              num_head, enc_n_points), num_encoder_layers, d_model)
        self.decoder = DeformableTransformerDecoder(
            DeformableTransformerDecoderLayer(d_model, dim_feedforward, dropout, activation, num_feature_levels,
                                              num_head, dec_n_points), num_decoder_layers, return_intermediate_dec)
        self.level_embed = nn.Parameter(torch.Tensor(num_feature_levels, d_model))
        self.enc_output = Linear(d_model, d_model)
        self.enc_output_norm = nn.LayerNorm(d_model)
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
        num_pos_feats, temperature, scale = 256, 10000, 2 * math.pi
        dim_t = torch.arange(num_pos_feats, dtype=torch.float32, device=proposals.device)
        dim_t = temperature ** (2 * (dim_t // 2) / num_pos_feats)
        pos = (proposals.sigmoid() * scale)[:, :, :, None] / dim_t
        return torch.stack((pos[:, :, :, 0::2].sin(), pos[:, :, :, 1::2].cos()), dim=4).flatten(2)

    def gen_encoder_output_proposals(self, memory, memory_padding_mask, temporal_shapes, process_output=True):
        """Per-token proposals (centre (i+0.5)/valid_l, length 0.05*2^l) in logit space, the
        invalid / padded ones at +inf, and the projected memory (reference :101-145).
        :return output_memory (B, S, d), output_proposals (B, S, 2), valid token count (B,)"""
        N, S, _ = memory.shape
        lengths = getattr(temporal_shapes, "_mfl_host", None) or [int(t) for t in temporal_shapes]
        proposals, cur = [], 0
        for lvl, t in enumerate(lengths):
            valid_l = torch.sum(~memory_padding_mask[:, cur:cur + t], 1)
            grid = torch.linspace(0, t - 1, t, dtype=torch.float32, device=memory.device)
            grid = (grid.unsqueeze(0).expand(N, -1) + 0.5) / valid_l.unsqueeze(-1)
            wh = torch.full(grid.shape, 0.05 * (2.0 ** lvl), device=grid.device)
            proposals.append(torch.cat((grid, wh), -1).view(N, -1, 2))
            cur += t
        output_proposals = torch.cat(proposals, 1)
        valid = ((output_proposals > 0.01) & (output_proposals < 0.99)).all(-1, keepdim=True)
        output_proposals = torch.log(output_proposals / (1 - output_proposals))
        output_proposals = output_proposals.masked_fill(memory_padding_mask.unsqueeze(-1), float("inf"))
        output_proposals = output_proposals.masked_fill(~valid, float("inf"))
        output_memory = memory
        if process_output:
            output_memory = output_memory.masked_fill(memory_padding_mask.unsqueeze(-1), float(0))
            output_memory = output_memory.masked_fill(~valid, float(0))
            output_memory = self.enc_output_norm(self.enc_output(output_memory))
        return output_memory, output_proposals, (~memory_padding_mask).sum(axis=-1)

    def get_valid_ratio(self, mask):
        return torch.sum(~mask, 1).float() / mask.shape[1]

    def prepare_encoder_inputs(self, srcs, masks, pos_embeds):
        """Flatten the pyramid and pick the encoder's top-k tokens (reference :152-227).
        :return src_flatten, temporal_shapes, level_start_index, valid_ratios, lvl_pos_embed_flatten,
                mask_flatten, backbone_output_proposals, backbone_topk_proposals (B, k),
                backbone_mask_prediction (B, S), sparse_token_nums (B,)"""
        src_flatten = flatten_levels(srcs)
        lvl_pos_embed_flatten = level_pos_flatten(pos_embeds, self.level_embed)
        mask_flatten = torch.cat(list(masks), 1)
        temporal_shapes, level_start_index = level_metadata([s.shape[-1] for s in srcs], src_flatten.device)
        valid_ratios = torch.stack([self.get_valid_ratio(m) for m in masks], 1)
        backbone_output_proposals = None
        if self.rho or self.use_enc_aux_loss:
            backbone_output_memory, backbone_output_proposals, valid_token_nums = self.gen_encoder_output_proposals(
                src_flatten + lvl_pos_embed_flatten, mask_flatten, temporal_shapes, process_output=bool(self.rho))
            self.valid_token_nums = valid_token_nums
        if self.rho:
            sparse_token_nums = (valid_token_nums * self.rho).int() + 1
            S_tok = backbone_output_memory.shape[1]
            if self.static_topk:
                backbone_topk = min(int(S_tok * self.rho) + 1, S_tok)
            else:
                backbone_topk = min(int(max(sparse_token_nums)), S_tok)  # host sync, as :212
            self.sparse_token_nums = sparse_token_nums
            backbone_mask_prediction = self.enc_mask_predictor(backbone_output_memory).squeeze(-1)
            # masked_fill(mask, tensor.min()) reads the 0-dim value on the host; where() keeps it on the device
            backbone_mask_prediction = torch.where(mask_flatten, backbone_mask_prediction.min(),
                                                   backbone_mask_prediction)
            backbone_topk_proposals = torch.topk(backbone_mask_prediction, backbone_topk, dim=1)[1]
        else:
            backbone_topk_proposals = backbone_mask_prediction = sparse_token_nums = None
        return (src_flatten, temporal_shapes, level_start_index, valid_ratios, lvl_pos_embed_flatten, mask_flatten,
                backbone_output_proposals, backbone_topk_proposals, backbone_mask_prediction, sparse_token_nums)

    def forward_encoder(self, src_flatten, temporal_shapes, level_start_index, valid_ratios, lvl_pos_embed_flatten,
                        mask_flatten, backbone_output_proposals, backbone_topk_proposals, sparse_token_nums):
        """:return memory, sampling_locations_enc, attn_weights_enc, aux count, aux segments (reference :230-250)"""
        output_proposals = backbone_output_proposals if self.use_enc_aux_loss else None
        return self.encoder(src_flatten, temporal_shapes, level_start_index, valid_ratios, lvl_pos_embed_flatten,
                            mask_flatten, backbone_topk_proposals, output_proposals, sparse_token_nums)

    def prepare_decoder_input_query(self, batch_size, query_embed):
        query_embed, tgt = torch.chunk(query_embed, 2, dim=1)
        query_embed = query_embed.unsqueeze(0).expand(batch_size, -1, -1)
        tgt = tgt.unsqueeze(0).expand(batch_size, -1, -1)
        reference_points = self.reference_points(query_embed).sigmoid()
        return reference_points, tgt, reference_points, query_embed

    def prepare_decoder_input_proposal(self, gt_reference_points):
        """reference :271-277 (needs pos_trans / pos_trans_norm, absent in the reference too)."""
        topk_coords_unact = inverse_sigmoid(gt_reference_points)
        pos_trans_out = self.pos_trans_norm(self.pos_trans(self.get_proposal_pos_embed(topk_coords_unact)))
        query_embed, tgt = torch.chunk(pos_trans_out, 2, dim=2)
        return gt_reference_points, tgt, gt_reference_points, query_embed

    def forward_decoder(self, *kargs):
        """:return hs, inter_references, sampling_locations_dec, attn_weights_dec"""
        return self.decoder(*kargs)


class DeformableTransformerEncoderLayer(nn.Module):
    """MSDA over the full pyramid for ``src`` (dense) or for the top-k ``tgt`` queries (sparse),
    then FFN; returns (out, sampling_locations, attn_weights) (reference :285-359)."""

    def __init__(self, d_model=256, d_ffn=1024, dropout=0.1, activation="relu", n_levels=4, n_heads=8, n_points=4):
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

    def forward(self, src, pos, reference_points, temporal_shapes, level_start_index, padding_mask=None, tgt=None):
        query = src if tgt is None else tgt
        attn, sampling_locations, attn_weights = self.self_attn(
            self.with_pos_embed(query, pos), reference_points, src, temporal_shapes, level_start_index, padding_mask,
            is_sparse=True)
        out = add_layer_norm(query, attn, self.norm1, dropout=self.dropout1)
        return self.forward_ffn(out), sampling_locations, attn_weights

    def forward_carry(self, value, tgt, query, next_pos, reference_points, temporal_shapes, level_start_index,
                      padding_mask=None):
        """``forward`` on the top-k tokens with the 16-bit operands carried between layers (bf16
        autocast on the GPU, as the dense encoder's ``forward_carry``): ``value`` is the whole
        memory in bf16 (the MSDA value), ``query`` this layer's ``tgt + pos`` (bf16 from the previous
        layer's fused add + LayerNorm, or fp32 in the first layer).  Returns (tgt, bf16(tgt),
        bf16(tgt + next_pos) or None, sampling_locations, attn_weights)."""
        attn, sampling_locations, attn_weights = self.self_attn(query, reference_points, value, temporal_shapes,
                                                                level_start_index, padding_mask, is_sparse=True)
        t1, t1_16, _ = add_layer_norm_carry(tgt, attn, self.norm1, dropout=self.dropout1)
        hidden = relu_dropout(self.linear1(t1_16), self.activation, self.dropout2)
        out, out16, q16 = add_layer_norm_carry(t1, self.linear2(hidden), self.norm2, next_pos, self.dropout3)
        return out, out16, q16, sampling_locations, attn_weights


class DeformableTransformerEncoder(nn.Module):
    """reference :363-470"""

    def __init__(self, encoder_layer, num_layers, d_model):
        super().__init__()
        self.layers = _get_clones(encoder_layer, num_layers)
        self.num_layers = num_layers
        self.aux_heads = False
        self.count_head = None
        self.segment_embedding = None

    @staticmethod
    def get_reference_points(temporal_shapes, valid_ratios, device):
        return encoder_reference_points(temporal_shapes, valid_ratios, device)

    def forward(self, src, temporal_shapes, level_start_index, valid_ratios, pos=None, padding_mask=None,
                backbone_topk_proposals=None, output_proposals=None, sparse_token_nums=None):
        if self.aux_heads:
            assert output_proposals is not None
        else:
            assert output_proposals is None
        output = src
        sparsified = backbone_topk_proposals is not None
        reference_points = self.get_reference_points(temporal_shapes, valid_ratios, device=src.device)
        tgt = None
        inv = None
        if sparsified:
            topk = backbone_topk_proposals
            if sparse_token_nums is not None:
                # (the keep mask below is by score rank: taken before the reorder)
                rank_keep = (torch.arange(topk.shape[1], device=topk.device)[None, :]
                             < sparse_token_nums.to(topk.device)[:, None])
            if topk.is_cuda:
                # the refined tokens in position order (their reference points; tokens of every level
                # interleaved): every layer treats them independently and scatters them back by index,
                # so the order is free — and with neighbouring tokens next to each other the MSDA
                # backward takes the row-block kernel (each query tile touches a short row interval of
                # every level) instead of the per-tap kernel.  The returned per-token tensors are put
                # back into score order (``inv``), as the reference returns them.
                key = reference_points[:, :, 0, 0].gather(1, topk)
                order = key.sort(dim=1, stable=True)[1]
                topk = topk.gather(1, order)
                inv = torch.argsort(order, dim=1)
                if sparse_token_nums is not None:
                    rank_keep = rank_keep.gather(1, order)
            B, N, S_, P_ = reference_points.shape
            reference_points = torch.gather(reference_points.view(B, N, -1), 1,
                                            topk.unsqueeze(-1).expand(-1, -1, S_ * P_)).view(B, -1, S_, P_)
            idx = topk.unsqueeze(-1).expand(-1, -1, output.size(-1))
            by_rows = (output.is_cuda and os.environ.get("MFL_SPARSE_ROWS", "1") != "0"
                       and pos is not None and pos.shape == output.shape)
            if by_rows:
                # flat row indices b * S + topk (unique per clip): gathers / scatters by row (_GatherRows)
                rows = (topk + torch.arange(B, device=topk.device)[:, None] * output.shape[1]).reshape(-1)
                tgt = _GatherRows.apply(output, rows, topk.shape[1])
                pos = _GatherRows.apply(pos.contiguous(), rows, topk.shape[1])
            else:
                tgt = torch.gather(output, 1, idx)
                pos = torch.gather(pos, 1, topk.unsqueeze(-1).expand(-1, -1, pos.size(-1)))
            if output_proposals is not None:
                output_proposals = output_proposals.gather(1, topk.unsqueeze(-1).expand(-1, -1,
                                                                                         output_proposals.size(-1)))
            if sparse_token_nums is not None:
                # clip i keeps only its first sparse_token_nums[i] top-k tokens (reference :445-448
                # scatters them one clip at a time): the others write back their own old value
                keep = rank_keep.unsqueeze(-1)
        locs, weights, inter = [], [], []
        carry = (sparsified and self.layers and os.environ.get("MFL_SPARSE_CARRY", "1") != "0"
                 and all(type(layer) is DeformableTransformerEncoderLayer for layer in self.layers)
                 and carry_supported(tgt, self.layers[0].norm1))
        if carry:
            # bf16 operands carried between the layers as the dense encoder does (no per-layer pos add,
            # casts of the whole memory or gradient-accumulation kernels): value16 is bf16(output)
            # kept up to date by the same scatter; the last one is the decoder's bf16 memory
            from ... import _trace
            _trace.hit("sparse_carry")
            value16 = output.to(torch.get_autocast_dtype("cuda"))
            if by_rows:
                return self._forward_carry_rows(output, value16, tgt, pos, rows, keep if sparse_token_nums is not None
                                                else None, reference_points, temporal_shapes, level_start_index,
                                                padding_mask, inv, output_proposals)
            query = tgt + pos
            for i, layer in enumerate(self.layers):
                next_pos = pos if i + 1 < len(self.layers) else None
                tgt, tgt16, q16, sampling_locations, attn_weights = layer.forward_carry(
                    value16, tgt, query, next_pos, reference_points, temporal_shapes, level_start_index,
                    padding_mask)
                locs.append(sampling_locations)
                weights.append(attn_weights)
                new, new16 = tgt, tgt16.to(value16.dtype)  # (a no-op on the fused path)
                if sparse_token_nums is not None:
                    new = torch.where(keep, tgt, torch.gather(output, 1, idx))
                    new16 = torch.where(keep, tgt16, torch.gather(value16, 1, idx))
                output = output.scatter(1, idx, new)
                value16 = value16.scatter(1, idx, new16)
                query = q16
                if self.aux_heads:
                    inter.append(tgt)
            output._mfl_bf16 = value16
        for layer in (self.layers if not carry else ()):
            tgt, sampling_locations, attn_weights = layer(output, pos, reference_points, temporal_shapes,
                                                          level_start_index, padding_mask,
                                                          tgt=tgt if sparsified else None)
            locs.append(sampling_locations)
            weights.append(attn_weights)
            if sparsified:
                new = tgt if sparse_token_nums is None else torch.where(keep, tgt, torch.gather(output, 1, idx))
                output = output.scatter(1, idx, new)
            else:
                output = tgt
            if self.aux_heads:
                inter.append(tgt)
        return self._encoder_returns(output, locs, weights, inter, inv, output_proposals)

    def _forward_carry_rows(self, src, value16, tgt, pos, rows, keep, reference_points, temporal_shapes,
                            level_start_index, padding_mask, inv, output_proposals):
        """The carry loop with the top-k tokens written back by row (_ScatterRows).  The fp32 memory is
        read by nothing but the next layer's write-back, and every layer writes the same rows, so it is
        written once, after the last layer: ``src`` with the kept top-k rows replaced by the last
        layer's output (the same memory the reference's per-layer scatters leave).  The bf16 value
        copy is rewritten per layer (the next layer's MSDA reads it); the rows a clip does not keep
        hold bf16(src)'s values throughout (``keep``: reference :445-448)."""
        from ... import _trace
        _trace.hit("sparse_rows")
        first = tgt
        const16 = first.to(value16.dtype) if keep is not None else None
        query = tgt + pos
        locs, weights, inter = [], [], []
        for i, layer in enumerate(self.layers):
            next_pos = pos if i + 1 < len(self.layers) else None
            # value16's two consumers (this layer's value projection, the write-back below) sum its
            # gradient in the projection's dgrad GEMM (mark_grad_sum)
            mark_grad_sum(value16)
            tgt, tgt16, q16, sampling_locations, attn_weights = layer.forward_carry(
                value16, tgt, query, next_pos, reference_points, temporal_shapes, level_start_index, padding_mask)
            locs.append(sampling_locations)
            weights.append(attn_weights)
            new16 = tgt16.to(value16.dtype)
            if keep is not None:
                new16 = torch.where(keep, new16, const16)
            value16 = _ScatterRows.apply(value16, rows, new16)
            query = q16
            if self.aux_heads:
                inter.append(tgt)
        new = tgt if keep is None else torch.where(keep, tgt, first)
        output = _ScatterRows.apply(src, rows, new)
        output._mfl_bf16 = value16
        return self._encoder_returns(output, locs, weights, inter, inv, output_proposals)

    def _encoder_returns(self, output, locs, weights, inter, inv, output_proposals):
        sampling_locations_enc = torch.stack(locs, dim=1)
        attn_weights_enc = torch.stack(weights, dim=1)
        if inv is not None:  # back into score order (B, layers, k, ...)
            def unsort(t, dim):
                shape = [1] * t.dim()
                shape[0], shape[dim] = inv.shape[0], inv.shape[1]
                return t.gather(dim, inv.view(shape).expand(*t.shape[:dim], inv.shape[1], *t.shape[dim + 1:]))
            sampling_locations_enc = unsort(sampling_locations_enc, 2)
            attn_weights_enc = unsort(attn_weights_enc, 2)
            inter = [unsort(t, 1) for t in inter]
            if output_proposals is not None:
                output_proposals = unsort(output_proposals, 1)
        if self.aux_heads:
            from ..modules.misc_modules import predict_event_num_with_depth
            enc_inter_tgt = torch.stack(inter)
            outputs_count = predict_event_num_with_depth(self.count_head, enc_inter_tgt[:-1])
            outputs_coords = (output_proposals.squeeze(0) + self.segment_embedding(enc_inter_tgt[:-1])).sigmoid()
            return output, sampling_locations_enc, attn_weights_enc, outputs_count, outputs_coords
        return output, sampling_locations_enc, attn_weights_enc, None, None


class DeformableTransformerDecoderLayer(nn.Module):
    """Query self-attention -> MSDA cross-attention (is_sparse returns) -> FFN (reference :474-551)."""

    def __init__(self, d_model=256, d_ffn=1024, dropout=0.1, activation="relu", n_levels=4, n_heads=8, n_points=4):
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
        out, _, _, sampling_locations, attn_weights = self.forward_carry(
            tgt, query_pos, reference_points, src, src_temporal_shapes, level_start_index, src_padding_mask,
            query_mask, value)
        return out, sampling_locations, attn_weights

    def forward_carry(self, tgt, query_pos, reference_points, src, src_temporal_shapes, level_start_index,
                      src_padding_mask=None, query_mask=None, value=None, carried=None, pos_acc=None):
        """``forward`` returning ``(out, out16, q16, sampling_locations, attn_weights)``: as the dense
        decoder's layer (unimodal_deformable_transformer.py), under bf16 autocast on the GPU the fused
        add + LayerNorms hand the cross-attention its bf16 query, linear1 its bf16 input and the next
        layer bf16(out) and bf16(out + query_pos) (``carried``); (out, None, None, ...) otherwise."""
        sa = mha_self_attention(self.self_attn, tgt, query_pos, query_mask, carried)
        if carry_supported(tgt, self.norm2) and (query_pos is None or query_pos.shape == tgt.shape):
            tgt, tgt16, q16 = add_layer_norm_carry(tgt, sa, self.norm2, query_pos, self.dropout2, pos_acc=pos_acc)
            ca, sampling_locations, attn_weights = self.cross_attn(
                q16 if q16 is not None else tgt16, reference_points, src, src_temporal_shapes, level_start_index,
                src_padding_mask, is_sparse=True, value=value)
            tgt, tgt16, _ = add_layer_norm_carry(tgt, ca, self.norm1, dropout=self.dropout1)
            hidden = relu_dropout(self.linear1(tgt16), self.activation, self.dropout3)
            out, out16, q16 = add_layer_norm_carry(tgt, self.linear2(hidden), self.norm3, query_pos, self.dropout4,
                                                   pos_acc=pos_acc)
            return out, out16, q16, sampling_locations, attn_weights
        tgt = add_layer_norm(tgt, sa, self.norm2, dropout=self.dropout2)
        ca, sampling_locations, attn_weights = self.cross_attn(self.with_pos_embed(tgt, query_pos), reference_points,
                                                               src, src_temporal_shapes, level_start_index,
                                                               src_padding_mask, is_sparse=True, value=value)
        tgt = add_layer_norm(tgt, ca, self.norm1, dropout=self.dropout1)
        return self.forward_ffn(tgt), None, None, sampling_locations, attn_weights


class DeformableTransformerDecoder(nn.Module):
    """reference :554-631: also stacks every layer's sampling locations / attention weights."""

    def __init__(self, decoder_layer, num_layers, return_intermediate=True):
        super().__init__()
        self.layers = _get_clones(decoder_layer, num_layers)
        self.num_layers = num_layers
        self.return_intermediate = return_intermediate
        self.bbox_head = None

    def flat_groups(self):
        """Parameters a flat-buffer trainer lays out back to back (train_step._flat_order), as the dense
        decoder's: each same-shape weight / bias of the layers and the query prologue pairs interleaved,
        so the batched gradient GEMMs write one view of the flat gradient buffer."""
        layers = [layer for layer in self.layers if type(layer) is DeformableTransformerDecoderLayer]
        if len(layers) < 2:
            return []
        names = ("linear1.weight", "linear2.weight", "self_attn.out_proj.weight", "cross_attn.value_proj.weight",
                 "cross_attn.value_proj.bias", "cross_attn.output_proj.weight")
        groups = [tuple(layer.get_parameter(n) for layer in layers) for n in names]
        for kind in ("weight", "bias"):
            groups.append(tuple(layer.get_parameter(f"cross_attn.{n}.{kind}") for layer in layers
                                for n in ("sampling_offsets", "attention_weights")))
        return groups

    def forward(self, tgt, reference_points, src, src_temporal_shapes, src_level_start_index, src_valid_ratios,
                query_pos=None, src_padding_mask=None, query_padding_mask=None, disable_iterative_refine=False):
        output = tgt
        hs, refs, locs, weights = [], [], [], []
        plain = all(type(layer) is DeformableTransformerDecoderLayer for layer in self.layers)
        values = carried = pos_acc = None
        if plain:
            attns = [layer.cross_attn for layer in self.layers]
            if layer_values_supported(attns, src, src_padding_mask):
                # every layer projects the same memory (its bf16 copy carried from the encoder): one
                # batched GEMM each way (value_proj.py), as the dense decoder
                values = layer_values(attns, src, src_padding_mask)
            if query_pos is not None and not query_pos.is_contiguous():
                query_pos = query_pos.contiguous()  # once, not per layer (the fused layers read it flat)
            query_pos, pos_acc = pos_sink(query_pos)  # its gradient summed in place (add_norm.pos_sink)
        for lid, layer in enumerate(self.layers):
            if reference_points.shape[-1] == 2:
                ref_in = reference_points[:, :, None] * torch.stack([src_valid_ratios, src_valid_ratios], -1)[:, None]
            else:
                assert reference_points.shape[-1] == 1
                ref_in = reference_points[:, :, None] * src_valid_ratios[:, None, :, None]
            if plain:
                # bf16 self-attention inputs carried from the previous layer's last add + LayerNorm
                output, out16, q16, sampling_locations, attn_weights = layer.forward_carry(
                    output, query_pos, ref_in, src, src_temporal_shapes, src_level_start_index, src_padding_mask,
                    query_padding_mask, values[lid] if values is not None else None, carried, pos_acc=pos_acc)
                carried = (out16, q16) if out16 is not None else None
            else:
                output, sampling_locations, attn_weights = layer(output, query_pos, ref_in, src, src_temporal_shapes,
                                                                 src_level_start_index, src_padding_mask,
                                                                 query_padding_mask)
            locs.append(sampling_locations)
            weights.append(attn_weights)
            if not disable_iterative_refine and self.bbox_head is not None:
                delta = self.bbox_head[lid](output)
                if reference_points.shape[-1] == 2:
                    refined = (delta + inverse_sigmoid(reference_points)).sigmoid()
                else:
                    refined = delta
                    refined[..., :1] = delta[..., :1] + inverse_sigmoid(reference_points)
                    refined = refined.sigmoid()
                reference_points = refined.detach()
            if self.return_intermediate:
                hs.append(output)
                refs.append(reference_points)
        sampling_locations_dec = torch.stack(locs, dim=1)
        attn_weights_dec = torch.stack(weights, dim=1)
        if self.return_intermediate:
            return torch.stack(hs), torch.stack(refs), sampling_locations_dec, attn_weights_dec
        return output, reference_points, sampling_locations_dec, attn_weights_dec


class MaskPredictor(nn.Module):
    """Token saliency scorer: LayerNorm -> Linear -> GELU, local half + clip-mean global half,
    then a 3-layer GELU MLP to one logit per token (reference :634-657)."""

    def __init__(self, in_dim, h_dim):
        super().__init__()
        self.h_dim = h_dim
        self.layer1 = nn.Sequential(nn.LayerNorm(in_dim), Linear(in_dim, h_dim), nn.GELU())
        self.layer2 = nn.Sequential(Linear(h_dim, h_dim // 2), nn.GELU(), Linear(h_dim // 2, h_dim // 4), nn.GELU(),
                                    Linear(h_dim // 4, 1))

    def forward(self, x):
        z = self.layer1(x)
        z_local, z_global = torch.split(z, self.h_dim // 2, dim=-1)
        z_global = z_global.mean(dim=1, keepdim=True).expand(-1, z_local.shape[1], -1)
        return self.layer2(torch.cat([z_local, z_global], dim=-1))


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


def build_sparse_deforamble_transformer(args):
    """reference :676-693 (name kept, typo included)."""
    return SparseDeformableTransformer(
        d_model=args.d_model, num_head=args.num_heads, num_encoder_layers=args.enc_layers,
        num_decoder_layers=args.dec_layers, dim_feedforward=args.transformer_ff_dim,
        dropout=args.transformer_dropout_prob, activation="relu", return_intermediate_dec=args.return_intermediate,
        num_feature_levels=args.num_feature_levels, dec_n_points=args.dec_n_points, enc_n_points=args.enc_n_points,
        rho=args.rho, use_enc_aux_loss=args.use_enc_aux_loss, eff_query_init=args.eff_query_init,
        eff_specific_head=args.eff_specific_head)
