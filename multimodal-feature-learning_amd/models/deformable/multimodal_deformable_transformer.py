"""Video + audio deformable encoder/decoder, same interface as the reference's
``models/deformable/multimodal_deformable_transformer.py``.

Every encoder layer makes four MSDA calls with ONE shared ``self_attn`` module
(video->video, audio->audio, audio queries over video values, video queries over
audio values; reference :256-270); every decoder layer two MSDA cross-attentions
(video, audio) followed by the concat / LayerNorm(2d) / Linear / ReLU bridge
(:410-428).  All MSDA calls run on the HIP kernel through ``MSDeformAttn``.
"""
import math

import torch
from torch import nn
from torch.nn.init import constant_, normal_, xavier_uniform_

from ..modules.pyramid import flatten_levels, level_pos_flatten
from ... import msda as _msda
from ..modules.attention import MSDeformAttn, joint_supported, mha_self_attention
from ..modules.misc_modules import inverse_sigmoid
from ..modules.linear import Linear, mark_grad_sum
from ..modules.add_norm import add_layer_norm, add_layer_norm_carry, carry_entry, carry_supported, pos_sink
from ..modules.ffn import relu_dropout
from ..modules.value_proj import layer_values, layer_values_supported
from .unimodal_deformable_transformer import (_get_activation_fn, _get_clones, encoder_reference_points,
                                              level_metadata)

__all__ = [
    "MultimodalDeformableTransformer", "MultimodalDeformableTransformerEncoderLayer",
    "MultimodalDeformableTransformerEncoder", "MultimodalDeformableTransformerDecoderLayer",
    "MultimodalDeformableTransformerDecoder", "build_multimodal_deformable_transformer",
]


class MultimodalDeformableTransformer(nn.Module):
    """reference multimodal_deformable_transformer.py:11-218 (same constructor, submodule
    names and init; ``pos_trans`` / ``pos_trans_norm`` exist here as in the reference)."""

    def __init__(self, d_model=256, num_head=8, num_encoder_layers=6, num_decoder_layers=6,
                 dim_feedforward=1024, dropout=0.1, activation="relu", return_intermediate_dec=False,
                 num_feature_levels=4, dec_n_points=4, enc_n_points=4):
        super().__init__()
        self.d_model = d_model
        self.num_head = num_head
        self.no_encoder = num_encoder_layers == 0
        self.num_feature_levels = num_feature_levels
        self.encoder = MultimodalDeformableTransformerEncoder(
            MultimodalDeformableTransformerEncoderLayer(d_model, dim_feedforward, dropout, activation,
                                                        num_feature_levels, num_head, enc_n_points),
            num_encoder_layers)
        self.decoder = MultimodalDeformableTransformerDecoder(
            MultimodalDeformableTransformerDecoderLayer(d_model, dim_feedforward, dropout, activation,
                                                        num_feature_levels, num_head, dec_n_points),
            num_decoder_layers, return_intermediate_dec)
        self.level_embed = nn.Parameter(torch.Tensor(num_feature_levels, d_model))
        self.pos_trans = Linear(d_model, d_model * 2)
        self.pos_trans_norm = nn.LayerNorm(d_model * 2)
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

    def get_valid_ratio(self, mask):
        return torch.sum(~mask, 1).float() / mask.shape[1]

    def prepare_encoder_inputs(self, srcs, masks, pos_embeds):
        """One modality's pyramid -> flattened inputs (reference :87-131)."""
        src_flatten = flatten_levels(srcs)
        lvl_pos_embed_flatten = level_pos_flatten(pos_embeds, self.level_embed)
        mask_flatten = torch.cat(list(masks), 1)
        temporal_shapes, level_start_index = level_metadata([s.shape[-1] for s in srcs], src_flatten.device)
        valid_ratios = torch.stack([self.get_valid_ratio(m) for m in masks], 1)
        return src_flatten, temporal_shapes, level_start_index, valid_ratios, lvl_pos_embed_flatten, mask_flatten

    def forward_encoder(self, video_src_flatten, video_temporal_shapes, video_level_start_index, video_valid_ratios,
                        video_lvl_pos_embed_flatten, video_mask_flatten, audio_src_flatten, audio_temporal_shapes,
                        audio_level_start_index, audio_valid_ratios, audio_lvl_pos_embed_flatten, audio_mask_flatten):
        """:return (audio_attended_visual (B, S_v, d), visual_attended_audio (B, S_a, d)) (reference :133-166)"""
        if self.no_encoder:
            return video_src_flatten, audio_src_flatten
        return self.encoder(video_src_flatten, video_temporal_shapes, video_level_start_index, video_valid_ratios,
                            video_lvl_pos_embed_flatten, video_mask_flatten, audio_src_flatten, audio_temporal_shapes,
                            audio_level_start_index, audio_valid_ratios, audio_lvl_pos_embed_flatten,
                            audio_mask_flatten)

    def prepare_decoder_input_query(self, batch_size, query_embed):
        query_embed, tgt = torch.chunk(query_embed, 2, dim=1)
        query_embed = query_embed.unsqueeze(0).expand(batch_size, -1, -1)
        tgt = tgt.unsqueeze(0).expand(batch_size, -1, -1)
        reference_points = self.reference_points(query_embed).sigmoid()
        return reference_points, tgt, reference_points, query_embed

    def prepare_decoder_input_proposal(self, gt_reference_points):
        topk_coords_unact = inverse_sigmoid(gt_reference_points)
        pos_trans_out = self.pos_trans_norm(self.pos_trans(self.get_proposal_pos_embed(topk_coords_unact)))
        query_embed, tgt = torch.chunk(pos_trans_out, 2, dim=2)
        return gt_reference_points, tgt, gt_reference_points, query_embed

    def forward_decoder(self, *kargs):
        return self.decoder(*kargs)


class MultimodalDeformableTransformerEncoderLayer(nn.Module):
    """reference :221-277.  Returns ``(audio_attended_visual, visual_attended_audio)``."""

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

    def forward_carry(self, video, audio, video_next_pos, audio_next_pos, video_reference_points,
                      video_temporal_shapes, video_level_start_index, video_padding_mask, audio_reference_points,
                      audio_temporal_shapes, audio_level_start_index, audio_padding_mask, pos_accs=(None, None)):
        """``forward`` with each stream as ``(src, value, query)``: the MSDA self-attention inputs
        arrive as bf16 copies (``src``, ``src + pos``) from the previous layer's fused FFN add +
        LayerNorm, and this layer's FFNs hand the next layer its copies (query = bf16(out +
        next_pos); None when next_pos is None).  ``pos_accs``: the (video, audio) next_pos came
        from ``pos_sink`` (their gradients summed in place by the fused backwards)."""
        def self_block(stream, ref, shapes, starts, mask):
            src, value, query = stream
            attn = self.self_attn(query, ref, value, shapes, starts, mask)
            return add_layer_norm_carry(src, attn, self.norm1, dropout=self.dropout1)[1]

        def ffn(x, next_pos, pos_acc):
            # x's two consumers (linear1, the residual) sum its gradient in one GEMM (mark_grad_sum)
            mark_grad_sum(x)
            hidden = relu_dropout(self.linear1(x), self.activation, self.dropout2)
            out, out16, q16 = add_layer_norm_carry(x, self.linear2(hidden), self.norm2, next_pos, self.dropout3,
                                                   pos_acc=pos_acc)
            return out, out16, (q16 if q16 is not None else out16)

        v16 = self_block(video, video_reference_points, video_temporal_shapes, video_level_start_index,
                         video_padding_mask)
        a16 = self_block(audio, audio_reference_points, audio_temporal_shapes, audio_level_start_index,
                         audio_padding_mask)
        # each stream is the value of one cross-modal call and the query of the other: the two input
        # gradients summed in one GEMM (mark_grad_sum)
        mark_grad_sum(v16)
        mark_grad_sum(a16)
        visual_attended_audio = self.self_attn(a16, audio_reference_points, v16, video_temporal_shapes,
                                               video_level_start_index, video_padding_mask)
        audio_attended_visual = self.self_attn(v16, video_reference_points, a16, audio_temporal_shapes,
                                               audio_level_start_index, audio_padding_mask)
        return (ffn(audio_attended_visual, video_next_pos, pos_accs[0]),
                ffn(visual_attended_audio, audio_next_pos, pos_accs[1]))

    def forward_joint(self, stream, next_pos, pos_acc, self_calls, cross_calls, padding_mask):
        """``forward_carry`` with the video and audio rows in ONE tensor each (``stream`` = (src, value,
        query) of the joint rows, video rows first): the shared self_attn runs both streams' self calls,
        then both cross-modal calls, as ONE value projection, ONE query projection and ONE output
        projection over all the rows (MSDeformAttn.forward_joint, one MSDA launch per call); the add +
        LayerNorms and the FFN run once over all the rows.  Same math per row as ``forward_carry``
        (reference :237-277): the cross calls' outputs come back in query row order, i.e. the video rows
        hold audio_attended_visual and the audio rows visual_attended_audio, each stream's FFN input."""
        src, value, query = stream
        attn = self.self_attn.forward_joint(query, value, padding_mask, self_calls)
        x16 = add_layer_norm_carry(src, attn, self.norm1, dropout=self.dropout1)[1]
        # x16 is the cross calls' value and their query: both input gradients summed in one GEMM
        mark_grad_sum(x16)
        x = self.self_attn.forward_joint(x16, x16, padding_mask, cross_calls)
        mark_grad_sum(x)  # (linear1's input and the add + LayerNorm's residual)
        hidden = relu_dropout(self.linear1(x), self.activation, self.dropout2)
        out, out16, q16 = add_layer_norm_carry(x, self.linear2(hidden), self.norm2, next_pos, self.dropout3,
                                               pos_acc=pos_acc)
        return out, out16, (q16 if q16 is not None else out16)

    def _self_block(self, src, pos, ref, shapes, starts, mask):
        """``norm1(src + dropout1(self_attn(src + pos, src)))`` as its bf16 copy (under bf16 autocast
        on the GPU, from the fused add + LayerNorm; else the fp32 tensor itself): its only
        consumers are the two cross-modal MSDA calls, as query of one and value of the other,
        which would otherwise each cast it."""
        attn = self.self_attn(self.with_pos_embed(src, pos), ref, src, shapes, starts, mask)
        return add_layer_norm_carry(src, attn, self.norm1, dropout=self.dropout1)[1]

    def forward(self, video_src, video_pos, video_reference_points, video_temporal_shapes, video_level_start_index,
                video_padding_mask, audio_src, audio_pos, audio_reference_points, audio_temporal_shapes,
                audio_level_start_index, audio_padding_mask):
        video_src = self._self_block(video_src, video_pos, video_reference_points, video_temporal_shapes,
                                     video_level_start_index, video_padding_mask)
        audio_src = self._self_block(audio_src, audio_pos, audio_reference_points, audio_temporal_shapes,
                                     audio_level_start_index, audio_padding_mask)
        # cross-modal: queries of one stream sample the other stream's values (no residual, no pos)
        visual_attended_audio = self.self_attn(audio_src, audio_reference_points, video_src, video_temporal_shapes,
                                               video_level_start_index, video_padding_mask)
        audio_attended_visual = self.self_attn(video_src, video_reference_points, audio_src, audio_temporal_shapes,
                                               audio_level_start_index, audio_padding_mask)
        return self.forward_ffn(audio_attended_visual), self.forward_ffn(visual_attended_audio)


class MultimodalDeformableTransformerEncoder(nn.Module):
    """reference :280-335"""

    def __init__(self, encoder_layer, num_layers):
        super().__init__()
        self.layers = _get_clones(encoder_layer, num_layers)
        self.num_layers = num_layers

    @staticmethod
    def get_reference_points(temporal_shapes, valid_ratios, device):
        return encoder_reference_points(temporal_shapes, valid_ratios, device)

    def forward(self, video_src, video_temporal_shapes, video_level_start_index, video_valid_ratios, video_pos,
                video_padding_mask, audio_src, audio_temporal_shapes, audio_level_start_index, audio_valid_ratios,
                audio_pos, audio_padding_mask):
        video_ref = self.get_reference_points(video_temporal_shapes, video_valid_ratios, device=video_src.device)
        audio_ref = self.get_reference_points(audio_temporal_shapes, audio_valid_ratios, device=audio_src.device)
        output = video_src, audio_src
        carry = (self.layers and all(type(layer) is MultimodalDeformableTransformerEncoderLayer for layer in self.layers)
                 and carry_supported(video_src, self.layers[0].norm2) and carry_supported(audio_src, self.layers[0].norm2)
                 and all(p is None or p.dtype == torch.float32 for p in (video_pos, audio_pos)))
        if carry and _joint_ok(self, video_src, audio_src, video_pos, audio_pos):
            return self._forward_joint(video_src, video_temporal_shapes, video_level_start_index, video_pos,
                                       video_padding_mask, video_ref, audio_src, audio_temporal_shapes,
                                       audio_level_start_index, audio_pos, audio_padding_mask, audio_ref)
        if carry:
            # bf16 MSDA operands carried from each layer's fused FFN add + LayerNorm to the next;
            # each pos's gradient summed in place by those fused backwards (add_norm.pos_sink)
            wp = MultimodalDeformableTransformerEncoderLayer.with_pos_embed
            video_pos, vacc = pos_sink(video_pos)
            audio_pos, aacc = pos_sink(audio_pos)
            # (src, bf16(src), bf16(src + pos)) of each stream in one pass where the fused kernel applies
            v = carry_entry(video_src, video_pos, vacc) or (video_src, video_src, wp(video_src, video_pos))
            a = carry_entry(audio_src, audio_pos, aacc) or (audio_src, audio_src, wp(audio_src, audio_pos))
            for i, layer in enumerate(self.layers):
                last = i + 1 == len(self.layers)
                v, a = layer.forward_carry(v, a, None if last else video_pos, None if last else audio_pos,
                                           video_ref, video_temporal_shapes, video_level_start_index,
                                           video_padding_mask, audio_ref, audio_temporal_shapes,
                                           audio_level_start_index, audio_padding_mask, pos_accs=(vacc, aacc))
            v[0]._mfl_bf16, a[0]._mfl_bf16 = v[1], a[1]  # bf16(out): the decoder's value projections read them
            return v[0], a[0]
        for layer in self.layers:
            v, a = output
            output = layer(v, video_pos, video_ref, video_temporal_shapes, video_level_start_index, video_padding_mask,
                           a, audio_pos, audio_ref, audio_temporal_shapes, audio_level_start_index, audio_padding_mask)
        return output


    def _forward_joint(self, video_src, video_temporal_shapes, video_level_start_index, video_pos, video_padding_mask,
                       video_ref, audio_src, audio_temporal_shapes, audio_level_start_index, audio_pos,
                       audio_padding_mask, audio_ref):
        """The carried layers on the joint rows (``forward_joint``): both streams' rows and position
        embeddings concatenated once (video first), split back into the two memories at the end."""
        B, Sv, d = video_src.shape
        Sa = audio_src.shape[1]
        nv, na = B * Sv, B * Sa
        v_shapes, v_starts = _msda.host_levels(video_temporal_shapes, video_level_start_index)
        a_shapes, a_starts = _msda.host_levels(audio_temporal_shapes, audio_level_start_index)
        src = torch.cat([video_src.reshape(nv, d), audio_src.reshape(na, d)])
        pos = None if video_pos is None else torch.cat([video_pos.reshape(nv, d), audio_pos.reshape(na, d)])
        mask = None
        if video_padding_mask is not None or audio_padding_mask is not None:
            vm = (video_padding_mask if video_padding_mask is not None
                  else torch.zeros((B, Sv), dtype=torch.bool, device=video_src.device))
            am = (audio_padding_mask if audio_padding_mask is not None
                  else torch.zeros((B, Sa), dtype=torch.bool, device=audio_src.device))
            mask = torch.cat([vm.reshape(nv), am.reshape(na)])
        # (q0, q1, v0, v1, B, reference points, value level shapes, starts): video rows first
        self_calls = ((0, nv, 0, nv, B, video_ref, v_shapes, v_starts),
                      (nv, nv + na, nv, nv + na, B, audio_ref, a_shapes, a_starts))
        cross_calls = ((0, nv, nv, nv + na, B, video_ref, a_shapes, a_starts),
                       (nv, nv + na, 0, nv, B, audio_ref, v_shapes, v_starts))
        pos, acc = pos_sink(pos)
        wp = MultimodalDeformableTransformerEncoderLayer.with_pos_embed
        stream = carry_entry(src, pos, acc) or (src, src, wp(src, pos))
        for i, layer in enumerate(self.layers):
            last = i + 1 == len(self.layers)
            stream = layer.forward_joint(stream, None if last else pos, acc, self_calls, cross_calls, mask)
        v_out, a_out = _SplitRows.apply(stream[0], nv, (B, Sv, d), (B, Sa, d))
        v16, a16 = _SplitRows.apply(stream[1], nv, (B, Sv, d), (B, Sa, d))
        v_out._mfl_bf16, a_out._mfl_bf16 = v16, a16  # bf16(out): the decoder's value projections read them
        return v_out, a_out


def _joint_ok(encoder, video_src, audio_src, video_pos, audio_pos):
    """Whether the encoder runs both streams on joint rows (``_forward_joint``; MFL_MM_JOINT=0 keeps the
    per-stream calls for A/B)."""
    import os
    if os.environ.get("MFL_MM_JOINT", "1") == "0":
        return False
    attn = encoder.layers[0].self_attn
    return (video_src.dim() == 3 and audio_src.dim() == 3 and video_src.shape[0] == audio_src.shape[0]
            and video_src.shape[2] == audio_src.shape[2] and video_src.dtype == audio_src.dtype == torch.float32
            and (video_pos is None) == (audio_pos is None)
            and all(p is None or p.shape == s.shape for p, s in ((video_pos, video_src), (audio_pos, audio_src)))
            and joint_supported(attn, video_src.reshape(-1, video_src.shape[-1]),
                                audio_src.reshape(-1, audio_src.shape[-1])))


class _SplitRows(torch.autograd.Function):
    """(x[:n] as shape_a, x[n:] as shape_b) of joint rows; backward ONE concatenation of the two
    gradients (zeros for a part that got none) instead of autograd's two zero-filled full-size slice
    gradients and their sum."""

    @staticmethod
    def forward(ctx, x, n, shape_a, shape_b):
        ctx.set_materialize_grads(False)
        ctx.n, ctx.shape, ctx.dtype = n, x.shape, x.dtype
        return x[:n].view(shape_a), x[n:].view(shape_b)

    @staticmethod
    def backward(ctx, ga, gb):
        if ga is None and gb is None:
            return None, None, None, None
        n, (R, d) = ctx.n, ctx.shape
        ref = ga if ga is not None else gb
        ga = ga.reshape(n, d) if ga is not None else ref.new_zeros((n, d))
        gb = gb.reshape(R - n, d) if gb is not None else ref.new_zeros((R - n, d))
        return torch.cat([ga, gb]), None, None, None


class MultimodalDeformableTransformerDecoderLayer(nn.Module):
    """reference :338-432"""

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
        self.norm4 = nn.LayerNorm(2 * d_model)
        self.linear3 = Linear(2 * d_model, d_model)
        self.dropout5 = nn.Dropout(dropout)

    @staticmethod
    def with_pos_embed(tensor, pos):
        return tensor if pos is None else tensor + pos

    def forward_ffn(self, tgt):
        hidden = relu_dropout(self.linear1(tgt), self.activation, self.dropout3)
        return add_layer_norm(tgt, self.linear2(hidden), self.norm3, dropout=self.dropout4)

    def _cross_block(self, tgt, query_pos, ref, src, shapes, starts, mask, value=None):
        attn = self.cross_attn(self.with_pos_embed(tgt, query_pos), ref, src, shapes, starts, mask, value=value)
        return add_layer_norm(tgt, attn, self.norm1, dropout=self.dropout1)

    def forward_carry(self, tgt, query_pos, reference_points_input_video, reference_points_input_audio, query_mask,
                      video_src, video_temporal_shapes, video_level_start_index, video_src_padding_mask, audio_src,
                      audio_temporal_shapes, audio_level_start_index, audio_src_padding_mask, video_value=None,
                      audio_value=None, carried=None, pos_acc=None):
        """``forward`` returning ``(out, out16, q16)`` with the bf16 operands carried between the fused
        add + LayerNorms (bf16 autocast on the GPU): the self-attention add + LayerNorm hands both
        cross-attentions ONE query bf16(tgt + query_pos) (no pos adds or casts, its two gradients
        summed by autograd once), the FFN's the next layer's self-attention inputs (``carried``);
        query_pos's gradient summed in place (``pos_acc``, add_norm.pos_sink).  Same math as
        ``forward`` (reference :410-432)."""
        sa = mha_self_attention(self.self_attn, tgt, query_pos, query_mask, carried)
        tgt, _, q16 = add_layer_norm_carry(tgt, sa, self.norm2, query_pos, self.dropout2, pos_acc=pos_acc)
        query = q16 if q16 is not None else tgt
        # the one query of both cross-attentions: their two prologue input gradients summed in one GEMM
        mark_grad_sum(query)
        ca_v = self.cross_attn(query, reference_points_input_video, video_src, video_temporal_shapes,
                               video_level_start_index, video_src_padding_mask, value=video_value)
        tgt_video = add_layer_norm(tgt, ca_v, self.norm1, dropout=self.dropout1)
        ca_a = self.cross_attn(query, reference_points_input_audio, audio_src, audio_temporal_shapes,
                               audio_level_start_index, audio_src_padding_mask, value=audio_value)
        tgt_audio = add_layer_norm(tgt, ca_a, self.norm1, dropout=self.dropout1)
        bridged = self.linear3(self.norm4(torch.cat([tgt_video, tgt_audio], dim=-1)))
        t = relu_dropout(bridged, self.activation, self.dropout5)
        mark_grad_sum(t)  # (linear1's input and the add + LayerNorm's residual)
        hidden = relu_dropout(self.linear1(t), self.activation, self.dropout3)
        return add_layer_norm_carry(t, self.linear2(hidden), self.norm3, query_pos, self.dropout4, pos_acc=pos_acc)

    def forward(self, tgt, query_pos, reference_points_input_video, reference_points_input_audio, query_mask,
                video_src, video_temporal_shapes, video_level_start_index, video_src_padding_mask, audio_src,
                audio_temporal_shapes, audio_level_start_index, audio_src_padding_mask, video_value=None,
                audio_value=None):
        """``video_value`` / ``audio_value``: this layer's cross-attention values of the two memories,
        when the decoder computed every layer's at once (models/modules/value_proj.py)."""
        sa = mha_self_attention(self.self_attn, tgt, query_pos, query_mask)
        tgt = add_layer_norm(tgt, sa, self.norm2, dropout=self.dropout2)
        tgt_video = self._cross_block(tgt, query_pos, reference_points_input_video, video_src, video_temporal_shapes,
                                      video_level_start_index, video_src_padding_mask, video_value)
        tgt_audio = self._cross_block(tgt, query_pos, reference_points_input_audio, audio_src, audio_temporal_shapes,
                                      audio_level_start_index, audio_src_padding_mask, audio_value)
        bridged = self.linear3(self.norm4(torch.cat([tgt_video, tgt_audio], dim=-1)))
        tgt = self.activation(self.dropout5(bridged))
        return self.forward_ffn(tgt)


class MultimodalDeformableTransformerDecoder(nn.Module):
    """reference :435-512"""

    def __init__(self, decoder_layer, num_layers, return_intermediate=False):
        super().__init__()
        self.layers = _get_clones(decoder_layer, num_layers)
        self.num_layers = num_layers
        self.return_intermediate = return_intermediate
        self.bbox_head = None

    def flat_groups(self):
        """Parameters a flat-buffer trainer should lay out back to back (train_step._flat_order): each
        same-shape weight of the layers, and the query prologue's [W_off; W_aw] pairs interleaved, so
        that the deferred short-K queue's batched gradient GEMMs write one view of the flat gradient
        buffer (linear._WgradQueue) — as the unimodal decoder's."""
        layers = [layer for layer in self.layers if type(layer) is MultimodalDeformableTransformerDecoderLayer]
        if len(layers) < 2:
            return []
        names = ("linear1.weight", "linear2.weight", "linear3.weight", "self_attn.out_proj.weight",
                 "cross_attn.value_proj.weight", "cross_attn.value_proj.bias", "cross_attn.output_proj.weight")
        groups = [tuple(layer.get_parameter(n) for layer in layers) for n in names]
        for kind in ("weight", "bias"):
            groups.append(tuple(layer.get_parameter(f"cross_attn.{n}.{kind}") for layer in layers
                                for n in ("sampling_offsets", "attention_weights")))
        return groups

    @staticmethod
    def _per_level(reference_points, valid_ratios):
        if reference_points.shape[-1] == 2:
            return reference_points[:, :, None] * torch.stack([valid_ratios, valid_ratios], -1)[:, None]
        assert reference_points.shape[-1] == 1
        return reference_points[:, :, None] * valid_ratios[:, None, :, None]

    def forward(self, tgt, reference_points, query_pos, query_padding_mask, video_src, video_temporal_shapes,
                video_level_start_index, video_valid_ratios, video_padding_mask, audio_src, audio_temporal_shapes,
                audio_level_start_index, audio_valid_ratios, audio_padding_mask, disable_iterative_refine=False):
        output = tgt
        hs, refs = [], []
        vvals = avals = None
        attns = [getattr(layer, "cross_attn", None) for layer in self.layers]
        if (all(type(layer) is MultimodalDeformableTransformerDecoderLayer for layer in self.layers)
                and layer_values_supported(attns, video_src, video_padding_mask)
                and layer_values_supported(attns, audio_src, audio_padding_mask)):
            # every layer projects the same two memories: one batched GEMM each way per memory
            vvals = layer_values(attns, video_src, video_padding_mask)
            avals = layer_values(attns, audio_src, audio_padding_mask)
        carry = (all(type(layer) is MultimodalDeformableTransformerDecoderLayer for layer in self.layers)
                 and carry_supported(output, self.layers[0].norm2)
                 and (query_pos is None or (query_pos.shape == output.shape and query_pos.dtype == torch.float32)))
        carried = pos_acc = None
        if carry:
            if query_pos is not None and not query_pos.is_contiguous():
                query_pos = query_pos.contiguous()  # once, not per layer (the fused layers read it flat)
            query_pos, pos_acc = pos_sink(query_pos)  # its gradient summed in place (add_norm.pos_sink)
        for lid, layer in enumerate(self.layers):
            ref_v = self._per_level(reference_points, video_valid_ratios)
            ref_a = self._per_level(reference_points, audio_valid_ratios)
            extra = {} if vvals is None else {"video_value": vvals[lid], "audio_value": avals[lid]}
            if carry:
                # bf16 operands carried between the fused add + LayerNorms (forward_carry)
                output, out16, q16 = layer.forward_carry(
                    output, query_pos, ref_v, ref_a, query_padding_mask, video_src, video_temporal_shapes,
                    video_level_start_index, video_padding_mask, audio_src, audio_temporal_shapes,
                    audio_level_start_index, audio_padding_mask, carried=carried, pos_acc=pos_acc, **extra)
                carried = (out16, q16)
            else:
                output = layer(output, query_pos, ref_v, ref_a, query_padding_mask, video_src, video_temporal_shapes,
                               video_level_start_index, video_padding_mask, audio_src, audio_temporal_shapes,
                               audio_level_start_index, audio_padding_mask, **extra)
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
        if self.return_intermediate:
            return torch.stack(hs), torch.stack(refs)
        return output, reference_points


def build_multimodal_deformable_transformer(args):
    return MultimodalDeformableTransformer(
        d_model=args.d_model, num_head=args.num_heads, num_encoder_layers=args.enc_layers,
        num_decoder_layers=args.dec_layers, dim_feedforward=args.transformer_ff_dim,
        dropout=args.transformer_dropout_prob, activation="relu",
        return_intermediate_dec=args.return_intermediate, num_feature_levels=args.num_feature_levels,
        dec_n_points=args.dec_n_points, enc_n_points=args.enc_n_points)
