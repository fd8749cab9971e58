"""``UnimodalSparseDVC``, reference models/sparse/unimodal_sparse_dvc.py:35-529 — the reference's
default model (config_dvc_train.py:135-136) and the only DVC wrapper that trains end to end at
HEAD, so its forward is pinned whole against a reference run (tests/golden/sparse_dvc_f64.pt):
heads, Hungarian matching, segment crop, caption decoder (teacher forcing and greedy decode).

Same constructor, state_dict keys and ``forward(obj, is_training=True, faster_eval=False,
val_mode="one_by_one")`` -> ``(out, captions, indices, indices_aux, mask)``.  The MSDA calls run on
the HIP kernel; matching makes one device->host copy; crop / denormalisation are device index math;
the one_by_one decode uses the KV-cached greedy loop (models/unimodal_caption_decoder.py)."""
import copy
import math
from math import ceil

import torch
from torch import nn

from ..base_encoder import build_base_encoder
from ..dvc_common import (append_end_token, context_mask, look_ahead_mask, make_padding_mask, segment_memory,
                          special_tokens)
from ..modules.embedding_layers import PositionEmbeddingVideoSine
from ..modules.layers import FFN, ContextMaskModel
from ..modules.linear import Linear
from ..modules.misc_modules import inverse_sigmoid, predict_event_num_with_depth
from ..unimodal_caption_decoder import build_unimodal_caption_decoder
from .unimodal_sparse_deformable_transformer import build_sparse_deforamble_transformer

__all__ = ["UnimodalSparseDVC", "decoder_reference_stack"]


def _get_clones(module, N):
    return nn.ModuleList([copy.deepcopy(module) for _ in range(N)])


def decoder_reference_stack(init_reference, inter_references):
    """The per-level reference points the segment head is offset by, as the reference computes
    them (:193-196): ``reference = inter_references; reference[0] = init_reference;
    reference[1:] = inter_references[:-1].clone()`` — the in-place first write is visible to the
    clone, so levels 0 and 1 both get init_reference.  Out of place here, same values."""
    parts = [init_reference[None]]
    if inter_references.shape[0] > 1:
        parts += [init_reference[None], inter_references[1:-1]]
    return torch.cat(parts, 0)


class UnimodalSparseDVC(nn.Module):
    def __init__(self, input_modalities, num_queries, d_model, num_classes, aux_loss, matcher, threshold,
                 max_eseq_length, vocab, seq_len, embedding_matrix, sparse_detr_args, caption_args,
                 use_differentiable_mask=False):
        super().__init__()
        self.input_modalities = input_modalities
        self.num_queries = num_queries
        self.aux_loss = aux_loss
        self.num_classes = num_classes
        self.threshold = threshold
        self.query_embedding = nn.Embedding(num_queries, d_model * 2)
        self.segment_embedding_encoder = FFN(in_dim=d_model, hidden_dim=d_model, out_dim=2, num_layers=3)
        self.segment_embedding_decoder = FFN(in_dim=d_model, hidden_dim=d_model, out_dim=2, num_layers=3)
        self.count_head_encoder = Linear(d_model, max_eseq_length + 1)
        self.count_head_decoder = Linear(d_model, max_eseq_length + 1)
        self.matcher = matcher
        assert 'video' in input_modalities or 'audio' in input_modalities, \
            f'input_modalities should contain one of "video" or "audio". You have {input_modalities}'
        self.pos_embed = PositionEmbeddingVideoSine(d_model // 2, normalize=True)
        self.rho = sparse_detr_args.rho
        self.use_enc_aux_loss = sparse_detr_args.use_enc_aux_loss
        self.base_encoder = build_base_encoder(sparse_detr_args)
        nn.init.constant_(self.segment_embedding_encoder.layers[-1].weight.data, 0.)
        nn.init.constant_(self.segment_embedding_encoder.layers[-1].bias.data, 0.)
        nn.init.constant_(self.segment_embedding_decoder.layers[-1].weight.data, 0.)
        nn.init.constant_(self.segment_embedding_decoder.layers[-1].bias.data[:2], 0.)
        nn.init.constant_(self.segment_embedding_decoder.layers[-1].bias.data[2:], -2.0)
        self.unimodal_sparse_transformer = build_sparse_deforamble_transformer(sparse_detr_args)
        if sparse_detr_args.use_enc_aux_loss:
            enc = self.unimodal_sparse_transformer.encoder
            enc.aux_heads = True
            enc.count_head = self.count_head_encoder
            enc.segment_embedding = self.segment_embedding_encoder
        self.num_feature_levels = sparse_detr_args.num_feature_levels
        self.video_rescale_len = sparse_detr_args.video_rescale_len
        self.num_tokens = ceil(((2 ** self.num_feature_levels - 1) / 2 ** (self.num_feature_levels - 1))
                               * self.video_rescale_len)
        self.use_differentiable_mask = use_differentiable_mask
        if use_differentiable_mask:
            self.context_mask_model = ContextMaskModel(in_dim=(2 + d_model), out_dim=self.num_tokens)
        self.seq_len = seq_len
        self.vocab = vocab
        self.unimodal_caption_decoder = build_unimodal_caption_decoder(caption_args, len(vocab), seq_len,
                                                                       embedding_matrix)

    def forward_proposals(self, video, video_mask, durations):
        """Proposal path (reference :145-229) -> (out, query_features, memory, outputs_segment, outputs_count, masks)."""
        tr = self.unimodal_sparse_transformer
        B = video.shape[0]
        srcs, masks, pos = self.base_encoder(video, video_mask, durations, self.pos_embed)
        (src_flatten, shapes, starts, valid, lvl_pos, mask_flatten, proposals, topk, mask_pred,
         sparse_token_nums) = tr.prepare_encoder_inputs(srcs, masks, pos)
        memory, sl_enc, aw_enc, enc_count, enc_segments = tr.forward_encoder(
            src_flatten, shapes, starts, valid, lvl_pos, mask_flatten, proposals, topk, sparse_token_nums)
        qw = self.query_embedding.weight
        proposals_mask = torch.ones(B, qw.shape[0], device=qw.device).bool()
        init_reference, tgt, reference_points, qw = tr.prepare_decoder_input_query(B, qw)
        query_features, inter_references, sl_dec, aw_dec = tr.forward_decoder(
            tgt, reference_points, memory, shapes, starts, valid, qw, mask_flatten, proposals_mask, False)
        outputs_segment = self.segment_embedding_decoder(query_features)
        outputs_count = predict_event_num_with_depth(self.count_head_decoder, query_features)
        reference = inverse_sigmoid(decoder_reference_stack(init_reference, inter_references))
        assert reference.shape[-1] in (1, 2)
        # ``outputs_segment[..., :2] += reference`` (:199-203): a (..., 1) reference offsets both terms
        outputs_segment = (outputs_segment + reference).sigmoid()
        out = {'pred_segments': outputs_segment[-1], 'pred_count': outputs_count[-1],
               'sampling_locations_enc': sl_enc, 'attn_weights_enc': aw_enc,
               'sampling_locations_dec': sl_dec, 'attn_weights_dec': aw_dec,
               'temporal_shapes': shapes, 'level_start_index': starts}
        if topk is not None:
            out["backbone_topk_proposals"] = topk
        if self.rho:
            out["backbone_mask_prediction"] = mask_pred
        if self.use_enc_aux_loss:
            out['aux_outputs_enc'] = self._set_aux_loss(enc_segments, enc_count, is_enc_aux=True)
        if self.rho:
            out["sparse_token_nums"] = sparse_token_nums
        out['mask_flatten'] = torch.cat([m.flatten(1) for m in masks], 1)
        return out, query_features, memory, outputs_segment, outputs_count

    def forward(self, obj, is_training=True, faster_eval=False, val_mode="one_by_one"):
        video = obj['video_tensor']
        durations = obj['video_length'][:, 1]
        out, query_features, memory, outputs_segment, outputs_count = self.forward_proposals(
            video, obj['video_mask'], durations)
        num_pred = outputs_segment.shape[0]
        aux = self._set_aux_loss(outputs_segment, outputs_count) if self.aux_loss else []
        # last level + aux levels matched in one device->host copy (reference: one .cpu() each, :233,291)
        all_indices = self.matcher.match_levels([out] + aux, obj['video_target'])
        indices = all_indices[0]
        idx, idx_dev, denorm, memory, memory_mask = segment_memory(
            memory, out, indices, durations, self.num_feature_levels, self.video_rescale_len)
        if self.use_differentiable_mask:
            pred_logits, pred_memory_mask = context_mask(self.context_mask_model, denorm, query_features[-1][idx_dev],
                                                         memory_mask)
            out['pred_memory_mask'] = pred_logits
        key_mask = pred_memory_mask if self.use_differentiable_mask else memory_mask
        mask_out = memory_mask.float() if self.use_differentiable_mask else None

        def teacher_forced():
            tgt_captions = obj['cap_tensor'][:, :-1]
            tgt_padding_mask = obj['cap_mask'][:, :-1]
            return self.unimodal_caption_decoder(tgt=tgt_captions, memory=memory,
                                                 tgt_mask=look_ahead_mask(tgt_captions.shape[1], memory.device),
                                                 memory_mask=None, tgt_padding_mask=tgt_padding_mask,
                                                 memory_padding_mask=key_mask)

        if is_training:
            outputs_caption = teacher_forced()
            out["pred_captions"] = outputs_caption[-1]
            captions_out = torch.argmax(outputs_caption[-1], dim=2)
        elif val_mode == "one_by_one":
            bos, eos, pad = special_tokens(self.vocab)
            captions, last_input = self.unimodal_caption_decoder.greedy_decode(memory, key_mask, bos, eos, pad,
                                                                               self.seq_len, faster_eval)
            outputs_caption = self._caption_probs(last_input, memory, key_mask)
            out['pred_captions'] = outputs_caption[-1]
            captions_out = append_end_token(captions, self.vocab, faster_eval)
        elif val_mode == "teacher_forcing":
            outputs_caption = teacher_forced()
            out["pred_captions"] = outputs_caption[-1]
            captions_out = torch.argmax(outputs_caption[-1], dim=2)
        else:
            raise ValueError(f"val_mode must be 'one_by_one' or 'teacher_forcing', got {val_mode!r}")

        indices_aux = []
        if self.aux_loss:
            out['aux_outputs'] = aux
            indices_aux = all_indices[1:]
            out['aux_outputs_caption'] = self._set_aux_loss_caption(outputs_caption)
        return out, captions_out, indices, indices_aux, mask_out

    @torch.no_grad()
    def _caption_probs(self, captions, memory, key_mask):
        """Full decoder output over ``captions`` (all depths), as the reference's last decode word."""
        return self.unimodal_caption_decoder(tgt=captions, memory=memory,
                                             tgt_mask=look_ahead_mask(captions.shape[1], memory.device),
                                             memory_mask=None, tgt_padding_mask=make_padding_mask(captions, self.vocab),
                                             memory_padding_mask=key_mask)

    def _set_aux_loss(self, outputs_segment, outputs_count, is_enc_aux=False):
        if is_enc_aux:
            return [{'pred_segments': a, 'pred_count': b} for a, b in zip(outputs_segment, outputs_count)]
        return [{'pred_segments': a, 'pred_count': b} for a, b in zip(outputs_segment[:-1], outputs_count[:-1])]

    def _set_aux_loss_caption(self, outputs_caption):
        return [{'pred_captions': a} for a in outputs_caption[:-1]]

    def make_tgt_mask(self, target, device):
        return look_ahead_mask(target.shape[1], device)

    def make_padding_mask(self, target):
        return make_padding_mask(target, self.vocab)

    def get_segment_features(self, features, denormalized_segments, idx, video_durations):
        return self.crop_segments(features, denormalized_segments, idx[0], video_durations)

    def crop_segments(self, features, denormalized_segments, segment_batch_id, video_durations):
        from ...utils.preds_postprocess import crop_segments
        return crop_segments(features, denormalized_segments, segment_batch_id, video_durations,
                             self.num_feature_levels, self.video_rescale_len)
