"""``MultimodalDeformableDVC``, reference models/deformable/multimodal_deformable_dvc.py:29-569:
video + audio streams through one shared BaseEncoder, the multimodal deformable transformer (HIP
MSDA: 4 calls per encoder layer, 2 per decoder layer), shared heads with reference-point offsets,
matching, per-modality crops and the MultimodalCaptionDecoder.  Constructor, state_dict keys and
``forward(obj, is_training=True, faster_eval=False)`` -> ``(out, captions, indices, indices_aux,
video_mask, audio_mask)`` as engine.py:71 consumes it.

The reference cannot be built or run at HEAD.  What is restated, each marked at the code:
* ``detr_args`` is used (:63,74,76,88) but the parameter is ``sparse_detr_args`` (:32): here the
  parameter is ``detr_args`` (what models/__init__.py:55-68 passes) and ``sparse_detr_args`` is
  accepted as an alias; ``max_eseq_length``, omitted by the builder, defaults to 10 (the config's).
* ``self.video_num_tokens`` (:95) is ``self.num_tokens``; ``memory`` (:284) is the video memory.
* the caption-decoder calls use the keyword convention of the working sparse wrappers
  (models/sparse/multimodal_sparse_dvc.py:299-305): the positional call (:320-322) shifts every mask
  by one slot and ``nn.MultiheadAttention`` rejects the (N,1,L,L) masks it builds.
* inference reads ``memory_list`` / ``memory_mask_list`` (:348-350), which do not exist: the video ones.
Everything else is computed as written — each level denormalises the LAST level's segments at its
own matching (:256), rebinds ``video_memory`` / ``audio_memory`` to its crop so the next level crops
that (:259-260), and crops audio on the video token ranges (``crop_segments`` reads
``video_rescale_len``, :530) — and the training forward is pinned against the reference run with
exactly these names bound (tests/golden/mm_dvc_f64.pt)."""
import math
from math import ceil

import torch
from torch import nn

from ..base_encoder import build_base_encoder
from ..dvc_common import append_end_token, context_mask, look_ahead_mask, make_padding_mask, segment_memory, \
    special_tokens
from ..modules.embedding_layers import PositionEmbeddingVideoSine
from ..modules.layers import FFN, ContextMaskModel
from ..modules.linear import Linear
from ..modules.misc_modules import inverse_sigmoid, predict_event_num, predict_event_num_with_depth
from ..multimodal_caption_decoder import build_multimodal_caption_decoder
from ...utils.preds_postprocess import crop_segments
from .multimodal_deformable_transformer import build_multimodal_deformable_transformer

__all__ = ["MultimodalDeformableDVC"]


class MultimodalDeformableDVC(nn.Module):
    def __init__(self, input_modalities, num_queries, d_model, num_classes, aux_loss, matcher, threshold,
                 max_eseq_length=10, vocab=None, seq_len=None, embedding_matrix=None, detr_args=None, caption_args=None,
                 use_differentiable_mask=False, sparse_detr_args=None):
        super().__init__()
        detr_args = detr_args if detr_args is not None else sparse_detr_args
        self.input_modalities = input_modalities
        self.num_queries = num_queries
        self.aux_loss = aux_loss
        self.num_classes = num_classes
        self.threshold = threshold
        self.query_embedding = nn.Embedding(num_queries, d_model * 2)
        self.class_embedding = Linear(d_model, num_classes + 1)
        self.segment_embedding = FFN(in_dim=d_model, hidden_dim=d_model, out_dim=2, num_layers=3)
        self.count_head = Linear(d_model, max_eseq_length + 1)
        self.matcher = matcher
        assert 'video' in input_modalities and 'audio' in input_modalities, \
            f'input_modalities should contain both, "video" and "audio". You have {input_modalities}'
        self.pos_embed = PositionEmbeddingVideoSine(d_model // 2, normalize=True)
        self.rho = getattr(detr_args, "rho", 0)
        self.use_enc_aux_loss = getattr(detr_args, "use_enc_aux_loss", False)
        self.base_encoder = build_base_encoder(detr_args)
        prior_prob = 0.01
        bias_value = -math.log((1 - prior_prob) / prior_prob)
        self.class_embedding.bias.data = torch.ones(num_classes + 1) * bias_value
        nn.init.constant_(self.segment_embedding.layers[-1].weight.data, 0)
        nn.init.constant_(self.segment_embedding.layers[-1].bias.data, 0)
        self.multimodal_deformable_transformer = build_multimodal_deformable_transformer(detr_args)
        num_pred = detr_args.dec_layers
        nn.init.constant_(self.segment_embedding.layers[-1].bias.data[2:], -2.0)
        self.class_embedding = nn.ModuleList([self.class_embedding for _ in range(num_pred)])
        self.count_head = nn.ModuleList([self.count_head for _ in range(num_pred)])
        self.segment_embedding = nn.ModuleList([self.segment_embedding for _ in range(num_pred)])
        self.num_feature_levels = detr_args.num_feature_levels
        self.video_rescale_len = detr_args.video_rescale_len
        self.audio_rescale_len = detr_args.audio_rescale_len
        self.num_tokens = ceil(((2 ** self.num_feature_levels - 1) / 2 ** (self.num_feature_levels - 1))
                               * self.video_rescale_len)
        self.audio_num_tokens = ceil(((2 ** self.num_feature_levels - 1) / 2 ** (self.num_feature_levels - 1))
                                     * self.audio_rescale_len)
        self.use_differentiable_mask = use_differentiable_mask
        if use_differentiable_mask:
            self.video_context_mask_model = ContextMaskModel(in_dim=(2 + d_model), out_dim=self.num_tokens)
            self.audio_context_mask_model = ContextMaskModel(in_dim=(2 + d_model), out_dim=self.audio_num_tokens)
        self.seq_len = seq_len
        self.vocab = vocab
        self.multimodal_caption_decoder = build_multimodal_caption_decoder(caption_args, len(vocab), seq_len,
                                                                           embedding_matrix)

    def forward_proposals(self, video, video_mask, audio, audio_mask, durations):
        tr = self.multimodal_deformable_transformer
        B = video.shape[0]
        v_srcs, v_masks, v_pos = self.base_encoder(video, video_mask, durations, self.pos_embed)
        a_srcs, a_masks, a_pos = self.base_encoder(audio, audio_mask, durations, self.pos_embed)
        v = tr.prepare_encoder_inputs(v_srcs, v_masks, v_pos)
        a = tr.prepare_encoder_inputs(a_srcs, a_masks, a_pos)
        video_memory, audio_memory = tr.forward_encoder(*v, *a)
        qw = self.query_embedding.weight
        proposals_mask = torch.ones(B, qw.shape[0], device=qw.device).bool()
        init_reference, tgt, reference_points, qw = tr.prepare_decoder_input_query(B, qw)
        query_features, inter_references = tr.forward_decoder(tgt, reference_points, qw, proposals_mask, video_memory,
                                                              v[1], v[2], v[3], v[5], audio_memory, a[1], a[2], a[3],
                                                              a[5], False)
        if not self.aux_loss:
            query_features, inter_references = query_features[-1:], inter_references[-1:]
        nl = query_features.shape[0]
        refs = [init_reference if lvl == 0 else inter_references[lvl - 1] for lvl in range(nl)]
        assert all(r.shape[-1] in (1, 2) for r in refs)
        shared = all(all(m is h[0] for m in h) for h in (self.class_embedding, self.segment_embedding, self.count_head))
        if shared and all(r.shape == refs[0].shape for r in refs):
            # the reference's heads are one shared module per kind (:72-74): one call over the stacked
            # levels (row-wise layers; each weight's gradient from one GEMM, not six accumulated)
            heads = (self.class_embedding[0](query_features).softmax(dim=-1),
                     # ``output_segment[..., :2] += reference`` (:220-226)
                     (self.segment_embedding[0](query_features) + inverse_sigmoid(torch.stack(refs))).sigmoid(),
                     predict_event_num_with_depth(self.count_head[0], query_features))
        else:
            classes, counts, segments = [], [], []
            for lvl in range(nl):
                classes.append(self.class_embedding[lvl](query_features[lvl]).softmax(dim=-1))
                seg = self.segment_embedding[lvl](query_features[lvl])
                counts.append(predict_event_num(self.count_head[lvl], query_features[lvl]))
                segments.append((seg + inverse_sigmoid(refs[lvl])).sigmoid())
            heads = (torch.stack(classes), torch.stack(segments), torch.stack(counts))
        out = {'pred_logits': heads[0][-1], 'pred_count': heads[2][-1], 'pred_segments': heads[1][-1]}
        return out, query_features, video_memory, audio_memory, heads

    def forward(self, obj, is_training=True, faster_eval=False):
        video, audio = obj['video_tensor'], obj['audio_tensor']
        durations = obj['video_length'][:, 1]
        out, query_features, video_memory, audio_memory, (outputs_class, outputs_segment, outputs_count) = \
            self.forward_proposals(video, obj['video_mask'], audio, obj['audio_mask'], durations)
        num_pred = query_features.shape[0]
        out_aux = [{'pred_logits': outputs_class[l], 'pred_segments': outputs_segment[l],
                    'pred_count': outputs_count[l]} for l in range(num_pred)]
        level_indices = self.matcher.match_levels(out_aux, obj['video_target'])
        vids, auds, outputs_captions = [], [], []
        for lvl in range(num_pred):
            indices = level_indices[lvl]
            # as written: the last level's segments at this level's matching (:256)
            idx, idx_dev, denorm, video_memory, v_mask = segment_memory(video_memory, out, indices, durations,
                                                                        self.num_feature_levels, self.video_rescale_len)
            audio_memory, a_mask = crop_segments(audio_memory, denorm, idx_dev[0], durations, self.num_feature_levels,
                                                 self.video_rescale_len)
            v_key, a_key = v_mask, a_mask
            if self.use_differentiable_mask:
                qsel = query_features[-1][idx_dev]
                v_pred, v_key = context_mask(self.video_context_mask_model, denorm, qsel, v_mask)
                a_pred, a_key = context_mask(self.audio_context_mask_model, denorm, qsel, a_mask)
                out['video_pred_memory_mask'], out['audio_pred_memory_mask'] = v_pred, a_pred
            vids.append((video_memory, v_mask, v_key))
            auds.append((audio_memory, a_mask, a_key))
            if is_training:
                captions = obj['cap_tensor'][:, :-1]
                padding_mask = obj['cap_mask'][:, :-1]
                output_caption = self.multimodal_caption_decoder(
                    tgt=captions, video_memory=video_memory, audio_memory=audio_memory,
                    tgt_mask=look_ahead_mask(captions.shape[1], captions.device), tgt_padding_mask=padding_mask,
                    video_memory_padding_mask=v_key, audio_memory_padding_mask=a_key)
                outputs_captions.append(output_caption[-1])

        masks_out = ((vids[-1][1].float(), auds[-1][1].float()) if self.use_differentiable_mask else (None, None))
        if is_training:
            outputs_caption = torch.stack(outputs_captions)
            out["pred_captions"] = outputs_captions[-1]
            outputs_caption_last_layer = torch.argmax(outputs_captions[-1], dim=2)
            indices_aux = []
            if self.aux_loss:
                out['aux_outputs'] = self._set_aux_loss(outputs_class, outputs_segment, outputs_count, outputs_caption)
                indices_aux = level_indices[:len(out['aux_outputs'])]
            return (out, outputs_caption_last_layer, indices, indices_aux) + masks_out

        bos, eos, pad = special_tokens(self.vocab)
        (v_mem, _, v_key), (a_mem, _, a_key) = vids[-1], auds[-1]
        captions, last_input = self.multimodal_caption_decoder.greedy_decode(v_mem, v_key, a_mem, a_key, bos, eos, pad,
                                                                             self.seq_len - 1, faster_eval)
        out['pred_captions'] = self._caption_probs(last_input, vids[-1], auds[-1])
        captions_with_eos = append_end_token(captions, self.vocab, faster_eval)
        indices_aux = []
        if self.aux_loss:
            first = torch.full_like(captions, pad)
            first[:, 0] = bos
            aux_caps = [self._caption_probs(first, vids[l], auds[l]) for l in range(num_pred - 1)]
            out['aux_outputs'] = self._set_aux_loss(outputs_class, outputs_segment, outputs_count, aux_caps + [None])
            indices_aux = level_indices[:len(out['aux_outputs'])]
        return (out, captions_with_eos, indices, indices_aux) + masks_out

    @torch.no_grad()
    def _caption_probs(self, captions, vid, aud):
        return self.multimodal_caption_decoder(
            tgt=captions, video_memory=vid[0], audio_memory=aud[0],
            tgt_mask=look_ahead_mask(captions.shape[1], captions.device),
            tgt_padding_mask=make_padding_mask(captions, self.vocab), video_memory_padding_mask=vid[2],
            audio_memory_padding_mask=aud[2])[-1]

    def _set_aux_loss(self, outputs_class, outputs_segment, outputs_count, outputs_caption=None):
        if outputs_caption is None:
            return [{'pred_logits': a, 'pred_segments': b, 'pred_count': c}
                    for a, b, c in zip(outputs_class, outputs_segment, outputs_count)]
        return [{'pred_logits': a, 'pred_segments': b, 'pred_count': c, 'pred_captions': d}
                for a, b, c, d in zip(outputs_class[:-1], outputs_segment[:-1], outputs_count[:-1], outputs_caption[:-1])]

    def make_tgt_mask(self, target, tgt_padding_mask):
        from ..dvc_common import make_tgt_mask
        return make_tgt_mask(target, tgt_padding_mask)

    def make_padding_mask(self, target):
        return make_padding_mask(target, self.vocab)
