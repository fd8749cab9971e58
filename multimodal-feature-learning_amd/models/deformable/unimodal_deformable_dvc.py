"""``UnimodalDeformableDVC``, reference models/deformable/unimodal_deformable_dvc.py:26-549, with the
reference constructor, state_dict keys and ``forward(obj, is_training=True, faster_eval=False)``
returning ``(out, captions, indices, indices_aux, mask)`` as engine.py:62 consumes it.

The proposal path (BaseEncoder -> deformable encoder / decoder on the HIP MSDA kernel -> shared
heads) is the bench workload; the caption path (matching, crop, caption decoder) follows.

At HEAD the reference forward cannot run: its caption-decoder call passes the
caption padding mask as ``memory_mask`` and the memory mask as ``tgt_padding_mask`` (:277-279 vs
models/unimodal_caption_decoder.py:68), and without the differentiable mask ``pred_memory_mask`` is
unbound (:264).  Restated intent, which is also what the working UnimodalSparseDVC does
(models/sparse/unimodal_sparse_dvc.py:279-281): captions self-attend under the look-ahead and
caption padding masks, and cross-attend to the matched segment's memory under its crop mask.
That argument order is the only change: everything else computes what the reference's code does
as written — including level l > 0 cropping level l-1's crop (``memory`` is rebound, :235) — and is
pinned against the reference run with just that call fixed (tests/golden/deformable_dvc_f64.pt;
the reference also needs ``use_differentiable_mask=True`` to run at all, :264).  Inference decodes
with a KV cache: the same rows as the reference's full re-decode, one pass per word, last level only
(the only level its token choice reads, :334-338)."""
import math
from math import ceil

import torch
from torch import nn

from ..base_encoder import build_base_encoder
from ..dvc_common import (append_end_token, context_mask, make_padding_mask, make_tgt_mask, segment_memory,
                          special_tokens)
from ..modules.embedding_layers import PositionEmbeddingVideoSine
from ..modules.layers import FFN, ContextMaskModel
from ..modules.linear import Linear
from ..modules.misc_modules import level_heads
from ...utils.preds_postprocess import SegmentMemory, crop_keep, denormalize_segments, get_src_permutation_idx
from ..unimodal_caption_decoder import build_unimodal_caption_decoder
from .unimodal_deformable_transformer import build_unimodal_deformable_transformer

__all__ = ["UnimodalDeformableDVC"]


class UnimodalDeformableDVC(nn.Module):
    def __init__(self, input_modalities, num_queries, d_model, num_classes, aux_loss, matcher, threshold,
                 max_eseq_length, vocab, seq_len, embedding_matrix, detr_args, caption_args,
                 use_differentiable_mask=False):
        super().__init__()
        self.input_modalities = input_modalities
        self.num_queries = num_queries
        self.aux_loss = aux_loss
        self.threshold = threshold
        self.query_embedding = nn.Embedding(num_queries, d_model * 2)
        self.class_embedding = Linear(d_model, num_classes + 1)
        self.segment_embedding = FFN(in_dim=d_model, hidden_dim=d_model, out_dim=2, num_layers=3)
        self.count_head = Linear(d_model, max_eseq_length + 1)
        self.matcher = matcher
        assert 'video' in input_modalities or 'audio' in input_modalities, \
            f'input_modalities should contain one of "video" or "audio". You have {input_modalities}'
        self.pos_embed = PositionEmbeddingVideoSine(d_model // 2, normalize=True)
        self.base_encoder = build_base_encoder(detr_args)
        prior_prob = 0.01
        bias_value = -math.log((1 - prior_prob) / prior_prob)
        self.class_embedding.bias.data = torch.ones(num_classes + 1) * bias_value
        nn.init.constant_(self.segment_embedding.layers[-1].weight.data, 0)
        nn.init.constant_(self.segment_embedding.layers[-1].bias.data, 0)
        self.unimodal_deformable_transformer = build_unimodal_deformable_transformer(detr_args)
        num_pred = detr_args.dec_layers
        nn.init.constant_(self.segment_embedding.layers[-1].bias.data[2:], -2.0)
        # heads shared by every decoder level (reference :72-74)
        self.class_embedding = nn.ModuleList([self.class_embedding for _ in range(num_pred)])
        self.count_head = nn.ModuleList([self.count_head for _ in range(num_pred)])
        self.segment_embedding = nn.ModuleList([self.segment_embedding for _ in range(num_pred)])
        self.num_feature_levels = detr_args.num_feature_levels
        self.video_rescale_len = detr_args.video_rescale_len
        self.num_tokens = ceil(((2 ** self.num_feature_levels - 1) / 2 ** (self.num_feature_levels - 1))
                               * self.video_rescale_len)
        self.use_differentiable_mask = use_differentiable_mask
        if use_differentiable_mask:
            self.context_mask_model = ContextMaskModel(in_dim=(2 + d_model), out_dim=self.num_tokens)
        self.seq_len = seq_len
        self.vocab = vocab
        self.unimodal_caption_decoder = build_unimodal_caption_decoder(caption_args, len(vocab), seq_len,
                                                                       embedding_matrix)

    # --- proposal path ------------------------------------------------------------------------
    def forward_proposals(self, video, video_mask, durations):
        """BaseEncoder + deformable encoder / decoder + shared heads (reference :135-203).
        -> (out, query_features (depth, B, Q, d), memory (B, S, d), heads stacked over depth)"""
        tr = self.unimodal_deformable_transformer
        B = video.shape[0]
        srcs, masks, pos = self.base_encoder(video, video_mask, durations, self.pos_embed)
        src_flatten, shapes, starts, valid, lvl_pos, mask_flatten = tr.prepare_encoder_inputs(srcs, masks, pos)
        memory = tr.forward_encoder(src_flatten, shapes, starts, valid, lvl_pos, mask_flatten)
        qw = self.query_embedding.weight
        proposals_mask = torch.ones(B, qw.shape[0], device=qw.device).bool()
        _, tgt, reference_points, qw = tr.prepare_decoder_input_query(B, qw)
        query_features, _ = tr.forward_decoder(tgt, reference_points, memory, shapes, starts, valid, qw,
                                               mask_flatten, proposals_mask, False)
        # reference :197-203 applies the (shared) heads level by level: one call over the stacked levels
        heads = level_heads(self, query_features)
        out = {'pred_logits': heads[0][-1], 'pred_segments': heads[1][-1], 'pred_count': heads[2][-1]}
        return out, query_features, memory, heads

    def forward(self, obj, is_training=True, faster_eval=False):
        st = self.forward_stage_proposals(obj)
        # every level's matching in one device->host copy (reference: one .cpu() per level, :227)
        level_indices = self.matcher.solve_levels(st['costs'].cpu(), st['cost_meta'])
        return self.forward_stage_captions(obj, st, level_indices, None, is_training, faster_eval)

    def forward_stage_proposals(self, obj):
        """The device work before the Hungarian matching: proposals and every level's cost
        matrix (``HungarianMatcher.level_costs``).  A graph-captured training step replays this
        stage, copies ``costs`` to the host for the assignment, then replays the caption stage."""
        video = obj['video_tensor']
        video_mask = obj['video_mask']
        durations = obj['video_length'][:, 1]
        out, query_features, memory, (outputs_class, outputs_segment, outputs_count) = \
            self.forward_proposals(video, video_mask, durations)
        num_pred = query_features.shape[0]
        out_aux = [{'pred_logits': outputs_class[l], 'pred_segments': outputs_segment[l],
                    'pred_count': outputs_count[l]} for l in range(num_pred)]
        costs, meta = self.matcher.level_costs(out_aux, obj['video_target'])
        return {'out': out, 'query_features': query_features, 'memory': memory, 'durations': durations,
                'heads': (outputs_class, outputs_segment, outputs_count), 'out_aux': out_aux, 'costs': costs,
                'cost_meta': meta}

    def forward_stage_captions(self, obj, st, level_indices, level_idx_dev=None, is_training=True,
                               faster_eval=False):
        """Everything after the matching (reference :227-372).  ``level_idx_dev``: per decoder level
        the (batch, prediction) indices of the matched segments already on the device (static
        buffers of a captured step), else derived from ``level_indices``."""
        out, query_features, memory = st['out'], st['query_features'], st['memory']
        outputs_class, outputs_segment, outputs_count = st['heads']
        out_aux = st['out_aux']
        num_pred = query_features.shape[0]
        video_durations = st['durations']
        indices = level_indices[-1]
        if is_training:
            # the levels' crops as views of the encoder memory: the caption decoder projects the
            # clips' rows once a step (utils/preds_postprocess.py, SegmentMemory)
            memory = SegmentMemory.of(memory)

        outputs_captions, memory_list, memory_mask_list, pred_memory_mask_list = [], [], [], []
        levels = self._level_crops(memory, outputs_segment, query_features, level_indices, level_idx_dev,
                                   video_durations) if is_training else None
        if levels is not None:
            memory_list, memory_mask_list, pred_memory_mask_list, pred_logits = levels
            if pred_logits is not None:
                out['pred_memory_mask'] = pred_logits
        for lvl in range(num_pred if levels is None else 0):
            # as the reference (:235): ``memory`` is rebound to this level's crop, which the next level crops
            idx, idx_dev, denorm, memory, key_mask = segment_memory(
                memory, out_aux[lvl], level_indices[lvl], video_durations, self.num_feature_levels,
                self.video_rescale_len, idx_dev=None if level_idx_dev is None else level_idx_dev[lvl])
            mem = memory
            memory_mask = key_mask.unsqueeze(1).unsqueeze(1)  # (n, 1, 1, K)
            pred_memory_mask = None
            if self.use_differentiable_mask:
                pred_logits, pred_bool = context_mask(self.context_mask_model, denorm, query_features[lvl][idx_dev],
                                                      key_mask)
                out['pred_memory_mask'] = pred_logits
                pred_memory_mask = pred_bool.unsqueeze(1).unsqueeze(1)
            memory_list.append(mem)
            memory_mask_list.append(memory_mask)
            pred_memory_mask_list.append(pred_memory_mask)
        if is_training:
            # the reference decodes every level's segments in its own caption decoder call (:261-283);
            # the calls are independent (same weights, per-segment rows), so they run as ONE call over
            # the levels' segments stacked along the batch — six times the rows per GEMM, and each
            # weight's gradient produced once instead of accumulated over the levels
            captions = obj['cap_tensor'][:, :-1]
            padding_mask = obj['cap_mask'][:, :-1]
            tgt_mask = make_tgt_mask(captions, padding_mask)
            cross = pred_memory_mask_list if self.use_differentiable_mask else memory_mask_list
            counts = [m.shape[0] for m in memory_list]
            reps = len(counts)
            stacked = (SegmentMemory.cat(memory_list) if all(isinstance(m, SegmentMemory) for m in memory_list)
                       else torch.cat(memory_list))
            # only the last caption layer's word probabilities are read (:281): the head runs on it alone
            output_caption = self.unimodal_caption_decoder(
                captions.repeat(reps, 1), stacked, tgt_mask=tgt_mask.repeat(reps, 1, 1, 1),
                memory_mask=torch.cat(cross), tgt_padding_mask=padding_mask.repeat(reps, 1), last_only=True)
            outputs_captions = list(output_caption[-1].split(counts))
            lg = getattr(output_caption, "_mfl_logits", None)
            if lg is not None:  # (each level's logits, for a loss's fused word gather: word_probs)
                for piece, lgp in zip(outputs_captions, lg[-1].split(counts)):
                    piece._mfl_logits = lgp

        mask_out = memory_mask_list[-1].squeeze().float() if self.use_differentiable_mask else None
        if is_training:
            # the levels' caption probabilities as the split views of the one decoder call (the
            # reference stacks them, :281; every consumer reads one level): no (levels, n, L, vocab)
            # stacking copy, and their gradients meet in the split's one concatenation
            outputs_caption = outputs_captions
            out['pred_captions'] = outputs_caption[-1]
            outputs_caption_last_layer = torch.argmax(outputs_caption[-1], dim=2)
            indices_aux = []
            if self.aux_loss:
                out['aux_outputs'] = self._set_aux_loss(outputs_class, outputs_segment, outputs_count, outputs_caption)
                indices_aux = level_indices[:len(out['aux_outputs'])]  # same segments -> same assignment
            # the same outputs stacked over the levels (a loss may read every level at once:
            # dvc_core.level_terms); private key, the reference's keys are untouched
            caps_all = output_caption[-1]
            if lg is not None:
                caps_all._mfl_logits = lg[-1]
            out['_levels'] = {'logits': outputs_class, 'segments': outputs_segment, 'counts': outputs_count,
                              'captions': caps_all}
            return out, outputs_caption_last_layer, indices, indices_aux, mask_out

        # inference: greedy decode of the last level (the reference's token choice reads only it, :334-338)
        bos, eos, pad = special_tokens(self.vocab)
        cross = pred_memory_mask_list if self.use_differentiable_mask else memory_mask_list
        key_mask = cross[-1][:, 0, 0, :]
        captions, last_input = self.unimodal_caption_decoder.greedy_decode(memory_list[-1], key_mask, bos, eos, pad,
                                                                           self.seq_len - 1, faster_eval)
        out['pred_captions'] = self._caption_probs(last_input, memory_list[-1], cross[-1])
        captions_with_eos = append_end_token(captions, self.vocab, faster_eval)
        indices_aux = []
        if self.aux_loss:
            # the reference's aux captions are the other levels' outputs at the first word (:367)
            first = torch.full_like(captions, pad)
            first[:, 0] = bos
            aux_caps = [self._caption_probs(first, memory_list[l], cross[l]) for l in range(num_pred - 1)]
            out['aux_outputs'] = self._set_aux_loss(outputs_class, outputs_segment, outputs_count, aux_caps + [None])
            indices_aux = level_indices[:len(out['aux_outputs'])]
        return out, captions_with_eos, indices, indices_aux, mask_out

    def _level_crops(self, memory, outputs_segment, query_features, level_indices, level_idx_dev, video_durations):
        """The per-level loop of ``forward_stage_captions`` (reference :227-260: each decoder level's matched
        segments denormalised, the memory cropped — level l cropping level l-1's crop — and the context
        mask predicted) with everything that does not chain from level to level run over all the levels'
        segments at once: the segment gathers, the denormalisation, the crop bounds and the context-mask
        model (row-wise: the same value per row; only the last level's logits reach the loss, the others
        feed the boolean mask).  The crops still compose level by level (``SegmentMemory.select``).  None
        (the loop runs) unless the memory is a SegmentMemory and every level matched the same number of
        segments.  -> (memories, key masks, predicted masks or Nones, last level's mask logits or None)"""
        if not isinstance(memory, SegmentMemory):
            return None
        L = query_features.shape[0]
        dev = outputs_segment.device
        idxs = []
        for lvl in range(L):
            if level_idx_dev is not None:
                idxs.append(level_idx_dev[lvl])
            else:
                idxs.append(tuple(t.to(dev) for t in get_src_permutation_idx(level_indices[lvl])))
        n = int(idxs[0][0].shape[0])
        if n == 0 or any(int(i[0].shape[0]) != n for i in idxs):
            return None
        from ... import _trace
        _trace.hit("level_crops_batched")
        b_all = torch.cat([i[0] for i in idxs])
        s_all = torch.cat([i[1] for i in idxs])
        lv_all = torch.arange(L, device=dev).repeat_interleave(n)
        denorm = denormalize_segments(outputs_segment[lv_all, b_all, s_all], video_durations, b_all)
        keep = crop_keep(denorm, b_all, video_durations, memory.shape[1], self.num_feature_levels,
                         self.video_rescale_len, dev)
        memories, key_masks = [], []
        for lvl in range(L):
            memory = memory.select(idxs[lvl][0], keep[lvl * n:(lvl + 1) * n])
            memories.append(memory)
            key_masks.append((~keep[lvl * n:(lvl + 1) * n]).unsqueeze(1).unsqueeze(1))
        if not self.use_differentiable_mask:
            return memories, key_masks, [None] * L, None
        pred_logits, pred_bool = context_mask(self.context_mask_model, denorm, query_features[lv_all, b_all, s_all],
                                              ~keep)
        preds = [pred_bool[lvl * n:(lvl + 1) * n].unsqueeze(1).unsqueeze(1) for lvl in range(L)]
        return memories, key_masks, preds, pred_logits[(L - 1) * n:]

    @torch.no_grad()
    def _caption_probs(self, captions, mem, cross_mask):
        padding = make_padding_mask(captions, self.vocab)
        return self.unimodal_caption_decoder(captions, mem, tgt_mask=make_tgt_mask(captions, padding),
                                             memory_mask=cross_mask, tgt_padding_mask=padding)[-1]

    def _set_aux_loss(self, outputs_class, outputs_segment, outputs_count, outputs_caption):
        return [{'pred_logits': a, 'pred_segments': b, 'pred_count': c, 'pred_captions': d}
                for a, b, c, d in zip(outputs_class[:-1], outputs_segment[:-1], outputs_count[:-1], outputs_caption[:-1])]

    def make_tgt_mask(self, target, tgt_padding_mask):
        return make_tgt_mask(target, tgt_padding_mask)

    def make_padding_mask(self, target):
        return make_padding_mask(target, self.vocab)

    def get_segment_features(self, features, denormalized_segments, idx, video_durations):
        return self.crop_segments(features, denormalized_segments, idx[0], video_durations)

    def crop_segments(self, features, denormalized_segments, segment_batch_id, video_durations):
        from ...utils.preds_postprocess import crop_segments
        return crop_segments(features, denormalized_segments, segment_batch_id, video_durations,
                             self.num_feature_levels, self.video_rescale_len)
