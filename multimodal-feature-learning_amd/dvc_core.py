"""The measured workload: the proposal path of the reference's ``UnimodalDeformableDVC``
(models/deformable/unimodal_deformable_dvc.py:26-203) — sine position + duration embedding,
Conv1d pyramid (BaseEncoder), deformable encoder / decoder, and the per-decoder-level
class / segment / count heads — without the Hungarian matching and caption decoder
(host-side / out of scope; the reference wrapper crashes past the
heads at HEAD).

Submodule names follow the reference wrapper (``pos_embed``, ``base_encoder``,
``unimodal_deformable_transformer``, ``query_embedding``, ``class_embedding``,
``segment_embedding``, ``count_head``) so its state_dict keys map one to one.
"""
import math

import torch
from torch import nn

from .models.base_encoder import BaseEncoder
from .models.deformable.multimodal_deformable_transformer import MultimodalDeformableTransformer
from .models.deformable.unimodal_deformable_transformer import DeformableTransformer
from .models.sparse.unimodal_sparse_deformable_transformer import SparseDeformableTransformer
from .models.modules.embedding_layers import FFN, PositionEmbeddingVideoSine
from .models.modules.misc_modules import inverse_sigmoid, level_heads, predict_event_num, predict_event_num_with_depth
from .models.unimodal_caption_decoder import word_probs
from .utils.dam import attn_map_to_flat_grid
from .models.modules.linear import Linear

__all__ = ["DeformableDVCCore", "MultimodalDVCCore", "SparseDVCCore", "synthetic_clips", "workload_loss",
           "multimodal_workload_loss", "sparse_workload_loss", "StagedDVCLoss", "level_terms"]


class DeformableDVCCore(nn.Module):
    def __init__(self, d_model=512, num_queries=100, num_classes=200, max_eseq_length=10, feature_dim=512,
                 num_heads=8, num_feature_levels=4, enc_layers=6, dec_layers=6, ff_dim=2048, dropout=0.1,
                 enc_n_points=4, dec_n_points=4):
        super().__init__()
        self.num_queries = num_queries
        self.query_embedding = nn.Embedding(num_queries, d_model * 2)
        class_embedding = Linear(d_model, num_classes + 1)
        segment_embedding = FFN(in_dim=d_model, hidden_dim=d_model, out_dim=2, num_layers=3)
        count_head = Linear(d_model, max_eseq_length + 1)
        self.pos_embed = PositionEmbeddingVideoSine(d_model // 2, normalize=True)
        self.base_encoder = BaseEncoder(num_feature_levels, feature_dim, d_model)
        # head init of unimodal_deformable_dvc.py:59-71
        prior_prob = 0.01
        class_embedding.bias.data = torch.ones(num_classes + 1) * -math.log((1 - prior_prob) / prior_prob)
        nn.init.constant_(segment_embedding.layers[-1].weight.data, 0)
        nn.init.constant_(segment_embedding.layers[-1].bias.data, 0)
        self.unimodal_deformable_transformer = DeformableTransformer(
            d_model=d_model, num_head=num_heads, num_encoder_layers=enc_layers, num_decoder_layers=dec_layers,
            dim_feedforward=ff_dim, dropout=dropout, activation="relu", return_intermediate_dec=True,
            num_feature_levels=num_feature_levels, dec_n_points=dec_n_points, enc_n_points=enc_n_points)
        nn.init.constant_(segment_embedding.layers[-1].bias.data[2:], -2.0)
        # heads shared across decoder levels, as the reference does (:72-74)
        self.class_embedding = nn.ModuleList([class_embedding for _ in range(dec_layers)])
        self.count_head = nn.ModuleList([count_head for _ in range(dec_layers)])
        self.segment_embedding = nn.ModuleList([segment_embedding for _ in range(dec_layers)])

    def forward(self, video, video_mask, durations):
        """video (B, T, feature_dim), video_mask (B, T) bool True = pad, durations (B,)
        -> dict with pred_logits / pred_segments / pred_count (last level), the stacked
        per-level head outputs, hs (dec_layers, B, Q, d) and memory (B, S, d)."""
        tr = self.unimodal_deformable_transformer
        B = video.shape[0]
        srcs, masks, pos = self.base_encoder(video, video_mask, durations, self.pos_embed)
        src_flatten, shapes, starts, valid, lvl_pos, mask_flatten = tr.prepare_encoder_inputs(srcs, masks, pos)
        memory = tr.forward_encoder(src_flatten, shapes, starts, valid, lvl_pos, mask_flatten)
        qw = self.query_embedding.weight
        query_mask = torch.ones(B, qw.shape[0], dtype=torch.bool, device=qw.device)
        _, tgt, refp, qpos = tr.prepare_decoder_input_query(B, qw)
        hs, inter = tr.forward_decoder(tgt, refp, memory, shapes, starts, valid, qpos, mask_flatten, query_mask,
                                       False)
        cls, seg, cnt = _level_heads(self, hs)
        return {"pred_logits": cls[-1], "pred_segments": seg[-1], "pred_count": cnt[-1],
                "all_logits": cls, "all_segments": seg, "all_counts": cnt,
                "hs": hs, "inter_references": inter, "memory": memory}


_level_heads = level_heads  # (models/modules/misc_modules.py)


def synthetic_clips(batch, T=1024, feature_dim=512, padded=False, seed=0, device="cpu", dtype=torch.float32):
    """ActivityNet-shaped synthetic inputs (BASELINE.md / SURVEY §8(d)): features ~ N(0,1)
    (seed), masks all valid or valid length U[T/2, T] (seed+1), durations U(30, 240) s (seed+2)."""
    g = torch.Generator().manual_seed(seed)
    video = torch.randn((batch, T, feature_dim), generator=g).to(dtype)
    mask = torch.zeros(batch, T, dtype=torch.bool)
    if padded:
        gm = torch.Generator().manual_seed(seed + 1)
        for b in range(batch):
            valid = int(torch.randint(T // 2, T + 1, (1,), generator=gm))
            mask[b, valid:] = True
    gd = torch.Generator().manual_seed(seed + 2)
    durations = torch.rand(batch, generator=gd, dtype=torch.float64) * 210.0 + 30.0
    return video.to(device), mask.to(device), durations.to(device)


def workload_loss(out):
    """hs.sum() + memory.sum() (isolates the path from matcher / criterion)
    plus the heads' outputs, so every head and decoder level carries gradient."""
    return (out["hs"].float().sum() + out["memory"].float().sum() + out["all_segments"].float().sum()
            + out["all_counts"].float().sum() + (out["all_logits"].float() * 1e-2).square().sum())


class MultimodalDVCCore(nn.Module):
    """Config 3: the proposal path of the reference's ``MultimodalDeformableDVC``
    (models/deformable/multimodal_deformable_dvc.py:112-230) — one BaseEncoder shared by the video
    and audio streams (:155-156), the multimodal deformable encoder (4 MSDA calls per layer:
    video->video, audio->audio and both cross-modal directions) and decoder (2 MSDA
    cross-attentions per layer + the fusion bridge), and the shared per-level heads.  Audio
    features are 512-d (the shared base encoder needs it; a 128-d VGGish input would need a
    projection the reference lacks)."""

    def __init__(self, d_model=512, num_queries=100, num_classes=200, max_eseq_length=10, feature_dim=512,
                 num_heads=8, num_feature_levels=4, enc_layers=6, dec_layers=6, ff_dim=2048, dropout=0.1,
                 enc_n_points=4, dec_n_points=4):
        super().__init__()
        self.query_embedding = nn.Embedding(num_queries, d_model * 2)
        class_embedding = Linear(d_model, num_classes + 1)
        segment_embedding = FFN(in_dim=d_model, hidden_dim=d_model, out_dim=2, num_layers=3)
        count_head = Linear(d_model, max_eseq_length + 1)
        self.pos_embed = PositionEmbeddingVideoSine(d_model // 2, normalize=True)
        self.base_encoder = BaseEncoder(num_feature_levels, feature_dim, d_model)
        prior_prob = 0.01
        class_embedding.bias.data = torch.ones(num_classes + 1) * -math.log((1 - prior_prob) / prior_prob)
        nn.init.constant_(segment_embedding.layers[-1].weight.data, 0)
        nn.init.constant_(segment_embedding.layers[-1].bias.data, 0)
        self.multimodal_deformable_transformer = MultimodalDeformableTransformer(
            d_model=d_model, num_head=num_heads, num_encoder_layers=enc_layers, num_decoder_layers=dec_layers,
            dim_feedforward=ff_dim, dropout=dropout, activation="relu", return_intermediate_dec=True,
            num_feature_levels=num_feature_levels, dec_n_points=dec_n_points, enc_n_points=enc_n_points)
        nn.init.constant_(segment_embedding.layers[-1].bias.data[2:], -2.0)
        self.class_embedding = nn.ModuleList([class_embedding for _ in range(dec_layers)])
        self.count_head = nn.ModuleList([count_head for _ in range(dec_layers)])
        self.segment_embedding = nn.ModuleList([segment_embedding for _ in range(dec_layers)])

    def forward(self, video, video_mask, audio, audio_mask, durations):
        tr = self.multimodal_deformable_transformer
        B = video.shape[0]
        v_srcs, v_masks, v_pos = self.base_encoder(video, video_mask, durations, self.pos_embed)
        a_srcs, a_masks, a_pos = self.base_encoder(audio, audio_mask, durations, self.pos_embed)
        v = tr.prepare_encoder_inputs(v_srcs, v_masks, v_pos)
        a = tr.prepare_encoder_inputs(a_srcs, a_masks, a_pos)
        mem_v, mem_a = tr.forward_encoder(*v, *a)
        qw = self.query_embedding.weight
        query_mask = torch.ones(B, qw.shape[0], dtype=torch.bool, device=qw.device)
        _, tgt, refp, qpos = tr.prepare_decoder_input_query(B, qw)
        hs, inter = tr.forward_decoder(tgt, refp, qpos, query_mask, mem_v, v[1], v[2], v[3], v[5], mem_a, a[1], a[2],
                                       a[3], a[5], False)
        cls, seg, cnt = _level_heads(self, hs)
        return {"all_logits": cls, "all_segments": seg, "all_counts": cnt, "hs": hs, "memory_video": mem_v,
                "memory_audio": mem_a}


def multimodal_workload_loss(out):
    return (out["hs"].float().sum() + out["memory_video"].float().sum() + out["memory_audio"].float().sum()
            + out["all_segments"].float().sum() + out["all_counts"].float().sum()
            + (out["all_logits"].float() * 1e-2).square().sum())


class SparseDVCCore(nn.Module):
    """The proposal path of the reference's ``UnimodalSparseDVC``
    (models/sparse/unimodal_sparse_dvc.py:111-230): BaseEncoder, Sparse-DETR transformer
    (rho = 0.3: only the top 30 % encoder tokens are refined, over the full pyramid), decoder with
    reference-point-relative segments and the count head.  The output also carries what the
    criterion's mask-prediction loss needs (models/criterion.py:246-280)."""

    def __init__(self, d_model=512, num_queries=100, max_eseq_length=10, feature_dim=512, num_heads=8,
                 num_feature_levels=4, enc_layers=6, dec_layers=6, ff_dim=2048, dropout=0.1, enc_n_points=4,
                 dec_n_points=4, rho=0.3):
        super().__init__()
        self.query_embedding = nn.Embedding(num_queries, d_model * 2)
        self.segment_embedding_decoder = FFN(in_dim=d_model, hidden_dim=d_model, out_dim=2, num_layers=3)
        self.count_head_decoder = Linear(d_model, max_eseq_length + 1)
        self.pos_embed = PositionEmbeddingVideoSine(d_model // 2, normalize=True)
        self.base_encoder = BaseEncoder(num_feature_levels, feature_dim, d_model)
        nn.init.constant_(self.segment_embedding_decoder.layers[-1].weight.data, 0.)
        nn.init.constant_(self.segment_embedding_decoder.layers[-1].bias.data[:2], 0.)
        nn.init.constant_(self.segment_embedding_decoder.layers[-1].bias.data[2:], -2.0)
        self.unimodal_sparse_transformer = SparseDeformableTransformer(
            d_model=d_model, num_head=num_heads, num_encoder_layers=enc_layers, num_decoder_layers=dec_layers,
            dim_feedforward=ff_dim, dropout=dropout, activation="relu", return_intermediate_dec=True,
            num_feature_levels=num_feature_levels, dec_n_points=dec_n_points, enc_n_points=enc_n_points, rho=rho)
        # top-k widths from the shapes, not from a device read: the step is graph-capturable
        self.unimodal_sparse_transformer.static_topk = True

    def forward(self, video, video_mask, durations):
        tr = self.unimodal_sparse_transformer
        B = video.shape[0]
        srcs, masks, pos = self.base_encoder(video, video_mask, durations, self.pos_embed)
        (src_flatten, shapes, starts, valid, lvl_pos, mask_flatten, proposals, topk, mask_pred,
         sparse_token_nums) = tr.prepare_encoder_inputs(srcs, masks, pos)
        memory, sl_enc, aw_enc, _, _ = tr.forward_encoder(src_flatten, shapes, starts, valid, lvl_pos, mask_flatten,
                                                          proposals, topk, sparse_token_nums)
        qw = self.query_embedding.weight
        query_mask = torch.ones(B, qw.shape[0], dtype=torch.bool, device=qw.device)
        init_ref, tgt, refp, qpos = tr.prepare_decoder_input_query(B, qw)
        hs, inter, sl_dec, aw_dec = tr.forward_decoder(tgt, refp, memory, shapes, starts, valid, qpos, mask_flatten,
                                                       query_mask, False)
        segments = self.segment_embedding_decoder(hs)
        counts = predict_event_num_with_depth(self.count_head_decoder, hs)
        reference = torch.cat([init_ref[None], inter[:-1]], 0)  # reference :194-196
        # (depth, B, Q, 1) broadcast over both segment terms, as ``outputs_segment[..., :2] += reference`` (:203)
        segments = (segments + inverse_sigmoid(reference)).sigmoid()
        return {"all_segments": segments, "all_counts": counts, "hs": hs, "memory": memory,
                "sparse_topk": topk.shape[1] if topk is not None else None,
                "backbone_mask_prediction": mask_pred, "sparse_token_nums": sparse_token_nums,
                "sampling_locations_dec": sl_dec, "attn_weights_dec": aw_dec, "temporal_shapes": shapes,
                "level_start_index": starts, "mask_flatten": mask_flatten}


def sparse_workload_loss(out):
    """hs / memory / heads as workload_loss, plus the criterion's mask-prediction loss
    (models/criterion.py:246-280): the decoder attention map (DAM kernel) summed over layers and
    heads, its top sparse_token_nums tokens as the target of the mask predictor."""
    dam = attn_map_to_flat_grid(out["temporal_shapes"], out["level_start_index"],
                                out["sampling_locations_dec"].detach(), out["attn_weights_dec"].detach()).sum(dim=(1, 2))
    dam = torch.where(out["mask_flatten"], dam.min() - 1, dam)  # masked_fill with a tensor value syncs
    nums = out["sparse_token_nums"]
    k = out.get("sparse_topk") or int(nums.max())  # the encoder's static width: no host read
    topk = torch.topk(dam, k)[1]
    keep = torch.arange(topk.shape[1], device=topk.device)[None, :] < nums[:, None]
    pred = out["backbone_mask_prediction"]
    target = torch.zeros_like(pred).scatter_(1, topk, keep.to(pred.dtype))
    mask_loss = torch.nn.functional.multilabel_soft_margin_loss(pred.float(), target.float())
    return (out["hs"].float().sum() + out["memory"].float().sum() + out["all_segments"].float().sum()
            + out["all_counts"].float().sum() + mask_loss)


# --- the full DVC training step (proposals + matching + crop + caption decoder) -------------------

DVC_SPECIALS = ['<unk>', '<pad>', '<bos>', '<eos>']


def dvc_vocab(size=10000):
    """A vocabulary of ``size`` tokens with the reference's special tokens first (pad 1, bos 2, eos 3;
    dataset/anet_video.py builds it from the captions, ~10k words on ActivityNet)."""
    return {w: i for i, w in enumerate(DVC_SPECIALS + [f"w{i}" for i in range(size - len(DVC_SPECIALS))])}


def build_dvc(d_model=512, num_queries=100, num_classes=200, T=1024, enc_layers=6, dec_layers=6, caption_depth=6,
              dropout=0.1, vocab_size=10000, seq_len=20, ff_dim=2048, num_heads=8):
    """UnimodalDeformableDVC at the reference's training configuration (config/config_dvc_train.py:
    dvc d_model 512, detr 6 + 6 layers / 8 heads / 4 levels / 4 points / ff 2048 / dropout 0.1,
    caption decoder depth 6 / 8 heads / mlp 4 / dropout 0.1 / post-norm, matcher costs 1 / 5 / 2,
    max_eseq_length 10, threshold 0.5) with BASELINE's 100 queries and T = video_rescale_len; the
    differentiable context mask on (the only setting in which the reference wrapper runs)."""
    from types import SimpleNamespace as ns
    from .models.deformable.unimodal_deformable_dvc import UnimodalDeformableDVC
    from .models.matcher import HungarianMatcher
    detr = ns(feature_dim=d_model, d_model=d_model, num_heads=num_heads, num_feature_levels=4, dec_n_points=4,
              enc_n_points=4, enc_layers=enc_layers, dec_layers=dec_layers, transformer_dropout_prob=dropout,
              transformer_ff_dim=ff_dim, video_rescale_len=T, return_intermediate=True, hidden_dropout_prob=dropout,
              layer_norm_eps=1e-12)
    caption = ns(d_model=d_model, depth=caption_depth, num_heads=num_heads, mlp_ratio=4, qkv_bias=True,
                 positional_embedding_dropout=dropout, attention_dropout=dropout, projection_dropout=dropout,
                 bridge_dropout=dropout, mlp_dropout_1=dropout, mlp_dropout_2=dropout, pre_norm=False,
                 model_official=None, weight_init=True, weight_load=False, emb_weights_req_grad=True,
                 return_intermediate=True)
    matcher = HungarianMatcher(cost_class=1, cost_segment=5, cost_giou=2, cost_alpha=0.25, cost_gamma=2.0)
    return UnimodalDeformableDVC(['video'], num_queries, d_model, num_classes, True, matcher, 0.5, 10,
                                 dvc_vocab(vocab_size), seq_len, None, detr, caption, use_differentiable_mask=True)


def synthetic_dvc_batch(batch, T=1024, feature_dim=512, vocab_size=10000, seq_len=20, seed=0, device="cpu",
                        events=(3, 4, 2, 5, 3, 4, 3, 4)):
    """engine.py-shaped ``obj`` (dataset/anet_video.py:262-384 collate keys): features ~ N(0,1),
    all frames valid, durations U(30, 240) s, ``events[b]`` target segments per clip (ActivityNet
    averages ~3.7) with random centres / lengths and captions of 8-19 random words."""
    video, mask, dur = synthetic_clips(batch, T=T, feature_dim=feature_dim, seed=seed)
    g = torch.Generator().manual_seed(seed + 7)
    targets, rows = [], []
    for b in range(batch):
        n = events[b % len(events)]
        c = torch.rand(n, generator=g) * 0.6 + 0.2
        ln = torch.rand(n, generator=g) * 0.3 + 0.05
        targets.append({'segments': torch.stack([c, ln], 1).to(device), 'labels': torch.zeros(n, dtype=torch.long,
                                                                                             device=device)})
        for _ in range(n):
            k = int(torch.randint(8, seq_len, (1,), generator=g))
            rows.append(torch.cat([torch.tensor([2]), torch.randint(4, vocab_size, (k - 2,), generator=g),
                                   torch.tensor([3]), torch.ones(seq_len - k, dtype=torch.long)]))
    cap = torch.stack(rows)
    length = torch.stack([torch.tensor([float(T), float(dur[b]), float(len(targets[b]['segments']))])
                          for b in range(batch)])
    return {'video_tensor': video.to(device), 'video_mask': mask.to(device), 'video_length': length.to(device),
            'video_target': targets, 'cap_tensor': cap.to(device), 'cap_mask': (cap == 1).to(device)}


def level_terms(levels, lidx, tgt_seg, n_events, words, live, live_sum):
    """The per-level terms of ``dvc_workload_loss`` summed over every decoder level at once: the heads
    stacked over the levels (``levels['segments' / 'logits' / 'counts']``, (L, B, Q, .), as
    misc_modules.level_heads makes them) and the levels' caption probabilities stacked along the
    segments (``levels['captions']``, (L n, W, V), the one caption decoder call), with ``lidx`` (L, 2, n)
    the (clip, prediction) pairs matched at each level.  Per level the same terms as the loop — L1 of the
    matched segments (x5), -log p(label) (x1), the count head's cross-entropy (x2), the captions' -log
    p(word) over non-pad words — each gather / reduction one launch for all levels instead of one per
    level (the loss had ~50 launches a level each way at the DVC bench shape)."""
    import torch.nn.functional as F
    L, n = lidx.shape[0], lidx.shape[2]
    lv = torch.arange(L, device=lidx.device)[:, None].expand(L, n)
    b, s = lidx[:, 0], lidx[:, 1]
    total = 5 * (levels['segments'][lv, b, s].float() - tgt_seg).abs().mean(dim=(1, 2)).sum()
    total = total - torch.log(levels['logits'][lv, b, s, 0].float().clamp_min(1e-9)).mean(dim=1).sum()
    counts = levels['counts']
    C = counts.shape[-1]
    ce = F.cross_entropy(counts.float().reshape(-1, C), n_events.clamp_max(C - 1).repeat(L), reduction='none')
    total = total + 2 * ce.view(L, -1).mean(dim=1).sum()
    caps = levels.get('captions')
    if caps is not None:
        p = word_probs(caps, words.repeat(L, 1))
        total = total - (torch.log(p.clamp_min(1e-9)) * live.repeat(L, 1)).view(L, -1).sum(dim=1).div(live_sum).sum()
    return total


def _stacked_levels(out):
    """``out['_levels']`` when it covers every level the loss reads (the aux levels present), else None."""
    lv = out.get('_levels')
    if lv is None or len(out.get('aux_outputs', [])) + 1 != lv['segments'].shape[0]:
        return None
    return lv


def dvc_workload_loss(result, obj):
    """A loss over every output of UnimodalDeformableDVC's training forward, shaped like the
    reference criterion's terms (models/criterion.py, coefficients of config_dvc_train.py): L1 of
    the matched segments (x5), -log p(label) of the matched predictions (x1), the count head's
    cross-entropy (x2), the captions' -log p(word) over non-pad words (x1), the context mask's
    BCE against the crop (x3) — on the last decoder level and every aux level."""
    import torch.nn.functional as F
    from .utils.preds_postprocess import get_src_permutation_idx
    out, _, indices, indices_aux, _ = result
    dev = out['pred_segments'].device
    tgt_seg = torch.cat([t['segments'] for t in obj['video_target']]).float()
    words = obj['cap_tensor'][:, 1:]
    live = (~obj['cap_mask'][:, 1:]).float()
    n_events = torch.tensor([len(t['segments']) for t in obj['video_target']], device=dev)
    total = 0.0
    stacked = _stacked_levels(out)
    if stacked is not None:
        # every level at once (level_terms): level l's pairs, the last level's being ``indices``
        lidx = torch.stack([torch.stack([t.to(dev) for t in get_src_permutation_idx(ind)])
                            for ind in list(indices_aux) + [indices]])
        total = level_terms(stacked, lidx, tgt_seg, n_events, words, live, live.sum())
        if 'pred_memory_mask' in out:
            total = total + 3 * F.binary_cross_entropy_with_logits(out['pred_memory_mask'].float(),
                                                                  (out['pred_memory_mask'].detach() > 0).float())
        return total
    levels = [(out, indices)] + list(zip(out.get('aux_outputs', []), indices_aux))
    for o, ind in levels:
        bidx, sidx = (t.to(dev) for t in get_src_permutation_idx(ind))
        total = total + 5 * (o['pred_segments'][bidx, sidx].float() - tgt_seg).abs().mean()
        total = total - torch.log(o['pred_logits'][bidx, sidx, 0].float().clamp_min(1e-9)).mean()
        total = total + 2 * F.cross_entropy(o['pred_count'].float(), n_events.clamp_max(o['pred_count'].shape[-1] - 1))
        if o.get('pred_captions') is not None:
            p = word_probs(o['pred_captions'], words)
            total = total - (torch.log(p.clamp_min(1e-9)) * live).sum() / live.sum()
    if 'pred_memory_mask' in out:
        # the crop's kept tokens as the context target (criterion.py loss_contexts)
        total = total + 3 * F.binary_cross_entropy_with_logits(out['pred_memory_mask'].float(),
                                                              (out['pred_memory_mask'].detach() > 0).float())
    return total


class StagedDVCLoss:
    """``dvc_workload_loss`` over ``UnimodalDeformableDVC``'s training forward, split around its
    host step (the Hungarian assignment, reference engine.py:62 -> models/matcher.py:86) so that
    ``FlatGradTrainer`` captures the step as two HIP graphs (train_step.py, staged losses):

    * ``stage_a``: the proposals and every decoder level's matching costs (device);
    * ``host``: scipy's assignment of the copied costs and the matched (batch, prediction) index
      pairs of each level, written into pinned buffers; ``upload`` copies them (stream-ordered)
      into static device buffers;
    * ``stage_b``: the crop, context mask and caption decoder of every level from those buffers,
      and the loss — with the batch's targets kept as device constants, so nothing in it reads
      the host.

    The number of matches is the batch's number of target segments (one per target), so every
    shape is fixed by the batch: a replay only changes which predictions are matched."""

    def __init__(self, obj, model):
        dev = obj['video_tensor'].device
        num_levels = len(model.class_embedding)
        self._matcher = model.matcher
        self.obj = obj
        tgts = obj['video_target']
        self.tgt_seg = torch.cat([t['segments'] for t in tgts]).float()
        self.words = obj['cap_tensor'][:, 1:]
        self.live = (~obj['cap_mask'][:, 1:]).float()
        self.live_sum = self.live.sum()
        self.n_events = torch.tensor([len(t['segments']) for t in tgts], device=dev)
        n = int(self.tgt_seg.shape[0])
        self.idx_host = torch.empty((num_levels, 2, n), dtype=torch.int64)
        if dev.type == "cuda":
            self.idx_host = self.idx_host.pin_memory()
        self.idx_dev = torch.zeros((num_levels, 2, n), dtype=torch.int64, device=dev)
        self.level_indices = None

    # --- the staged-loss protocol of FlatGradTrainer ---------------------------------------
    def stage_a(self, model, batch):
        return model.forward_stage_proposals(batch[0])

    @staticmethod
    def request(state):
        return state['costs']

    def host(self, state, cpu):
        """get_src_permutation_idx (utils/preds_postprocess.py) of every level, written with numpy
        into the pinned buffer: (clip, prediction) pairs ordered by target within each clip."""
        import numpy as np
        ih = self.idx_host.numpy()
        m = self._matcher
        if "solve_levels" not in vars(m):
            # the matching and the index lists in one native call where it applies (solve_levels_into)
            self.level_indices = type(m).solve_levels_into(cpu, state['cost_meta'], ih)
            return
        # (an instance's own solve_levels: a test pinning the assignment)
        self.level_indices = m.solve_levels(cpu, state['cost_meta'])
        for lvl, ind in enumerate(self.level_indices):
            off = 0
            for b, (src, tgt) in enumerate(ind):
                s, t = src.numpy(), tgt.numpy()
                k = len(s)
                ih[lvl, 0, off:off + k] = b
                ih[lvl, 1, off:off + k] = s[np.argsort(t, kind="stable")]
                off += k

    def upload(self):
        self.idx_dev.copy_(self.idx_host, non_blocking=True)

    def stage_b(self, model, batch, state):
        levels = [(self.idx_dev[l, 0], self.idx_dev[l, 1]) for l in range(self.idx_dev.shape[0])]
        result = model.forward_stage_captions(batch[0], state, self.level_indices, levels, is_training=True)
        return self.loss(result, levels)

    def loss(self, result, levels):
        """``dvc_workload_loss`` with the matched indices from ``levels`` (device) and the targets
        as device constants: the same terms in the same order."""
        import torch.nn.functional as F
        out = result[0]
        total = 0.0
        stacked = _stacked_levels(out)
        if stacked is not None:
            total = level_terms(stacked, self.idx_dev, self.tgt_seg, self.n_events, self.words, self.live,
                                self.live_sum)
            if 'pred_memory_mask' in out:
                total = total + 3 * F.binary_cross_entropy_with_logits(out['pred_memory_mask'].float(),
                                                                      (out['pred_memory_mask'].detach() > 0).float())
            return total
        outs = [out] + list(out.get('aux_outputs', []))
        lv = [levels[-1]] + levels[:len(outs) - 1]
        for o, (bidx, sidx) in zip(outs, lv):
            total = total + 5 * (o['pred_segments'][bidx, sidx].float() - self.tgt_seg).abs().mean()
            total = total - torch.log(o['pred_logits'][bidx, sidx, 0].float().clamp_min(1e-9)).mean()
            total = total + 2 * F.cross_entropy(o['pred_count'].float(),
                                                self.n_events.clamp_max(o['pred_count'].shape[-1] - 1))
            if o.get('pred_captions') is not None:
                p = word_probs(o['pred_captions'], self.words)
                total = total - (torch.log(p.clamp_min(1e-9)) * self.live).sum() / self.live_sum
        if 'pred_memory_mask' in out:
            total = total + 3 * F.binary_cross_entropy_with_logits(out['pred_memory_mask'].float(),
                                                                  (out['pred_memory_mask'].detach() > 0).float())
        return total
