"""Pieces the DVC wrappers share (reference models/deformable/*_dvc.py, models/sparse/*_dvc.py):
caption masks, the matched-segment memory crop, the differentiable context mask and the
caption end tokens.  All device-side; the only host round trip of a training step is the
matcher's single cost-matrix copy (models/matcher.py)."""
import torch

from ..utils.preds_postprocess import crop_segments, denormalize_segments, get_src_permutation_idx

__all__ = ["special_tokens", "make_tgt_mask", "look_ahead_mask", "make_padding_mask", "segment_memory",
           "context_mask", "append_end_token"]


def special_tokens(vocab):
    return vocab['<bos>'], vocab['<eos>'], vocab['<pad>']


def look_ahead_mask(seq_len, device):
    """(L, L) bool, True above the diagonal (reference unimodal_sparse_dvc.py:410-426)."""
    return torch.ones(seq_len, seq_len, dtype=torch.bool, device=device).triu(1)


def make_tgt_mask(target, tgt_padding_mask):
    """(N, 1, L, L) = look-ahead | key padding (reference unimodal_deformable_dvc.py:384-403)."""
    L = target.shape[1]
    return tgt_padding_mask[:, None, None, :] | look_ahead_mask(L, tgt_padding_mask.device)


def make_padding_mask(target, vocab):
    """True where the token is <pad> (reference :419-431)."""
    return target == vocab['<pad>']


def segment_memory(memory, out_aux, indices, video_durations, num_feature_levels, rescale_len, idx_dev=None):
    """Matched segments of one decoder level -> (idx, idx on the device, denormalised (n, 2),
    cropped memory (n, K, d), key mask (n, K)) (reference unimodal_deformable_dvc.py:229-240,
    434-493).  ``idx_dev``: the level's (batch, prediction) index pair already on the device (a
    graph-captured step uploads it from the host matching; ``idx`` is then ``indices``)."""
    if idx_dev is not None:
        idx = indices
    else:
        idx = get_src_permutation_idx(indices)
        dev = out_aux['pred_segments'].device
        idx_dev = (idx[0].to(dev), idx[1].to(dev))
    denorm = denormalize_segments(out_aux['pred_segments'][idx_dev], video_durations, idx_dev[0])
    mem, key_mask = crop_segments(memory, denorm, idx_dev[0], video_durations, num_feature_levels, rescale_len)
    return idx, idx_dev, denorm, mem, key_mask


def context_mask(model, denorm, query_features_selected, key_mask):
    """Differentiable context mask (reference :243-260): the predicted logits (returned for the
    criterion) and the boolean mask the caption decoder reads (sigmoid > 0.5)."""
    x = torch.cat([denorm.to(query_features_selected.dtype), query_features_selected], 1)
    pred = model(x)
    # the reference blends ``seg_confidence * pred + (1 - seg_confidence) * key_mask`` with
    # seg_confidence = ones (:255-257): exactly pred (1 * p = p, (1 - 1) * m = 0, p + 0 = p) and a gradient
    # of exactly 1 — five launches each way per level that change nothing, so pred is used as it is
    return pred, pred.sigmoid() > 0.5


def append_end_token(captions, vocab, faster_eval):
    """(N, L) -> (N, L+1): <eos> always (faster_eval), else <pad> if the caption already holds <eos>
    and <eos> otherwise (reference :356-363)."""
    bos, eos, pad = special_tokens(vocab)
    if faster_eval:
        last = torch.full((captions.shape[0], 1), eos, dtype=torch.int32, device=captions.device)
    else:
        has = (captions == eos).any(1, keepdim=True)
        last = torch.where(has, torch.full_like(has, pad, dtype=torch.int32),
                           torch.full_like(has, eos, dtype=torch.int32))
    return torch.cat((captions, last), 1)
