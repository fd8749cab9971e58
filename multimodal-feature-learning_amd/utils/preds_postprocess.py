"""Post-decoder index math of the DVC wrappers, on the device:
``get_src_permutation_idx`` and ``denormalize_segments`` (reference utils/preds_postprocess.py:16-80)
and the memory crop of the wrappers' ``crop_segments``
(models/deformable/unimodal_deformable_dvc.py:457-493).

The reference runs these as Python loops over segments with one device->host read per element
(``min(max(tensor, 0), d)``, ``torch.tensor([...])``) and builds the crop on the host followed by
an upload (:476-493, ``.to(device)`` :237).  Here each is a handful of vectorised device ops with
the same float32 operation order, so the token boundaries are bit-identical."""
from math import floor

import torch

__all__ = ["get_src_permutation_idx", "denormalize_segments", "crop_segments", "crop_keep", "SegmentMemory",
           "level_token_ranges",
           "captions_to_string", "pre_process"]


def get_src_permutation_idx(indices):
    """(batch_idx, src_idx) of the matched predictions, ordered by target index within each clip
    (reference :16-29: ``src[argsort(tgt)]``)."""
    batch_idx = torch.cat([torch.full_like(src, i) for i, (src, _) in enumerate(indices)])
    src_idx = torch.cat([src[torch.sort(tgt)[1]].long() for (src, tgt) in indices])
    return batch_idx, src_idx


def _durations(video_durations, device):
    if isinstance(video_durations, torch.Tensor):
        return video_durations.to(device)
    return torch.stack([torch.as_tensor(d) for d in video_durations]).to(device)


def denormalize_segments(segments, video_durations, segment_batch_id):
    """(centre, length) in [0, 1] -> (start, end) seconds, clamped to [0, duration] and ordered
    (reference :54-80).  segments (n, 2) on any device; video_durations (B,) tensor or list of
    0-dim tensors; segment_batch_id (n,).  Returns float32 (n, 2) on ``segments``' device."""
    dev = segments.device
    segments = segments.detach()  # the reference rebuilds them with torch.tensor(...): no gradient (:70-78)
    d = _durations(video_durations, dev)[segment_batch_id.to(dev)]
    c, l = segments[:, 0], segments[:, 1]
    # the 16-bit (2c - l) / (2c + l) converted to the promoted dtype explicitly (exact: the values the
    # mixed-dtype multiply promotes to), so the multiply is a same-dtype kernel — ROCm's mixed-dtype
    # elementwise path took ~40 us a call here for a few dozen elements
    pt = torch.promote_types(c.dtype, d.dtype)
    start = torch.minimum(torch.clamp(d / 2 * (2 * c - l).to(pt), min=0), d)
    end = torch.clamp(torch.minimum(d / 2 * (2 * c + l).to(pt), d), min=0)
    seg = torch.stack([start, end], 1).float()
    swap = ~(seg[:, 0] < seg[:, 1])
    return torch.where(swap[:, None], seg.flip(1), seg)


def level_token_ranges(num_feature_levels, video_rescale_len):
    """[(lower, upper)) token range of each pyramid level in the flattened memory (reference
    crop_segments :481-484)."""
    out = []
    for n in range(num_feature_levels):
        lower = floor(video_rescale_len * ((2 ** n - 1) / 2 ** (n - 1)))
        upper = floor(video_rescale_len * ((2 ** (n + 1) - 1) / 2 ** n))
        out.append((lower, upper))
    return out


_RANGES = {}


def _range_tensors(num_feature_levels, video_rescale_len, dev):
    """level_token_ranges as device tensors (lower, upper - lower as float32; lower, upper - 1 as int64),
    made once per device (the first, eager step: nothing is copied from the host inside a captured
    graph)."""
    key = (num_feature_levels, video_rescale_len, str(dev))
    t = _RANGES.get(key)
    if t is None:
        rng = level_token_ranges(num_feature_levels, video_rescale_len)
        t = (torch.tensor([lo for lo, _ in rng], dtype=torch.float32, device=dev),
             torch.tensor([up - lo for lo, up in rng], dtype=torch.float32, device=dev),
             torch.tensor([lo for lo, _ in rng], dtype=torch.int64, device=dev),
             torch.tensor([up - 1 for _, up in rng], dtype=torch.int64, device=dev))
        _RANGES[key] = t
    return t


def crop_segments(features, denormalized_segments, segment_batch_id, video_durations, num_feature_levels,
                  video_rescale_len):
    """Memory rows of each matched segment: per level, tokens [start, end) with
    start / end = clamp(round(lower + diff * t / duration), lower, upper - 1) (reference :457-493);
    other rows 0 and masked.  -> (features (n, K, d), padding mask (n, K) bool, True = masked)."""
    bid = segment_batch_id.to(features.device)
    keep = crop_keep(denormalized_segments, bid, video_durations, features.shape[1], num_feature_levels,
                     video_rescale_len, features.device)
    if isinstance(features, SegmentMemory):
        return features.select(bid, keep), ~keep
    cropped = torch.where(keep[..., None], features[bid], features.new_zeros(()))
    return cropped, ~keep


def crop_keep(denormalized_segments, bid, video_durations, K, num_feature_levels, video_rescale_len, dev):
    """crop_segments' (n, K) bool mask of the tokens each segment keeps (any row count: the DVC wrapper
    computes every decoder level's segments at once)."""
    seg = denormalized_segments.to(dev, torch.float32)
    bid = bid.to(dev)
    dur = _durations(video_durations, dev)[bid]  # its own dtype: the reference promotes seg / dur the same way
    tok = torch.arange(K, device=dev)
    # every level's token range at once, (n, levels) bounds (the reference loops over the levels,
    # :481-490; ~12 small kernels a level and decoder level in a step): the same float32 / float64
    # arithmetic per element, the same rounding and clamps, the union of the ranges
    lower, diff, lo_i, hi_i = _range_tensors(num_feature_levels, video_rescale_len, dev)
    dcol = dur[:, None] if dur.dim() == 1 else dur
    s = torch.clamp((lower + (diff * seg[:, 0:1] / dcol)).round().long(), min=lo_i, max=hi_i)
    e = torch.clamp((lower + (diff * seg[:, 1:2] / dcol)).round().long(), min=lo_i, max=hi_i)
    return ((tok[None, None, :] >= s[:, :, None]) & (tok[None, None, :] < e[:, :, None])).any(1)


class SegmentMemory:
    """The cropped memory of the matched segments, (n, K, d), without materialising it: row s is
    ``source[index[s]]`` where ``keep[s]`` and 0 elsewhere (crop_segments).  A crop of a crop (the
    reference's level l > 0 crops level l-1's crop, unimodal_deformable_dvc.py:235) is again one:
    ``select`` composes the index and ANDs the keep masks, so every level's memory refers to the
    one (B, K, d) encoder memory.

    What it saves is the caption decoder's cross-attention projections (models/modules/attention.py
    CrossAttention): k_linear / v_linear of a cropped row are those of its source row where kept and
    the bias where zeroed (0 . W + b), so ``project`` runs each projection over the B clips' K rows
    ONCE per step — shared by every segment and every decoder level, since they all read the same
    caption decoder — and gathers per segment, instead of a GEMM over the n K rows of every level.
    The projected rows are the same values the materialised crop gives (each output row is its
    own product); ``materialize`` returns the crop itself."""

    def __init__(self, source, index, keep, cache=None):
        self.source, self.index, self.keep = source, index, keep
        self.cache = {} if cache is None else cache
        self.shape = (int(index.shape[0]),) + tuple(source.shape[1:])
        self.dtype, self.device = source.dtype, source.device

    @classmethod
    def of(cls, memory):
        """The uncropped memory (B, K, d) as the source of the crops."""
        B, K = memory.shape[0], memory.shape[1]
        return cls(memory, torch.arange(B, device=memory.device),
                   torch.ones(B, K, dtype=torch.bool, device=memory.device))

    @staticmethod
    def cat(memories):
        """The segments of several crops of one source, stacked (torch.cat along the segments)."""
        first = memories[0]
        if any(m.source is not first.source for m in memories):
            raise ValueError("SegmentMemory.cat: crops of different sources")
        return SegmentMemory(first.source, torch.cat([m.index for m in memories]),
                             torch.cat([m.keep for m in memories]), first.cache)

    def __getitem__(self, rows):
        if not isinstance(rows, torch.Tensor) or rows.dim() != 1:
            raise TypeError("SegmentMemory: only 1-D index tensors select segments")
        return SegmentMemory(self.source, self.index[rows], self.keep[rows], self.cache)

    def select(self, rows, keep):
        """Rows ``rows`` of this memory with everything outside ``keep`` (n, K) zeroed."""
        return SegmentMemory(self.source, self.index[rows], self.keep[rows] & keep, self.cache)

    def materialize(self):
        return torch.where(self.keep[..., None], self.source[self.index], self.source.new_zeros(()))

    def projected(self, linear):
        """(``linear(source)`` — computed once per step and cached —, the bias a zeroed row projects
        to, or None): what a kernel reading the crop in place needs (models/modules/seg_attention.py)."""
        P = self.cache.get(linear)
        if P is None:
            P = linear(self.source)
            self.cache[linear] = P
        return P, (linear.bias.to(P.dtype) if linear.bias is not None else None)

    def project_group(self, linears):
        """Project the source by every Linear of ``linears`` not cached yet, all at once (one batched
        GEMM each way, value_proj.linear_group: the caption decoder's cross-attention key / value
        projections of all its layers), and cache them for ``projected``."""
        from ..models.modules.value_proj import linear_group, linear_group_supported
        todo = [lin for lin in linears if lin not in self.cache]
        if not linear_group_supported(todo, self.source):
            return
        from .. import _trace
        _trace.hit("memory_projection_group")
        for lin, p in zip(todo, linear_group(todo, self.source)):
            self.cache[lin] = p

    def project(self, linear):
        """``linear(self.materialize())`` from one projection of the source per step."""
        P, bias = self.projected(linear)
        if bias is None:
            bias = P.new_zeros(P.shape[-1])
        return _GatherKeep.apply(P, bias, self.index, self.keep)


class _GatherKeep(torch.autograd.Function):
    """``where(keep[..., None], P[index], bias)``.  The backward sums each source row's gradient
    over the segments that read it, and the bias's over the positions that read it, in fp32 and
    rounds once — autograd's index_select backward would accumulate 16-bit P's gradient in 16 bits
    (segments of one clip adding into the same rows)."""

    @staticmethod
    def forward(ctx, P, bias, index, keep):
        ctx.save_for_backward(index, keep)
        ctx.p_shape, ctx.dtypes = P.shape, (P.dtype, bias.dtype)
        return torch.where(keep[..., None], P.index_select(0, index), bias)

    @staticmethod
    def backward(ctx, g):
        index, keep = ctx.saved_tensors
        B, K, d = ctx.p_shape
        if (g.is_cuda and g.dtype == torch.bfloat16 and ctx.dtypes[0] == torch.bfloat16 and d % 8 == 0 and d <= 512
                and all(ctx.needs_input_grad[:2])):
            # one HIP pass over g: each source row's sum over the segments that read it, and the
            # bias's partial sums per token (csrc/ffn_glue.hip, gather_keep_bwd_kernel)
            from .. import _native
            lib = _native.load_library()
            g = g.contiguous()
            gP = torch.empty(ctx.p_shape, dtype=torch.bfloat16, device=g.device)
            part = torch.empty(K, d, dtype=torch.float32, device=g.device)
            rc = lib.mfl_gather_keep_backward(g.data_ptr(), index.contiguous().data_ptr(),
                                              keep.contiguous().data_ptr(), g.shape[0], B, K, d, gP.data_ptr(),
                                              part.data_ptr(), _native.stream_handle(g.device))
            if rc != 0:
                raise RuntimeError("mfl_gather_keep_backward failed: " + lib.mfl_relu_dropout_last_error().decode())
            return gP, part.sum(0).to(ctx.dtypes[1]), None, None
        k = keep[..., None]
        acc = torch.promote_types(g.dtype, torch.float32)  # fp32, or fp64 for fp64 memories
        g32 = g.to(acc)
        gP = gb = None
        if ctx.needs_input_grad[0]:
            gP = torch.zeros(ctx.p_shape, dtype=acc, device=g.device)
            gP.index_add_(0, index, torch.where(k, g32, 0.0))
            gP = gP.to(ctx.dtypes[0])
        if ctx.needs_input_grad[1]:
            gb = torch.where(k, 0.0, g32).sum((0, 1)).to(ctx.dtypes[1])
        return gP, gb, None, None


def captions_to_string(captions, vocab):
    """Token rows -> strings without <pad>/<bos>/<eos>/<unk> (reference :83-104)."""
    unwanted = {vocab['<pad>'], vocab['<bos>'], vocab['<eos>'], vocab['<unk>']}
    itos = vocab.get_itos()
    rows = captions.tolist() if isinstance(captions, torch.Tensor) else captions
    return pre_process([' '.join([itos[t] for t in row if t not in unwanted][1:-1]) for row in rows])


def pre_process(captions):
    """Drop punctuation tokens and immediate repeats (reference :138-152)."""
    for i, caption in enumerate(captions):
        tokens = caption.split()
        if len(tokens) == 0:
            captions[i] = ''
            continue
        res = [tokens[0]]
        for t in tokens[1:]:
            if t in ['.', ',', '/', "'"] or res[-1] == t:
                continue
            res.append(t)
        captions[i] = ' '.join(res)
    return captions
