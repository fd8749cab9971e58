"""The flattened level position embedding of ``prepare_encoder_inputs``.

Reference (models/deformable/unimodal_deformable_transformer.py:90-134, and the multimodal / sparse
transformers): ``lvl_pos_embed_flatten = torch.cat([pos_l.transpose(1, 2) + level_embed[l].view(1, 1, -1)
for l], 1)``.  ATen runs that as four transposed adds and a cat (one more pass over the (B, S, d)
result), and its backward sums ``level_embed``'s gradient with four ``sum_to_size`` reductions —
24-71 us each at the bench shape (keep-last-dim reductions over 1-8 K rows on 128 workgroups) —
plus a zero fill, copy and add per level: ~0.25 ms a step.  Here (bf16 training on the GPU and fp32
position embeddings) one HIP kernel writes the flattened sum (include/ffn_glue.h,
mfl_level_pos_flatten) and two write the level embedding's gradient (mfl_level_colsum); the
position embeddings' gradients are transposed views of the incoming gradient, as autograd's own.
"""
import ctypes

import torch
from torch.autograd import Function

__all__ = ["level_pos_flatten", "LevelPositions", "group_norm_cl", "flatten_levels"]


def _reference(pos_embeds, level_embed):
    return torch.cat([p.transpose(1, 2) + level_embed[lvl].view(1, 1, -1) for lvl, p in enumerate(pos_embeds)], 1)


class _LevelPosFlatten(Function):
    @staticmethod
    def forward(ctx, level_embed, *poses):
        from ... import _native, _trace
        _trace.hit("level_pos_flatten")
        lib = _native.load_library()
        L = len(poses)
        B, N = poses[0].shape[0], poses[0].shape[1]
        T = [p.shape[2] for p in poses]
        out = torch.empty(B, sum(T), N, dtype=torch.float32, device=level_embed.device)
        ptrs = (ctypes.c_void_p * L)(*[p.data_ptr() for p in poses])
        cl = (ctypes.c_int * L)(*[0 if p.is_contiguous() else 1 for p in poses])
        rc = lib.mfl_level_pos_flatten_ex(ptrs, cl, (ctypes.c_int64 * L)(*T), L, B, N, level_embed.data_ptr(),
                                          out.data_ptr(), _native.stream_handle(out.device))
        if rc != 0:
            raise RuntimeError("mfl_level_pos_flatten failed: " + lib.mfl_relu_dropout_last_error().decode())
        ctx.T, ctx.B, ctx.N = T, B, N
        ctx.level_embed = level_embed
        return out

    @staticmethod
    def backward(ctx, g):
        from ... import _native
        from .linear import _accum_target, _claim
        T, B, N = ctx.T, ctx.B, ctx.N
        L = len(T)
        nig = ctx.needs_input_grad
        g = g.contiguous()
        dlevel = None
        if nig[0]:
            lib = _native.load_library()
            t64 = (ctypes.c_int64 * L)(*T)
            ws = torch.empty(lib.mfl_level_colsum_workspace_bytes(t64, L, B, N), dtype=torch.uint8, device=g.device)
            # the trainer's flat gradient view: claimed, or (a second pyramid — the multimodal audio
            # stream shares level_embed) added into where the first call wrote
            acc = _accum_target(ctx.level_embed)
            out = acc if acc is not None else _claim(ctx.level_embed)
            if out is None:
                out = torch.empty(ctx.level_embed.shape, dtype=torch.float32, device=g.device)
            rc = lib.mfl_level_colsum(g.data_ptr(), t64, L, B, N, out.data_ptr(), 1 if acc is not None else 0,
                                      ws.data_ptr(), _native.stream_handle(g.device))
            dlevel = None if acc is not None else out
            if rc != 0:
                raise RuntimeError("mfl_level_colsum failed: " + lib.mfl_relu_dropout_last_error().decode())
        dposes, s = [], 0
        for lvl, t in enumerate(T):
            dposes.append(g[:, s:s + t].transpose(1, 2) if nig[1 + lvl] else None)
            s += t
        return (dlevel, *dposes)


def _supported(pos_embeds, level_embed):
    if not (level_embed.is_cuda and level_embed.dtype == torch.float32 and level_embed.is_contiguous()
            and torch.is_autocast_enabled("cuda") and torch.get_autocast_dtype("cuda") == torch.bfloat16):
        return False
    if not 1 <= len(pos_embeds) <= 16 or level_embed.dim() != 2 or level_embed.shape[0] != len(pos_embeds):
        return False
    B, N = pos_embeds[0].shape[0], pos_embeds[0].shape[1]
    if N % 4 or level_embed.shape[1] != N:
        return False
    # (B, N, T) contiguous, or the transposed view of contiguous (B, T, N) rows (the position
    # embedding's own layout)
    return all(p.is_cuda and p.device == level_embed.device and p.dtype == torch.float32 and p.dim() == 3
               and p.shape[0] == B and p.shape[1] == N and p.shape[2] > 0
               and (p.is_contiguous() or p.transpose(1, 2).is_contiguous()) for p in pos_embeds)


class LevelPositions(list):
    """The per-level position embeddings of a pyramid (BaseEncoder's ``poses``), computed when first
    read: ``pos_embed(NestedTensor(src_l, mask_l, duration))`` per level, as the reference does
    (base_encoder.py:62-89).  ``level_pos_flatten`` reads the masks and durations instead and writes the
    flattened embedding in one kernel (``_PyramidPos``) without ever building the per-level tensors."""

    def __init__(self, pos_embed, srcs, masks, duration, dtypes):
        super().__init__()
        self.pos_embed, self.srcs, self.masks, self.duration, self.dtypes = pos_embed, srcs, masks, duration, dtypes
        self._done = False

    def _materialise(self):
        if not self._done:
            from .misc_modules import NestedTensor
            super().extend(self.pos_embed(NestedTensor(s, m, self.duration)).to(dt)
                           for s, m, dt in zip(self.srcs, self.masks, self.dtypes))
            self._done = True

    def __getitem__(self, i):
        self._materialise()
        return super().__getitem__(i)

    def __iter__(self):
        self._materialise()
        return super().__iter__()

    def __len__(self):
        return len(self.masks)


class _PyramidPos(Function):
    """lvl_pos_embed_flatten of a pyramid from its masks and durations (mfl_pyramid_pos_flatten);
    gradients for level_embed (per-level column sums) and for the duration embedding (per-clip column
    sums of the duration half), the position embedding's only learned input."""

    @staticmethod
    def forward(ctx, level_embed, dur, masks, dim_t, npf, normalize, scale, eps):
        from ... import _native, _trace
        _trace.hit("pyramid_pos")
        lib = _native.load_library()
        L = len(masks)
        B = masks[0].shape[0]
        T = [m.shape[1] for m in masks]
        out = torch.empty(B, sum(T), 2 * npf, dtype=torch.float32, device=level_embed.device)
        ptrs = (ctypes.c_void_p * L)(*[m.data_ptr() for m in masks])
        rc = lib.mfl_pyramid_pos_flatten(ptrs, (ctypes.c_int64 * L)(*T), L, B, npf, dim_t.data_ptr(), dur.data_ptr(),
                                         level_embed.data_ptr(), 1 if normalize else 0, float(scale), float(eps),
                                         out.data_ptr(), _native.stream_handle(out.device))
        if rc != 0:
            raise RuntimeError("mfl_pyramid_pos_flatten failed: " + lib.mfl_relu_dropout_last_error().decode())
        ctx.T, ctx.B, ctx.npf = T, B, npf
        ctx.level_embed = level_embed
        return out

    @staticmethod
    def backward(ctx, g):
        from ... import _native
        from .linear import _accum_target, _claim
        T, B, npf = ctx.T, ctx.B, ctx.npf
        L, N = len(T), 2 * npf
        nig = ctx.needs_input_grad
        g = g.contiguous()
        lib = _native.load_library()

        def colsum(t_list, nb, out, accumulate):
            t64 = (ctypes.c_int64 * len(t_list))(*t_list)
            ws = torch.empty(lib.mfl_level_colsum_workspace_bytes(t64, len(t_list), nb, N), dtype=torch.uint8,
                             device=g.device)
            rc = lib.mfl_level_colsum(g.data_ptr(), t64, len(t_list), nb, N, out.data_ptr(), 1 if accumulate else 0,
                                      ws.data_ptr(), _native.stream_handle(g.device))
            if rc != 0:
                raise RuntimeError("mfl_level_colsum failed: " + lib.mfl_relu_dropout_last_error().decode())

        dlevel = ddur = None
        if nig[0]:
            acc = _accum_target(ctx.level_embed)  # (the multimodal audio pyramid shares level_embed)
            out = acc if acc is not None else _claim(ctx.level_embed)
            if out is None:
                out = torch.empty(ctx.level_embed.shape, dtype=torch.float32, device=g.device)
            colsum(T, B, out, acc is not None)
            dlevel = None if acc is not None else out
        if nig[1]:
            if B <= 16:  # per-clip column sums: the clips as the "levels" of one batch
                per_clip = torch.empty(B, N, dtype=torch.float32, device=g.device)
                colsum([sum(T)] * B, 1, per_clip, False)
                ddur = per_clip[:, npf:]
            else:
                ddur = g[..., npf:].sum(1)
        return dlevel, ddur, None, None, None, None, None, None


def _pyramid_supported(pos, level_embed):
    import os
    from .embedding_layers import PositionEmbeddingVideoSine
    if os.environ.get("MFL_PYRAMID_POS", "1") == "0":  # (A/B: the per-level embeddings + mfl_level_pos_flatten)
        return False
    mod = pos.pos_embed
    if not (type(mod) is PositionEmbeddingVideoSine and level_embed.is_cuda and level_embed.dtype == torch.float32
            and level_embed.is_contiguous() and level_embed.dim() == 2 and level_embed.shape[0] == len(pos.masks)
            and level_embed.shape[1] == 2 * mod.num_pos_feats and 1 <= len(pos.masks) <= 16
            and torch.is_autocast_enabled("cuda") and torch.get_autocast_dtype("cuda") == torch.bfloat16
            and pos.duration is not None and all(dt == torch.float32 for dt in pos.dtypes)):
        return False
    B = pos.masks[0].shape[0]
    return all(m.is_cuda and m.device == level_embed.device and m.dtype == torch.bool and m.dim() == 2
               and m.shape[0] == B and m.shape[1] > 0 and m.is_contiguous() for m in pos.masks)


def _pyramid_pos(pos, level_embed):
    mod = pos.pos_embed
    npf = mod.num_pos_feats
    dev = level_embed.device
    # dim_t exactly as the module computes it (embedding_layers.py: PositionEmbeddingVideoSine.forward)
    dim_t = torch.arange(npf, dtype=torch.float32, device=dev)
    dim_t = mod.temperature ** (2 * torch.div(dim_t, 2, rounding_mode='trunc') / npf)
    dur = mod.duration_embedding(pos.duration).float().contiguous()
    return _PyramidPos.apply(level_embed, dur, list(pos.masks), dim_t, npf, mod.normalize, mod.scale, 1e-6)


def level_pos_flatten(pos_embeds, level_embed):
    """``torch.cat([p.transpose(1, 2) + level_embed[l].view(1, 1, -1) for l, p in enumerate(pos_embeds)], 1)``
    (pos_embeds: (B, d, T_l) per level): the HIP kernels under bf16 autocast on the GPU, the reference
    composition elsewhere.  A ``LevelPositions`` is flattened from its masks and durations in one kernel
    (its per-level tensors are never built)."""
    if isinstance(pos_embeds, LevelPositions) and not pos_embeds._done and _pyramid_supported(pos_embeds,
                                                                                              level_embed):
        return _pyramid_pos(pos_embeds, level_embed)
    if not _supported(pos_embeds, level_embed):
        return _reference(pos_embeds, level_embed)
    return _LevelPosFlatten.apply(level_embed, *pos_embeds)


class _GroupNormCL(Function):
    """GroupNorm of channels-last bf16 rows x (B, T, C) (include/add_layernorm.h mfl_groupnorm_cl_*):
    the fp32 output is written into ``flat`` (B, S, C) at rows [start, start + T) and returned as that
    view; with ``want16`` also its bf16 copy (the next level's convolution input)."""

    @staticmethod
    def forward(ctx, x, weight, bias, groups, eps, flat, start, want16):
        from ... import _native, _trace
        _trace.hit("groupnorm_cl")
        lib = _native.load_library()
        B, T, C = x.shape
        out32 = flat[:, start:start + T]
        out16 = torch.empty(B, T, C, dtype=torch.bfloat16, device=x.device) if want16 else None
        mean = torch.empty(B, groups, dtype=torch.float32, device=x.device)
        rstd = torch.empty(B, groups, dtype=torch.float32, device=x.device)
        ws = torch.empty(lib.mfl_groupnorm_cl_workspace_bytes(B, T, C, groups), dtype=torch.uint8, device=x.device)
        rc = lib.mfl_groupnorm_cl_forward(x.data_ptr(), weight.data_ptr(), bias.data_ptr(), B, T, C, groups,
                                          float(eps), out32.data_ptr(), flat.stride(0),
                                          None if out16 is None else out16.data_ptr(), mean.data_ptr(),
                                          rstd.data_ptr(), ws.data_ptr(), _native.stream_handle(x.device))
        if rc != 0:
            raise RuntimeError("mfl_groupnorm_cl_forward failed: " + lib.mfl_add_layernorm_last_error().decode())
        ctx.save_for_backward(x, weight, mean, rstd)
        ctx.groups, ctx.params = groups, (weight, bias)
        ctx.set_materialize_grads(False)
        return out32, out16

    @staticmethod
    def backward(ctx, g32, g16):
        from ... import _native
        from .linear import _accum_target, _claim
        x, weight, mean, rstd = ctx.saved_tensors
        B, T, C = x.shape
        G = ctx.groups
        lib = _native.load_library()
        if g32 is not None and (g32.dtype != torch.float32 or g32.stride(2) != 1 or g32.stride(1) != C):
            g32 = g32.float().contiguous()
        if g16 is not None:
            g16 = g16.to(torch.bfloat16).contiguous()
        dx = torch.empty(B, T, C, dtype=torch.bfloat16, device=x.device)
        nig = ctx.needs_input_grad
        w, b = ctx.params
        accs = (_accum_target(w), _accum_target(b)) if nig[1] and nig[2] else (None, None)
        accumulate = accs[0] is not None and accs[1] is not None
        if accumulate:  # (the multimodal audio pyramid shares the BaseEncoder)
            dw, db = accs
        else:
            dw = (_claim(w) if nig[1] else None)
            db = (_claim(b) if nig[2] else None)
            dw = dw if dw is not None else torch.empty(C, dtype=torch.float32, device=x.device)
            db = db if db is not None else torch.empty(C, dtype=torch.float32, device=x.device)
        ws = torch.empty(lib.mfl_groupnorm_cl_workspace_bytes(B, T, C, G), dtype=torch.uint8, device=x.device)
        rc = lib.mfl_groupnorm_cl_backward(None if g32 is None else g32.data_ptr(),
                                           0 if g32 is None else g32.stride(0),
                                           None if g16 is None else g16.data_ptr(), x.data_ptr(), weight.data_ptr(),
                                           mean.data_ptr(), rstd.data_ptr(), B, T, C, G, dx.data_ptr(),
                                           dw.data_ptr(), db.data_ptr(), 1 if accumulate else 0, ws.data_ptr(),
                                           _native.stream_handle(x.device))
        if rc != 0:
            raise RuntimeError("mfl_groupnorm_cl_backward failed: " + lib.mfl_add_layernorm_last_error().decode())
        if accumulate:
            dw = db = None
        return (dx, dw if nig[1] else None, db if nig[2] else None, None, None, None, None, None)


def group_norm_cl_supported(x, norm):
    import os
    from ... import _native
    if os.environ.get("MFL_GROUPNORM_CL", "1") == "0":  # (A/B: the reference's transposes + nn.GroupNorm)
        return False
    if not (x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 3 and x.is_contiguous()
            and isinstance(norm, torch.nn.GroupNorm) and norm.affine and norm.weight.dtype == torch.float32
            and norm.weight.device == x.device and norm.num_channels == x.shape[2]
            and torch.is_autocast_enabled("cuda") and torch.get_autocast_dtype("cuda") == torch.bfloat16):
        return False
    B, T, C = x.shape
    return _native.load_library().mfl_groupnorm_cl_workspace_bytes(B, T, C, norm.num_groups) > 0


def group_norm_cl(x, norm, flat, start, want16):
    """(out32, out16): ``F.group_norm`` of the channels-last x (B, T, C) as the reference's nn.GroupNorm on
    its (B, C, T) transpose, the fp32 result written into ``flat`` (B, S, C) at rows [start, start + T)
    (returned as that view, channels last) and its bf16 copy when ``want16``."""
    with torch.autocast("cuda", enabled=False):
        return _GroupNormCL.apply(x, norm.weight, norm.bias, norm.num_groups, norm.eps, flat, start, want16)


class _JoinLevels(Function):
    """The levels' rows, written by _GroupNormCL into one (B, S, C) buffer, as that buffer (no copy);
    the backward hands each level its rows of the gradient."""

    @staticmethod
    def forward(ctx, flat, *levels):
        ctx.bounds = [(lv.storage_offset() - flat.storage_offset()) // flat.shape[2] for lv in levels]
        ctx.sizes = [lv.shape[1] for lv in levels]
        return flat.view_as(flat)

    @staticmethod
    def backward(ctx, g):
        return (None,) + tuple(g[:, s:s + t] for s, t in zip(ctx.bounds, ctx.sizes))


def flatten_levels(srcs):
    """``torch.cat([s.transpose(1, 2) for s in srcs], 1)`` (prepare_encoder_inputs, reference
    unimodal_deformable_transformer.py:90-134) — without the copy when the levels are the consecutive
    rows of one buffer (BaseEncoder's channels-last GroupNorm wrote them there)."""
    rows = [s.transpose(1, 2) for s in srcs]
    flat = getattr(srcs[0], "_mfl_flat", None)
    if flat is not None and all(getattr(s, "_mfl_flat", None) is flat for s in srcs):
        run = 0
        ok = True
        for r in rows:
            if (r.untyped_storage().data_ptr() != flat.untyped_storage().data_ptr() or r.stride() != flat.stride()
                    or r.storage_offset() != flat.storage_offset() + run * flat.shape[2]):
                ok = False
                break
            run += r.shape[1]
        if ok and run == flat.shape[1]:
            from ... import _trace
            _trace.hit("flatten_levels_view")
            return _JoinLevels.apply(flat, *rows)
    return torch.cat(rows, 1)

