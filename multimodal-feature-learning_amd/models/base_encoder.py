"""Conv1d feature pyramid + position embedding, the reference's ``models/base_encoder.py``.

Stays stock PyTorch-ROCm (BASELINE.json north_star): the Conv1d/GroupNorm stacks are library
GEMM / normalisation work, not part of the hand-written hot path.  Same module tree and
parameter names as the reference (``input_proj.{l}.{0,1}``) so state_dicts load unchanged.

Under 16-bit autocast on the GPU each Conv1d (k=1, or k=3 stride 2 padding 1) runs as ONE GEMM
over the channels-last input (``_Conv1dGemm``: the k taps' shifted rows side by side, K = k*C)
instead of MIOpen's convolution: at the bench shape MIOpen's bf16 kernels took 0.53 ms of the
step (~100 TFLOP/s) and their forward is not reproducible run to run (tools/determinism_diag.py:
the same inputs gave different outputs; every later difference of the bf16 DVC step followed
from it).  The arithmetic is the convolution's: bf16 operands, fp32 accumulation, one rounding
of the output; the input gradient is folded in fp32 and rounded once; weight / bias gradients
in fp32.
"""
import torch
import torch.nn.functional as F
from torch import nn

from .modules.misc_modules import NestedTensor

__all__ = ["BaseEncoder", "build_base_encoder", "conv1d_gemm"]


class _Conv1dGemm(torch.autograd.Function):
    """y (B, T_out, O) = conv1d of x (B, T, C) (channels-last, 16-bit) with weight (O, C, k), k = 1
    or k = 3 with stride 2 and padding 1 (reference base_encoder.py:27-36), as one GEMM."""

    @staticmethod
    def forward(ctx, x, weight, bias):
        B, T, C = x.shape
        O, _, k = weight.shape
        dt = x.dtype
        # [o][tap][c] in the input dtype: the permute and the cast in one copy kernel (reshape of the
        # permuted fp32 weight would first clone it in fp32)
        w2 = torch.empty((O, k, C), dtype=dt, device=weight.device).copy_(weight.permute(0, 2, 1)).view(O, k * C)
        if k == 1:
            t_out = T
            cols = x.reshape(B * T, C)
        else:
            t_out = (T - 1) // 2 + 1
            xp = F.pad(x, (0, 0, 1, 1))  # zero rows at t = -1 and t = T
            cols = torch.cat([xp[:, j:j + 2 * t_out - 1:2] for j in range(3)], 2).reshape(B * t_out, 3 * C)
        y = torch.mm(cols, w2.t()) if bias is None else torch.addmm(bias.to(dt), cols, w2.t())
        ctx.save_for_backward(cols, w2)
        ctx.meta = (B, T, C, O, k, t_out, bias is not None)
        ctx.params = (weight, bias)  # (whose flat gradient views the backward may claim)
        return y.view(B, t_out, O)

    @staticmethod
    def backward(ctx, gy):
        from .modules.linear import _accum_target, _bias_grad, _claim, _weight_grad
        cols, w2 = ctx.saved_tensors
        weight, bias = ctx.params
        B, T, C, O, k, t_out, has_bias = ctx.meta
        g2 = gy.reshape(B * t_out, O).to(w2.dtype)
        half = g2.is_cuda and g2.dtype in (torch.bfloat16, torch.float16)  # (else: fp32 / fp64 unit tests)
        gx = gw = gb = None
        if ctx.needs_input_grad[0]:
            if k == 1:
                gx = torch.mm(g2, w2).view(B, T, C)
            else:
                acc = torch.float32 if half else g2.dtype
                gc = (torch.mm(g2, w2, out_dtype=acc) if half else torch.mm(g2, w2)).view(B, t_out, 3, C)
                gxp = torch.zeros(B, 2 * t_out + 1, C, dtype=acc, device=gy.device)
                gxp[:, 0:2 * t_out:2] = gc[:, :, 0]
                gxp[:, 1:2 * t_out:2] = gc[:, :, 1]
                gxp[:, 2:2 * t_out + 1:2] += gc[:, :, 2]
                gx = gxp[:, 1:T + 1].to(w2.dtype)
        if ctx.needs_input_grad[1]:
            gw_t = (_weight_grad(g2, cols) if half else torch.mm(g2.t(), cols)).view(O, k, C).permute(0, 2, 1)
            # the trainer's flat gradient view: written in place (claimed), or added into when the
            # encoder ran twice (configs[2]: the video and audio streams share the BaseEncoder)
            acc = _accum_target(weight)
            if acc is not None:
                acc.add_(gw_t)
            else:
                v = _claim(weight)
                gw = gw_t.contiguous() if v is None else v.copy_(gw_t)
        if has_bias and ctx.needs_input_grad[2]:
            acc = _accum_target(bias)
            if acc is not None:
                _bias_grad(g2, acc, accumulate=True) if half else acc.add_(g2.sum(0))
            else:
                gb = _bias_grad(g2, _claim(bias)) if half else g2.sum(0)
        return gx, gw, gb


def _gemm_conv_ok(conv, x):
    return (isinstance(conv, nn.Conv1d) and x.is_cuda and torch.is_autocast_enabled("cuda")
            and torch.get_autocast_dtype("cuda") in (torch.bfloat16, torch.float16)
            and conv.weight.dtype == torch.float32 and conv.groups == 1 and conv.dilation == (1,)
            and conv.padding_mode == "zeros"
            and ((conv.kernel_size == (1,) and conv.stride == (1,) and conv.padding == (0,))
                 or (conv.kernel_size == (3,) and conv.stride == (2,) and conv.padding == (1,))))


def conv1d_gemm(conv, x_cl):
    """``conv`` (nn.Conv1d) applied to the channels-last x_cl (B, T, C) -> (B, T_out, O) in the
    autocast dtype (see the module docstring)."""
    dt = torch.get_autocast_dtype("cuda")
    with torch.autocast("cuda", enabled=False):
        return _Conv1dGemm.apply(x_cl.to(dt).contiguous(), conv.weight, conv.bias)


class BaseEncoder(nn.Module):
    """reference base_encoder.py:13-89: level 0 = 1x1 Conv1d + GroupNorm(32) on the input
    features; levels 1.. = k3 s2 p1 Conv1d + GroupNorm, each on the previous level
    (T, T/2, T/4, T/8 for 4 levels); masks nearest-resized per level."""

    def __init__(self, num_feature_levels, vf_dim, d_model):
        super(BaseEncoder, self).__init__()
        self.num_feature_levels = num_feature_levels
        self.d_model = d_model
        if num_feature_levels > 1:
            input_proj_list = []
            in_channels = vf_dim
            input_proj_list.append(nn.Sequential(
                nn.Conv1d(in_channels, d_model, kernel_size=1),
                nn.GroupNorm(32, d_model),
            ))
            for _ in range(num_feature_levels - 1):
                input_proj_list.append(nn.Sequential(
                    nn.Conv1d(in_channels, d_model, kernel_size=3, stride=2, padding=1),
                    nn.GroupNorm(32, d_model),
                ))
                in_channels = d_model
            self.input_proj = nn.ModuleList(input_proj_list)
        else:
            self.input_proj = nn.ModuleList([
                nn.Sequential(
                    nn.Conv2d(vf_dim, d_model, kernel_size=1),
                    nn.GroupNorm(32, d_model),
                )])
        for proj in self.input_proj:
            nn.init.xavier_uniform_(proj[0].weight, gain=1)
            nn.init.constant_(proj[0].bias, 0)

    def _forward_gemm(self, vf, mask, duration, pos_embed):
        """``forward`` with every Conv1d as one GEMM on channels-last rows (_Conv1dGemm) and the
        GroupNorm on the (B, C, T) transpose, as the reference computes it; the returned srcs are
        (B, d_model, T_l) views of channels-last tensors (prepare_encoder_inputs transposes them back)."""
        from .modules.pyramid import LevelPositions, group_norm_cl, group_norm_cl_supported
        vf_nt = NestedTensor(vf.transpose(1, 2), mask, duration)
        srcs, masks, dtypes = [], [], []
        # the levels' lengths (k3 s2 p1 halves them), so the channels-last GroupNorm can write every
        # level's rows into the encoder's flattened input directly (pyramid.flatten_levels)
        Ts = [vf.shape[1]]
        for _ in range(1, self.num_feature_levels):
            Ts.append((Ts[-1] - 1) // 2 + 1)
        flat = None

        def level(l, x_cl, want16):
            nonlocal flat
            conv, norm = self.input_proj[l][0], self.input_proj[l][1]
            y = conv1d_gemm(conv, x_cl)
            if group_norm_cl_supported(y, norm) and y.shape[1] == Ts[l]:
                if flat is None:
                    flat = torch.empty(y.shape[0], sum(Ts), y.shape[2], dtype=torch.float32, device=y.device)
                out32, out16 = group_norm_cl(y, norm, flat, sum(Ts[:l]), want16)
                src = out32.transpose(1, 2)
                src._mfl_flat = flat
                return src, out16
            src = F.group_norm(y.transpose(1, 2).contiguous(), norm.num_groups, norm.weight, norm.bias, norm.eps)
            return src, src.transpose(1, 2)

        # level 1 convolves the input features as level 0 does, every later level the previous level
        # (reference base_encoder.py:79-86)
        src, _ = level(0, vf, False)
        srcs.append(src)
        masks.append(mask)
        prev_cl = vf
        for l in range(1, self.num_feature_levels):
            src, prev_cl = level(l, prev_cl, l + 1 < self.num_feature_levels)
            m = vf_nt.mask
            lmask = F.interpolate(m[None].float(), size=src.shape[-1:]).to(torch.bool)[0]
            srcs.append(src)
            masks.append(lmask)
        # level 0's embedding in pos_embed's own dtype, the others cast to the level's (reference
        # :62-89); computed when read — prepare_encoder_inputs flattens them from the masks instead
        dtypes = [torch.float32] + [s.dtype for s in srcs[1:]]
        poses = LevelPositions(pos_embed, [vf_nt.tensors] + srcs[1:], masks, duration, dtypes)
        return srcs, masks, poses

    def forward(self, vf, mask, duration, pos_embed):
        """
        :param vf: (batch_size, num_tokens, vf_dim)
        :param mask: (batch_size, num_tokens) bool, True = padding
        :param duration: (batch_size,)
        :param pos_embed: PositionEmbeddingVideoSine
        :return srcs [(B, d_model, T_l)], masks [(B, T_l)], poses [(B, d_model, T_l)]
        """
        if (mask is not None and self.num_feature_levels > 1
                and all(isinstance(p[1], nn.GroupNorm) and _gemm_conv_ok(p[0], vf) for p in self.input_proj)):
            return self._forward_gemm(vf, mask, duration, pos_embed)
        vf = vf.transpose(1, 2)
        vf_nt = NestedTensor(vf, mask, duration)
        pos0 = pos_embed(vf_nt)
        srcs, masks, poses = [], [], []
        src0, mask0 = vf_nt.decompose()
        srcs.append(self.input_proj[0](src0))
        masks.append(mask0)
        poses.append(pos0)
        assert mask is not None
        for l in range(1, self.num_feature_levels):
            if l == 1:
                src = self.input_proj[l](vf_nt.tensors)
            else:
                src = self.input_proj[l](srcs[-1])
            m = vf_nt.mask
            mask = F.interpolate(m[None].float(), size=src.shape[-1:]).to(torch.bool)[0]
            pos_l = pos_embed(NestedTensor(src, mask, duration)).to(src.dtype)
            srcs.append(src)
            masks.append(mask)
            poses.append(pos_l)
        return srcs, masks, poses


def build_base_encoder(args):
    return BaseEncoder(args.num_feature_levels, args.feature_dim, args.d_model)
