"""Conv1d feature pyramid + position embedding, the reference's ``models/base_encoder.py``.

Stays stock PyTorch-ROCm (BASELINE.json north_star): the Conv1d/GroupNorm stacks are
MIOpen/hipBLASLt work, not part of the hand-written hot path.  Same module tree and
parameter names as the reference (``input_proj.{l}.{0,1}``) so state_dicts load unchanged.
"""
import torch
import torch.nn.functional as F
from torch import nn

from .modules.misc_modules import NestedTensor

__all__ = ["BaseEncoder", "build_base_encoder"]


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

    def forward(self, vf, mask, duration, pos_embed):
        """
        :param vf: (batch_size, num_tokens, vf_dim)
        :param mask: (batch_size, num_tokens) bool, True = padding
        :param duration: (batch_size,)
        :param pos_embed: PositionEmbeddingVideoSine
        :return srcs [(B, d_model, T_l)], masks [(B, T_l)], poses [(B, d_model, T_l)]
        """
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
