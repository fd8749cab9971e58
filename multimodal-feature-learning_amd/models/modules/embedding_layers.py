"""Position embedding of the deformable path: the reference's ``PositionEmbeddingVideoSine``
(models/modules/embedding_layers.py:185-227) and the ``FFN`` head MLP
(models/modules/layers.py:871-906)."""
import math

import torch
from torch import nn

from .misc_modules import NestedTensor
from .linear import Linear

__all__ = ["PositionEmbeddingVideoSine", "FFN"]


class PositionEmbeddingVideoSine(nn.Module):
    """Sine position embedding over time + a learned clip-duration embedding.

    Output (B, 2*num_pos_feats, T): ``num_pos_feats`` sine/cosine channels of the
    cumulative valid-frame count, then ``num_pos_feats`` channels of
    ``duration_embed_layer(1[i < int(duration)])``.  The reference builds the duration
    one-hot with a per-clip Python loop (embedding_layers.py:221-227, one device->host
    sync per clip); here it is one comparison against ``arange``, same values for
    durations in [0, num_pos_feats].
    """

    def __init__(self, num_pos_feats, temperature=10000, normalize=False, scale=None):
        super().__init__()
        self.num_pos_feats = num_pos_feats
        self.temperature = temperature
        self.normalize = normalize
        if scale is not None and normalize is False:
            raise ValueError("normalize should be True if scale is passed")
        if scale is None:
            scale = 2 * math.pi
        self.scale = scale
        self.duration_embed_layer = Linear(self.num_pos_feats, self.num_pos_feats)

    def forward(self, tensor_list: NestedTensor):
        x = tensor_list.tensors
        mask = tensor_list.mask
        duration = tensor_list.duration
        assert mask is not None
        not_mask = ~mask
        x_embed = not_mask.cumsum(1, dtype=torch.float32)
        if self.normalize:
            eps = 1e-6
            x_embed = (x_embed - 0.5) / (x_embed[:, -1:] + eps) * self.scale
        dim_t = torch.arange(self.num_pos_feats, dtype=torch.float32, device=x.device)
        dim_t = self.temperature ** (2 * torch.div(dim_t, 2, rounding_mode='trunc') / self.num_pos_feats)
        pos_x = x_embed[:, :, None] / dim_t
        pos_x = torch.stack((pos_x[:, :, 0::2].sin(), pos_x[:, :, 1::2].cos()), dim=3).flatten(2)
        dur_embed = self.duration_embedding(duration).reshape(-1, 1, self.num_pos_feats).expand_as(pos_x)
        pos = torch.cat((pos_x, dur_embed), dim=2).permute(0, 2, 1)
        return pos

    def duration_embedding(self, durations):
        idx = torch.arange(self.num_pos_feats, device=durations.device)
        # default dtype, like the reference's torch.zeros (embedding_layers.py:222)
        out = (idx[None, :] < durations.int()[:, None]).to(torch.get_default_dtype())
        return self.duration_embed_layer(out)


class FFN(nn.Module):
    """n-layer MLP with ReLU between layers (reference layers.py:871-906)."""

    def __init__(self, in_dim, hidden_dim, out_dim, num_layers, dropout=0.):
        super().__init__()
        self.num_layers = num_layers
        h = [hidden_dim] * (num_layers - 1)
        self.layers = nn.ModuleList(Linear(n, k) for n, k in zip([in_dim] + h, h + [out_dim]))
        self.relu = nn.ReLU()

    def forward(self, x):
        for i, layer in enumerate(self.layers):
            x = self.relu(layer(x)) if i < self.num_layers - 1 else layer(x)
        return x
