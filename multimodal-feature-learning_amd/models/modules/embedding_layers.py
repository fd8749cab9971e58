"""Embeddings of the DVC path, reference models/modules/embedding_layers.py: the video position +
duration embedding ``PositionEmbeddingVideoSine`` (:185-227), the caption decoder's
``PositionalEncoding`` (:167-181) and ``VocabularyEmbedder`` (:231-261).  ``FFN`` (layers.py:871-906)
is re-exported from ``layers`` for the importers of the first round."""
import math

import torch
from torch import nn

from .misc_modules import NestedTensor
from .linear import Linear
from .layers import FFN  # noqa: F401  (re-export)

__all__ = ["PositionEmbeddingVideoSine", "FFN", "PositionalEncoding", "VocabularyEmbedder"]


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


class PositionalEncoding(nn.Module):
    """Sinusoidal token positions added to the caption embedding, then dropout (reference
    embedding_layers.py:167-181; buffer ``pos_embedding`` (1, maxlen, d_model))."""

    def __init__(self, d_model, dropout, maxlen=5000):
        super().__init__()
        den = torch.exp(- torch.arange(0, d_model, 2) * math.log(10000) / d_model)
        pos = torch.arange(0, maxlen).reshape(maxlen, 1)
        pos_embedding = torch.zeros((maxlen, d_model))
        pos_embedding[:, 0::2] = torch.sin(pos * den)
        pos_embedding[:, 1::2] = torch.cos(pos * den)
        self.dropout = nn.Dropout(dropout)
        self.register_buffer('pos_embedding', pos_embedding.unsqueeze(0))

    def forward(self, token_embedding, start=0):
        """``start``: position of the first token (the incremental decode feeds single rows)."""
        return self.dropout(token_embedding
                            + self.pos_embedding[:, start:start + token_embedding.size(1), :].to(token_embedding.dtype))


class VocabularyEmbedder(nn.Module):
    """Token embedding times sqrt(d_model) (reference embedding_layers.py:231-261); GloVe-style
    ``embedding_matrix`` loaded as the reference does (frozen unless emb_weights_req_grad; projected
    by Linear + ReLU when its width differs from d_model)."""

    def __init__(self, vocab_size, d_model):
        super().__init__()
        self.vocab_size = vocab_size
        self.d_model = d_model
        self.embedder = nn.Embedding(vocab_size, d_model)

    def forward(self, x):
        return self.embedder(x) * math.sqrt(self.d_model)

    def init_word_embeddings(self, embedding_matrix, emb_weights_req_grad=True):
        if embedding_matrix is None:
            return
        embedding_matrix = torch.as_tensor(embedding_matrix)
        _, pretrained_embed_dim = embedding_matrix.shape
        if self.d_model == pretrained_embed_dim:
            self.embedder = self.embedder.from_pretrained(embedding_matrix)
            self.embedder.weight.requires_grad = emb_weights_req_grad
        else:
            self.embedder = nn.Sequential(
                nn.Embedding(self.vocab_size, pretrained_embed_dim).from_pretrained(embedding_matrix),
                Linear(pretrained_embed_dim, self.d_model),
                nn.ReLU())
            self.embedder[0].weight.requires_grad = emb_weights_req_grad
