"""Weight initialisation used by the caption decoders (reference models/load_weights.py:11-29).
The pretrained-checkpoint loaders of that file (ViViT / timm weights) are off the DVC path."""
from torch import nn
from torch.nn.init import constant_, xavier_uniform_

__all__ = ["init_encoder_block_weights"]


def init_encoder_block_weights(module):
    """xavier-uniform Linear weights with zero bias, unit / zero LayerNorm (reference :11-29).
    A Linear built without bias (qkv_bias=False) keeps None; the reference would raise on it."""
    if isinstance(module, nn.Linear):
        xavier_uniform_(module.weight)
        if module.bias is not None:
            constant_(module.bias, 0.)
    elif isinstance(module, nn.LayerNorm):
        constant_(module.weight, 1.)
        constant_(module.bias, 0.)
