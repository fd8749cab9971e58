"""Multimodal caption decoder, reference models/multimodal_caption_decoder.py:19-141, with the
KV-cached greedy decode of the unimodal decoder.

The reference class cannot be constructed at HEAD: ``super()`` names an undefined
class (:29), the layer class name is misspelt (:42) and it passes ``dropout_1`` / ``dropout_2`` to
a layer that takes ``mlp_dropout_1`` / ``mlp_dropout_2`` (:49-50; ``build_multimodal_caption_decoder``
reads ``args.dropout_1`` which the training config does not define — it has ``mlp_dropout_*``).
Restated intent: the same submodules and forward; ``dropout_1`` / ``dropout_2`` feed the MLP
dropouts, and the builder accepts either name."""
import torch
from torch import nn

from .load_weights import init_encoder_block_weights
from .modules.embedding_layers import PositionalEncoding, VocabularyEmbedder
from .modules.layers import MultimodalCaptionDecoderLayer
from .modules.linear import Linear
from .unimodal_caption_decoder import greedy_decode

__all__ = ["MultimodalCaptionDecoder", "build_multimodal_caption_decoder"]


class MultimodalCaptionDecoder(nn.Module):
    def __init__(self, vocab_size, seq_len=20, d_model=768, embedding_matrix=None, emb_weights_req_grad=False,
                 depth=12, num_heads=12, mlp_ratio=4., qkv_bias=True, positional_embedding_dropout=0.,
                 attention_dropout=0., projection_dropout=0., dropout_1=0., dropout_2=0., pre_norm=True,
                 weight_init=False, weight_load=False, model_official=None, return_intermediate=False,
                 bridge_dropout=0.):
        super().__init__()
        self.vocab_size = vocab_size
        self.target_embedding = VocabularyEmbedder(vocab_size, d_model)
        self.positional_encoding = PositionalEncoding(d_model, dropout=positional_embedding_dropout)
        self.d_model = d_model
        self.depth = depth
        self.return_intermediate = return_intermediate
        self.decoder = nn.ModuleList([
            MultimodalCaptionDecoderLayer(d_model=d_model, num_heads=num_heads, mlp_ratio=mlp_ratio, qkv_bias=qkv_bias,
                                          attention_dropout=attention_dropout, projection_dropout=projection_dropout,
                                          bridge_dropout=bridge_dropout, mlp_dropout_1=dropout_1,
                                          mlp_dropout_2=dropout_2, pre_norm=pre_norm)
            for _ in range(depth)])
        self.head = Linear(d_model, vocab_size)
        self.init_weights(embedding_matrix, emb_weights_req_grad)

    def forward(self, tgt, video_memory, audio_memory, tgt_mask=None, video_memory_mask=None, audio_memory_mask=None,
                tgt_padding_mask=None, video_memory_padding_mask=None, audio_memory_padding_mask=None):
        tgt = self.positional_encoding(self.target_embedding(tgt))
        intermediate = []
        for layer in self.decoder:
            tgt = layer(tgt, video_memory, audio_memory, tgt_mask, video_memory_mask, audio_memory_mask,
                        tgt_padding_mask, video_memory_padding_mask, audio_memory_padding_mask)
            if self.return_intermediate:
                intermediate.append(tgt)
        tgt = torch.stack(intermediate) if self.return_intermediate else tgt.unsqueeze(0)
        return self.head(tgt).softmax(dim=-1)

    def init_weights(self, embedding_matrix, emb_weights_req_grad):
        self.target_embedding.init_word_embeddings(embedding_matrix, emb_weights_req_grad)
        self.decoder.apply(init_encoder_block_weights)

    def greedy_decode(self, video_memory, video_key_mask, audio_memory, audio_key_mask, bos, eos, pad, length,
                      faster_eval=False):
        """Greedy captions over both memories (key masks (N, K) bool, True = masked, or None)."""
        memories = {"video": (video_memory, video_key_mask), "audio": (audio_memory, audio_key_mask)}

        def prime(cache):
            for i, layer in enumerate(self.decoder):
                layer.prime(cache, i, memories)

        def step(x, cache, pos):
            for i, layer in enumerate(self.decoder):
                x = layer.step(x, cache, i, pos)
            return x

        return greedy_decode(self, prime, step, video_memory.shape[0], length, bos, eos, pad, faster_eval,
                             video_memory.device)


def build_multimodal_caption_decoder(args, vocab_size, seq_len, embedding_matrix):
    """reference :121-141 (``dropout_1`` / ``dropout_2``, or the config's ``mlp_dropout_*``)."""
    get = lambda *names: next(getattr(args, n) for n in names if hasattr(args, n))  # noqa: E731
    return MultimodalCaptionDecoder(vocab_size=vocab_size, seq_len=seq_len, d_model=args.d_model,
                                    embedding_matrix=embedding_matrix, emb_weights_req_grad=args.emb_weights_req_grad,
                                    depth=args.depth, num_heads=args.num_heads, mlp_ratio=args.mlp_ratio,
                                    qkv_bias=args.qkv_bias,
                                    positional_embedding_dropout=args.positional_embedding_dropout,
                                    attention_dropout=args.attention_dropout,
                                    projection_dropout=args.projection_dropout,
                                    dropout_1=get("dropout_1", "mlp_dropout_1"),
                                    dropout_2=get("dropout_2", "mlp_dropout_2"), pre_norm=args.pre_norm,
                                    weight_init=args.weight_init, weight_load=args.weight_load,
                                    model_official=args.model_official, return_intermediate=args.return_intermediate,
                                    bridge_dropout=getattr(args, "bridge_dropout", 0.))
