"""Caption decoder, reference models/unimodal_caption_decoder.py:19-144, plus a KV-cached greedy
decode (``greedy_decode``) for the DVC wrappers' inference loop.

The reference decodes by re-running the whole decoder over the full (seq_len - 1)-token prefix
for every word (models/deformable/unimodal_deformable_dvc.py:318-354): at word w the output row w
is read, its input token being <pad>, with causal + <pad>-key masks.  ``greedy_decode`` computes
exactly those rows: per word one decoder pass over two rows — the token chosen at w-1 (its keys /
values enter ``CaptionKVCache``) and the <pad> probe at w — against cached keys of the earlier
words and the memory projected once.  No host synchronisation inside the loop."""
import torch
from torch import nn

from .. import _trace
from .load_weights import init_encoder_block_weights
from .modules.embedding_layers import PositionalEncoding, VocabularyEmbedder
from .modules.layers import CaptionKVCache, UnimodalCaptionDecoderLayer
from .modules.linear import Linear
from ..utils.preds_postprocess import SegmentMemory

__all__ = ["UnimodalCaptionDecoder", "build_unimodal_caption_decoder", "greedy_decode"]


def _probs(logits):
    """``logits.softmax(dim=-1)`` as autocast runs it (softmax is on its fp32 list: the 16-bit logits
    cast to fp32, then an fp32 softmax): one kernel reading the 16-bit logits and writing fp32 (same
    values), whose backward writes the logits' 16-bit gradient directly — no (n, L, vocab) fp32 cast
    pass either way (vocab 10,000: 128 MB a pass at the DVC bench shape)."""
    if logits.is_cuda and logits.dtype in (torch.bfloat16, torch.float16) and torch.is_autocast_enabled("cuda"):
        with torch.autocast("cuda", enabled=False):
            probs = torch.softmax(logits, dim=-1, dtype=torch.float32)
        # (word_probs: a loss's gather of one word a row, fused backward).  This keeps the 16-bit logits
        # alive while probs is: half the fp32 probabilities' size (63.8 MB beside 127.7 MB at the DVC bench
        # shape: 168 segments x 19 words x 10,000), both freed at the loss backward
        probs._mfl_logits = logits
        return probs
    return logits.softmax(dim=-1)


class _WordProbs(torch.autograd.Function):
    """probs[..., words] of softmax probabilities computed from ``logits``, the gradient going to the
    logits directly (include/ffn_glue.h mfl_word_prob_backward) instead of through a dense
    (rows x vocabulary) gradient of the probabilities and softmax's backward."""

    @staticmethod
    def forward(ctx, logits, probs, words):
        p = probs.gather(-1, words[..., None])[..., 0]
        ctx.save_for_backward(probs, words, p)
        ctx.logits_shape, ctx.logits_dtype = logits.shape, logits.dtype
        return p

    @staticmethod
    def backward(ctx, g):
        from .. import _native
        probs, words, p = ctx.saved_tensors
        lib = _native.load_library()
        V = probs.shape[-1]
        coef = (g.float() * p).contiguous()
        dx = torch.empty(ctx.logits_shape, dtype=ctx.logits_dtype, device=probs.device)
        rc = lib.mfl_word_prob_backward(probs.data_ptr(), words.data_ptr(), coef.data_ptr(), probs.numel() // V, V,
                                        dx.data_ptr(), _native.stream_handle(probs.device))
        if rc != 0:
            raise RuntimeError(lib.mfl_relu_dropout_last_error().decode())
        return dx, None, None


def word_probs(probs, words):
    """``probs.float().gather(-1, words[..., None])[..., 0]`` — one word's probability a row, the caption
    loss's read of the decoder's output.  When ``probs`` came from ``_probs`` on the GPU (it carries
    its logits), the gradient is written to the logits in one pass (``_WordProbs``); the value is the
    same."""
    lg = getattr(probs, "_mfl_logits", None)
    if (lg is None or not probs.is_cuda or probs.dtype != torch.float32 or not probs.is_contiguous()
            or lg.shape != probs.shape or probs.shape[-1] % 4 or words.shape != probs.shape[:-1]):
        return probs.float().gather(-1, words[..., None])[..., 0]
    _trace.hit("word_prob_fused")
    return _WordProbs.apply(lg, probs.detach(), words.contiguous().to(torch.int64))


@torch.no_grad()
def greedy_decode(decoder, prime, step, n, length, bos, eos, pad, faster_eval, device):
    """Shared greedy loop of both caption decoders (reference unimodal_deformable_dvc.py:304-363).

    ``prime(cache)`` projects the memories; ``step(x, cache, pos)`` runs the layers on rows x
    (N, 2, d) — row 0 the token at ``pos`` (committed), row 1 the <pad> probe at pos + 1.
    Returns (captions (n, length) int32, captions as they were before the last word's update — the
    decoder input of the reference's final ``out['pred_captions']`` — or None if no word ran)."""
    captions = torch.full((n, length), pad, dtype=torch.int32, device=device)
    captions[:, 0] = bos
    cache = CaptionKVCache(n, length, device)
    prime(cache)
    done = torch.zeros(n, dtype=torch.bool, device=device)
    last_input = None
    pad_col = torch.full((n,), pad, dtype=torch.int32, device=device)
    for w in range(1, length):
        prev = captions[:, w - 1]
        cache.key_valid[:, w - 1] = prev != pad
        tokens = torch.stack([prev, pad_col], 1).long()
        x = decoder.positional_encoding(decoder.target_embedding(tokens), start=w - 1)
        x = step(x, cache, w - 1)
        tok = decoder.head(x[:, 1]).softmax(dim=-1).argmax(dim=-1).to(torch.int32)
        if w == length - 1:
            last_input = captions.clone()
        if faster_eval:
            captions[:, w] = tok
        else:
            live = ~done
            captions[:, w] = torch.where(live, tok, captions[:, w])
            done = done | (live & (tok == eos))
    return captions, last_input


class UnimodalCaptionDecoder(nn.Module):
    """Token embedding * sqrt(d) + sinusoidal positions, ``depth`` UnimodalCaptionDecoderLayers,
    vocabulary head with softmax; returns (depth or 1, N, L, vocab) (reference :19-107)."""

    def __init__(self, vocab_size, seq_len=20, d_model=768, embedding_matrix=None, emb_weights_req_grad=False,
                 depth=12, num_heads=12, mlp_ratio=4., qkv_bias=True, positional_embedding_dropout=0.,
                 attention_dropout=0., projection_dropout=0., bridge_dropout=0., mlp_dropout_1=0., mlp_dropout_2=0.,
                 pre_norm=True, weight_init=False, weight_load=False, model_official=None, return_intermediate=False):
        super().__init__()
        self.vocab_size = vocab_size
        self.target_embedding = VocabularyEmbedder(vocab_size, d_model)
        self.positional_encoding = PositionalEncoding(d_model, dropout=positional_embedding_dropout)
        self.d_model = d_model
        self.depth = depth
        self.return_intermediate = return_intermediate
        self.decoder = nn.ModuleList([
            UnimodalCaptionDecoderLayer(d_model=d_model, num_heads=num_heads, mlp_ratio=mlp_ratio, qkv_bias=qkv_bias,
                                        attention_dropout=attention_dropout, projection_dropout=projection_dropout,
                                        bridge_dropout=bridge_dropout, mlp_dropout_1=mlp_dropout_1,
                                        mlp_dropout_2=mlp_dropout_2, pre_norm=pre_norm)
            for _ in range(depth)])
        self.head = Linear(d_model, vocab_size)
        self.init_weights(embedding_matrix, emb_weights_req_grad)

    def forward(self, tgt, memory, tgt_mask=None, memory_mask=None, tgt_padding_mask=None, memory_padding_mask=None,
                last_only=False):
        """``last_only``: the head and softmax on the last layer only, (1, N, L, vocab) — the row
        ``[-1]`` of the full result, for callers that read nothing else (the DVC training forward)."""
        tgt = self.positional_encoding(self.target_embedding(tgt))
        if isinstance(memory, SegmentMemory):
            # every layer's cross-attention keys / values of the clip memory in one GEMM each way
            memory.project_group([lin for layer in self.decoder
                                  for lin in (layer.cross_attention.k_linear, layer.cross_attention.v_linear)])
        intermediate = []
        for layer in self.decoder:
            tgt = layer(tgt, memory, tgt_mask, memory_mask, tgt_padding_mask, memory_padding_mask)
            if self.return_intermediate and not last_only:
                intermediate.append(tgt)
        tgt = torch.stack(intermediate) if self.return_intermediate and not last_only else tgt.unsqueeze(0)
        return _probs(self.head(tgt))

    def init_weights(self, embedding_matrix, emb_weights_req_grad):
        self.target_embedding.init_word_embeddings(embedding_matrix, emb_weights_req_grad)
        self.decoder.apply(init_encoder_block_weights)

    def greedy_decode(self, memory, memory_key_mask, bos, eos, pad, length, faster_eval=False):
        """Greedy captions of ``length`` tokens for memory (N, K, d); memory_key_mask (N, K) bool
        (True = masked) or None.  See ``greedy_decode``."""
        mask4 = None if memory_key_mask is None else memory_key_mask[:, None, None, :]

        def prime(cache):
            for i, layer in enumerate(self.decoder):
                layer.prime(cache, i, memory, mask4)

        def step(x, cache, pos):
            for i, layer in enumerate(self.decoder):
                x = layer.step(x, cache, i, pos)
            return x

        return greedy_decode(self, prime, step, memory.shape[0], length, bos, eos, pad, faster_eval, memory.device)


def build_unimodal_caption_decoder(args, vocab_size, seq_len, embedding_matrix):
    """reference :123-144"""
    return UnimodalCaptionDecoder(vocab_size=vocab_size, seq_len=seq_len, d_model=args.d_model,
                                  embedding_matrix=embedding_matrix, emb_weights_req_grad=args.emb_weights_req_grad,
                                  depth=args.depth, num_heads=args.num_heads, mlp_ratio=args.mlp_ratio,
                                  qkv_bias=args.qkv_bias, positional_embedding_dropout=args.positional_embedding_dropout,
                                  attention_dropout=args.attention_dropout, projection_dropout=args.projection_dropout,
                                  bridge_dropout=args.bridge_dropout, mlp_dropout_1=args.mlp_dropout_1,
                                  mlp_dropout_2=args.mlp_dropout_2, pre_norm=args.pre_norm,
                                  weight_init=args.weight_init, weight_load=args.weight_load,
                                  model_official=args.model_official, return_intermediate=args.return_intermediate)
