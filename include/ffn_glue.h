/*
 * ffn_glue.h — C-ABI of the fused FFN activation dropout(relu(h)) of the deformable transformer
 * layers (multimodal-feature-learning_amd/csrc/ffn_glue.hip, built into libmsda_hip.so).
 *
 * Replaces, under bf16 autocast, `self.dropout2(self.activation(self.linear1(src)))` of the
 * reference's encoder FFN (models/deformable/unimodal_deformable_transformer.py:233-236) and the
 * decoder's `dropout3(activation(linear1(tgt)))` (:360-362): ATen's relu, dropout (+ byte mask)
 * and, in the backward, masked-scale and threshold_backward kernels.
 *
 * n bf16 elements, contiguous, n % 8 == 0, 16-byte aligned pointers.  seed: a device int64
 * (null = no dropout, relu only); keep bits are a pure function of (seed, element index).
 * The backward needs only the forward's output: dx = dy / (1 - p) where out > 0, else 0
 * (`dropped` = whether the forward had a seed).  0 <= p_drop < 1.  Asynchronous on `stream`;
 * 0 or non-zero with mfl_relu_dropout_last_error().
 */
#ifndef MFL_FFN_GLUE_H
#define MFL_FFN_GLUE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

int mfl_relu_dropout_forward(const void* x, int64_t n, float p_drop, const int64_t* seed, void* out, void* stream);

int mfl_relu_dropout_backward(const void* dy, const void* out, int64_t n, float p_drop, int dropped, void* dx,
                              void* stream);

/* dropout(gelu(x)) (exact erf GELU, reference layers.py:827-869 MLP: nn.GELU() then nn.Dropout) on n bf16
 * elements (n % 8 == 0, 16-byte aligned), rounded as ATen rounds it under bf16 autocast (gelu to bf16,
 * then the dropout scale); keep bits from `seed` as mfl_relu_dropout_forward (NULL: no dropout).
 * Backward from x and the same seed: dx = bf16(bf16(dy keep / (1 - p)) gelu'(x)).
 * (reference: the caption decoder MLP, models/modules/layers.py:827-869) */
int mfl_gelu_dropout_forward(const void* x, int64_t n, float p_drop, const int64_t* seed, void* out, void* stream);
int mfl_gelu_dropout_backward(const void* dy, const void* x, int64_t n, float p_drop, const int64_t* seed, void* dx,
                              void* stream);

/* The logits' gradient when a loss reads one word's probability a row, p_w = softmax(x)[row, words[row]]
 * (the caption loss's gather of the decoder's probabilities, reference criterion over
 * unimodal_caption_decoder.py's softmax): dx[row, j] = coef[row] (delta_{j, w} - probs[row, j]) as bf16,
 * coef = dL/dp_w * p_w; probs (rows x vocab) fp32, vocab % 4 == 0, dx rows 8-byte aligned. */
int mfl_word_prob_backward(const float* probs, const int64_t* words, const float* coef, int64_t rows, int64_t vocab,
                           void* dx, void* stream);

/* mfl_relu_dropout_backward on a (rows x cols) row-major matrix (cols % 8 == 0) that also writes
 * colsum[j] = sum over rows of dx[:, j] as stored (bf16, summed in fp32, fixed order): the bias
 * gradient of the Linear layer whose output the activation read (reference linear1.bias.grad).
 * `workspace`: mfl_relu_dropout_colsum_workspace_bytes(rows, cols) bytes. */
size_t mfl_relu_dropout_colsum_workspace_bytes(int64_t rows, int64_t cols);
int mfl_relu_dropout_backward_colsum(const void* dy, const void* out, int64_t rows, int64_t cols, float p_drop,
                                     int dropped, void* dx, float* colsum, void* workspace, void* stream);

/*
 * x.view(rows, row_bytes).masked_fill_(mask[:, None], 0) in place: `value.masked_fill(
 * input_padding_mask[..., None], 0)` of MSDeformAttn.forward (reference
 * models/modules/attention.py:462-463) and its backward (the same on the value gradient).
 * mask: rows bytes (torch.bool), non-zero = padding.  row_bytes % 16 == 0, x 16-byte aligned.
 * Only padding rows are written.  Errors via mfl_relu_dropout_last_error().
 */
int mfl_zero_masked_rows(void* x, int64_t rows, int64_t row_bytes, const uint8_t* mask, void* stream);

/* The same on nbatch consecutive (rows x row_bytes) matrices sharing one mask of rows bytes: the
 * decoder's value projections of all layers, computed as one batch (models/modules/value_proj.py). */
/* Backward of the DVC segment memory's gathered projections (utils/preds_postprocess.py,
 * SegmentMemory.project: out[s, t] = keep[s, t] ? P[index[s], t] : bias, s < n segments, t < K tokens):
 *   grad_src[b, t, :]  = sum of grad[s, t, :] over s with index[s] == b and keep[s, t]   (bf16, every row written)
 *   bias_part[t, :]    = sum of grad[s, t, :] over s with !keep[s, t]                   (fp32; the bias gradient
 *                        is its sum over t)
 * fp32 sums in segment order.  grad (n, K, d) bf16, index (n,) int64 in [0, B), keep (n, K) bool (1 byte);
 * d % 8 == 0, d <= 512, 16-byte aligned grad / grad_src. */
int mfl_gather_keep_backward(const void* grad, const int64_t* index, const void* keep, int64_t n, int64_t B, int64_t K,
                             int64_t d, void* grad_src, float* bias_part, void* stream);

int mfl_zero_masked_rows_batched(void* x, int64_t nbatch, int64_t rows, int64_t row_bytes, const uint8_t* mask,
                                 void* stream);

/* The augmented operands of the batched value / key projections' bias-in-K GEMM
 * (models/modules/value_proj.py layer_values, y_i = [x | 1] . [W_i^T ; b_i] with K padded to ca):
 *   mfl_augment_rows:    out (k, ca) bf16 = [x (k, c) | 1 | 0 ...]                  (c, ca multiples of 8, 16-B aligned)
 *   mfl_augment_weights: out (n, ca, co) bf16, out[i][j][o] = w[i][o][j] (j < c), b[i][o] (j == c), 0 (j > c),
 *                        w (n, co, c) / b (n, co) bf16 contiguous.
 * One pass each. */
int mfl_augment_rows(const void* x, int64_t k, int64_t c, int64_t ca, void* out, void* stream);
int mfl_augment_weights(const void* w, const void* b, int64_t n, int64_t c, int64_t ca, int64_t co, void* out,
                        void* stream);

/* The flattened level position embedding of prepare_encoder_inputs (reference
 * models/deformable/unimodal_deformable_transformer.py:90-134, `torch.cat([pos_l.transpose(1, 2) +
 * level_embed[l].view(1, 1, -1) for l], 1)`): out[b, start_l + t, c] = pos[l][b, c, t] +
 * level_embed[l, c], fp32; pos: a host array of L device pointers to contiguous (B, N, T[l]) fp32
 * tensors, out (B, sum T, N) contiguous, start_l the running sum of T.  1 <= L <= 16. */
int mfl_level_pos_flatten(const float* const* pos, const int64_t* T, int64_t L, int64_t B, int64_t N,
                          const float* level_embed, float* out, void* stream);
/* As mfl_level_pos_flatten; channels_last (host array of L flags, may be NULL): level l's (B, N, T[l])
 * tensor is the transposed view of contiguous (B, T[l], N) rows (element (b, c, t) at (b T + t) N + c),
 * as the position embedding module returns it. */
int mfl_level_pos_flatten_ex(const float* const* pos, const int* channels_last, const int64_t* T, int64_t L,
                             int64_t B, int64_t N, const float* level_embed, float* out, void* stream);

/* Its backward for the level embedding: out[l, c] (+)= sum over b and t < T[l] of g[b, start_l + t, c]
 * (g (B, sum T, N) fp32 contiguous, N % 4 == 0, 16-byte aligned; fixed summation order).
 * accumulate != 0 adds into out.  workspace: mfl_level_colsum_workspace_bytes(T, L, B, N) bytes. */
size_t mfl_level_colsum_workspace_bytes(const int64_t* T, int64_t L, int64_t B, int64_t N);
int mfl_level_colsum(const float* g, const int64_t* T, int64_t L, int64_t B, int64_t N, float* out, int accumulate,
                     void* workspace, void* stream);

/* The whole flattened level position embedding of a pyramid (reference PositionEmbeddingVideoSine,
 * models/modules/embedding_layers.py:185-227, per level, then prepare_encoder_inputs' level_embed add
 * and flatten, unimodal_deformable_transformer.py:90-134): for level l, clip b, position t and
 * x = the number of non-padding positions in [0, t] of masks[l][b] (normalize: (x - 0.5) /
 * (x_last + eps) * scale), out[b, start_l + t, c] = sin(x / dim_t[c]) for even c < npf, cos(x /
 * dim_t[c]) for odd c < npf, dur[b, c - npf] for c >= npf; plus level_embed[l, c].  masks: host array
 * of L device pointers to (B, T[l]) bool; dim_t (npf) fp32; dur (B, npf) fp32; level_embed (L, 2 npf)
 * fp32; out (B, sum T, 2 npf) fp32.  1 <= L <= 16. */
int mfl_pyramid_pos_flatten(const uint8_t* const* masks, const int64_t* T, int64_t L, int64_t B, int64_t npf,
                            const float* dim_t, const float* dur, const float* level_embed, int normalize,
                            float scale, float eps, float* out, void* stream);

const char* mfl_relu_dropout_last_error(void);

#ifdef __cplusplus
}
#endif

#endif /* MFL_FFN_GLUE_H */
