/*
 * gemm_small.h — C-ABI of the short-M bf16 GEMM of the training step (multimodal-feature-learning_amd/
 * csrc/gemm_small.hip, built into libmsda_hip.so).
 *
 * C[M, N] = A[M, K] . Bt[N, K]^T (+ bias[N]), bf16 operands, fp32 accumulation, bf16 result rounded
 * once (to nearest even) after the bias is added: what torch.addmm / torch.mm compute for the
 * Linear layers of the deformable decoder (800 query rows at the bench shape, models/deformable/
 * unimodal_deformable_transformer.py:342-373) and of the caption decoder (models/modules/layers.py),
 * i.e. `x @ W^T + b` with W stored (out, in) as nn.Linear does — both operands contiguous along K.
 * At these sizes the library GEMMs are launch / latency bound (0.4 GFLOP in ~10 us): here every
 * 32 x 32 output tile is one workgroup whose waves split K and add their partial sums in LDS.
 *
 * Requirements (else MFL_GEMM_UNSUPPORTED, and the caller keeps the library GEMM): N % 32 == 0,
 * K % 32 == 0, lda / ldb >= K and multiples of 8, 16-byte aligned A / Bt / C, ldc % 8 == 0.
 * bias may be NULL.  Asynchronous on `stream`.
 */
#ifndef MFL_GEMM_SMALL_H
#define MFL_GEMM_SMALL_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MFL_GEMM_UNSUPPORTED 2

int mfl_gemm_nt_bf16(const void* A, const void* Bt, const void* bias, void* C, int64_t M, int64_t N, int64_t K,
                     int64_t lda, int64_t ldb, int64_t ldc, void* stream);

/* C[M, N] = A[M, K] . B[K, N] (+ bias[N]) with B row-major (K, N): a Linear layer's input gradient
 * dX = dY . W, W stored (out, in).  Same requirements with ldb >= N (B's rows N-contiguous). */
int mfl_gemm_nn_bf16(const void* A, const void* B, const void* bias, void* C, int64_t M, int64_t N, int64_t K,
                     int64_t lda, int64_t ldb, int64_t ldc, void* stream);

const char* mfl_gemm_last_error(void);

#ifdef __cplusplus
}
#endif

#endif
