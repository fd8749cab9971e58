/*
 * flat_adamw.h — C-ABI of the training step's fused optimizer over one flat fp32 parameter
 * buffer (multimodal-feature-learning_amd/csrc/flat_adamw.hip, built into libmsda_hip.so).
 *
 * Runtime component, not part of the MSDA boundary: it replaces, for the flat-buffer trainer
 * (train_step.py), the reference step's clip_grad_norm_ + AdamW
 * (reference engine.py:125-127, main.py:113) with the semantics of
 * torch.nn.utils.clip_grad_norm_(max_norm) followed by torch.optim.AdamW(lr, (beta1, beta2), eps,
 * weight_decay), and refreshes the bf16 shadow of the parameters in the same pass.
 * Graph-capturable: the step count (`step`, one fp32 device scalar) and the clip coefficient
 * stay on the device.  Gradients are read, not modified (the clip is applied on the fly).
 * Also the bias-gradient column sum of the autocast Linear (mfl_colsum).
 */
#ifndef FLAT_ADAMW_H_
#define FLAT_ADAMW_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Bytes of device scratch flat_adamw_step needs (8-byte aligned). */
size_t flat_adamw_workspace_bytes(void);

/* One optimizer step over n parameters (16-byte aligned fp32 buffers; bf16_shadow may be NULL).
 * max_norm <= 0 disables clipping.  lr_wd: NULL, or a device array {lr, weight_decay} read by the
 * kernels in place of the lr / weight_decay arguments, so that a captured HIP graph follows a
 * learning-rate schedule (reference main.py:99 StepLR) instead of replaying the capture's values.
 * Returns 0, or non-zero with flat_adamw_last_error(). */
int flat_adamw_step(float* params, const float* grads, float* exp_avg, float* exp_avg_sq, uint16_t* bf16_shadow,
                    int64_t n, float* step, void* workspace, float lr, float beta1, float beta2, float eps,
                    float weight_decay, float max_norm, const float* lr_wd, void* stream);

/* Column sums in fp32 of a row-major (K, N) matrix x (dtype tag as msda_hip.h: 0 fp32, 2 bf16,
 * 3 fp16; N*elt a multiple of 16 bytes, x 16-byte aligned): the bias gradient of the autocast
 * Linear (models/modules/linear.py), sum over the K token rows of dY.  Fixed summation order.
 * workspace: mfl_colsum_workspace_bytes(K, N) bytes. */
size_t mfl_colsum_workspace_bytes(int64_t K, int64_t N);
int mfl_colsum(const void* x, int dtype, int64_t K, int64_t N, float* out, void* workspace, void* stream);
/* As mfl_colsum; accumulate != 0: out += the column sums (each sum formed first, then added). */
int mfl_colsum_ex(const void* x, int dtype, int64_t K, int64_t N, float* out, int accumulate, void* workspace,
                  void* stream);

/* out[i] = sum over k < s of part[k * n + i] (fp32, chunk order): the split-K partial products of
 * the autocast Linear's weight gradient summed into the fp32 gradient.  n % 4 == 0, 16-byte
 * aligned pointers. */
int mfl_sum_slabs(const float* part, int64_t s, int64_t n, float* out, void* stream);
/* groups sums at once: out[g * n + i] = sum over k < s of part[(g * s + k) * n + i]; accumulate != 0:
 * out[g * n + i] += that sum (formed first, then added: the accumulation of a finished gradient).
 * The weight gradients of a layer used several times in one backward (a shared module, the
 * trainer's flat gradient views; models/modules/linear.py). */
int mfl_sum_slabs_ex(const float* part, int64_t groups, int64_t s, int64_t n, float* out, int accumulate,
                     void* stream);

/* A HIP stream of its own on `device` (hipStreamNonBlocking), outside PyTorch's round-robin stream pool:
 * the trainer's capture / comm streams (train_step.py).  A pool stream can be the RCCL process group's
 * own NCCL stream, and HIP refuses hipEventQuery of an event whose stream is capturing — even one
 * recorded before the capture — which the RCCL watchdog takes as fatal.  Lives for the
 * process. */
int mfl_stream_create(int device, void** stream);

/* Text of the last error of flat_adamw_step / mfl_colsum / mfl_sum_slabs on the calling thread. */
const char* flat_adamw_last_error(void);

#ifdef __cplusplus
}
#endif

#endif /* FLAT_ADAMW_H_ */
