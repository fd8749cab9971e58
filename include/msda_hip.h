/*
 * msda_hip.h — C-ABI of the MI355X (gfx950) multi-scale temporal deformable
 * attention (MSDA) kernels.
 *
 * This is the drop-in boundary for the reference's native op
 *   module `MultiScaleDeformableAttention`            (reference: models/ops/setup.py:53)
 *   ms_deform_attn_forward / ms_deform_attn_backward   (reference: models/ops/src/vision.cpp:14-15,
 *                                                       models/ops/src/ms_deform_attn.h:20-61)
 * and for the live pure-PyTorch core it shadows
 *   ms_deform_attn_core_pytorch                        (reference: models/modules/attention.py:331-383)
 *
 * Differences from the reference's pybind signature, all deliberate:
 *   - plain device pointers + sizes, no torch types;
 *   - level shapes / start indices are HOST arrays (the reference passes device
 *     tensors and syncs on them at models/modules/attention.py:346,458);
 *   - the 1-D temporal layout is native: sampling_loc is (B, Lq, M, L, P) and
 *     spatial_shapes holds T_l (the 2-D (H=1, W=T) form of
 *     models/ops/modules/ms_deform_attn.py:114-117 is unpacked by the host shim);
 *   - a padding-mode tag picks the live semantics (BORDER: grid_sample
 *     bilinear/border/align_corners=False, models/modules/attention.py:367-368)
 *     or the dormant CUDA kernel's zero padding
 *     (models/ops/src/cuda/ms_deform_im2col_cuda.cuh:34-85,289);
 *   - errors come back as a non-zero status + msda_hip_last_error() text instead
 *     of the reference's printf (ms_deform_im2col_cuda.cuh:949-953,1322-1326).
 *
 * Ownership: inputs are borrowed, read-only and must be contiguous (as asserted at
 * models/ops/src/cuda/ms_deform_attn_cuda.cu:28-38,93-105). Outputs are caller
 * allocated (the shim allocates them through the framework allocator). All work is
 * enqueued asynchronously on `stream`; nothing in here synchronises the host.
 */
#ifndef MSDA_HIP_H_
#define MSDA_HIP_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* dtype tags for value / output / grad_value / grad_output storage */
#define MSDA_DTYPE_F32 0
#define MSDA_DTYPE_F64 1
#define MSDA_DTYPE_BF16 2
#define MSDA_DTYPE_F16 3

/* padding-mode tags */
#define MSDA_PAD_BORDER 0 /* live path: grid_sample(border, align_corners=False) */
#define MSDA_PAD_ZEROS 1  /* dormant CUDA kernel: taps outside the map read 0    */

/* status codes */
#define MSDA_OK 0
#define MSDA_ERR_ARG 1    /* bad size / dtype / pointer                          */
#define MSDA_ERR_LAUNCH 2 /* hipGetLastError after a launch                       */
#define MSDA_ERR_UNSUPPORTED 3 /* a valid request this call's kernel path cannot honour (ABI v8:
                                  msda_hip_backward_ex's strided grad_value); nothing was launched */

#define MSDA_MAX_LEVELS 16

/* Coordinate dtype rule: sampling_loc / attn_weight / grad_loc / grad_attn are
 * f64 when value_dtype == MSDA_DTYPE_F64 and f32 otherwise (bf16/f16 values keep
 * fp32 locations: loc*T_l up to 4096 needs a 24-bit mantissa). */

/* Forward.  Replaces ms_deform_attn_cuda_forward
 * (reference: models/ops/src/cuda/ms_deform_attn_cuda.cu:20-80) and
 * ms_deform_attn_core_pytorch (models/modules/attention.py:331-383).
 *   value          (batch, spatial_size, num_heads, channels)   value_dtype
 *   sampling_loc   (batch, num_query, num_heads, num_levels, num_point)  in [0,1] (any real accepted)
 *   attn_weight    (batch, num_query, num_heads, num_levels, num_point)
 *   output         (batch, num_query, num_heads*channels)        value_dtype (written, not accumulated)
 * spatial_shapes[l] = T_l, level_start[l] = offset of level l along spatial_size (host arrays). */
int msda_hip_forward(const void* value, int value_dtype, const int64_t* spatial_shapes,
                     const int64_t* level_start, int64_t num_levels, const void* sampling_loc,
                     const void* attn_weight, void* output, int64_t batch, int64_t spatial_size,
                     int64_t num_heads, int64_t channels, int64_t num_query, int64_t num_point,
                     int padding_mode, void* stream);

/* Bytes of device scratch msda_hip_backward needs (ABI v2: depends on the query side).
 * Holds the per-row tap lists of the backward's sort pass (B*M*L*2*Lq*P entries) and the
 * row table (B*M*S).  No floating-point atomics
 * are used; with MSDA_HIP_DETERMINISTIC=1 in the environment every sum also has a fixed
 * order (bitwise reproducible backward, slower sort pass). */
size_t msda_hip_backward_workspace_bytes(int value_dtype, int64_t batch, int64_t spatial_size,
                                         int64_t num_heads, int64_t channels, int64_t num_query,
                                         int64_t num_levels, int64_t num_point);

/* Backward.  Replaces ms_deform_attn_cuda_backward
 * (reference: models/ops/src/cuda/ms_deform_attn_cuda.cu:83-153) and the autograd
 * graph of ms_deform_attn_core_pytorch (grid_sampler_2d_backward + stack/mul/sum).
 *   grad_output    (batch, num_query, num_heads*channels)        value_dtype
 *   grad_value     (batch, spatial_size, num_heads, channels)    value_dtype (overwritten)
 *   grad_loc       (batch, num_query, num_heads, num_levels, num_point)  coord dtype (overwritten)
 *   grad_attn      (batch, num_query, num_heads, num_levels, num_point)  coord dtype (overwritten)
 *   workspace      msda_hip_backward_workspace_bytes(...) bytes of device memory, 256-B aligned
 * Any of grad_value / grad_loc / grad_attn may be NULL to skip it.
 * BORDER mode: grad_loc is 0 where loc*T_l-0.5 is clamped (<=0 or >=T_l-1), exactly
 * as ATen's clip_coordinates_set_grad treats the border as out of bounds. */
int msda_hip_backward(const void* value, int value_dtype, const int64_t* spatial_shapes,
                      const int64_t* level_start, int64_t num_levels, const void* sampling_loc,
                      const void* attn_weight, const void* grad_output, void* grad_value,
                      void* grad_loc, void* grad_attn, void* workspace, int64_t batch,
                      int64_t spatial_size, int64_t num_heads, int64_t channels,
                      int64_t num_query, int64_t num_point, int padding_mode, void* stream);

/* ABI v8: msda_hip_backward with grad_value rows grad_value_row_stride elements apart (element
 * (b, s, h, c) at (b * spatial_size + s) * grad_value_row_stride + h * channels + c; a multiple of 8,
 * >= num_heads * channels; 0 = contiguous): lets a caller collect several calls' value gradients
 * side by side in one buffer (the decoder layers' value projections read them as one GEMM operand,
 * models/modules/value_proj.py) without a stacking copy.  Honoured by the per-tap fused backward
 * (sparse / decoder-like calls); other calls return MSDA_ERR_UNSUPPORTED and launch nothing. */
int msda_hip_backward_ex(const void* value, int value_dtype, const int64_t* spatial_shapes,
                         const int64_t* level_start, int64_t num_levels, const void* sampling_loc,
                         const void* attn_weight, const void* grad_output, void* grad_value,
                         void* grad_loc, void* grad_attn, void* workspace, int64_t batch,
                         int64_t spatial_size, int64_t num_heads, int64_t channels,
                         int64_t num_query, int64_t num_point, int padding_mode, int64_t grad_value_row_stride,
                         void* stream);

/* Forward that also hands the backward its row intervals (ABI v5; an extension: the reference's
 * extension has no forward-to-backward state beyond the saved inputs).  For calls whose backward
 * takes the row-block MFMA path (bf16 values, channels == 64, encoder-like calls: the queries
 * cover the pyramid; csrc/msda.hip win_takes) the backward first computes, for every
 * (batch, head, level, tile of 32 queries), the value rows the tile's samples touch: a pass over
 * all of sampling_loc.  The forward already reads sampling_loc, so it can write them instead.
 *   msda_hip_forward_tiles_bytes  size of that interval buffer for a call, 0 when the call's
 *                                 backward does not take the row-block path (then use the
 *                                 plain entry points)
 *   msda_hip_forward_tiles        msda_hip_forward + fills `tiles` (that many bytes)
 *   msda_hip_backward_tiles       msda_hip_backward on the same inputs with the filled `tiles`
 *                                 (the row-block path needs no other workspace; `workspace` is
 *                                 then only read if the call takes another path, e.g. under
 *                                 MSDA_HIP_BWD_WIN=0, and must be sized as for msda_hip_backward
 *                                 whenever msda_hip_backward_workspace_bytes differs from the
 *                                 tiles size)
 * The buffer is opaque: after the intervals it holds a 128-byte tail (the query order the forward
 * grouped its tiles by, which the backward reads, so both always agree); one forward's tiles serve
 * any number of backwards on the same inputs. */
size_t msda_hip_forward_tiles_bytes(int value_dtype, const int64_t* spatial_shapes, int64_t num_levels,
                                    int64_t batch, int64_t spatial_size, int64_t num_heads, int64_t channels,
                                    int64_t num_query, int64_t num_point);
int msda_hip_forward_tiles(const void* value, int value_dtype, const int64_t* spatial_shapes,
                           const int64_t* level_start, int64_t num_levels, const void* sampling_loc,
                           const void* attn_weight, void* output, void* tiles, int64_t batch, int64_t spatial_size,
                           int64_t num_heads, int64_t channels, int64_t num_query, int64_t num_point,
                           int padding_mode, void* stream);
int msda_hip_backward_tiles(const void* value, int value_dtype, const int64_t* spatial_shapes,
                            const int64_t* level_start, int64_t num_levels, const void* sampling_loc,
                            const void* attn_weight, const void* grad_output, void* grad_value,
                            void* grad_loc, void* grad_attn, void* workspace, const void* tiles, int64_t batch,
                            int64_t spatial_size, int64_t num_heads, int64_t channels,
                            int64_t num_query, int64_t num_point, int padding_mode, void* stream);

/* MSDA prologue.  Replaces the elementwise chain of MSDeformAttn.forward
 * between its two query projections and the core (reference models/modules/attention.py:468-483):
 *   attn_weight  = softmax(attn_logits over num_levels*num_point)                 (coord dtype)
 *   sampling_loc = ref[..., 0] + sampling_offsets / T_l                          (ref_dim == 1)
 *   sampling_loc = ref[..., 0] + sampling_offsets / num_point * ref[..., 1] * 0.5 (ref_dim == 2)
 *   sampling_offsets, attn_logits  (batch, num_query, num_heads, num_levels, num_point)  dtype
 *   reference_points               (batch, num_query, num_levels, ref_dim)          coord dtype
 *   sampling_loc, attn_weight      (batch, num_query, num_heads, num_levels, num_point)  coord dtype
 * 16-bit dtypes reproduce PyTorch's promotion under autocast (offsets / T_l rounded to the
 * 16-bit dtype once; the softmax in fp32).  num_heads*num_levels*num_point must be <= 1024. */
int msda_hip_prologue_forward(const void* sampling_offsets, const void* attn_logits, int dtype,
                              const void* reference_points, int ref_dim, const int64_t* spatial_shapes,
                              int64_t num_levels, int64_t batch, int64_t num_query, int64_t num_heads,
                              int64_t num_point, void* sampling_loc, void* attn_weight, void* stream);

/* Backward of msda_hip_prologue_forward: from grad_loc / grad_attn (coord dtype, the outputs of
 * msda_hip_backward) and the forward's attn_weight, writes grad_offsets and grad_logits (dtype)
 * and grad_ref (coord dtype, (batch, num_query, num_levels, ref_dim), summed over heads and
 * points).  Any output may be NULL to skip it; sampling_offsets / reference_points are read
 * only for ref_dim == 2. */
int msda_hip_prologue_backward(const void* grad_loc, const void* grad_attn, const void* attn_weight,
                               const void* sampling_offsets, int dtype, const void* reference_points,
                               int ref_dim, const int64_t* spatial_shapes, int64_t num_levels,
                               int64_t batch, int64_t num_query, int64_t num_heads, int64_t num_point,
                               void* grad_offsets, void* grad_logits, void* grad_ref, void* stream);

/* The same with the (batch, num_query) rows of sampling_offsets / attn_logits (and of
 * grad_offsets / grad_logits) `in_stride` elements apart (>= num_heads*num_levels*num_point;
 * ABI v6): both query projections can then be ONE GEMM writing [offsets | logits] rows of
 * 2*num_heads*num_levels*num_point, read in place, and the backward writes both gradients into
 * one such buffer, the input of one dgrad GEMM (models/modules/attention.py, _QueryPrologue). */
int msda_hip_prologue_forward_ex(const void* sampling_offsets, const void* attn_logits, int dtype,
                                 const void* reference_points, int ref_dim, const int64_t* spatial_shapes,
                                 int64_t num_levels, int64_t batch, int64_t num_query, int64_t num_heads,
                                 int64_t num_point, int64_t in_stride, void* sampling_loc, void* attn_weight,
                                 void* stream);
int msda_hip_prologue_backward_ex(const void* grad_loc, const void* grad_attn, const void* attn_weight,
                                  const void* sampling_offsets, int dtype, const void* reference_points,
                                  int ref_dim, const int64_t* spatial_shapes, int64_t num_levels,
                                  int64_t batch, int64_t num_query, int64_t num_heads, int64_t num_point,
                                  int64_t in_stride, void* grad_offsets, void* grad_logits, void* grad_ref,
                                  void* stream);

/* Coordinate layouts (ABI v7).  The reference's (and every entry point above) is
 * (batch, num_query, num_heads, num_levels, num_point): one (query, head)'s 64 bytes hold its
 * four levels, so in the backward four row blocks (one per level) each write 16 of them and the
 * line leaves L2 four times partially written.  Level-major puts one (batch, head, level)'s
 * coordinates of consecutive queries side by side, (batch, num_heads, num_levels, num_query,
 * num_point): a row block reads and writes whole lines.  It is internal to the fused MSDeformAttn
 * path (prologue -> forward -> backward -> prologue backward all in this library); the
 * extension API keeps the reference layout. */
#define MSDA_COORD_API 0
#define MSDA_COORD_LEVEL_MAJOR 1

/* Whether a call may use MSDA_COORD_LEVEL_MAJOR: its backward takes the row-block path fed by the
 * forward's tile intervals (msda_hip_forward_tiles_bytes > 0) and the prologue's level-major
 * kernel covers it (num_levels * num_point == 16, num_point % 4 == 0, num_heads <= 8). */
int msda_hip_level_major_ok(int value_dtype, const int64_t* spatial_shapes, int64_t num_levels, int64_t batch,
                            int64_t spatial_size, int64_t num_heads, int64_t channels, int64_t num_query,
                            int64_t num_point);

/* msda_hip_forward_tiles / msda_hip_backward_tiles / the _ex prologue pair with a coordinate
 * layout tag; sampling_loc, attn_weight, grad_loc and grad_attn are in that layout (the prologue's
 * offsets / logits rows and reference points are as in the _ex entry points). */
int msda_hip_forward_tiles_layout(const void* value, int value_dtype, const int64_t* spatial_shapes,
                                  const int64_t* level_start, int64_t num_levels, const void* sampling_loc,
                                  const void* attn_weight, void* output, void* tiles, int64_t batch,
                                  int64_t spatial_size, int64_t num_heads, int64_t channels, int64_t num_query,
                                  int64_t num_point, int padding_mode, int coord_layout, void* stream);
int msda_hip_backward_tiles_layout(const void* value, int value_dtype, const int64_t* spatial_shapes,
                                   const int64_t* level_start, int64_t num_levels, const void* sampling_loc,
                                   const void* attn_weight, const void* grad_output, void* grad_value,
                                   void* grad_loc, void* grad_attn, void* workspace, const void* tiles,
                                   int64_t batch, int64_t spatial_size, int64_t num_heads, int64_t channels,
                                   int64_t num_query, int64_t num_point, int padding_mode, int coord_layout,
                                   void* stream);
int msda_hip_prologue_forward_layout(const void* sampling_offsets, const void* attn_logits, int dtype,
                                     const void* reference_points, int ref_dim, const int64_t* spatial_shapes,
                                     int64_t num_levels, int64_t batch, int64_t num_query, int64_t num_heads,
                                     int64_t num_point, int64_t in_stride, int coord_layout, void* sampling_loc,
                                     void* attn_weight, void* stream);
int msda_hip_prologue_backward_layout(const void* grad_loc, const void* grad_attn, const void* attn_weight,
                                      const void* sampling_offsets, int dtype, const void* reference_points,
                                      int ref_dim, const int64_t* spatial_shapes, int64_t num_levels,
                                      int64_t batch, int64_t num_query, int64_t num_heads, int64_t num_point,
                                      int64_t in_stride, int coord_layout, void* grad_offsets, void* grad_logits,
                                      void* grad_ref, void* stream);

/* Sparse-DETR decoder attention map.  Replaces attn_map_to_flat_grid
 * (reference utils/dam.py:20-73): per (row, head), the attention weight of every sample is
 * scattered onto the two tokens around loc * T_l of its level with the reference's margins
 * (floor token: loc*T_l - floor - 1, next token: loc*T_l - floor), in-level tokens only.
 *   sampling_loc, attn_weight  (rows, num_query, num_heads, num_levels, num_point)  fp32
 *                              (rows = batch * decoder layers)
 *   flat_grid                  (rows, num_heads, sum_l T_l) fp32 (overwritten)
 * Float atomics in LDS: the summation order is not fixed (as the reference's scatter_add_). */
int msda_hip_dam_flat_grid(const void* sampling_loc, const void* attn_weight, const int64_t* spatial_shapes,
                           const int64_t* level_start, int64_t num_levels, int64_t rows, int64_t num_query,
                           int64_t num_heads, int64_t num_point, void* flat_grid, void* stream);

/* Text of the last error raised on the calling thread ("" if none). */
const char* msda_hip_last_error(void);

/* ABI version (bumped on any signature change). */
int msda_hip_abi_version(void);

#ifdef __cplusplus
}
#endif

#endif /* MSDA_HIP_H_ */
