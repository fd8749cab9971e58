// FFN activation of the deformable transformer layers: dropout(relu(linear1(x))) (reference
// unimodal_deformable_transformer.py:233-236 forward_ffn, :360-362; the multimodal and sparse
// layers repeat it).  Under bf16 autocast ATen runs it as a relu kernel, a dropout kernel that
// also writes a byte mask, and in the backward a masked-scale kernel plus relu's
// threshold_backward, each a full pass over the (tokens x d_ffn) hidden tensor.  Here:
//   forward : out = relu(x) * keep * 1/(1-p), one read of x and one write of out; keep bits from a
//             64-bit mix of (device seed, element index / 4), 16 bits per element;
//   backward: dx = dy * 1/(1-p) where out > 0, else 0 (out > 0 exactly when x > 0 and the element
//             was kept), from the output linear2 keeps anyway: no mask, no RNG.
// bf16 in and out, 8 elements (16 bytes) per lane, grid-stride over n / 8 vectors.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#include "../../include/ffn_glue.h"

namespace {

thread_local char g_err[256];

constexpr int kThreads = 256;

__device__ __forceinline__ uint32_t rne(float f) {
  const uint32_t u = __float_as_uint(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (u >> 16) | 0x40u;
  return (u + 0x7fffu + ((u >> 16) & 1u)) >> 16;
}

// 64 random bits per 4 consecutive elements (one 64-bit mix of (seed, e / 4)), 16 per element:
// the mix's 64-bit multiplies, not HBM, bounded the forward with one mix per element
__device__ __forceinline__ uint64_t drop_bits4(uint64_t seed, uint64_t quad) {
  uint64_t x = seed * 0x9E3779B97F4A7C15ull + quad;
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ull;
  x ^= x >> 33;
  return x;
}

__device__ __forceinline__ float relu_nan(float x) { return x > 0.f ? x : (x != x ? x : 0.f); }
__device__ __forceinline__ float lo(uint32_t w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float hi(uint32_t w) { return __uint_as_float(w & 0xffff0000u); }

__global__ __launch_bounds__(kThreads) void relu_dropout_fwd(const uint4* __restrict__ x, long long nvec,
                                                            const int64_t* __restrict__ seed_ptr, uint32_t thresh,
                                                            float scale, uint4* __restrict__ out) {
  const uint64_t seed = seed_ptr ? (uint64_t)seed_ptr[0] : 0;
  for (long long i = (long long)blockIdx.x * kThreads + threadIdx.x; i < nvec; i += (long long)gridDim.x * kThreads) {
    const uint4 v = x[i];
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
    uint32_t o[4];
    uint64_t bits[2] = {0ull, 0ull};
    if (seed_ptr) {
      bits[0] = drop_bits4(seed, (uint64_t)i * 2);
      bits[1] = drop_bits4(seed, (uint64_t)i * 2 + 1);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      // relu as ATen's: NaN stays NaN (fmaxf would turn it into 0 and hide a diverging FFN)
      float a = relu_nan(lo(w[j])), b = relu_nan(hi(w[j]));
      if (seed_ptr) {  // elements 2j, 2j+1 of the vector: 16-bit draws (2j % 4), (2j % 4) + 1 of bits[j / 2]
        const uint64_t q = bits[j >> 1] >> (32 * (j & 1));
        // dropped: x * 0 as ATen's x * mask (a NaN stays NaN)
        a *= (uint32_t)(q & 0xffffu) >= thresh ? scale : 0.f;
        b *= (uint32_t)((q >> 16) & 0xffffu) >= thresh ? scale : 0.f;
      }
      o[j] = rne(a) | (rne(b) << 16);
    }
    out[i] = make_uint4(o[0], o[1], o[2], o[3]);
  }
}

__global__ __launch_bounds__(kThreads) void relu_dropout_bwd(const uint4* __restrict__ dy, const uint4* __restrict__ out,
                                                            long long nvec, float scale, uint4* __restrict__ dx) {
  for (long long i = (long long)blockIdx.x * kThreads + threadIdx.x; i < nvec; i += (long long)gridDim.x * kThreads) {
    const uint4 g = dy[i], y = out[i];
    const uint32_t gw[4] = {g.x, g.y, g.z, g.w}, yw[4] = {y.x, y.y, y.z, y.w};
    uint32_t o[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      // ATen's threshold_backward: zero where out <= 0 (a NaN output passes its gradient)
      const float a = !(lo(yw[j]) <= 0.f) ? lo(gw[j]) * scale : 0.f;
      const float b = !(hi(yw[j]) <= 0.f) ? hi(gw[j]) * scale : 0.f;
      o[j] = rne(a) | (rne(b) << 16);
    }
    dx[i] = make_uint4(o[0], o[1], o[2], o[3]);
  }
}

// dropout(gelu(x)) of the caption decoder's MLP (reference layers.py:827-869: fc1 -> nn.GELU() ->
// dropout), the exact erf form, as ATen computes it under bf16 autocast: gelu in fp32 rounded to bf16,
// then (dropout) the bf16 value times keep / (1 - p) rounded again; the keep bits as relu_dropout's.
// Backward from x and the seed: g = bf16(dy * keep / (1 - p)), dx = bf16(g * gelu'(x)) — ATen's
// dropout backward then gelu_backward, each rounding to bf16.  One pass each way (ATen: gelu, a
// dropout writing a byte mask, a masked scale and gelu_backward: four full passes and a mask).
__device__ __forceinline__ float gelu_f(float x) { return 0.5f * x * (1.f + erff(x * 0.70710678118654752f)); }
__device__ __forceinline__ float gelu_grad_f(float x) {
  const float cdf = 0.5f * (1.f + erff(x * 0.70710678118654752f));
  const float pdf = expf(-0.5f * x * x) * 0.39894228040143268f;
  return cdf + x * pdf;
}
__device__ __forceinline__ float bfr(float f) { return __uint_as_float(rne(f) << 16); }

__global__ __launch_bounds__(kThreads) void gelu_dropout_fwd(const uint4* __restrict__ x, long long nvec,
                                                            const int64_t* __restrict__ seed_ptr, uint32_t thresh,
                                                            float scale, uint4* __restrict__ out) {
  const uint64_t seed = seed_ptr ? (uint64_t)seed_ptr[0] : 0;
  for (long long i = (long long)blockIdx.x * kThreads + threadIdx.x; i < nvec; i += (long long)gridDim.x * kThreads) {
    const uint4 v = x[i];
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
    uint32_t o[4];
    uint64_t bits[2] = {0ull, 0ull};
    if (seed_ptr) {
      bits[0] = drop_bits4(seed, (uint64_t)i * 2);
      bits[1] = drop_bits4(seed, (uint64_t)i * 2 + 1);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float a = gelu_f(lo(w[j])), b = gelu_f(hi(w[j]));
      if (seed_ptr) {
        const uint64_t q = bits[j >> 1] >> (32 * (j & 1));
        a = bfr(a) * ((uint32_t)(q & 0xffffu) >= thresh ? scale : 0.f);
        b = bfr(b) * ((uint32_t)((q >> 16) & 0xffffu) >= thresh ? scale : 0.f);
      }
      o[j] = rne(a) | (rne(b) << 16);
    }
    out[i] = make_uint4(o[0], o[1], o[2], o[3]);
  }
}

__global__ __launch_bounds__(kThreads) void gelu_dropout_bwd(const uint4* __restrict__ dy, const uint4* __restrict__ x,
                                                            long long nvec, const int64_t* __restrict__ seed_ptr,
                                                            uint32_t thresh, float scale, uint4* __restrict__ dx) {
  const uint64_t seed = seed_ptr ? (uint64_t)seed_ptr[0] : 0;
  for (long long i = (long long)blockIdx.x * kThreads + threadIdx.x; i < nvec; i += (long long)gridDim.x * kThreads) {
    const uint4 g = dy[i], v = x[i];
    const uint32_t gw[4] = {g.x, g.y, g.z, g.w}, xw[4] = {v.x, v.y, v.z, v.w};
    uint32_t o[4];
    uint64_t bits[2] = {0ull, 0ull};
    if (seed_ptr) {
      bits[0] = drop_bits4(seed, (uint64_t)i * 2);
      bits[1] = drop_bits4(seed, (uint64_t)i * 2 + 1);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float ga = lo(gw[j]), gb = hi(gw[j]);
      if (seed_ptr) {
        const uint64_t q = bits[j >> 1] >> (32 * (j & 1));
        ga = bfr(ga * ((uint32_t)(q & 0xffffu) >= thresh ? scale : 0.f));
        gb = bfr(gb * ((uint32_t)((q >> 16) & 0xffffu) >= thresh ? scale : 0.f));
      }
      o[j] = rne(ga * gelu_grad_f(lo(xw[j]))) | (rne(gb * gelu_grad_f(hi(xw[j]))) << 16);
    }
    dx[i] = make_uint4(o[0], o[1], o[2], o[3]);
  }
}

// Gradient of the caption logits when a loss reads one word's probability a row (p_w = softmax(x)_w,
// the caption loss's gather): dx_j = c (delta_jw - p_j), c = dL/dp_w * p_w, from the stored fp32
// probabilities; one workgroup a row, float4 reads, bf16 writes.  The dense path (the gather's
// scatter_add into zeros, the level split's concatenation, softmax's backward, the bf16 cast) makes
// ~8 passes over the (rows x vocabulary) tensor; this one reads it once.
__global__ __launch_bounds__(kThreads) void word_prob_bwd(const float4* __restrict__ probs, const int64_t* __restrict__ words,
                                                         const float* __restrict__ coef, int v4, uint2* __restrict__ dx) {
  const long long r = blockIdx.x;
  const float c = coef[r];
  const long long w = words[r];
  const float4* pr = probs + r * v4;
  uint2* out = dx + r * v4;
  for (int i = threadIdx.x; i < v4; i += kThreads) {
    const float4 p = pr[i];
    float o[4] = {-c * p.x, -c * p.y, -c * p.z, -c * p.w};
    const long long j0 = 4ll * i;
    if (w >= j0 && w < j0 + 4) o[w - j0] += c;  // c (1 - p_w) as c - c p_w
    out[i] = make_uint2(rne(o[0]) | (rne(o[1]) << 16), rne(o[2]) | (rne(o[3]) << 16));
  }
}

// relu_dropout_bwd on a (rows x cols) matrix that also sums each column of dx as stored (bf16): the
// bias gradient of the Linear layer that produced the hidden (linear1), which then needs no
// column-sum pass over dx.  One block = rpb rows x blockDim.x vectors of 8 columns; per-block column
// partials in fixed order, summed by relu_dropout_colsum_final in fixed order (deterministic).
// rpb = 32 rows and 256-thread blocks for the encoder's ~16 K rows; the decoder / audio calls (760-800
// rows) take 8 rows and one-wave blocks (rd_rows_per_block): with 32 they ran 25 blocks of 32
// dependent-row rounds (15-20 us for 3 MB; 4-5 us now)
constexpr int kRdRows = 32;
constexpr int kRdRowsSmall = 8;
constexpr int kRdUnroll = 8;  // rows whose loads are in flight together (one dependent row at a time: 2x slower)

int rd_rows_per_block(long long rows, long long cvec) {
  const long long waves = (rows + kRdRows - 1) / kRdRows * ((cvec + 63) / 64);
  return waves >= 1024 ? kRdRows : kRdRowsSmall;
}

__global__ __launch_bounds__(kThreads) void relu_dropout_bwd_colsum(const uint4* __restrict__ dy,
                                                                   const uint4* __restrict__ out, long long rows,
                                                                   int cvec, int rpb, float scale,
                                                                   uint4* __restrict__ dx, float* __restrict__ part) {
  const int c = blockIdx.y * blockDim.x + threadIdx.x;
  if (c >= cvec) return;
  const long long r0 = (long long)blockIdx.x * rpb;
  // (the last block's rows past the end re-read its last row and add nothing: branch-free loads, so
  // the compiler keeps kRdUnroll rows of loads in flight — with guarded loads it waited on each)
  const int nr = (int)min((long long)rpb, rows - r0);
  float sum[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  const uint4* __restrict__ dyc = dy + r0 * cvec + c;
  const uint4* __restrict__ outc = out + r0 * cvec + c;
  uint4* __restrict__ dxc = dx + r0 * cvec + c;
  for (int rr = 0; rr < rpb; rr += kRdUnroll) {
    uint4 g[kRdUnroll], y[kRdUnroll];
#pragma unroll
    for (int u = 0; u < kRdUnroll; ++u) {
      const int rw = min(rr + u, nr - 1);
      g[u] = dyc[(long long)rw * cvec];
      y[u] = outc[(long long)rw * cvec];
    }
#pragma unroll
    for (int u = 0; u < kRdUnroll; ++u) {
      const bool live = rr + u < nr;
      const uint32_t gw[4] = {g[u].x, g[u].y, g[u].z, g[u].w}, yw[4] = {y[u].x, y[u].y, y[u].z, y[u].w};
      uint32_t o[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float a = !(lo(yw[j]) <= 0.f) ? lo(gw[j]) * scale : 0.f;
        const float b = !(hi(yw[j]) <= 0.f) ? hi(gw[j]) * scale : 0.f;
        o[j] = rne(a) | (rne(b) << 16);
        sum[2 * j] += live ? lo(o[j]) : 0.f;
        sum[2 * j + 1] += live ? hi(o[j]) : 0.f;
      }
      if (live) dxc[(long long)(rr + u) * cvec] = make_uint4(o[0], o[1], o[2], o[3]);
    }
  }
  float4* pp = reinterpret_cast<float4*>(part + (long long)blockIdx.x * cvec * 8 + (long long)c * 8);
  pp[0] = make_float4(sum[0], sum[1], sum[2], sum[3]);
  pp[1] = make_float4(sum[4], sum[5], sum[6], sum[7]);
}

// colsum[j] = sum over the row groups' partials: a block = 16 row strides x 64 columns (the row
// groups dealt over the 16, eight independent chains each, then the 16 added in LDS; fixed order)
__global__ __launch_bounds__(1024) void relu_dropout_colsum_final(const float* __restrict__ part, int ngroups,
                                                                 int cols, float* __restrict__ colsum) {
  __shared__ float red[16][64];
  const int cl = threadIdx.x & 63, grp = threadIdx.x >> 6;
  const int j = blockIdx.x * 64 + cl;
  float sc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (j < cols) {
    int k = grp;
    for (; k + 112 < ngroups; k += 128) {
#pragma unroll
      for (int u = 0; u < 8; ++u) sc[u] += part[(long long)(k + 16 * u) * cols + j];
    }
    for (; k < ngroups; k += 16) sc[0] += part[(long long)k * cols + j];
  }
  red[grp][cl] = ((sc[0] + sc[1]) + (sc[2] + sc[3])) + ((sc[4] + sc[5]) + (sc[6] + sc[7]));
  __syncthreads();
  if (grp == 0 && j < cols) {
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) t += red[i][cl];
    colsum[j] = t;
  }
}

// value.masked_fill(padding_mask[..., None], 0) of MSDeformAttn (reference attention.py:462-463) in
// place, and the same on its gradient: a wave reads the mask bytes of 64 rows (one a lane) and zeroes
// only the padding rows among them, one row at a time with all its lanes, so an all-valid batch
// costs the mask read, not a pass over value.  (One wave per row before: 16 K waves that each read
// one byte, ~5 us a call at the encoder's 15,360 rows.)  Row i of x uses mask[i % mask_rows] (a batch
// of matrices sharing one token mask).
__global__ __launch_bounds__(kThreads) void zero_masked_rows_kernel(uint4* __restrict__ x, long long rows,
                                                                   int vec_per_row,
                                                                   const uint8_t* __restrict__ mask,
                                                                   long long mask_rows) {
  const int lane = threadIdx.x & 63;
  const long long row0 = ((long long)blockIdx.x * (kThreads / 64) + (threadIdx.x >> 6)) * 64;
  const long long row = row0 + lane;
  unsigned long long pad = __ballot(row < rows && mask[row % mask_rows] != 0);
  while (pad != 0ull) {  // (wave-uniform)
    const int r = __builtin_ctzll(pad);
    pad &= pad - 1ull;
    uint4* p = x + (row0 + r) * vec_per_row;
    for (int i = lane; i < vec_per_row; i += 64) p[i] = make_uint4(0u, 0u, 0u, 0u);
  }
}

unsigned grid_for(long long nvec) {
  const long long want = (nvec + kThreads - 1) / kThreads;
  return (unsigned)(want < 256 * 32 ? (want > 0 ? want : 1) : 256 * 32);  // <= 32 blocks per CU, grid-stride
}

bool args_ok(const char* who, int64_t n, const void* a, const void* b, const void* c, float p) {
  if (n < 0 || n % 8 != 0) {
    snprintf(g_err, sizeof(g_err), "%s: n must be a non-negative multiple of 8", who);
    return false;
  }
  if (!(p >= 0.f && p < 1.f)) {
    snprintf(g_err, sizeof(g_err), "%s: dropout p must be in [0, 1)", who);
    return false;
  }
  if (n > 0 && (!a || !b || !c)) {
    snprintf(g_err, sizeof(g_err), "%s: null pointer", who);
    return false;
  }
  if (((uintptr_t)a | (uintptr_t)b | (uintptr_t)c) & 15u) {
    snprintf(g_err, sizeof(g_err), "%s: pointers must be 16-byte aligned", who);
    return false;
  }
  return true;
}

int status(const char* what) {
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    snprintf(g_err, sizeof(g_err), "ffn_glue: %s launch failed: %s", what, hipGetErrorString(e));
    return 2;
  }
  return 0;
}

// Backward of the DVC segment memory's gathered projections (utils/preds_postprocess.py,
// _GatherKeep): forward out[s, t] = keep[s, t] ? P[index[s], t] : bias.  Here
//   grad_P[b, t] = sum over segments s with index[s] == b and keep[s, t] of g[s, t]
//   bias partial row t = sum over segments s with !keep[s, t] of g[s, t]
// in fp32, in segment order (deterministic).  One workgroup per token t: wave w sums clips
// b = w, w + 4, ... (the segments' clip ids are read as scalars), each lane 8 channels; the four
// waves' bias sums meet in LDS.  Every (s, t) row of g is read once.
__global__ __launch_bounds__(256) void gather_keep_bwd_kernel(const uint16_t* __restrict__ g,
                                                              const long long* __restrict__ index,
                                                              const uint8_t* __restrict__ keep, int n, int B, int K,
                                                              int d, uint16_t* __restrict__ gsrc,
                                                              float* __restrict__ bpart) {
  __shared__ float red[4][512];
  const int t = blockIdx.x, lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c0 = lane * 8;
  const bool act = c0 < d;
  float bacc[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) bacc[i] = 0.f;
  for (int b = w; b < B; b += 4) {
    float acc[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] = 0.f;
    for (int s = 0; s < n; ++s) {
      if (index[s] != b) continue;  // wave-uniform
      const long long row = (long long)s * K + t;
      const bool k = keep[row] != 0;
      if (act) {
        const uint4 v = *reinterpret_cast<const uint4*>(g + row * d + c0);
        const uint32_t u[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float lo = __uint_as_float(u[i] << 16), hi = __uint_as_float(u[i] & 0xffff0000u);
          if (k) {
            acc[2 * i] += lo;
            acc[2 * i + 1] += hi;
          } else {
            bacc[2 * i] += lo;
            bacc[2 * i + 1] += hi;
          }
        }
      }
    }
    if (act) {
      uint4 o;
      uint32_t* op = reinterpret_cast<uint32_t*>(&o);
#pragma unroll
      for (int i = 0; i < 4; ++i)
        op[i] = rne(acc[2 * i]) | (rne(acc[2 * i + 1]) << 16);
      *reinterpret_cast<uint4*>(gsrc + ((long long)b * K + t) * d + c0) = o;
    }
  }
  if (act) {
#pragma unroll
    for (int i = 0; i < 8; ++i) red[w][c0 + i] = bacc[i];
  }
  __syncthreads();
  for (int j = threadIdx.x; j < d; j += 256) bpart[(long long)t * d + j] = red[0][j] + red[1][j] + red[2][j] + red[3][j];
}


// ---------------------------------------------------------------------------------------------
// The flattened level position embedding of prepare_encoder_inputs (reference
// models/deformable/unimodal_deformable_transformer.py:90-134, also the multimodal and sparse
// transformers): lvl_pos[b, start_l + t, :] = pos_l[b, :, t] + level_embed[l, :], and the level
// embedding's gradient, the per-level column sums of lvl_pos's gradient.  ATen ran the forward as
// four transposed adds and a cat (an extra pass over the (B, S, d) result), the backward as four
// sum_to_size reductions (24-71 us each at the bench shape: a keep-last-dim reduction over 1-8 K
// rows with 128 workgroups) plus a zero fill, copy and add per level.
constexpr int kLpMaxL = 16;
struct LevelTable {
  const float* pos[kLpMaxL];
  long long sb[kLpMaxL];  // pos[l] element strides: batch; channel (1 or T, the other is the t stride)
  int sc1[kLpMaxL];       // 1: channels contiguous ((B, T, N) rows viewed as (B, N, T)), 0: positions contiguous
  int T[kLpMaxL], start[kLpMaxL];
  int blk0[kLpMaxL + 1];  // first workgroup / chunk of each level
  int L, tiles_c;         // levels; 64-column tiles (flatten) or 256-column groups (colsum)
};
constexpr int kLpT = 32;  // positions per transpose tile
// one workgroup a (level, b, 32 positions, 64 channels) tile: coalesced reads along t, LDS
// transpose (33-float rows), coalesced writes along channels
__global__ __launch_bounds__(256) void level_pos_flatten_kernel(const LevelTable tb, const float* __restrict__ emb,
                                                                long long B, int N, long long S, float* __restrict__ out) {
  __shared__ float tile[64][kLpT + 1];
  int l = 0;
  while (l + 1 < tb.L && (int)blockIdx.x >= tb.blk0[l + 1]) ++l;
  const int j = (int)blockIdx.x - tb.blk0[l];
  const int nt = (tb.T[l] + kLpT - 1) / kLpT;
  const int ct = j % tb.tiles_c, tt = (j / tb.tiles_c) % nt;
  const long long b = j / (tb.tiles_c * nt);
  const int T = tb.T[l], c0 = ct * 64, t0 = tt * kLpT;
  const float* __restrict__ pl = tb.pos[l] + b * tb.sb[l];
  if (tb.sc1[l]) {  // element (c, t) at t N + c: 64 c-lanes x 4 t-rows, coalesced along c
    const int cx = threadIdx.x & 63, ry = threadIdx.x >> 6;
#pragma unroll
    for (int i = 0; i < kLpT / 4; ++i) {
      const int c = c0 + cx, t = t0 + ry + 4 * i;
      tile[cx][ry + 4 * i] = (c < N && t < T) ? pl[(long long)t * N + c] : 0.f;
    }
  } else {  // element (c, t) at c T + t: 32 t-lanes x 8 c-rows, coalesced along t
    const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int c = c0 + ty + 8 * i, t = t0 + tx;
      tile[ty + 8 * i][tx] = (c < N && t < T) ? pl[(long long)c * T + t] : 0.f;
    }
  }
  __syncthreads();
  const int cx = threadIdx.x & 63, ry = threadIdx.x >> 6;  // 64 c-lanes x 4 t-rows
  const int c = c0 + cx;
  const float e = c < N ? emb[(long long)l * N + c] : 0.f;
  float* __restrict__ ob = out + (b * S + tb.start[l]) * (long long)N;
#pragma unroll
  for (int i = 0; i < kLpT / 4; ++i) {
    const int tl = ry + 4 * i, t = t0 + tl;
    if (c < N && t < T) ob[(long long)t * N + c] = tile[cx][tl] + e;
  }
}

constexpr int kLcRows = 64;  // rows per colsum chunk (within one (level, b) segment)
// partial column sums of one chunk: 64 column lanes (float4) x 4 row lanes, fixed order
__global__ __launch_bounds__(256) void level_colsum_partial(const LevelTable tb, const float* __restrict__ g,
                                                            long long B, int N, long long S, float* __restrict__ part) {
  __shared__ float4 red[4][64];
  const int k = (int)blockIdx.y;
  int l = 0;
  while (l + 1 < tb.L && k >= tb.blk0[l + 1]) ++l;
  const int nch = (tb.T[l] + kLcRows - 1) / kLcRows;
  const int j = k - tb.blk0[l];
  const long long b = j / nch;
  const int r0 = (j % nch) * kLcRows;
  const int r1 = min(tb.T[l], r0 + kLcRows);
  const int cl = threadIdx.x & 63, rl = threadIdx.x >> 6;
  const int c = ((int)blockIdx.x * 64 + cl) * 4;
  float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
  if (c < N) {
    const float* __restrict__ gb = g + (b * S + tb.start[l]) * (long long)N + c;
    for (int r = r0 + rl; r < r1; r += 4) {
      const float4 v = *reinterpret_cast<const float4*>(gb + (long long)r * N);
      a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
    }
  }
  red[rl][cl] = a;
  __syncthreads();
  if (rl == 0 && c < N) {
    float4 t = red[0][cl];
#pragma unroll
    for (int i = 1; i < 4; ++i) {
      const float4 v = red[i][cl];
      t.x += v.x; t.y += v.y; t.z += v.z; t.w += v.w;
    }
    *reinterpret_cast<float4*>(part + (long long)k * N + c) = t;
  }
}

// out[l, c] (+)= sum over the level's chunks (4 chunk lanes x 64 columns a workgroup, fixed order)
__global__ __launch_bounds__(256) void level_colsum_final(const LevelTable tb, const float* __restrict__ part, int N,
                                                          float* __restrict__ out, int accumulate) {
  __shared__ float red[4][64];
  const int l = (int)blockIdx.y;
  const int cl = threadIdx.x & 63, kl = threadIdx.x >> 6;
  const int c = (int)blockIdx.x * 64 + cl;
  float a = 0.f;
  if (c < N)
    for (int k = tb.blk0[l] + kl; k < tb.blk0[l + 1]; k += 4) a += part[(long long)k * N + c];
  red[kl][cl] = a;
  __syncthreads();
  if (kl == 0 && c < N) {
    const float t = (red[0][cl] + red[1][cl]) + (red[2][cl] + red[3][cl]);
    out[(long long)l * N + c] = accumulate ? out[(long long)l * N + c] + t : t;
  }
}

// The whole level position embedding of a pyramid in one pass (models/modules/pyramid.py,
// pyramid_pos_flatten): for level l, clip b, position t with x = the count of non-padding positions
// in [0, t] of that level's mask (reference PositionEmbeddingVideoSine, embedding_layers.py:203-219:
// cumsum, normalised (x - 0.5) / (x_last + eps) * scale),
//   out[b, start_l + t, c]        = sin(x / dim_t[c]) (c even) or cos(x / dim_t[c]) (c odd), c < npf
//   out[b, start_l + t, npf + c]  = dur[b, c]                 (the duration embedding, every t)
// plus level_embed[l, :] (prepare_encoder_inputs, unimodal_deformable_transformer.py:90-134).  The
// reference's chain: ~15 kernels per level (cumsum, arange, pow, div, sin, cos, stack, duration
// Linear, compare, cat, permute) and the flatten.  fp32 with the reference's operation order (no
// contraction); dim_t is the module's own tensor.  One workgroup per (level, clip, 32 positions):
// the mask counts before the chunk and over the level are recounted per workgroup (T <= 2^24 bytes).
struct PosTable {
  const unsigned char* mask[kLpMaxL];  // (B, T_l) bool, non-zero = padding
  int T[kLpMaxL], start[kLpMaxL];
  int blk0[kLpMaxL + 1];
  int L;
};
constexpr int kPpRows = 32;
__global__ __launch_bounds__(256) void pyramid_pos_kernel(const PosTable tb, const float* __restrict__ dim_t,
                                                          const float* __restrict__ dur,
                                                          const float* __restrict__ emb, int npf, long long S,
                                                          int normalize, float scale, float eps,
                                                          float* __restrict__ out) {
#pragma clang fp contract(off)
  __shared__ int s_red[2][4];
  __shared__ float s_x[kPpRows];
  int l = 0;
  while (l + 1 < tb.L && (int)blockIdx.x >= tb.blk0[l + 1]) ++l;
  const int T = tb.T[l];
  const int nch = (T + kPpRows - 1) / kPpRows;
  const int j = (int)blockIdx.x - tb.blk0[l];
  const long long b = j / nch;
  const int r0 = (j % nch) * kPpRows;
  const unsigned char* __restrict__ m = tb.mask[l] + b * T;
  int before = 0, total = 0;
  for (int t = threadIdx.x; t < T; t += 256) {
    const int nm = m[t] == 0 ? 1 : 0;
    total += nm;
    before += t < r0 ? nm : 0;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    total += __shfl_xor(total, o);
    before += __shfl_xor(before, o);
  }
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    s_red[0][w] = before;
    s_red[1][w] = total;
  }
  __syncthreads();
  before = s_red[0][0] + s_red[0][1] + s_red[0][2] + s_red[0][3];
  total = s_red[1][0] + s_red[1][1] + s_red[1][2] + s_red[1][3];
  if (threadIdx.x < kPpRows) {
    const int r = r0 + (int)threadIdx.x;
    int c = before;
    for (int t = r0; t <= r && t < T; ++t) c += m[t] == 0 ? 1 : 0;
    float x = (float)c;  // (an exact integer, as the fp32 cumsum)
    if (normalize) x = ((x - 0.5f) / ((float)total + eps)) * scale;
    s_x[threadIdx.x] = x;
  }
  __syncthreads();
  const int C = 2 * npf;
  const int rows = min(kPpRows, T - r0);
  float* __restrict__ ob = out + (b * S + tb.start[l] + r0) * (long long)C;
  const float* __restrict__ el = emb + (long long)l * C;
  const float* __restrict__ db = dur + b * npf;
  for (int i = threadIdx.x; i < rows * C; i += 256) {
    const int r = i / C, c = i - r * C;
    float v;
    if (c < npf) {
      const float a = s_x[r] / dim_t[c];
      v = (c & 1) ? cosf(a) : sinf(a);
    } else {
      v = db[c - npf];
    }
    ob[(long long)r * C + c] = v + el[c];
  }
}

bool level_table(const int64_t* T, int64_t L, int64_t B, int64_t N, int rows_per_unit, int cols_per_unit,
                 LevelTable& tb) {
  if (L < 1 || L > kLpMaxL || B < 1 || N < 1) return false;
  tb.L = (int)L;
  tb.tiles_c = (int)((N + cols_per_unit - 1) / cols_per_unit);
  long long run = 0, blk = 0;
  for (int l = 0; l < L; ++l) {
    if (T[l] < 1 || T[l] > (1 << 24)) return false;
    tb.T[l] = (int)T[l];
    tb.start[l] = (int)run;
    tb.blk0[l] = (int)blk;
    run += T[l];
    blk += B * ((T[l] + rows_per_unit - 1) / rows_per_unit) * (cols_per_unit == 64 ? tb.tiles_c : 1);
    if (blk > (1LL << 30) || run > (1LL << 30)) return false;
  }
  tb.blk0[L] = (int)blk;
  return true;
}

// The augmented operands of value_proj.layer_values' bias-in-K GEMM (models/modules/value_proj.py):
// x_aug (k, ca) = [x | 1 | 0 ...] and w_aug (n, ca, co) = [W_i^T ; b_i ; 0 ...], each in ONE pass
// (against zeros + a strided copy + a column fill, and zeros + two stacks + two strided copies).
// One thread a 16-B chunk of an x_aug row (c % 8 == 0, ca % 8 == 0).
__global__ __launch_bounds__(kThreads) void augment_rows_kernel(const uint4* __restrict__ x, long long k, int cv,
                                                                int cav, uint4* __restrict__ out) {
  const long long i = (long long)blockIdx.x * kThreads + threadIdx.x;
  if (i >= k * cav) return;
  const long long r = i / cav;
  const int v = (int)(i - r * cav);
  uint4 o = make_uint4(0u, 0u, 0u, 0u);
  if (v < cv) o = x[r * cv + v];
  else if (v == cv) o.x = 0x3F80u;  // bf16 1.0 in the chunk's first element
  out[i] = o;
}

// w_aug[i][j][o] = j < c ? w[i][o][j] : (j == c ? b[i][o] : 0): one thread an output element (bf16;
// the (n x ca x co) operand is at most a few MB)
__global__ __launch_bounds__(kThreads) void augment_weights_kernel(const uint16_t* __restrict__ w,
                                                                   const uint16_t* __restrict__ b, int n, int c,
                                                                   int ca, int co, uint16_t* __restrict__ out) {
  const long long e = (long long)blockIdx.x * kThreads + threadIdx.x;
  if (e >= (long long)n * ca * co) return;
  const int o = (int)(e % co);
  const long long ij = e / co;
  const int j = (int)(ij % ca), i = (int)(ij / ca);
  uint16_t v = 0;
  if (j < c) v = w[((long long)i * co + o) * c + j];
  else if (j == c) v = b[(long long)i * co + o];
  out[e] = v;
}
}  // namespace

extern "C" {

int mfl_relu_dropout_forward(const void* x, int64_t n, float p_drop, const int64_t* seed, void* out, void* stream) {
  g_err[0] = 0;
  if (!args_ok("mfl_relu_dropout_forward", n, x, out, out, p_drop)) return 1;
  if (n == 0) return 0;
  const long long nvec = n / 8;
  const uint32_t thresh = (uint32_t)fminf(p_drop * 65536.f + 0.5f, 65536.f);  // keep iff 16-bit draw >= p * 2^16
  const float scale = seed ? 1.f / (1.f - p_drop) : 1.f;
  hipLaunchKernelGGL(relu_dropout_fwd, dim3(grid_for(nvec)), dim3(kThreads), 0, static_cast<hipStream_t>(stream),
                     static_cast<const uint4*>(x), nvec, seed, thresh, scale, static_cast<uint4*>(out));
  return status("forward");
}

int mfl_relu_dropout_backward(const void* dy, const void* out, int64_t n, float p_drop, int dropped, void* dx,
                              void* stream) {
  g_err[0] = 0;
  if (!args_ok("mfl_relu_dropout_backward", n, dy, out, dx, p_drop)) return 1;
  if (n == 0) return 0;
  const long long nvec = n / 8;
  const float scale = dropped ? 1.f / (1.f - p_drop) : 1.f;
  hipLaunchKernelGGL(relu_dropout_bwd, dim3(grid_for(nvec)), dim3(kThreads), 0, static_cast<hipStream_t>(stream),
                     static_cast<const uint4*>(dy), static_cast<const uint4*>(out), nvec, scale,
                     static_cast<uint4*>(dx));
  return status("backward");
}

int mfl_gelu_dropout_forward(const void* x, int64_t n, float p_drop, const int64_t* seed, void* out, void* stream) {
  g_err[0] = 0;
  if (!args_ok("mfl_gelu_dropout_forward", n, x, out, out, p_drop)) return 1;
  if (n == 0) return 0;
  const long long nvec = n / 8;
  const uint32_t thresh = (uint32_t)fminf(p_drop * 65536.f + 0.5f, 65536.f);
  const float scale = seed ? 1.f / (1.f - p_drop) : 1.f;
  hipLaunchKernelGGL(gelu_dropout_fwd, dim3(grid_for(nvec)), dim3(kThreads), 0, static_cast<hipStream_t>(stream),
                     static_cast<const uint4*>(x), nvec, seed, thresh, scale, static_cast<uint4*>(out));
  return status("gelu forward");
}

int mfl_gelu_dropout_backward(const void* dy, const void* x, int64_t n, float p_drop, const int64_t* seed, void* dx,
                              void* stream) {
  g_err[0] = 0;
  if (!args_ok("mfl_gelu_dropout_backward", n, dy, x, dx, p_drop)) return 1;
  if (n == 0) return 0;
  const long long nvec = n / 8;
  const uint32_t thresh = (uint32_t)fminf(p_drop * 65536.f + 0.5f, 65536.f);
  const float scale = seed ? 1.f / (1.f - p_drop) : 1.f;
  hipLaunchKernelGGL(gelu_dropout_bwd, dim3(grid_for(nvec)), dim3(kThreads), 0, static_cast<hipStream_t>(stream),
                     static_cast<const uint4*>(dy), static_cast<const uint4*>(x), nvec, seed, thresh, scale,
                     static_cast<uint4*>(dx));
  return status("gelu backward");
}

int mfl_word_prob_backward(const float* probs, const int64_t* words, const float* coef, int64_t rows, int64_t vocab,
                           void* dx, void* stream) {
  g_err[0] = 0;
  if (rows < 0 || vocab <= 0 || vocab % 4 != 0 || (rows > 0 && (!probs || !words || !coef || !dx))) {
    snprintf(g_err, sizeof(g_err), "mfl_word_prob_backward: bad arguments (vocab %% 4 == 0, non-null buffers)");
    return 1;
  }
  if (rows == 0) return 0;
  hipLaunchKernelGGL(word_prob_bwd, dim3((unsigned)rows), dim3(kThreads), 0, static_cast<hipStream_t>(stream),
                     reinterpret_cast<const float4*>(probs), words, coef, (int)(vocab / 4), static_cast<uint2*>(dx));
  return status("word prob backward");
}

size_t mfl_relu_dropout_colsum_workspace_bytes(int64_t rows, int64_t cols) {
  if (rows <= 0 || cols <= 0) return 0;
  const int rpb = rd_rows_per_block(rows, cols / 8);
  return (size_t)((rows + rpb - 1) / rpb) * (size_t)cols * sizeof(float);
}

int mfl_relu_dropout_backward_colsum(const void* dy, const void* out, int64_t rows, int64_t cols, float p_drop,
                                     int dropped, void* dx, float* colsum, void* workspace, void* stream) {
  g_err[0] = 0;
  if (rows < 0 || cols <= 0 || cols % 8 != 0 || cols / 8 > 65535LL * kThreads || rows / kRdRows >= (1LL << 31)) {
    snprintf(g_err, sizeof(g_err), "mfl_relu_dropout_backward_colsum: cols must be a positive multiple of 8");
    return 1;
  }
  if (!args_ok("mfl_relu_dropout_backward_colsum", rows * cols, dy, out, dx, p_drop)) return 1;
  if (!colsum || (rows > 0 && !workspace)) {
    snprintf(g_err, sizeof(g_err), "mfl_relu_dropout_backward_colsum: null colsum / workspace");
    return 1;
  }
  hipStream_t st = static_cast<hipStream_t>(stream);
  const float scale = dropped ? 1.f / (1.f - p_drop) : 1.f;
  const int cvec = (int)(cols / 8);
  const int rpb = rd_rows_per_block(rows, cvec);
  const int bt = rpb == kRdRows ? kThreads : 64;
  const long long groups = (rows + rpb - 1) / rpb;
  if (groups > 0) {
    hipLaunchKernelGGL(relu_dropout_bwd_colsum, dim3((unsigned)groups, (unsigned)((cvec + bt - 1) / bt)), dim3(bt), 0,
                       st, static_cast<const uint4*>(dy), static_cast<const uint4*>(out), (long long)rows, cvec, rpb,
                       scale, static_cast<uint4*>(dx), static_cast<float*>(workspace));
    int rc;
    if ((rc = status("backward (column sums)"))) return rc;
  }
  hipLaunchKernelGGL(relu_dropout_colsum_final, dim3((unsigned)((cols + 63) / 64)), dim3(1024), 0, st,
                     static_cast<const float*>(workspace), (int)groups, (int)cols, colsum);
  return status("backward (column sums, final)");
}

int mfl_augment_rows(const void* x, int64_t k, int64_t c, int64_t ca, void* out, void* stream) {
  g_err[0] = 0;
  if (k < 0 || c <= 0 || ca <= c || c % 8 || ca % 8 || !x || !out || ((uintptr_t)x & 15u) || ((uintptr_t)out & 15u) ||
      k * (ca / 8) >= (1LL << 40)) {
    snprintf(g_err, sizeof(g_err), "mfl_augment_rows: bad arguments (c %% 8 == 0, ca %% 8 == 0, ca > c, 16-B aligned)");
    return 1;
  }
  const long long total = k * (ca / 8);
  if (total == 0) return 0;
  hipLaunchKernelGGL(augment_rows_kernel, dim3((unsigned)((total + kThreads - 1) / kThreads)), dim3(kThreads), 0,
                     static_cast<hipStream_t>(stream), static_cast<const uint4*>(x), k, (int)(c / 8), (int)(ca / 8),
                     static_cast<uint4*>(out));
  return status("augment rows");
}

int mfl_augment_weights(const void* w, const void* b, int64_t n, int64_t c, int64_t ca, int64_t co, void* out,
                        void* stream) {
  g_err[0] = 0;
  if (n < 0 || c <= 0 || ca <= c || co <= 0 || !w || !b || !out || n * ca * co >= (1LL << 31)) {
    snprintf(g_err, sizeof(g_err), "mfl_augment_weights: bad arguments (ca > c, n * ca * co < 2^31)");
    return 1;
  }
  const long long total = n * ca * co;
  if (total == 0) return 0;
  hipLaunchKernelGGL(augment_weights_kernel, dim3((unsigned)((total + kThreads - 1) / kThreads)), dim3(kThreads), 0,
                     static_cast<hipStream_t>(stream), static_cast<const uint16_t*>(w),
                     static_cast<const uint16_t*>(b), (int)n, (int)c, (int)ca, (int)co, static_cast<uint16_t*>(out));
  return status("augment weights");
}

int mfl_zero_masked_rows_batched(void* x, int64_t nbatch, int64_t rows, int64_t row_bytes, const uint8_t* mask,
                                 void* stream) {
  g_err[0] = 0;
  if (nbatch < 0 || rows < 0 || row_bytes <= 0 || row_bytes % 16 != 0 || row_bytes / 16 > (1 << 30)) {
    snprintf(g_err, sizeof(g_err), "mfl_zero_masked_rows: rows >= 0 and row_bytes a positive multiple of 16 needed");
    return 1;
  }
  if (rows == 0 || nbatch == 0) return 0;
  if (!x || !mask || ((uintptr_t)x & 15u)) {
    snprintf(g_err, sizeof(g_err), "mfl_zero_masked_rows: null pointer or x not 16-byte aligned");
    return 1;
  }
  const long long total = nbatch * rows;
  const long long blocks = (total + kThreads - 1) / kThreads;  // 64 rows a wave
  hipLaunchKernelGGL(zero_masked_rows_kernel, dim3((unsigned)blocks), dim3(kThreads), 0,
                     static_cast<hipStream_t>(stream), static_cast<uint4*>(x), total, (int)(row_bytes / 16), mask,
                     (long long)rows);
  return status("zero masked rows");
}

int mfl_zero_masked_rows(void* x, int64_t rows, int64_t row_bytes, const uint8_t* mask, void* stream) {
  return mfl_zero_masked_rows_batched(x, 1, rows, row_bytes, mask, stream);
}

int mfl_gather_keep_backward(const void* grad, const int64_t* index, const void* keep, int64_t n, int64_t B, int64_t K,
                             int64_t d, void* grad_src, float* bias_part, void* stream) {
  g_err[0] = 0;
  if (n < 0 || B < 0 || K < 0 || d <= 0 || d % 8 || d > 512 || (n > 0 && (!grad || !index || !keep)) ||
      (B > 0 && K > 0 && (!grad_src || !bias_part)) || ((uintptr_t)grad & 15u) || ((uintptr_t)grad_src & 15u) ||
      n > (1 << 20) || B > (1 << 20)) {
    snprintf(g_err, sizeof(g_err), "mfl_gather_keep_backward: bad arguments (d %% 8 == 0, d <= 512, 16-B aligned)");
    return 1;
  }
  if (K == 0) return 0;
  hipLaunchKernelGGL(gather_keep_bwd_kernel, dim3((unsigned)K), dim3(256), 0, static_cast<hipStream_t>(stream),
                     static_cast<const uint16_t*>(grad), reinterpret_cast<const long long*>(index),
                     static_cast<const uint8_t*>(keep), (int)n, (int)B, (int)K, (int)d,
                     static_cast<uint16_t*>(grad_src), bias_part);
  return status("gather-keep backward");
}

int mfl_level_pos_flatten(const float* const* pos, const int64_t* T, int64_t L, int64_t B, int64_t N,
                          const float* level_embed, float* out, void* stream) {
  return mfl_level_pos_flatten_ex(pos, nullptr, T, L, B, N, level_embed, out, stream);
}

int mfl_level_pos_flatten_ex(const float* const* pos, const int* channels_last, const int64_t* T, int64_t L,
                             int64_t B, int64_t N, const float* level_embed, float* out, void* stream) {
  g_err[0] = 0;
  LevelTable tb{};
  if (!pos || !T || !level_embed || !out || !level_table(T, L, B, N, kLpT, 64, tb)) {
    snprintf(g_err, sizeof(g_err), "mfl_level_pos_flatten: bad arguments (1 <= L <= %d levels, B, N >= 1)", kLpMaxL);
    return 1;
  }
  for (int l = 0; l < L; ++l) {
    if (!pos[l]) {
      snprintf(g_err, sizeof(g_err), "mfl_level_pos_flatten: null level pointer");
      return 1;
    }
    tb.pos[l] = pos[l];
    tb.sb[l] = N * T[l];
    tb.sc1[l] = channels_last != nullptr && channels_last[l] ? 1 : 0;
  }
  long long S = 0;
  for (int l = 0; l < L; ++l) S += T[l];
  hipLaunchKernelGGL(level_pos_flatten_kernel, dim3((unsigned)tb.blk0[L]), dim3(256), 0, static_cast<hipStream_t>(stream),
                     tb, level_embed, (long long)B, (int)N, S, out);
  return status("level pos flatten");
}

size_t mfl_level_colsum_workspace_bytes(const int64_t* T, int64_t L, int64_t B, int64_t N) {
  LevelTable tb{};
  if (!T || !level_table(T, L, B, N, kLcRows, 256, tb)) return 0;
  return (size_t)tb.blk0[L] * (size_t)N * sizeof(float);
}

int mfl_level_colsum(const float* g, const int64_t* T, int64_t L, int64_t B, int64_t N, float* out, int accumulate,
                     void* workspace, void* stream) {
  g_err[0] = 0;
  LevelTable tb{};
  if (!g || !T || !out || !workspace || N % 4 != 0 || ((uintptr_t)g & 15u) || ((uintptr_t)workspace & 15u) ||
      !level_table(T, L, B, N, kLcRows, 256, tb)) {
    snprintf(g_err, sizeof(g_err),
             "mfl_level_colsum: bad arguments (1 <= L <= %d, N %% 4 == 0, 16-B aligned g and workspace)", kLpMaxL);
    return 1;
  }
  long long S = 0;
  for (int l = 0; l < L; ++l) S += T[l];
  hipStream_t st = static_cast<hipStream_t>(stream);
  auto* part = static_cast<float*>(workspace);
  hipLaunchKernelGGL(level_colsum_partial, dim3((unsigned)((N / 4 + 63) / 64), (unsigned)tb.blk0[L]), dim3(256), 0, st,
                     tb, g, (long long)B, (int)N, S, part);
  int rc;
  if ((rc = status("level colsum partial"))) return rc;
  hipLaunchKernelGGL(level_colsum_final, dim3((unsigned)((N + 63) / 64), (unsigned)L), dim3(256), 0, st, tb, part,
                     (int)N, out, accumulate);
  return status("level colsum final");
}

int mfl_pyramid_pos_flatten(const uint8_t* const* masks, const int64_t* T, int64_t L, int64_t B, int64_t npf,
                            const float* dim_t, const float* dur, const float* level_embed, int normalize,
                            float scale, float eps, float* out, void* stream) {
  g_err[0] = 0;
  if (!masks || !T || !dim_t || !dur || !level_embed || !out || L < 1 || L > kLpMaxL || B < 1 || npf < 1 ||
      npf > (1 << 16)) {
    snprintf(g_err, sizeof(g_err), "mfl_pyramid_pos_flatten: bad arguments (1 <= L <= %d)", kLpMaxL);
    return 1;
  }
  PosTable tb{};
  tb.L = (int)L;
  long long run = 0, blk = 0;
  for (int l = 0; l < L; ++l) {
    if (!masks[l] || T[l] < 1 || T[l] > (1 << 24)) {
      snprintf(g_err, sizeof(g_err), "mfl_pyramid_pos_flatten: bad level %d", l);
      return 1;
    }
    tb.mask[l] = masks[l];
    tb.T[l] = (int)T[l];
    tb.start[l] = (int)run;
    tb.blk0[l] = (int)blk;
    run += T[l];
    blk += B * ((T[l] + kPpRows - 1) / kPpRows);
  }
  if (blk > (1LL << 31) - 1) {
    snprintf(g_err, sizeof(g_err), "mfl_pyramid_pos_flatten: too many rows");
    return 1;
  }
  tb.blk0[L] = (int)blk;
  hipLaunchKernelGGL(pyramid_pos_kernel, dim3((unsigned)blk), dim3(256), 0, static_cast<hipStream_t>(stream), tb, dim_t,
                     dur, level_embed, (int)npf, run, normalize, scale, eps, out);
  return status("pyramid pos flatten");
}

const char* mfl_relu_dropout_last_error(void) { return g_err; }

}  // extern "C"
