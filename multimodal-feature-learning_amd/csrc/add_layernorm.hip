// Residual add + LayerNorm of the deformable transformer layers, forward and backward
// (reference unimodal_deformable_transformer.py:238-249 / 362-373: norm(x + dropout(y)), and the
// same pattern in the multimodal and sparse layers).  Under bf16 autocast the reference runs an
// fp32 add of the residual stream and the 16-bit branch output, then an fp32 LayerNorm; the
// backward is LayerNorm's input-gradient and gamma/beta kernels plus a cast of the gradient back
// to the branch's 16-bit dtype.  Here:
//   forward : z = r + y and out = (z - mean) * rstd * gamma + beta in one pass; mean / rstd kept;
//   backward: dz from (dout, z recomputed from r and y), written once as dr (r's dtype) and dy
//             (y's dtype); per-block gamma / beta partials, summed by a second small kernel.
// One wave per row, d % 256 == 0 and d <= 1024 (4 consecutive elements per lane per 256-wide
// chunk): the row stays in registers between the statistics and the output.
#include <hip/hip_runtime.h>

#include <algorithm>

#include <cstdint>
#include <cstdio>

#include "../../include/add_layernorm.h"

namespace {

thread_local char g_err[256];

constexpr int kWaves = 4;     // rows in flight per block (one per wave)
constexpr int kBwdRows = 16;  // rows per backward block (kWaves waves x 4 rows): gamma/beta partials
// Short calls (the decoder's 800 query rows) take one row per wave instead: 16-row blocks gave them
// 50 workgroups, each wave walking 4 dependent rows (14 us per call); 4-row blocks give 200.
constexpr int kBwdRowsShort = 4;
constexpr long long kBwdShortMax = 4096;
inline int bwd_rows_per_block(long long rows) { return rows <= kBwdShortMax ? kBwdRowsShort : kBwdRows; }

template <typename T> struct Vec4;
template <> struct Vec4<float> {
  __device__ static void load(const float* p, float (&v)[4]) {
    const float4 x = *reinterpret_cast<const float4*>(p);
    v[0] = x.x; v[1] = x.y; v[2] = x.z; v[3] = x.w;
  }
  __device__ static void store(float* p, const float (&v)[4]) {
    *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
  }
};
template <> struct Vec4<uint16_t> {  // bf16
  __device__ static void load(const uint16_t* p, float (&v)[4]) {
    const uint2 x = *reinterpret_cast<const uint2*>(p);
    v[0] = __uint_as_float(x.x << 16); v[1] = __uint_as_float(x.x & 0xffff0000u);
    v[2] = __uint_as_float(x.y << 16); v[3] = __uint_as_float(x.y & 0xffff0000u);
  }
  __device__ static uint32_t rne(float f) {  // round to nearest even, NaN kept quiet
    const uint32_t u = __float_as_uint(f);
    if ((u & 0x7fffffffu) > 0x7f800000u) return (u >> 16) | 0x40u;
    return (u + 0x7fffu + ((u >> 16) & 1u)) >> 16;
  }
  __device__ static void store(uint16_t* p, const float (&v)[4]) {
    *reinterpret_cast<uint2*>(p) = make_uint2(rne(v[0]) | (rne(v[1]) << 16), rne(v[2]) | (rne(v[3]) << 16));
  }
};

__device__ __forceinline__ float wave_sum(float x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
  return x;
}

// Dropout of the branch (nn.Dropout(p) in training, reference :238/:249): element e of the call is
// kept when a 64-bit mix of (seed, e) clears p; the backward regenerates the same bits from the
// same device-side seed (no mask in HBM).  Kept values are scaled by 1 / (1 - p) and, for a bf16
// branch, rounded to bf16 as ATen's dropout of a bf16 tensor is.
struct Drop {
  const int64_t* seed_ptr;  // null: no dropout
  float p, scale;
};

__device__ __forceinline__ uint32_t drop_bits(uint64_t seed, uint64_t e) {
  uint64_t x = seed * 0x9E3779B97F4A7C15ull + e;
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ull;
  x ^= x >> 33;
  return (uint32_t)x;
}

template <typename YT>
__device__ __forceinline__ void drop4(float (&b)[4], uint64_t seed, uint32_t thresh, float scale, long long e0,
                                      float (&keep)[4]) {
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    keep[k] = (drop_bits(seed, (uint64_t)(e0 + k)) >> 8) >= thresh ? scale : 0.f;
    float v = b[k] * keep[k];
    if (sizeof(YT) == 2) v = __uint_as_float(Vec4<uint16_t>::rne(v) << 16);
    b[k] = v;
  }
}

__device__ __forceinline__ uint32_t drop_thresh(float p) {  // keep iff 24-bit draw >= p * 2^24
  return (uint32_t)fminf(p * 16777216.f, 16777216.f);
}

// z = r + y: with both operands bf16 the reference's autocast add is a bf16 op (its result is
// rounded to bf16 before the fp32 LayerNorm); otherwise the add is fp32.
template <typename RT, typename YT>
__device__ __forceinline__ float add_z(float a, float b) {
  const float z = a + b;
  if (sizeof(RT) == 2 && sizeof(YT) == 2) return __uint_as_float(Vec4<uint16_t>::rne(z) << 16);
  return z;
}

template <typename RT, typename YT, int CH>
__global__ __launch_bounds__(kWaves * 64) void add_ln_fwd(const RT* __restrict__ r, const YT* __restrict__ y,
                                                         const float* __restrict__ gamma,
                                                         const float* __restrict__ beta, long long rows, int d,
                                                         float eps, float* __restrict__ out,
                                                         float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                         uint16_t* __restrict__ out16, const float* __restrict__ pos,
                                                         uint16_t* __restrict__ q16, Drop drop) {
  const int lane = threadIdx.x & 63;
  const uint64_t seed = drop.seed_ptr ? (uint64_t)drop.seed_ptr[0] : 0;
  const uint32_t thresh = drop_thresh(drop.p);
  // (the wave index as a scalar: row, its bounds test and the row's base address stay scalar)
  const long long row = (long long)blockIdx.x * kWaves + __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  if (row >= rows) return;  // wave-uniform
  const long long base = row * d;
  float z[CH][4];
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    const int col = c * 256 + lane * 4;
    float a[4], b[4];
    Vec4<RT>::load(r + base + col, a);
    Vec4<YT>::load(y + base + col, b);
    if (drop.seed_ptr) {
      float keep[4];
      drop4<YT>(b, seed, thresh, drop.scale, base + col, keep);
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      z[c][k] = add_z<RT, YT>(a[k], b[k]);
      s += z[c][k];
    }
  }
  const float mean = wave_sum(s) / (float)d;
  float q = 0.f;
#pragma unroll
  for (int c = 0; c < CH; ++c)
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float t = z[c][k] - mean;
      q += t * t;
    }
  const float rstd = rsqrtf(wave_sum(q) / (float)d + eps);
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    const int col = c * 256 + lane * 4;
    float g[4], bb[4], o[4];
    Vec4<float>::load(gamma + col, g);
    Vec4<float>::load(beta + col, bb);
#pragma unroll
    for (int k = 0; k < 4; ++k) o[k] = (z[c][k] - mean) * rstd * g[k] + bb[k];
    Vec4<float>::store(out + base + col, o);
    if (out16) Vec4<uint16_t>::store(out16 + base + col, o);  // the bf16 operand of the next GEMM
    if (q16) {  // bf16(out + pos): the next MSDA query, rounded once from fp32 as autocast would
      float p[4];
      Vec4<float>::load(pos + base + col, p);
#pragma unroll
      for (int k = 0; k < 4; ++k) p[k] += o[k];
      Vec4<uint16_t>::store(q16 + base + col, p);
    }
  }
  if (lane == 0) {
    mean_out[row] = mean;
    rstd_out[row] = rstd;
  }
}

template <typename RT, typename YT, int CH, int RPB>
__global__ __launch_bounds__(kWaves * 64) void add_ln_bwd(
    const float* __restrict__ dout, const RT* __restrict__ r, const YT* __restrict__ y,
    const float* __restrict__ gamma, const float* __restrict__ mean_in, const float* __restrict__ rstd_in,
    long long rows, int d, RT* __restrict__ dr, YT* __restrict__ dy, float* __restrict__ part,
    const uint16_t* __restrict__ dout16, const uint16_t* __restrict__ dq16, float* __restrict__ dpos, Drop drop,
    int dpos_acc, int ysum) {
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));  // (scalar)
  const uint64_t seed = drop.seed_ptr ? (uint64_t)drop.seed_ptr[0] : 0;
  const uint32_t thresh = drop_thresh(drop.p);
  float dg[CH][4], db[CH][4], ys[CH][4];
#pragma unroll
  for (int c = 0; c < CH; ++c)
#pragma unroll
    for (int k = 0; k < 4; ++k) dg[c][k] = db[c][k] = ys[c][k] = 0.f;
  for (int i = 0; i < RPB / kWaves; ++i) {
    const long long row = (long long)blockIdx.x * RPB + i * kWaves + wave;
    if (row >= rows) break;  // wave-uniform
    const long long base = row * d;
    const float mean = mean_in[row], rstd = rstd_in[row];
    float xh[CH][4], g[CH][4], kp[CH][4];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const int col = c * 256 + lane * 4;
      float a[4], b[4], go[4] = {0.f, 0.f, 0.f, 0.f}, ga[4];
      Vec4<RT>::load(r + base + col, a);
      Vec4<YT>::load(y + base + col, b);
      if (drop.seed_ptr) {
        drop4<YT>(b, seed, thresh, drop.scale, base + col, kp[c]);
      } else {
#pragma unroll
        for (int k = 0; k < 4; ++k) kp[c][k] = 1.f;
      }
      // d out = its fp32 gradient + the bf16 copy's + the (out + pos) copy's, summed in fp32
      if (dout) Vec4<float>::load(dout + base + col, go);
      if (dout16) {
        float t[4];
        Vec4<uint16_t>::load(dout16 + base + col, t);
#pragma unroll
        for (int k = 0; k < 4; ++k) go[k] += t[k];
      }
      if (dq16) {
        float t[4];
        Vec4<uint16_t>::load(dq16 + base + col, t);
        if (dpos) {
          if (dpos_acc) {  // the gradient of a pos shared by several layers, summed in place
            float o[4];
            Vec4<float>::load(dpos + base + col, o);
            float sum[4] = {o[0] + t[0], o[1] + t[1], o[2] + t[2], o[3] + t[3]};
            Vec4<float>::store(dpos + base + col, sum);
          } else {
            Vec4<float>::store(dpos + base + col, t);
          }
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) go[k] += t[k];
      }
      Vec4<float>::load(gamma + col, ga);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        xh[c][k] = (add_z<RT, YT>(a[k], b[k]) - mean) * rstd;
        g[c][k] = go[k] * ga[k];
        s1 += g[c][k];
        s2 += g[c][k] * xh[c][k];
        dg[c][k] += go[k] * xh[c][k];
        db[c][k] += go[k];
      }
    }
    const float m1 = wave_sum(s1) / (float)d, m2 = wave_sum(s2) / (float)d;
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const int col = c * 256 + lane * 4;
      float dx[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) dx[k] = rstd * (g[c][k] - m1 - xh[c][k] * m2);
      Vec4<RT>::store(dr + base + col, dx);
#pragma unroll
      for (int k = 0; k < 4; ++k) dx[k] *= kp[c][k];
      Vec4<YT>::store(dy + base + col, dx);
      if (ysum) {  // column sums of dy as stored (the producing Linear's bias gradient)
#pragma unroll
        for (int k = 0; k < 4; ++k)
          ys[c][k] += sizeof(YT) == 2 ? __uint_as_float(Vec4<uint16_t>::rne(dx[k]) << 16) : dx[k];
      }
    }
  }
  // gamma / beta partials of the block: waves meet in LDS, fixed order
  __shared__ float red[kWaves][3][CH * 256];
  const int np = ysum ? 3 : 2;  // partial rows per block: dgamma, dbeta (, dy column sums)
#pragma unroll
  for (int c = 0; c < CH; ++c)
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      red[wave][0][c * 256 + lane * 4 + k] = dg[c][k];
      red[wave][1][c * 256 + lane * 4 + k] = db[c][k];
      red[wave][2][c * 256 + lane * 4 + k] = ys[c][k];
    }
  __syncthreads();
  for (int j = threadIdx.x; j < np * d; j += kWaves * 64) {
    const int which = j / d, col = j - which * d;
    float t = 0.f;
#pragma unroll
    for (int w = 0; w < kWaves; ++w) t += red[w][which][col];
    part[(long long)blockIdx.x * np * d + j] = t;
  }
}

// dgamma / dbeta = sum over the backward blocks' partials (16 groups x 64 columns per block)
__global__ __launch_bounds__(1024) void add_ln_param_final(const float* __restrict__ part, int nblk, int d2,
                                                          float* __restrict__ dgamma, float* __restrict__ dbeta,
                                                          float* __restrict__ dysum, int d) {
  __shared__ float red[16][64];
  const int c_l = threadIdx.x & 63, grp = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + c_l;
  // eight independent chains (the encoder backward has 960 partial rows: a single dependent chain
  // of 60 L2 loads per thread made this 24-workgroup kernel latency-bound, ~20 us; four chains
  // ~5.5 us a call); fixed order
  float sc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (c < d2) {
    int k = grp;
    for (; k + 112 < nblk; k += 128) {
#pragma unroll
      for (int u = 0; u < 8; ++u) sc[u] += part[(long long)(k + 16 * u) * d2 + c];
    }
    for (; k < nblk; k += 16) sc[0] += part[(long long)k * d2 + c];
  }
  red[grp][c_l] = ((sc[0] + sc[1]) + (sc[2] + sc[3])) + ((sc[4] + sc[5]) + (sc[6] + sc[7]));
  __syncthreads();
  if (grp == 0 && c < d2) {
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) t += red[i][c_l];
    if (c < d) dgamma[c] = t;
    else if (c < 2 * d) dbeta[c - d] = t;
    else dysum[c - 2 * d] = t;
  }
}

// The carried operands of an encoder's first layer (models/modules/add_norm.py, carry_entry): the
// layer reads src (fp32) as its residual, bf16(src) as the value projection's input and
// bf16(src + pos) as the query (reference with_pos_embed, unimodal_deformable_transformer.py:241;
// autocast casts each at its Linear).  One pass writes both bf16 copies; its backward sums the
// three gradients of src in one pass (dr + dv16 + dq16, fp32) and dq16 into pos's gradient (or
// its shared accumulator).  8 elements a thread.
__global__ __launch_bounds__(256) void carry_entry_fwd(const float* __restrict__ src, const float* __restrict__ pos,
                                                       long long n8, uint16_t* __restrict__ v16,
                                                       uint16_t* __restrict__ q16) {
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n8; i += (long long)gridDim.x * 256) {
    float a[4], b[4], pa[4], pb[4];
    Vec4<float>::load(src + 8 * i, a);
    Vec4<float>::load(src + 8 * i + 4, b);
    if (v16) {
      Vec4<uint16_t>::store(v16 + 8 * i, a);
      Vec4<uint16_t>::store(v16 + 8 * i + 4, b);
    }
    if (pos) {
      Vec4<float>::load(pos + 8 * i, pa);
      Vec4<float>::load(pos + 8 * i + 4, pb);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        pa[k] = a[k] + pa[k];
        pb[k] = b[k] + pb[k];
      }
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        pa[k] = a[k];
        pb[k] = b[k];
      }
    }
    Vec4<uint16_t>::store(q16 + 8 * i, pa);
    Vec4<uint16_t>::store(q16 + 8 * i + 4, pb);
  }
}

__global__ __launch_bounds__(256) void carry_entry_bwd(const float* __restrict__ dr, const uint16_t* __restrict__ dv16,
                                                       const uint16_t* __restrict__ dq16, long long n4,
                                                       float* __restrict__ dsrc, float* __restrict__ dpos,
                                                       int dpos_accumulate) {
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n4; i += (long long)gridDim.x * 256) {
    float s[4] = {0.f, 0.f, 0.f, 0.f}, v[4], q[4] = {0.f, 0.f, 0.f, 0.f};
    if (dr) Vec4<float>::load(dr + 4 * i, s);
    if (dv16) {
      Vec4<uint16_t>::load(dv16 + 4 * i, v);
#pragma unroll
      for (int k = 0; k < 4; ++k) s[k] += v[k];
    }
    if (dq16) {
      Vec4<uint16_t>::load(dq16 + 4 * i, q);
#pragma unroll
      for (int k = 0; k < 4; ++k) s[k] += q[k];
    }
    Vec4<float>::store(dsrc + 4 * i, s);
    if (dpos) {
      if (dpos_accumulate) {
        float o[4];
        Vec4<float>::load(dpos + 4 * i, o);
#pragma unroll
        for (int k = 0; k < 4; ++k) q[k] = o[k] + q[k];
      }
      Vec4<float>::store(dpos + 4 * i, q);
    }
  }
}

// GroupNorm over channels-last rows (models/base_encoder.py, BaseEncoder's
// nn.GroupNorm(32, d_model) after each level's Conv1d; reference base_encoder.py:27-36): x (B, T, C)
// bf16 (the convolution GEMM's output), G groups of C / G consecutive channels, statistics over
// (T, C / G) per (b, g) in fp32 — ATen's group_norm on the (B, C, T) transpose, which autocast runs in
// fp32.  The normalised rows go straight into the encoder's flattened (B, S, C) fp32 input at the
// level's rows (no transpose copies, no cat) and, for the next level's convolution, as bf16.
// Lanes: C / 8 column lanes of 8 channels (one 16-B load; 8 | C / G, so a lane lies in one group) x
// 256 / (C / 8) row lanes; 32 rows a workgroup.
constexpr int kGnRows = 32;
__device__ __forceinline__ void load_bf16x8(const uint16_t* p, float (&v)[8]) {
  const uint4 u = *reinterpret_cast<const uint4*>(p);
  const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    v[2 * k] = __uint_as_float(w[k] << 16);
    v[2 * k + 1] = __uint_as_float(w[k] & 0xffff0000u);
  }
}
__device__ __forceinline__ void store_bf16x8(uint16_t* p, const float (&v)[8]) {
  uint4 u;
  u.x = Vec4<uint16_t>::rne(v[0]) | (Vec4<uint16_t>::rne(v[1]) << 16);
  u.y = Vec4<uint16_t>::rne(v[2]) | (Vec4<uint16_t>::rne(v[3]) << 16);
  u.z = Vec4<uint16_t>::rne(v[4]) | (Vec4<uint16_t>::rne(v[5]) << 16);
  u.w = Vec4<uint16_t>::rne(v[6]) | (Vec4<uint16_t>::rne(v[7]) << 16);
  *reinterpret_cast<uint4*>(p) = u;
}

// per-workgroup statistics of every group over the workgroup's rows: (mean, M2 = sum of squared
// deviations from that mean), two passes over the rows (the second from cache) — merged per (b, g)
// by gn_cl_apply (Chan et al.'s pairwise update), as robust as ATen's Welford moments when a group's
// mean is large against its spread (a one-pass E[x^2] - mean^2 cancels there)
__global__ __launch_bounds__(256) void gn_cl_stats(const uint16_t* __restrict__ x, int T, int C, int G, int nch,
                                                   float* __restrict__ part) {
  __shared__ float rs[256], s_m[128];
  const int blk = (int)blockIdx.x;
  const long long b = blk / nch;
  const int r0 = (blk % nch) * kGnRows, r1 = min(T, r0 + kGnRows);
  const int CL = C / 8, RL = 256 / CL;
  const int cl = (int)threadIdx.x % CL, rl = (int)threadIdx.x / CL;
  const int lpg = C / G / 8;
  const float nb = (float)(r1 - r0) * (float)(C / G);
  float sum = 0.f;
  for (int r = r0 + rl; r < r1; r += RL) {
    float v[8];
    load_bf16x8(x + ((b * T + r) * C + cl * 8), v);
#pragma unroll
    for (int k = 0; k < 8; ++k) sum += v[k];
  }
  rs[threadIdx.x] = sum;
  __syncthreads();
  if ((int)threadIdx.x < G) {
    const int g = (int)threadIdx.x;
    float a = 0.f;
    for (int r = 0; r < RL; ++r)
      for (int l = g * lpg; l < (g + 1) * lpg; ++l) a += rs[r * CL + l];
    s_m[g] = a / nb;
  }
  __syncthreads();
  const float m = s_m[cl / lpg];
  float sq = 0.f;
  for (int r = r0 + rl; r < r1; r += RL) {
    float v[8];
    load_bf16x8(x + ((b * T + r) * C + cl * 8), v);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float d = v[k] - m;
      sq += d * d;
    }
  }
  __syncthreads();
  rs[threadIdx.x] = sq;
  __syncthreads();
  if ((int)threadIdx.x < G) {
    const int g = (int)threadIdx.x;
    float q = 0.f;
    for (int r = 0; r < RL; ++r)
      for (int l = g * lpg; l < (g + 1) * lpg; ++l) q += rs[r * CL + l];
    part[((long long)blk * G + g) * 2] = s_m[g];
    part[((long long)blk * G + g) * 2 + 1] = q;
  }
}

// per (b, g) statistics from the partials, then out = x * (rstd gamma) + (beta - mean rstd gamma)
// (ATen's fused parameters) in fp32 into out32 (rows of the level, batch stride sb) and bf16 out16
__global__ __launch_bounds__(256) void gn_cl_apply(const uint16_t* __restrict__ x, const float* __restrict__ part,
                                                   const float* __restrict__ gamma, const float* __restrict__ beta,
                                                   int T, int C, int G, int nch, float eps, float* __restrict__ out32,
                                                   long long sb, uint16_t* __restrict__ out16,
                                                   float* __restrict__ mean_out, float* __restrict__ rstd_out) {
  __shared__ float s_mean[128], s_rstd[128];
  const int blk = (int)blockIdx.x;
  const long long b = blk / nch;
  if ((int)threadIdx.x < G) {
    const int g = (int)threadIdx.x;
    // merge the workgroups' (mean, M2): the mean weighted by rows, M2 += n_c (mean_c - mean)^2
    const float per = (float)(C / G);
    const float n = (float)T * per;
    float a = 0.f;
    for (int c = 0; c < nch; ++c) a += part[((b * nch + c) * G + g) * 2] * ((float)(min(T, (c + 1) * kGnRows) - c * kGnRows) * per);
    const float mean = a / n;
    float q = 0.f;
    for (int c = 0; c < nch; ++c) {
      const float nc = (float)(min(T, (c + 1) * kGnRows) - c * kGnRows) * per;
      const float d = part[((b * nch + c) * G + g) * 2] - mean;
      q += part[((b * nch + c) * G + g) * 2 + 1] + nc * d * d;
    }
    const float var = fmaxf(q / n, 0.f);
    const float rstd = 1.f / sqrtf(var + eps);
    s_mean[g] = mean;
    s_rstd[g] = rstd;
    if (blk % nch == 0) {
      mean_out[b * G + g] = mean;
      rstd_out[b * G + g] = rstd;
    }
  }
  __syncthreads();
  const int r0 = (blk % nch) * kGnRows, r1 = min(T, r0 + kGnRows);
  const int CL = C / 8, RL = 256 / CL;
  const int cl = (int)threadIdx.x % CL, rl = (int)threadIdx.x / CL;
  const int g = cl * 8 / (C / G);
  float sc[8], bi[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    sc[k] = s_rstd[g] * gamma[cl * 8 + k];
    bi[k] = -sc[k] * s_mean[g] + beta[cl * 8 + k];
  }
  for (int r = r0 + rl; r < r1; r += RL) {
    float v[8];
    load_bf16x8(x + ((b * T + r) * C + cl * 8), v);
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = v[k] * sc[k] + bi[k];
    float* o = out32 + (b * sb + (long long)r * C + cl * 8);
    *reinterpret_cast<float4*>(o) = make_float4(v[0], v[1], v[2], v[3]);
    *reinterpret_cast<float4*>(o + 4) = make_float4(v[4], v[5], v[6], v[7]);
    if (out16 != nullptr) store_bf16x8(out16 + ((b * T + r) * C + cl * 8), v);
  }
}

// backward partials per channel over one workgroup's rows: S1 = sum gt x, S0 = sum gt, gt = g32 + g16
__global__ __launch_bounds__(256) void gn_cl_bwd_partial(const float* __restrict__ g32, long long sb,
                                                         const uint16_t* __restrict__ g16,
                                                         const uint16_t* __restrict__ x, int T, int C, int nch,
                                                         float* __restrict__ part) {
  __shared__ float s1[256][8], s0[256][8];
  const int blk = (int)blockIdx.x;
  const long long b = blk / nch;
  const int r0 = (blk % nch) * kGnRows, r1 = min(T, r0 + kGnRows);
  const int CL = C / 8, RL = 256 / CL;
  const int cl = (int)threadIdx.x % CL, rl = (int)threadIdx.x / CL;
  float a1[8], a0[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) a1[k] = a0[k] = 0.f;
  for (int r = r0 + rl; r < r1; r += RL) {
    float xv[8], gt[8];
    load_bf16x8(x + ((b * T + r) * C + cl * 8), xv);
#pragma unroll
    for (int k = 0; k < 8; ++k) gt[k] = 0.f;
    if (g32 != nullptr) {
      const float* p = g32 + (b * sb + (long long)r * C + cl * 8);
      const float4 u = *reinterpret_cast<const float4*>(p), w = *reinterpret_cast<const float4*>(p + 4);
      gt[0] = u.x; gt[1] = u.y; gt[2] = u.z; gt[3] = u.w; gt[4] = w.x; gt[5] = w.y; gt[6] = w.z; gt[7] = w.w;
    }
    if (g16 != nullptr) {
      float h[8];
      load_bf16x8(g16 + ((b * T + r) * C + cl * 8), h);
#pragma unroll
      for (int k = 0; k < 8; ++k) gt[k] += h[k];
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      a1[k] += gt[k] * xv[k];
      a0[k] += gt[k];
    }
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    s1[threadIdx.x][k] = a1[k];
    s0[threadIdx.x][k] = a0[k];
  }
  __syncthreads();
  for (int c = (int)threadIdx.x; c < C; c += 256) {
    const int l = c / 8, k = c % 8;
    float t1 = 0.f, t0 = 0.f;
    for (int r = 0; r < RL; ++r) {
      t1 += s1[r * CL + l][k];
      t0 += s0[r * CL + l][k];
    }
    part[((long long)blk * 2) * C + c] = t1;
    part[((long long)blk * 2 + 1) * C + c] = t0;
  }
}

// per clip: the channels' sums over the clip's chunks (kept for dgamma / dbeta) and the group
// coefficients of dx = rstd gamma gt + c2 x + c3 (ATen's group_norm backward)
__global__ __launch_bounds__(256) void gn_cl_bwd_coef(const float* __restrict__ part, const float* __restrict__ gamma,
                                                      const float* __restrict__ mean, const float* __restrict__ rstd,
                                                      int T, int C, int G, int nch, float* __restrict__ sbc,
                                                      float* __restrict__ coef) {
  __shared__ float sds[1024], sdb[1024];
  const long long b = blockIdx.x;
  for (int c = (int)threadIdx.x; c < C; c += 256) {
    float t1 = 0.f, t0 = 0.f;
    for (int k = 0; k < nch; ++k) {
      t1 += part[((b * nch + k) * 2) * C + c];
      t0 += part[((b * nch + k) * 2 + 1) * C + c];
    }
    sbc[(b * 2) * C + c] = t1;
    sbc[(b * 2 + 1) * C + c] = t0;
    sds[c] = t1 * gamma[c];
    sdb[c] = t0 * gamma[c];
  }
  __syncthreads();
  if ((int)threadIdx.x < G) {
    const int g = (int)threadIdx.x, cpg = C / G;
    float ds = 0.f, db = 0.f;
    for (int c = g * cpg; c < (g + 1) * cpg; ++c) {
      ds += sds[c];
      db += sdb[c];
    }
    const float m = mean[b * G + g], rs = rstd[b * G + g];
    const float s = 1.f / ((float)cpg * (float)T);
    const float c2 = (db * m - ds) * rs * rs * rs * s;
    const float c3 = -c2 * m - db * rs * s;
    coef[(b * G + g) * 2] = c2;
    coef[(b * G + g) * 2 + 1] = c3;
  }
}

// dgamma[c] = sum_b (S1 - mean S0) rstd, dbeta[c] = sum_b S0 (added into out with accumulate)
__global__ __launch_bounds__(256) void gn_cl_bwd_params(const float* __restrict__ sbc, const float* __restrict__ mean,
                                                        const float* __restrict__ rstd, int B, int C, int G,
                                                        float* __restrict__ dgamma, float* __restrict__ dbeta,
                                                        int accumulate) {
  const int c = (int)(blockIdx.x * 256 + threadIdx.x);
  if (c >= C) return;
  const int g = c / (C / G);
  float dg = 0.f, dbt = 0.f;
  for (int b = 0; b < B; ++b) {
    const float s1 = sbc[((long long)b * 2) * C + c], s0 = sbc[((long long)b * 2 + 1) * C + c];
    dg += (s1 - mean[b * G + g] * s0) * rstd[b * G + g];
    dbt += s0;
  }
  if (dgamma != nullptr) dgamma[c] = accumulate ? dgamma[c] + dg : dg;
  if (dbeta != nullptr) dbeta[c] = accumulate ? dbeta[c] + dbt : dbt;
}

__global__ __launch_bounds__(256) void gn_cl_bwd_apply(const float* __restrict__ g32, long long sb,
                                                       const uint16_t* __restrict__ g16,
                                                       const uint16_t* __restrict__ x, const float* __restrict__ gamma,
                                                       const float* __restrict__ rstd, const float* __restrict__ coef,
                                                       int T, int C, int G, int nch, uint16_t* __restrict__ dx) {
  const int blk = (int)blockIdx.x;
  const long long b = blk / nch;
  const int r0 = (blk % nch) * kGnRows, r1 = min(T, r0 + kGnRows);
  const int CL = C / 8, RL = 256 / CL;
  const int cl = (int)threadIdx.x % CL, rl = (int)threadIdx.x / CL;
  const int g = cl * 8 / (C / G);
  const float rs = rstd[b * G + g], c2 = coef[(b * G + g) * 2], c3 = coef[(b * G + g) * 2 + 1];
  float c1[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) c1[k] = rs * gamma[cl * 8 + k];
  for (int r = r0 + rl; r < r1; r += RL) {
    float xv[8], gt[8];
    load_bf16x8(x + ((b * T + r) * C + cl * 8), xv);
#pragma unroll
    for (int k = 0; k < 8; ++k) gt[k] = 0.f;
    if (g32 != nullptr) {
      const float* p = g32 + (b * sb + (long long)r * C + cl * 8);
      const float4 u = *reinterpret_cast<const float4*>(p), w = *reinterpret_cast<const float4*>(p + 4);
      gt[0] = u.x; gt[1] = u.y; gt[2] = u.z; gt[3] = u.w; gt[4] = w.x; gt[5] = w.y; gt[6] = w.z; gt[7] = w.w;
    }
    if (g16 != nullptr) {
      float h[8];
      load_bf16x8(g16 + ((b * T + r) * C + cl * 8), h);
#pragma unroll
      for (int k = 0; k < 8; ++k) gt[k] += h[k];
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) gt[k] = c1[k] * gt[k] + c2 * xv[k] + c3;
    store_bf16x8(dx + ((b * T + r) * C + cl * 8), gt);
  }
}

int status(const char* what) {
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    snprintf(g_err, sizeof(g_err), "add_layernorm: %s launch failed: %s", what, hipGetErrorString(e));
    return 2;
  }
  return 0;
}

bool shape_ok(int64_t rows, int64_t d) { return rows >= 0 && d > 0 && d % 256 == 0 && d <= 1024; }

#define MFL_ALN_FWD(CHN)                                                                                   \
  hipLaunchKernelGGL((add_ln_fwd<RT, YT, CHN>), dim3(blocks), dim3(kWaves * 64), 0, st, rp, yp, gamma, beta, \
                     (long long)rows, (int)d, eps, out, mean, rstd, out16, pos, q16, drop)

template <typename RT, typename YT>
int fwd(const void* r, const void* y, const float* gamma, const float* beta, int64_t rows, int64_t d, float eps,
        float* out, float* mean, float* rstd, uint16_t* out16, const float* pos, uint16_t* q16, Drop drop,
        hipStream_t st) {
  const unsigned blocks = (unsigned)((rows + kWaves - 1) / kWaves);
  auto* rp = static_cast<const RT*>(r);
  auto* yp = static_cast<const YT*>(y);
  switch (d / 256) {
    case 1: MFL_ALN_FWD(1); break;
    case 2: MFL_ALN_FWD(2); break;
    case 3: MFL_ALN_FWD(3); break;
    default: MFL_ALN_FWD(4); break;
  }
  return status("forward");
}
#undef MFL_ALN_FWD

#define MFL_ALN_BWD_R(CHN, R)                                                                              \
  hipLaunchKernelGGL((add_ln_bwd<RT, YT, CHN, R>), dim3(blocks), dim3(kWaves * 64), 0, st, dout, rp, yp, gamma, \
                     mean, rstd, (long long)rows, (int)d, drp, dyp, part, dout16, dq16, dpos, drop, dpos_acc, \
                     dysum != nullptr ? 1 : 0)
#define MFL_ALN_BWD(CHN)                                                                                   \
  do {                                                                                                     \
    if (rpb == kBwdRowsShort) MFL_ALN_BWD_R(CHN, kBwdRowsShort); else MFL_ALN_BWD_R(CHN, kBwdRows);        \
  } while (0)

template <typename RT, typename YT>
int bwd(const float* dout, const void* r, const void* y, const float* gamma, const float* mean, const float* rstd,
        int64_t rows, int64_t d, void* dr, void* dy, float* dgamma, float* dbeta, void* workspace,
        const uint16_t* dout16, const uint16_t* dq16, float* dpos, Drop drop, hipStream_t st, int dpos_acc = 0,
        float* dysum = nullptr) {
  const int rpb = bwd_rows_per_block(rows);
  const unsigned blocks = (unsigned)((rows + rpb - 1) / rpb);
  auto* rp = static_cast<const RT*>(r);
  auto* yp = static_cast<const YT*>(y);
  auto* drp = static_cast<RT*>(dr);
  auto* dyp = static_cast<YT*>(dy);
  auto* part = static_cast<float*>(workspace);
  switch (d / 256) {
    case 1: MFL_ALN_BWD(1); break;
    case 2: MFL_ALN_BWD(2); break;
    case 3: MFL_ALN_BWD(3); break;
    default: MFL_ALN_BWD(4); break;
  }
  int rc;
  if ((rc = status("backward"))) return rc;
  const int d2 = (int)((dysum != nullptr ? 3 : 2) * d);
  hipLaunchKernelGGL(add_ln_param_final, dim3((unsigned)((d2 + 63) / 64)), dim3(1024), 0, st, part, (int)blocks, d2,
                     dgamma, dbeta, dysum, (int)d);
  return status("backward params");
}
#undef MFL_ALN_BWD
#undef MFL_ALN_BWD_R

// Zero fill as a kernel, not hipMemsetAsync: under the HIP runtime's graph packet capture a
// captured memset node did not take effect on replays that followed eager work
// (tools/packet_capture_unit.py), so nothing this library launches is a memset.
__global__ void zero_f32_kernel(float* __restrict__ p, long long n) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
    p[i] = 0.f;
}

hipError_t zero_f32(float* p, long long n, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  const long long blocks = std::min<long long>((n + 255) / 256, 4096);
  hipLaunchKernelGGL(zero_f32_kernel, dim3((unsigned)blocks), dim3(256), 0, st, p, n);
  return hipGetLastError();
}

}  // namespace

extern "C" {

size_t mfl_add_layernorm_workspace_bytes(int64_t rows, int64_t d) {
  if (rows <= 0 || d <= 0) return 0;
  const int rpb = bwd_rows_per_block(rows);
  return (size_t)((rows + rpb - 1) / rpb) * 3 * (size_t)d * sizeof(float);  // (dgamma, dbeta, dy column sums)
}

int mfl_add_layernorm_forward_ex(const void* r, int r_dtype, const void* y, int y_dtype, const float* gamma,
                                 const float* beta, int64_t rows, int64_t d, float eps, float* out, float* mean,
                                 float* rstd, uint16_t* out16, const float* pos, uint16_t* q16, float p_drop,
                                 const int64_t* seed, void* stream) {
  g_err[0] = 0;
  if (seed && !(p_drop >= 0.f && p_drop < 1.f)) {
    snprintf(g_err, sizeof(g_err), "mfl_add_layernorm_forward: dropout p must be in [0, 1)");
    return 1;
  }
  if (!shape_ok(rows, d) || (r_dtype != 0 && r_dtype != 2) || (y_dtype != 0 && y_dtype != 2)) {
    snprintf(g_err, sizeof(g_err), "mfl_add_layernorm_forward: needs d %% 256 == 0, d <= 1024, fp32/bf16 inputs");
    return 1;
  }
  if (rows == 0) return 0;
  if (!r || !y || !gamma || !beta || !out || !mean || !rstd || (q16 && !pos)) {
    snprintf(g_err, sizeof(g_err), "mfl_add_layernorm_forward: null pointer");
    return 1;
  }
  hipStream_t st = static_cast<hipStream_t>(stream);
  const Drop drop{seed, p_drop, seed ? 1.f / (1.f - p_drop) : 1.f};
#define MFL_ALN_FWD_ARGS r, y, gamma, beta, rows, d, eps, out, mean, rstd, out16, pos, q16, drop, st
  if (r_dtype == 0)
    return y_dtype == 0 ? fwd<float, float>(MFL_ALN_FWD_ARGS) : fwd<float, uint16_t>(MFL_ALN_FWD_ARGS);
  return y_dtype == 0 ? fwd<uint16_t, float>(MFL_ALN_FWD_ARGS) : fwd<uint16_t, uint16_t>(MFL_ALN_FWD_ARGS);
#undef MFL_ALN_FWD_ARGS
}

int mfl_add_layernorm_forward(const void* r, int r_dtype, const void* y, int y_dtype, const float* gamma,
                              const float* beta, int64_t rows, int64_t d, float eps, float* out, float* mean,
                              float* rstd, void* stream) {
  return mfl_add_layernorm_forward_ex(r, r_dtype, y, y_dtype, gamma, beta, rows, d, eps, out, mean, rstd, nullptr,
                                      nullptr, nullptr, 0.f, nullptr, stream);
}

int mfl_add_layernorm_backward_ex(const float* dout, const uint16_t* dout16, const uint16_t* dq16, const void* r,
                                  int r_dtype, const void* y, int y_dtype, const float* gamma, const float* mean,
                                  const float* rstd, int64_t rows, int64_t d, void* dr, void* dy, float* dgamma,
                                  float* dbeta, float* dpos, float p_drop, const int64_t* seed, void* workspace,
                                  void* stream) {
  g_err[0] = 0;
  if (seed && !(p_drop >= 0.f && p_drop < 1.f)) {
    snprintf(g_err, sizeof(g_err), "mfl_add_layernorm_backward: dropout p must be in [0, 1)");
    return 1;
  }
  if (!shape_ok(rows, d) || (r_dtype != 0 && r_dtype != 2) || (y_dtype != 0 && y_dtype != 2)) {
    snprintf(g_err, sizeof(g_err), "mfl_add_layernorm_backward: needs d %% 256 == 0, d <= 1024, fp32/bf16 inputs");
    return 1;
  }
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (rows == 0) {
    if (zero_f32(dgamma, d, st) != hipSuccess || zero_f32(dbeta, d, st) != hipSuccess)
      return 2;
    return 0;
  }
  if ((!dout && !dout16 && !dq16) || !r || !y || !gamma || !mean || !rstd || !dr || !dy || !dgamma || !dbeta ||
      !workspace) {
    snprintf(g_err, sizeof(g_err), "mfl_add_layernorm_backward: null pointer");
    return 1;
  }
  const Drop drop{seed, p_drop, seed ? 1.f / (1.f - p_drop) : 1.f};
#define MFL_ALN_BWD_ARGS \
  dout, r, y, gamma, mean, rstd, rows, d, dr, dy, dgamma, dbeta, workspace, dout16, dq16, dpos, drop, st
  if (r_dtype == 0)
    return y_dtype == 0 ? bwd<float, float>(MFL_ALN_BWD_ARGS) : bwd<float, uint16_t>(MFL_ALN_BWD_ARGS);
  return y_dtype == 0 ? bwd<uint16_t, float>(MFL_ALN_BWD_ARGS) : bwd<uint16_t, uint16_t>(MFL_ALN_BWD_ARGS);
#undef MFL_ALN_BWD_ARGS
}

int mfl_add_layernorm_backward_ex2(const float* dout, const uint16_t* dout16, const uint16_t* dq16, const void* r,
                                   int r_dtype, const void* y, int y_dtype, const float* gamma, const float* mean,
                                   const float* rstd, int64_t rows, int64_t d, void* dr, void* dy, float* dgamma,
                                   float* dbeta, float* dpos, int dpos_accumulate, float* dy_colsum, float p_drop,
                                   const int64_t* seed, void* workspace, void* stream) {
  g_err[0] = 0;
  if (seed && !(p_drop >= 0.f && p_drop < 1.f)) {
    snprintf(g_err, sizeof(g_err), "mfl_add_layernorm_backward: dropout p must be in [0, 1)");
    return 1;
  }
  if (!shape_ok(rows, d) || (r_dtype != 0 && r_dtype != 2) || (y_dtype != 0 && y_dtype != 2)) {
    snprintf(g_err, sizeof(g_err), "mfl_add_layernorm_backward: needs d %% 256 == 0, d <= 1024, fp32/bf16 inputs");
    return 1;
  }
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (rows == 0) {
    if (zero_f32(dgamma, d, st) != hipSuccess || zero_f32(dbeta, d, st) != hipSuccess ||
        (dy_colsum && zero_f32(dy_colsum, d, st) != hipSuccess))
      return 2;
    return 0;
  }
  if ((!dout && !dout16 && !dq16) || !r || !y || !gamma || !mean || !rstd || !dr || !dy || !dgamma || !dbeta ||
      !workspace || (dpos_accumulate && !dpos)) {
    snprintf(g_err, sizeof(g_err), "mfl_add_layernorm_backward: null pointer");
    return 1;
  }
  const Drop drop{seed, p_drop, seed ? 1.f / (1.f - p_drop) : 1.f};
  const int acc = dpos_accumulate ? 1 : 0;
#define MFL_ALN_BWD_ARGS \
  dout, r, y, gamma, mean, rstd, rows, d, dr, dy, dgamma, dbeta, workspace, dout16, dq16, dpos, drop, st, acc, dy_colsum
  if (r_dtype == 0)
    return y_dtype == 0 ? bwd<float, float>(MFL_ALN_BWD_ARGS) : bwd<float, uint16_t>(MFL_ALN_BWD_ARGS);
  return y_dtype == 0 ? bwd<uint16_t, float>(MFL_ALN_BWD_ARGS) : bwd<uint16_t, uint16_t>(MFL_ALN_BWD_ARGS);
#undef MFL_ALN_BWD_ARGS
}

int mfl_add_layernorm_backward(const float* dout, const void* r, int r_dtype, const void* y, int y_dtype,
                               const float* gamma, const float* mean, const float* rstd, int64_t rows, int64_t d,
                               void* dr, void* dy, float* dgamma, float* dbeta, void* workspace, void* stream) {
  if (!dout) {
    g_err[0] = 0;
    snprintf(g_err, sizeof(g_err), "mfl_add_layernorm_backward: null pointer");
    return 1;
  }
  return mfl_add_layernorm_backward_ex(dout, nullptr, nullptr, r, r_dtype, y, y_dtype, gamma, mean, rstd, rows, d, dr,
                                       dy, dgamma, dbeta, nullptr, 0.f, nullptr, workspace, stream);
}

int mfl_carry_entry_forward(const float* src, const float* pos, int64_t n, uint16_t* v16, uint16_t* q16,
                            void* stream) {
  g_err[0] = 0;
  if (n < 0 || n % 8 || (n > 0 && (!src || !q16)) ||
      (((uintptr_t)src | (uintptr_t)pos | (uintptr_t)v16 | (uintptr_t)q16) & 15u)) {
    snprintf(g_err, sizeof(g_err), "mfl_carry_entry_forward: n %% 8 == 0 and 16-byte aligned buffers needed");
    return 1;
  }
  if (n == 0) return 0;
  const long long n8 = n / 8;
  const unsigned blocks = (unsigned)std::min<long long>((n8 + 255) / 256, 8192);
  hipLaunchKernelGGL(carry_entry_fwd, dim3(blocks), dim3(256), 0, static_cast<hipStream_t>(stream), src, pos, n8,
                     v16, q16);
  return status("carry entry forward");
}

int mfl_carry_entry_backward(const float* dr, const uint16_t* dv16, const uint16_t* dq16, int64_t n, float* dsrc,
                             float* dpos, int dpos_accumulate, void* stream) {
  g_err[0] = 0;
  if (n < 0 || n % 8 || (n > 0 && !dsrc) ||
      (((uintptr_t)dr | (uintptr_t)dv16 | (uintptr_t)dq16 | (uintptr_t)dsrc | (uintptr_t)dpos) & 15u)) {
    snprintf(g_err, sizeof(g_err), "mfl_carry_entry_backward: n %% 8 == 0 and 16-byte aligned buffers needed");
    return 1;
  }
  if (n == 0) return 0;
  const long long n4 = n / 4;
  const unsigned blocks = (unsigned)std::min<long long>((n4 + 255) / 256, 8192);
  hipLaunchKernelGGL(carry_entry_bwd, dim3(blocks), dim3(256), 0, static_cast<hipStream_t>(stream), dr, dv16, dq16,
                     n4, dsrc, dpos, dpos_accumulate);
  return status("carry entry backward");
}

static bool gn_cl_ok(int64_t B, int64_t T, int64_t C, int64_t G) {
  return B >= 1 && T >= 1 && G >= 1 && G <= 128 && C % G == 0 && (C / G) % 8 == 0 && C % 8 == 0 && C <= 1024 &&
         256 % (C / 8) == 0 && B * T * C < (1LL << 40) && T < (1 << 30);
}

size_t mfl_groupnorm_cl_workspace_bytes(int64_t B, int64_t T, int64_t C, int64_t G) {
  if (!gn_cl_ok(B, T, C, G)) return 0;
  const long long nch = (T + kGnRows - 1) / kGnRows;
  const long long fwd = B * nch * G * 2, bwd = B * nch * 2 * C + B * 2 * C + B * G * 2;
  return (size_t)std::max(fwd, bwd) * sizeof(float);
}

int mfl_groupnorm_cl_forward(const uint16_t* x, const float* gamma, const float* beta, int64_t B, int64_t T, int64_t C,
                             int64_t G, float eps, float* out32, int64_t out32_batch_stride, uint16_t* out16,
                             float* mean, float* rstd, void* workspace, void* stream) {
  g_err[0] = 0;
  if (!gn_cl_ok(B, T, C, G) || !x || !gamma || !beta || !out32 || !mean || !rstd || !workspace ||
      out32_batch_stride < T * C || (((uintptr_t)x | (uintptr_t)out32 | (uintptr_t)out16) & 15u) ||
      out32_batch_stride % 4) {
    snprintf(g_err, sizeof(g_err), "mfl_groupnorm_cl_forward: bad arguments (C in {256, 512, 1024}, (C/G) %% 8 == 0, "
                                   "16-B aligned buffers)");
    return 1;
  }
  const int nch = (int)((T + kGnRows - 1) / kGnRows);
  const unsigned grid = (unsigned)(B * nch);
  hipStream_t st = static_cast<hipStream_t>(stream);
  auto* part = static_cast<float*>(workspace);
  hipLaunchKernelGGL(gn_cl_stats, dim3(grid), dim3(256), 0, st, x, (int)T, (int)C, (int)G, nch, part);
  int rc;
  if ((rc = status("groupnorm stats"))) return rc;
  hipLaunchKernelGGL(gn_cl_apply, dim3(grid), dim3(256), 0, st, x, part, gamma, beta, (int)T, (int)C, (int)G, nch, eps,
                     out32, (long long)out32_batch_stride, out16, mean, rstd);
  return status("groupnorm apply");
}

int mfl_groupnorm_cl_backward(const float* g32, int64_t g32_batch_stride, const uint16_t* g16, const uint16_t* x,
                              const float* gamma, const float* mean, const float* rstd, int64_t B, int64_t T,
                              int64_t C, int64_t G, uint16_t* dx, float* dgamma, float* dbeta, int accumulate,
                              void* workspace, void* stream) {
  g_err[0] = 0;
  if (!gn_cl_ok(B, T, C, G) || !x || !gamma || !mean || !rstd || !dx || !workspace ||
      (g32 != nullptr && (g32_batch_stride < T * C || g32_batch_stride % 4)) ||
      (((uintptr_t)x | (uintptr_t)g32 | (uintptr_t)g16 | (uintptr_t)dx) & 15u)) {
    snprintf(g_err, sizeof(g_err), "mfl_groupnorm_cl_backward: bad arguments");
    return 1;
  }
  const int nch = (int)((T + kGnRows - 1) / kGnRows);
  const unsigned grid = (unsigned)(B * nch);
  hipStream_t st = static_cast<hipStream_t>(stream);
  auto* part = static_cast<float*>(workspace);
  float* sbc = part + B * nch * 2 * C;
  float* coef = sbc + B * 2 * C;
  hipLaunchKernelGGL(gn_cl_bwd_partial, dim3(grid), dim3(256), 0, st, g32, (long long)g32_batch_stride, g16, x,
                     (int)T, (int)C, nch, part);
  int rc;
  if ((rc = status("groupnorm backward partials"))) return rc;
  hipLaunchKernelGGL(gn_cl_bwd_coef, dim3((unsigned)B), dim3(256), 0, st, part, gamma, mean, rstd, (int)T, (int)C,
                     (int)G, nch, sbc, coef);
  if ((rc = status("groupnorm backward coefficients"))) return rc;
  if (dgamma != nullptr || dbeta != nullptr) {
    hipLaunchKernelGGL(gn_cl_bwd_params, dim3((unsigned)((C + 255) / 256)), dim3(256), 0, st, sbc, mean, rstd, (int)B,
                       (int)C, (int)G, dgamma, dbeta, accumulate);
    if ((rc = status("groupnorm backward parameters"))) return rc;
  }
  hipLaunchKernelGGL(gn_cl_bwd_apply, dim3(grid), dim3(256), 0, st, g32, (long long)g32_batch_stride, g16, x, gamma,
                     rstd, coef, (int)T, (int)C, (int)G, nch, dx);
  return status("groupnorm backward apply");
}

const char* mfl_add_layernorm_last_error(void) { return g_err; }

}  // extern "C"
