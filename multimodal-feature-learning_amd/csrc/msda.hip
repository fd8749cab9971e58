// msda.hip — multi-scale temporal deformable attention (MSDA) for MI355X / gfx950.
//
// What it computes (the live semantics of the reference):
//   out[b,q,m,:] = sum_l sum_p aw[b,q,m,l,p] * lerp(V_l[b,:,m,:], y)
//   y = clamp(fma((2*loc-1)+1, T_l/2, -0.5), 0, T_l-1)           (BORDER)
// i.e. F.grid_sample(bilinear, border, align_corners=False) on a (B*M, D, T_l, 1)
// image at grid x=-1 — reference models/modules/attention.py:349-383 — and its
// autograd backward (ATen grid_sampler_2d_backward + stack/mul/sum).  The dormant
// CUDA extension's zero padding (models/ops/src/cuda/ms_deform_im2col_cuda.cuh:34-85,
// 238-300) is available as MSDA_PAD_ZEROS for the models/ops API.
//
// Layout in HBM (all row-major, contiguous):
//   value  (B, S, M, D)   one (b,s,m) row = D channels, rows of one token are M*D apart
//   loc/aw (B, Lq, M, L, P) fp32 (fp64 for fp64 values)
//   out    (B, Lq, M*D)
//
// Work decomposition: one "item" = one (b, q, m) output row.  G = D/VEC lanes of a
// 64-wide wavefront own one item (VEC channels per lane, 16-byte loads), so every
// tap is one coalesced G*16-byte row read; 64/G items share a wavefront.  The
// per-sample coordinate arithmetic is uniform inside a lane group.
// Backward: grad_aw / grad_loc are reductions over the item's D channels = a
// butterfly over the G lanes of the group (__shfl_xor, no LDS, no barriers);
// grad_value is NOT scattered with global atomics: msda_gvalue_kernel gives every
// (b, head, level, row-range) slab one owner workgroup that accumulates it in LDS.
//
// Coordinates are computed with FP contraction OFF in exactly the operation order of
// ATen's CPU grid sampler (g = 2*loc-1, then y = fma(g+1, T/2, -0.5)), so the tap index
// and the clamp decision are bit-identical to the CPU reference: the loc-gradient jumps
// at integer positions, and a one-ulp different y would flip the segment.

#include <hip/hip_runtime.h>

#include <algorithm>
#include <mutex>
#include <type_traits>
#include <hip/hip_bf16.h>
#include <hip/hip_fp16.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "msda_hip.h"
#include "msda_win.h"

namespace {

thread_local char g_last_error[512] = {0};

template <typename... A>
void set_error(const char* fmt, A... a) {
  snprintf(g_last_error, sizeof(g_last_error), fmt, a...);
}
void set_error(const char* msg) { snprintf(g_last_error, sizeof(g_last_error), "%s", msg); }

struct Levels {
  int T[MSDA_MAX_LEVELS];
  int start[MSDA_MAX_LEVELS];
};

// XCD-aware block order (MI355X_MICROARCH.md, workgroup dispatch; cdna guide T1): blocks are
// dealt round-robin over the 8 XCDs, each with a private 4 MB L2.  Renumber so that the
// blocks sharing an XCD get one contiguous range of logical ids: a clip's value / grad_out
// rows (2 MB in bf16 at the bench shape) then stay in one XCD's L2 instead of being fetched
// by all eight.  Bijective for any block count; speed only, never correctness.
__device__ __forceinline__ unsigned xcd_block(unsigned orig, unsigned nwg) {
  const unsigned xcd = orig % 8u, q = nwg / 8u, r = nwg % 8u;
  return (xcd < r ? xcd * (q + 1u) : r * (q + 1u) + (xcd - r) * q) + orig / 8u;
}

// ---------------------------------------------------------------------------------
// storage types and 16-byte vector I/O
// ---------------------------------------------------------------------------------
struct bf16_t { uint16_t x; };
struct f16_t { uint16_t x; };

template <typename scalar_t> struct AccOf { using type = float; };
template <> struct AccOf<double> { using type = double; };

__device__ __forceinline__ float to_acc(float v) { return v; }
__device__ __forceinline__ double to_acc(double v) { return v; }
__device__ __forceinline__ float to_acc(bf16_t v) { return __uint_as_float(((uint32_t)v.x) << 16); }
__device__ __forceinline__ float to_acc(f16_t v) {
  return __half2float(__ushort_as_half(v.x));
}

__device__ __forceinline__ void from_acc(float a, float* d) { *d = a; }
__device__ __forceinline__ void from_acc(double a, double* d) { *d = a; }
__device__ __forceinline__ void from_acc(float a, bf16_t* d) {
  __hip_bfloat16 h = __float2bfloat16(a);  // RNE, NaN stays NaN
  d->x = *reinterpret_cast<uint16_t*>(&h);
}
__device__ __forceinline__ void from_acc(float a, f16_t* d) {
  d->x = __half_as_ushort(__float2half(a));
}

// Load VEC consecutive elements (one 16- or 8-byte access when VEC*sizeof is 16 or 8).
template <typename scalar_t, int VEC>
__device__ __forceinline__ void load_vec(const scalar_t* __restrict__ p,
                                         typename AccOf<scalar_t>::type (&r)[VEC]) {
  if constexpr (VEC * sizeof(scalar_t) == 16) {
    const uint4 raw = *reinterpret_cast<const uint4*>(p);
    const scalar_t* e = reinterpret_cast<const scalar_t*>(&raw);
#pragma unroll
    for (int i = 0; i < VEC; ++i) r[i] = to_acc(e[i]);
  } else if constexpr (VEC * sizeof(scalar_t) == 8) {
    const uint2 raw = *reinterpret_cast<const uint2*>(p);
    const scalar_t* e = reinterpret_cast<const scalar_t*>(&raw);
#pragma unroll
    for (int i = 0; i < VEC; ++i) r[i] = to_acc(e[i]);
  } else {
#pragma unroll
    for (int i = 0; i < VEC; ++i) r[i] = to_acc(p[i]);
  }
}

template <typename scalar_t, int VEC>
__device__ __forceinline__ void store_vec(scalar_t* __restrict__ p,
                                          const typename AccOf<scalar_t>::type (&r)[VEC]) {
  if constexpr (VEC * sizeof(scalar_t) == 16) {
    uint4 raw;
    scalar_t* e = reinterpret_cast<scalar_t*>(&raw);
#pragma unroll
    for (int i = 0; i < VEC; ++i) from_acc(r[i], &e[i]);
    *reinterpret_cast<uint4*>(p) = raw;
  } else if constexpr (VEC * sizeof(scalar_t) == 8) {
    uint2 raw;
    scalar_t* e = reinterpret_cast<scalar_t*>(&raw);
#pragma unroll
    for (int i = 0; i < VEC; ++i) from_acc(r[i], &e[i]);
    *reinterpret_cast<uint2*>(p) = raw;
  } else {
#pragma unroll
    for (int i = 0; i < VEC; ++i) from_acc(r[i], &p[i]);
  }
}

template <typename scalar_t, int VEC>
__device__ __forceinline__ void store_vec_nt(scalar_t* __restrict__ p,
                                             const typename AccOf<scalar_t>::type (&r)[VEC]) {
#ifdef MSDA_NT
  if constexpr (VEC * sizeof(scalar_t) == 16) {
    uint4 raw;
    scalar_t* e = reinterpret_cast<scalar_t*>(&raw);
#pragma unroll
    for (int i = 0; i < VEC; ++i) from_acc(r[i], &e[i]);
    typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
    __builtin_nontemporal_store(u32x4_t{raw.x, raw.y, raw.z, raw.w}, reinterpret_cast<u32x4_t*>(p));
    return;
  }
#endif
  store_vec<scalar_t, VEC>(p, r);
}

// One 16-byte row fragment kept raw (4 VGPRs) until it is consumed; zero when not loaded.
template <typename scalar_t>
__device__ __forceinline__ uint4 load16_if(bool ok, const scalar_t* __restrict__ p) {
  return ok ? *reinterpret_cast<const uint4*>(p) : make_uint4(0u, 0u, 0u, 0u);
}
// Streaming variants (MSDA_NT builds): data touched once per kernel (value rows of the fused
// backward, grad_value) marked non-temporal so it does not evict the gathered grad_out rows.
template <typename scalar_t>
__device__ __forceinline__ uint4 load16_if_nt(bool ok, const scalar_t* __restrict__ p) {
#ifdef MSDA_NT
  typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
  if (!ok) return make_uint4(0u, 0u, 0u, 0u);
  const u32x4_t v = __builtin_nontemporal_load(reinterpret_cast<const u32x4_t*>(p));
  return make_uint4(v.x, v.y, v.z, v.w);
#else
  return load16_if(ok, p);
#endif
}
template <typename scalar_t, int VEC>
__device__ __forceinline__ void cvt16(const uint4& raw, typename AccOf<scalar_t>::type (&r)[VEC]) {
  static_assert(VEC * sizeof(scalar_t) == 16, "16-byte fragment");
  const scalar_t* e = reinterpret_cast<const scalar_t*>(&raw);
#pragma unroll
  for (int i = 0; i < VEC; ++i) r[i] = to_acc(e[i]);
}

// Packed fp32 pairs: the fast kernels' channel math runs as v_pk_fma_f32 (two channels per
// instruction); a bf16 pair unpacks with one shift and one mask.
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));

template <typename scalar_t, int VEC>
__device__ __forceinline__ void cvt16x2(const uint4& raw, f32x2 (&r)[VEC / 2]) {
  static_assert(VEC * sizeof(scalar_t) == 16, "16-byte fragment");
  if constexpr (std::is_same<scalar_t, bf16_t>::value) {
    const uint32_t d[4] = {raw.x, raw.y, raw.z, raw.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) r[i] = f32x2{__uint_as_float(d[i] << 16), __uint_as_float(d[i] & 0xffff0000u)};
  } else {
    const scalar_t* e = reinterpret_cast<const scalar_t*>(&raw);
#pragma unroll
    for (int i = 0; i < VEC / 2; ++i) r[i] = f32x2{(float)to_acc(e[2 * i]), (float)to_acc(e[2 * i + 1])};
  }
}

__device__ __forceinline__ f32x2 pk_fma(f32x2 a, f32x2 b, f32x2 c) {
  return __builtin_elementwise_fma(a, b, c);
}

// Dot product of two raw 16-byte fragments, fp32 accumulation: v_dot2_f32_bf16 / v_dot2_f32_f16
// on the packed pairs (no unpacking), plain FMAs for fp32.
typedef _Float16 f16x2_t __attribute__((ext_vector_type(2)));
template <typename scalar_t>
__device__ __forceinline__ float dot16(const uint4& a, const uint4& b) {
  const uint32_t x[4] = {a.x, a.y, a.z, a.w}, y[4] = {b.x, b.y, b.z, b.w};
  float r = 0.f;
  if constexpr (std::is_same<scalar_t, bf16_t>::value) {
#pragma unroll
    for (int e = 0; e < 4; ++e)
      r = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2_t, x[e]), __builtin_bit_cast(bf16x2_t, y[e]), r,
                                          false);
  } else if constexpr (std::is_same<scalar_t, f16_t>::value) {
#pragma unroll
    for (int e = 0; e < 4; ++e)
      r = __builtin_amdgcn_fdot2(__builtin_bit_cast(f16x2_t, x[e]), __builtin_bit_cast(f16x2_t, y[e]), r, false);
  } else {
    static_assert(std::is_same<scalar_t, float>::value, "dot16: 16-bit or fp32 fragments");
#pragma unroll
    for (int e = 0; e < 4; ++e) r = fmaf(__uint_as_float(x[e]), __uint_as_float(y[e]), r);
  }
  return r;
}

// ---------------------------------------------------------------------------------
// sampling coordinates
// ---------------------------------------------------------------------------------
template <typename coord_t>
struct Taps {
  int i0, i1;      // tap rows inside the level (always valid addresses)
  coord_t w0, w1;  // interpolation weights (0 for a tap outside the map)
  bool ok0, ok1;   // tap inside the map
  coord_t gmul;    // d(y)/d(loc) with the clamp folded in (0 where clamped / skipped)
};

// BORDER: grid_sample(bilinear, padding_mode='border', align_corners=False) along a
// T-long axis at normalized grid coordinate g = 2*loc-1 (attention.py:349,367-368).
template <typename coord_t>
__device__ __forceinline__ Taps<coord_t> taps_border(coord_t loc, int T) {
#pragma clang fp contract(off)
  Taps<coord_t> t;
  const coord_t g = loc * (coord_t)2 - (coord_t)1;
  // ATen's CPU sampler fuses the unnormalize into one FMA (pinned in tests/test_oracle.py)
  const coord_t y = fma(g + (coord_t)1, (coord_t)T * (coord_t)0.5, (coord_t)-0.5);
  const coord_t ymax = (coord_t)(T - 1);
  // ATen clip_coordinates_get_grad: the border itself counts as out of bounds.
  const bool inb = (y > (coord_t)0) && (y < ymax);
  const coord_t yc = y > (coord_t)0 ? (y < ymax ? y : ymax) : (coord_t)0;
  const coord_t y0 = floor(yc);
  const coord_t n = yc - y0;
  t.i0 = (int)y0;
  t.i1 = t.i0 + 1;
  t.ok0 = true;
  t.ok1 = t.i1 <= T - 1;
  if (!t.ok1) t.i1 = t.i0;
  t.w0 = (coord_t)1 - n;
  t.w1 = n;
  // dy/dloc = 2 (from g) * T/2 (unnormalize)
  t.gmul = inb ? (coord_t)T : (coord_t)0;
  return t;
}

// ZEROS: the dormant CUDA kernel's 1-D (H=1) semantics: w_im = loc*T - 0.5, the sample is
// skipped unless -1 < w_im < T, taps outside [0, T-1] read 0
// (ms_deform_im2col_cuda.cuh:34-85 and :276-290; ms_deform_attn.py:114-117 lift).
template <typename coord_t>
__device__ __forceinline__ Taps<coord_t> taps_zeros(coord_t loc, int T) {
#pragma clang fp contract(off)
  Taps<coord_t> t;
  const coord_t x = loc * (coord_t)T - (coord_t)0.5;
  const bool live = (x > (coord_t)-1) && (x < (coord_t)T);
  const coord_t x0 = floor(live ? x : (coord_t)0);
  const coord_t lw = (live ? x : (coord_t)0) - x0;
  const int lo = (int)x0;
  t.ok0 = live && lo >= 0;
  t.ok1 = live && lo + 1 <= T - 1;
  t.i0 = t.ok0 ? lo : 0;
  t.i1 = t.ok1 ? lo + 1 : 0;
  t.w0 = t.ok0 ? (coord_t)1 - lw : (coord_t)0;
  t.w1 = t.ok1 ? lw : (coord_t)0;
  t.gmul = live ? (coord_t)T : (coord_t)0;
  return t;
}

template <typename coord_t, bool ZEROS>
__device__ __forceinline__ Taps<coord_t> make_taps(coord_t loc, int T) {
  if constexpr (ZEROS) return taps_zeros(loc, T);
  else return taps_border(loc, T);
}

// ---------------------------------------------------------------------------------
// forward
// ---------------------------------------------------------------------------------
template <typename scalar_t, typename coord_t, int VEC, bool ZEROS>
__global__ __launch_bounds__(256) void msda_fwd_kernel(
    const scalar_t* __restrict__ value, const coord_t* __restrict__ loc,
    const coord_t* __restrict__ aw, scalar_t* __restrict__ out, const Levels lv, const int L,
    const int P, const int S, const int M, const int D, const int Lq, const long long n_items,
    const int gshift) {
  using acc_t = typename AccOf<scalar_t>::type;
  const long long tid = (long long)xcd_block(blockIdx.x, gridDim.x) * blockDim.x + threadIdx.x;
  const long long item = tid >> gshift;
  if (item >= n_items) return;
  const int G = 1 << gshift;
  const int lg = (int)(tid & (G - 1));
  const int m = (int)(item % M);
  const long long b = item / M / Lq;
  const long long rowstride = (long long)M * D;
  const coord_t* __restrict__ locp = loc + item * (L * P);
  const coord_t* __restrict__ awp = aw + item * (L * P);
  const scalar_t* __restrict__ vb = value + (b * S * M + m) * (long long)D;
  scalar_t* __restrict__ op = out + item * D;
  const int nchunk = D / VEC;
  for (int ck = lg; ck < nchunk; ck += G) {
    acc_t acc[VEC];
#pragma unroll
    for (int e = 0; e < VEC; ++e) acc[e] = (acc_t)0;
    for (int l = 0; l < L; ++l) {
      const int T = lv.T[l];
      const scalar_t* __restrict__ vl = vb + (long long)lv.start[l] * rowstride + ck * VEC;
      for (int p = 0; p < P; ++p) {
        const coord_t a = awp[l * P + p];
        const Taps<coord_t> t = make_taps<coord_t, ZEROS>(locp[l * P + p], T);
        acc_t v0[VEC], v1[VEC];
        load_vec<scalar_t, VEC>(vl + t.i0 * rowstride, v0);
        load_vec<scalar_t, VEC>(vl + t.i1 * rowstride, v1);
        const acc_t w0 = (acc_t)t.w0, w1 = (acc_t)t.w1, aa = (acc_t)a;
#pragma unroll
        for (int e = 0; e < VEC; ++e) {
          const acc_t x0 = t.ok0 ? v0[e] : (acc_t)0;
          const acc_t x1 = t.ok1 ? v1[e] : (acc_t)0;
          acc[e] += aa * (x0 * w0 + x1 * w1);
        }
      }
    }
    store_vec<scalar_t, VEC>(op + ck * VEC, acc);
  }
}

// Forward fast path: fp32 coordinates, L*P <= 16 with L*P % 4 == 0 (the reference's 4 levels
// x 4 points), D = G * VEC (every lane owns one 16-byte chunk).  The item's 2*L*P coordinates
// are loaded up front as float4s (one dependent round trip instead of one per sample), and
// the 8 row fragments of 4 samples are in flight together, kept raw until use.
constexpr int kLPMax = 16;

template <int N>
__device__ __forceinline__ void load_coords16(const float* __restrict__ p, int LP, float (&r)[N]) {
#pragma unroll
  for (int c = 0; c < N / 4; ++c) {
    if (4 * c < LP) {
      const float4 x = reinterpret_cast<const float4*>(p)[c];
      r[4 * c] = x.x; r[4 * c + 1] = x.y; r[4 * c + 2] = x.z; r[4 * c + 3] = x.w;
    } else {
      r[4 * c] = r[4 * c + 1] = r[4 * c + 2] = r[4 * c + 3] = 0.f;
    }
  }
}

// The same L*P coordinates from the level-major layout (MSDA_COORD_LEVEL_MAJOR, (B, M, L, Lq, P)):
// level l's P floats at base + l * cl.
template <int N>
__device__ __forceinline__ void load_coords16_lm(const float* __restrict__ base, long long cl, int L, int P,
                                                 float (&r)[N]) {
  if (P % 4 == 0) {
#pragma unroll
    for (int c = 0; c < N / 4; ++c) {
      const int l = (4 * c) / P, p0 = (4 * c) % P;
      if (4 * c < L * P) {
        const float4 x = *reinterpret_cast<const float4*>(base + l * cl + p0);
        r[4 * c] = x.x; r[4 * c + 1] = x.y; r[4 * c + 2] = x.z; r[4 * c + 3] = x.w;
      } else {
        r[4 * c] = r[4 * c + 1] = r[4 * c + 2] = r[4 * c + 3] = 0.f;
      }
    }
  } else {
#pragma unroll
    for (int j = 0; j < N; ++j) r[j] = j < L * P ? base[(j / P) * cl + j % P] : 0.f;
  }
}

// One (b, q, m) item's output chunk: the body of msda_fwd16_kernel (vb: the item's head and
// lane offset in its clip's value rows; rs: the row stride, tap offsets inside a clip fit 32 bits)
template <typename scalar_t, int VEC, bool ZEROS>
__device__ __forceinline__ void fwd16_item(const scalar_t* __restrict__ vb, const float (&lr)[kLPMax],
                                           const float (&ar)[kLPMax], const Levels& lv, int P, int LP, int rs,
                                           scalar_t* __restrict__ op) {
  using acc_t = float;
  f32x2 acc2[VEC / 2];
#pragma unroll
  for (int e = 0; e < VEC / 2; ++e) acc2[e] = f32x2{0.f, 0.f};
#pragma unroll
  for (int j0 = 0; j0 < kLPMax; j0 += 4) {
    if (j0 < LP) {
      uint4 r0[4], r1[4];
      float c0[4], c1[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int l = (j0 + u) / P;
        const Taps<float> t = make_taps<float, ZEROS>(lr[j0 + u], lv.T[l]);
        const scalar_t* __restrict__ vl = vb + (long long)lv.start[l] * rs;
        r0[u] = load16_if(t.ok0, vl + t.i0 * rs);
        r1[u] = load16_if(t.ok1, vl + t.i1 * rs);
        c0[u] = ar[j0 + u] * t.w0;
        c1[u] = ar[j0 + u] * t.w1;
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        f32x2 x0[VEC / 2], x1[VEC / 2];
        cvt16x2<scalar_t, VEC>(r0[u], x0);
        cvt16x2<scalar_t, VEC>(r1[u], x1);
        const f32x2 k0{c0[u], c0[u]}, k1{c1[u], c1[u]};
#pragma unroll
        for (int e = 0; e < VEC / 2; ++e) acc2[e] = pk_fma(x1[e], k1, pk_fma(x0[e], k0, acc2[e]));
      }
    }
  }
  acc_t acc[VEC];
#pragma unroll
  for (int e = 0; e < VEC / 2; ++e) {
    acc[2 * e] = acc2[e].x;
    acc[2 * e + 1] = acc2[e].y;
  }
  store_vec<scalar_t, VEC>(op, acc);
}

template <typename scalar_t, int VEC, int G, bool ZEROS, bool LM>
__global__ __launch_bounds__(256) void msda_fwd16_kernel(
    const scalar_t* __restrict__ value, const float* __restrict__ loc, const float* __restrict__ aw,
    scalar_t* __restrict__ out, const Levels lv, const int L, const int P, const int S, const int M,
    const int D, const int Lq, const long long n_items) {
  const long long tid = (long long)xcd_block(blockIdx.x, gridDim.x) * blockDim.x + threadIdx.x;
  const long long item = tid / G;
  if (item >= n_items) return;
  const int lg = (int)(tid % G);
  const int m = (int)(item % M);
  const long long b = item / M / Lq;
  const int LP = L * P;
  float lr[kLPMax], ar[kLPMax];
  if constexpr (LM) {
    const long long q = (item / M) % Lq;
    const long long c0 = ((b * M + m) * L * Lq + q) * P;
    load_coords16_lm(loc + c0, (long long)Lq * P, L, P, lr);
    load_coords16_lm(aw + c0, (long long)Lq * P, L, P, ar);
  } else {
    load_coords16(loc + item * LP, LP, lr);
    load_coords16(aw + item * LP, LP, ar);
  }
  fwd16_item<scalar_t, VEC, ZEROS>(value + (b * S * M + m) * (long long)D + lg * VEC, lr, ar, lv, P, LP, M * D,
                                   out + item * D + lg * VEC);
}

// The tiles buffer's tail (msda_win.h): the persistent backward's queue words zeroed and the tile
// order stored, by one lane of the forward's first workgroup (plain vector stores)
__device__ __forceinline__ void write_tiles_tail(int2* tiles, long long ntiles_all, const QOrder& qo) {
  if (blockIdx.x != 0 || threadIdx.x != 0) return;
  unsigned* t = reinterpret_cast<unsigned*>(tiles + ntiles_all);
#pragma unroll
  for (int i = 0; i < (int)(kWinTailBytes / sizeof(unsigned)); ++i) t[i] = 0u;  // (every tail byte defined)
  QOrder* o = reinterpret_cast<QOrder*>(reinterpret_cast<char*>(t) + kWinQOrderOffset);
  o->cs = qo.cs;
  o->inv_cs = qo.inv_cs;
  o->L = qo.L;
#pragma unroll
  for (int l = 0; l < kQOrderMaxL; ++l) {
    o->n[l] = qo.n[l];
    o->start[l] = qo.start[l];
  }
}

// msda_fwd16_kernel for D = 64 16-bit values (G = 8 lanes an item) that also writes the
// row-block backward's tile intervals (msda_win.hip): for every (b, m, level, query tile of 32)
// the rows [lo, hi] its samples touch or own (win_sample_rows, msda_win.h).  One 256-thread
// workgroup per (b, m, tile): its 32 items are the tile's queries of one head, so the intervals
// are reduced in the workgroup (xor shuffles over the 8 items of a wave, then LDS over the 4
// waves) and written once, no atomics — the backward then skips its interval prepass (a kernel
// that re-read all of loc: 11 us at the bench's encoder call).  Items in (b, m, q) order: each
// still reads its 64-B loc / aw rows and writes its 128-B output row whole.
template <typename scalar_t, bool ZEROS, int P, bool LM>
__global__ __launch_bounds__(256) void msda_fwd16_tiles_kernel(
    const scalar_t* __restrict__ value, const float* __restrict__ loc, const float* __restrict__ aw,
    scalar_t* __restrict__ out, int2* __restrict__ tiles, const Levels lv, const int L, const int S, const int M,
    const int Lq, const int ntile, const QOrder qo) {
  constexpr int VEC = 8, D = 64, NL = kLPMax / P;
  __shared__ int2 s_iv[4][NL];
  write_tiles_tail(tiles, (long long)gridDim.x * L, qo);
  const unsigned wg = xcd_block(blockIdx.x, gridDim.x);
  const unsigned bm = wg / (unsigned)ntile;
  const int tile = (int)(wg % (unsigned)ntile);
  const int m = (int)(bm % (unsigned)M);
  const long long b = bm / (unsigned)M;
  const int i = threadIdx.x >> 3, lg = threadIdx.x & 7;
  const int q = tile * kWinQT + i < Lq ? qo_query(qo, tile * kWinQT + i) : Lq;  // (msda_win.h: the tile order)
  const int LP = L * P;
  int lo[NL], hi[NL];
#pragma unroll
  for (int l = 0; l < NL; ++l) {
    lo[l] = kWinNone;
    hi[l] = -kWinNone;
  }
  if (q < Lq) {
    const long long item = (b * Lq + q) * M + m;
    float lr[kLPMax], ar[kLPMax];
    if constexpr (LM) {
      const long long c0 = ((b * M + m) * L * Lq + q) * P;
      load_coords16_lm(loc + c0, (long long)Lq * P, L, P, lr);
      load_coords16_lm(aw + c0, (long long)Lq * P, L, P, ar);
    } else {
      load_coords16(loc + item * LP, LP, lr);
      load_coords16(aw + item * LP, LP, ar);
    }
    fwd16_item<scalar_t, VEC, ZEROS>(value + (b * S * M + m) * (long long)D + lg * VEC, lr, ar, lv, P, LP, M * D,
                                     out + item * D + lg * VEC);
#pragma unroll
    for (int j = 0; j < kLPMax; ++j) {
      if (j < LP) {
        const int2 r = win_sample_rows(lr[j], lv.T[j / P], ZEROS);
        lo[j / P] = min(lo[j / P], r.x);
        hi[j / P] = max(hi[j / P], r.y);
      }
    }
  }
#pragma unroll
  for (int l = 0; l < NL; ++l) {
#pragma unroll
    for (int o = 8; o < 64; o <<= 1) {
      lo[l] = min(lo[l], __shfl_xor(lo[l], o));
      hi[l] = max(hi[l], __shfl_xor(hi[l], o));
    }
  }
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
#pragma unroll
    for (int l = 0; l < NL; ++l) s_iv[w][l] = make_int2(lo[l], hi[l]);
  }
  __syncthreads();
  if ((int)threadIdx.x < L) {
    int2 iv = s_iv[0][threadIdx.x];
#pragma unroll
    for (int v = 1; v < 4; ++v) {
      const int2 o = s_iv[v][threadIdx.x];
      iv.x = min(iv.x, o.x);
      iv.y = max(iv.y, o.y);
    }
    tiles[((long long)bm * L + threadIdx.x) * ntile + tile] = iv;
  }
}


// msda_fwd16_tiles_kernel with each wave's value rows staged in its own LDS slice (no workgroup
// barrier on the data path).  A wave holds 8 consecutive queries of one (b, m) (8 lanes an item, as
// msda_fwd16_tiles_kernel); in an encoder call their samples of one level fall in a short window of
// rows (8 consecutive tokens of a level cover 1-64 rows of another, plus the sampling spread: 18-24 %
// of the 64 rows their taps gather, tools/win_visits.py-style count over the microbench sampling), so
// per level the wave reduces its window [lo, hi], loads those rows once (8 lanes a 128-B row,
// coalesced) into its LDS slice and reads the taps there; a level whose window exceeds CAP
// (CAP) rows keeps the global gathers.  The next level's rows are loaded into registers while the current
// level's taps are read (one LDS slice: a wave's LDS accesses are in order).  Same taps, same weights,
// same fp32 accumulation order as fwd16_item: the output is msda_fwd16_tiles_kernel's bit for bit;
// the tile intervals are written the same way (win_sample_rows).  VERDICT r4 item 6: the gathering
// forward moved 503 MB of row fragments out of L2 per encoder call (14.7 TB/s, 34 us).
// CAP: staged rows a wave (48: 6 KB, three waves a SIMD by registers; 32: 4 KB, four)
template <typename scalar_t, bool ZEROS, int P, bool LM, int CAP>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(CAP <= 32 ? 4 : 3))) void msda_fwd16_stage_kernel(
    const scalar_t* __restrict__ value, const float* __restrict__ loc, const float* __restrict__ aw,
    scalar_t* __restrict__ out, int2* __restrict__ tiles, const Levels lv, const int L, const int S, const int M,
    const int Lq, const int ntile, const QOrder qo) {
  constexpr int VEC = 8, D = 64, NL = kLPMax / P, NR = CAP / 8;
  __shared__ int2 s_iv[4][NL];
  __shared__ uint4 s_rows[4][CAP * 8];  // per wave: row k, chunk c at [k * 8 + c]
  write_tiles_tail(tiles, (long long)gridDim.x * L, qo);
  const unsigned wg = xcd_block(blockIdx.x, gridDim.x);
  const unsigned bm = wg / (unsigned)ntile;
  const int tile = (int)(wg % (unsigned)ntile);
  const int m = (int)(bm % (unsigned)M);
  const long long b = bm / (unsigned)M;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int i = threadIdx.x >> 3, lg = threadIdx.x & 7, kr = lane >> 3;
  const int q = tile * kWinQT + i < Lq ? qo_query(qo, tile * kWinQT + i) : Lq;  // (msda_win.h: the tile order)
  const bool valid = q < Lq;
  const int LP = L * P;
  const int rs = M * D;
  uint4* const slice = s_rows[w];
  float lr[kLPMax], ar[kLPMax];
  if (valid) {
    if constexpr (LM) {
      const long long c0 = ((b * M + m) * L * Lq + q) * P;
      load_coords16_lm(loc + c0, (long long)Lq * P, L, P, lr);
      load_coords16_lm(aw + c0, (long long)Lq * P, L, P, ar);
    } else {
      const long long item = (b * Lq + q) * M + m;
      load_coords16(loc + item * LP, LP, lr);
      load_coords16(aw + item * LP, LP, ar);
    }
  } else {
#pragma unroll
    for (int j = 0; j < kLPMax; ++j) lr[j] = ar[j] = 0.f;
  }
  const scalar_t* __restrict__ vb = value + (b * S * M + m) * (long long)D + lg * VEC;
  // the rows level l's valid taps of this wave touch: (lo, n); n = 0 without any
  auto window = [&](int l, int& lo, int& n) {
    int a = 1 << 30, z = -1;
#pragma unroll
    for (int p = 0; p < P; ++p) {
      if (valid && l * P + p < LP) {
        const Taps<float> t = make_taps<float, ZEROS>(lr[l * P + p], lv.T[l]);
        if (t.ok0) { a = min(a, t.i0); z = max(z, t.i0); }
        if (t.ok1) { a = min(a, t.i1); z = max(z, t.i1); }
      }
    }
#pragma unroll
    for (int o = 8; o < 64; o <<= 1) {
      a = min(a, __shfl_xor(a, o));
      z = max(z, __shfl_xor(z, o));
    }
    lo = a;
    n = z >= a ? z - a + 1 : 0;
  };
  uint4 rg[NR];
  auto load_rows = [&](int l, int lo, int n) {
    const scalar_t* __restrict__ vl = vb + (long long)(lv.start[l] + lo) * rs;
#pragma unroll
    for (int k = 0; k < NR; ++k)
      if (kr + 8 * k < n) rg[k] = *reinterpret_cast<const uint4*>(vl + (kr + 8 * k) * rs);
  };
  auto store_rows = [&](int n) {
#pragma unroll
    for (int k = 0; k < NR; ++k)
      if (kr + 8 * k < n) slice[(kr + 8 * k) * 8 + lg] = rg[k];
  };
  f32x2 acc2[VEC / 2];
#pragma unroll
  for (int e = 0; e < VEC / 2; ++e) acc2[e] = f32x2{0.f, 0.f};
  int lo_c = 0, n_c = 0;
  window(0, lo_c, n_c);
  bool st_c = n_c > 0 && n_c <= CAP;
  if (st_c) {
    load_rows(0, lo_c, n_c);
    store_rows(n_c);
  }
  for (int l = 0; l < L; ++l) {
    int lo_n = 0, n_n = 0;
    bool st_n = false;
    if (l + 1 < L) {  // the next level's rows in flight while this level's taps are read
      window(l + 1, lo_n, n_n);
      st_n = n_n > 0 && n_n <= CAP;
      if (st_n) load_rows(l + 1, lo_n, n_n);
    }
    const scalar_t* __restrict__ vl = vb + (long long)lv.start[l] * rs;
#pragma unroll
    for (int p = 0; p < P; ++p) {
      const int j = l * P + p;
      if (j < LP) {
        const Taps<float> t = make_taps<float, ZEROS>(lr[j], lv.T[l]);
        uint4 r0, r1;
        if (st_c) {
          r0 = t.ok0 ? slice[(t.i0 - lo_c) * 8 + lg] : make_uint4(0u, 0u, 0u, 0u);
          r1 = t.ok1 ? slice[(t.i1 - lo_c) * 8 + lg] : make_uint4(0u, 0u, 0u, 0u);
        } else {
          r0 = load16_if(t.ok0, vl + t.i0 * rs);
          r1 = load16_if(t.ok1, vl + t.i1 * rs);
        }
        const float c0 = ar[j] * t.w0, c1 = ar[j] * t.w1;
        f32x2 x0[VEC / 2], x1[VEC / 2];
        cvt16x2<scalar_t, VEC>(r0, x0);
        cvt16x2<scalar_t, VEC>(r1, x1);
        const f32x2 k0{c0, c0}, k1{c1, c1};
#pragma unroll
        for (int e = 0; e < VEC / 2; ++e) acc2[e] = pk_fma(x1[e], k1, pk_fma(x0[e], k0, acc2[e]));
      }
    }
    if (st_n) store_rows(n_n);  // (after this level's LDS reads: in order within the wave)
    lo_c = lo_n;
    n_c = n_n;
    st_c = st_n;
  }
  if (valid) {
    float acc[VEC];
#pragma unroll
    for (int e = 0; e < VEC / 2; ++e) {
      acc[2 * e] = acc2[e].x;
      acc[2 * e + 1] = acc2[e].y;
    }
    store_vec<scalar_t, VEC>(out + ((b * Lq + q) * M + m) * D + lg * VEC, acc);
  }
  // tile intervals (as msda_fwd16_tiles_kernel)
  int lo[NL], hi[NL];
#pragma unroll
  for (int l = 0; l < NL; ++l) {
    lo[l] = kWinNone;
    hi[l] = -kWinNone;
  }
  if (valid) {
#pragma unroll
    for (int j = 0; j < kLPMax; ++j) {
      if (j < LP) {
        const int2 r = win_sample_rows(lr[j], lv.T[j / P], ZEROS);
        lo[j / P] = min(lo[j / P], r.x);
        hi[j / P] = max(hi[j / P], r.y);
      }
    }
  }
#pragma unroll
  for (int l = 0; l < NL; ++l) {
#pragma unroll
    for (int o = 8; o < 64; o <<= 1) {
      lo[l] = min(lo[l], __shfl_xor(lo[l], o));
      hi[l] = max(hi[l], __shfl_xor(hi[l], o));
    }
  }
  if (lane == 0) {
#pragma unroll
    for (int l = 0; l < NL; ++l) s_iv[w][l] = make_int2(lo[l], hi[l]);
  }
  __syncthreads();
  if ((int)threadIdx.x < L) {
    int2 iv = s_iv[0][threadIdx.x];
#pragma unroll
    for (int v = 1; v < 4; ++v) {
      const int2 o = s_iv[v][threadIdx.x];
      iv.x = min(iv.x, o.x);
      iv.y = max(iv.y, o.y);
    }
    tiles[((long long)bm * L + threadIdx.x) * ntile + tile] = iv;
  }
}

// LDS-staged variant of msda_fwd16_tiles_kernel (same items, same output and tile intervals bit
// for bit).  The workgroup's 32 queries of one head sample each level inside the row interval the
// tiles kernel reduces anyway; here the interval is reduced FIRST, the value rows of every level
// whose interval fits the workgroup's row budget are copied into LDS once (8 lanes a 128-B row,
// coalesced), and the taps then read LDS instead of gathering 16-B fragments from L2: an encoder
// tile touches ~90 rows per head (~12 KB) where its taps gathered 128 KB.  Levels that do not fit
// (a coarse-level query tile spans a quarter of the finest level) keep the global gathers, as
// does any tap outside its level's staged rows (never, by construction: make_taps and
// win_sample_rows give the same rows).
constexpr int kFwdStageRows = 256;  // staged rows a workgroup (144-B stride: 36 KB)
constexpr int kFwdRowStride = 144;

template <typename scalar_t, bool ZEROS, int P, bool LM>
__global__ __launch_bounds__(256) void msda_fwd16_lds_kernel(
    const scalar_t* __restrict__ value, const float* __restrict__ loc, const float* __restrict__ aw,
    scalar_t* __restrict__ out, int2* __restrict__ tiles, const Levels lv, const int L, const int S, const int M,
    const int Lq, const int ntile, const QOrder qo) {
  constexpr int VEC = 8, D = 64, NL = kLPMax / P;
  __shared__ int2 s_iv[4][NL];
  __shared__ int s_off[NL], s_lo[NL], s_n[NL + 1];
  __shared__ __attribute__((aligned(16))) unsigned char s_rows[kFwdStageRows * kFwdRowStride];
  write_tiles_tail(tiles, (long long)gridDim.x * L, qo);
  const unsigned wg = xcd_block(blockIdx.x, gridDim.x);
  const unsigned bm = wg / (unsigned)ntile;
  const int tile = (int)(wg % (unsigned)ntile);
  const int m = (int)(bm % (unsigned)M);
  const long long b = bm / (unsigned)M;
  const int i = threadIdx.x >> 3, lg = threadIdx.x & 7;
  const int q = tile * kWinQT + i < Lq ? qo_query(qo, tile * kWinQT + i) : Lq;  // (msda_win.h: the tile order)
  const int LP = L * P;
  const int rs = M * D;
  int lo[NL], hi[NL];
#pragma unroll
  for (int l = 0; l < NL; ++l) {
    lo[l] = kWinNone;
    hi[l] = -kWinNone;
  }
  float lr[kLPMax], ar[kLPMax];
  const bool valid = q < Lq;
  const long long item = (b * Lq + (valid ? q : 0)) * M + m;
  if (valid) {
    if constexpr (LM) {
      const long long c0 = ((b * M + m) * L * Lq + q) * P;
      load_coords16_lm(loc + c0, (long long)Lq * P, L, P, lr);
      load_coords16_lm(aw + c0, (long long)Lq * P, L, P, ar);
    } else {
      load_coords16(loc + item * LP, LP, lr);
      load_coords16(aw + item * LP, LP, ar);
    }
#pragma unroll
    for (int j = 0; j < kLPMax; ++j) {
      if (j < LP) {
        const int2 r = win_sample_rows(lr[j], lv.T[j / P], ZEROS);
        lo[j / P] = min(lo[j / P], r.x);
        hi[j / P] = max(hi[j / P], r.y);
      }
    }
  }
#pragma unroll
  for (int l = 0; l < NL; ++l) {
#pragma unroll
    for (int o = 8; o < 64; o <<= 1) {
      lo[l] = min(lo[l], __shfl_xor(lo[l], o));
      hi[l] = max(hi[l], __shfl_xor(hi[l], o));
    }
  }
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
#pragma unroll
    for (int l = 0; l < NL; ++l) s_iv[w][l] = make_int2(lo[l], hi[l]);
  }
  __syncthreads();
  if ((int)threadIdx.x < L) {
    int2 iv = s_iv[0][threadIdx.x];
#pragma unroll
    for (int v = 1; v < 4; ++v) {
      const int2 o = s_iv[v][threadIdx.x];
      iv.x = min(iv.x, o.x);
      iv.y = max(iv.y, o.y);
    }
    tiles[((long long)bm * L + threadIdx.x) * ntile + tile] = iv;
    s_iv[0][threadIdx.x] = iv;  // (each thread rewrites only its own level's slot)
  }
  __syncthreads();
  if (threadIdx.x == 0) {  // levels staged greedily in order while they fit the row budget
    int used = 0;
    for (int l = 0; l < L; ++l) {
      const int a = max(s_iv[0][l].x, 0), z = min(s_iv[0][l].y, lv.T[l] - 1);
      const int n = z - a + 1;
      if (n > 0 && used + n <= kFwdStageRows) {
        s_off[l] = used;
        s_lo[l] = a;
        s_n[l] = n;
        used += n;
      } else {
        s_off[l] = -1;
        s_lo[l] = 0;
        s_n[l] = 0;
      }
    }
    s_n[NL] = used;
  }
  __syncthreads();
  const int used = s_n[NL];
  const scalar_t* __restrict__ vb = value + (b * S * M + m) * (long long)D + lg * VEC;
  {  // stage: row k of the budget is row s_lo[l] + (k - s_off[l]) of its level l (8 loads in flight)
    constexpr int kU = 8;
    uint4 v[kU];
    int dst[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int k = i + 32 * u;
      dst[u] = -1;
      v[u] = make_uint4(0u, 0u, 0u, 0u);
      if (k < used) {
        // (levels are packed in level order: the staged level holding k is the last with s_off <= k)
        int l = 0;
        for (int x = 0; x < L; ++x)
          if (s_off[x] >= 0 && k >= s_off[x]) l = x;
        const int row = s_lo[l] + (k - s_off[l]);
        v[u] = *reinterpret_cast<const uint4*>(vb + (long long)(lv.start[l] + row) * rs);
        dst[u] = k;
      }
    }
#pragma unroll
    for (int u = 0; u < kU; ++u)
      if (dst[u] >= 0) *reinterpret_cast<uint4*>(s_rows + dst[u] * kFwdRowStride + lg * 16) = v[u];
  }
  __syncthreads();
  if (!valid) return;
  int soff[NL], slo[NL], sn[NL];
#pragma unroll
  for (int l = 0; l < NL; ++l) {
    soff[l] = s_off[l];
    slo[l] = s_lo[l];
    sn[l] = s_n[l];
  }
  f32x2 acc2[VEC / 2];
#pragma unroll
  for (int e = 0; e < VEC / 2; ++e) acc2[e] = f32x2{0.f, 0.f};
  auto fetch = [&](bool ok, int l, int row) -> uint4 {
    if (!ok) return make_uint4(0u, 0u, 0u, 0u);
    const int k = row - slo[l];
    if (soff[l] >= 0 && (unsigned)k < (unsigned)sn[l])
      return *reinterpret_cast<const uint4*>(s_rows + (soff[l] + k) * kFwdRowStride + lg * 16);
    return *reinterpret_cast<const uint4*>(vb + (long long)(lv.start[l] + row) * rs);
  };
#pragma unroll
  for (int j0 = 0; j0 < kLPMax; j0 += 4) {
    if (j0 < LP) {
      uint4 r0[4], r1[4];
      float c0[4], c1[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int l = (j0 + u) / P;
        const Taps<float> t = make_taps<float, ZEROS>(lr[j0 + u], lv.T[l]);
        r0[u] = fetch(t.ok0, l, t.i0);
        r1[u] = fetch(t.ok1, l, t.i1);
        c0[u] = ar[j0 + u] * t.w0;
        c1[u] = ar[j0 + u] * t.w1;
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        f32x2 x0[VEC / 2], x1[VEC / 2];
        cvt16x2<scalar_t, VEC>(r0[u], x0);
        cvt16x2<scalar_t, VEC>(r1[u], x1);
        const f32x2 k0{c0[u], c0[u]}, k1{c1[u], c1[u]};
#pragma unroll
        for (int e = 0; e < VEC / 2; ++e) acc2[e] = pk_fma(x1[e], k1, pk_fma(x0[e], k0, acc2[e]));
      }
    }
  }
  float acc[VEC];
#pragma unroll
  for (int e = 0; e < VEC / 2; ++e) {
    acc[2 * e] = acc2[e].x;
    acc[2 * e + 1] = acc2[e].y;
  }
  store_vec<scalar_t, VEC>(out + item * D + lg * VEC, acc);
}

// ---------------------------------------------------------------------------------
// backward
// ---------------------------------------------------------------------------------
// The backward is the transpose of the forward's sparse gather.  Every tap (sample, k)
// adds aw*w_k*grad_out[b,q,m,:] to value row (b, level_start + i_k, m) and needs the dot
// product d_k = <grad_out[b,q,m,:], value row> for grad_aw / grad_loc.  Three kernels and
// no floating-point atomics anywhere (ds_add_f32 measured ~12x slower than a plain LDS
// read+write pair on gfx950, tools/lds_probe.hip; global fp32 atomics ~1.3 TB/s):
//   1. msda_bwd_sort_kernel  — one workgroup per (b, m, level): histogram of the in-map
//      taps per row with LDS integer atomics, exclusive scan, per-row entry lists
//      {tap id, aw*w} (staged in LDS and written contiguously when they fit) and a row
//      table {first entry, count}.  With MSDA_HIP_DETERMINISTIC=1 the entries of a row are
//      sorted by tap id, so every sum below has a fixed order (bitwise reproducible
//      backward); by default their order is the LDS-atomic arrival order.
//   2. msda_bwd_pull_kernel  — the forward's mirror: 64/NS lanes (one 16-byte access per
//      lane, as the forward) per destination value row walk the row's entries, gather
//      grad_out rows, accumulate in registers and write the row once; the same loop reduces
//      each entry's dot product with the row's values (DPP butterfly over the row's
//      lanes) into the per-tap buffer d.
//   3. msda_bwd_coord_kernel — per sample: grad_aw = w0 d0 + w1 d1,
//      grad_loc = aw * dy/dloc * (d1 - d0)   (d_k = 0 for a tap outside the map).
template <typename coord_t>
struct Entry {
  int q;      // query whose grad_out row this tap pulls
  coord_t w;  // aw * w_k
};

// Deterministic mode's order of a row's list: by query, then weight.  Entries that tie on
// both add the same product, so any order of them gives the same sum.
template <typename coord_t>
__device__ __forceinline__ bool entry_after(const Entry<coord_t>& a, const Entry<coord_t>& b) {
  return a.q > b.q || (a.q == b.q && a.w > b.w);
}

constexpr int kSortThreads = 512;
constexpr long long kSortLdsMax = 150 * 1024;  // LDS staging of a level's entry lists

// exclusive scan of one value per thread over the workgroup; returns the thread's prefix,
// *total gets the sum.  scratch: >= kSortThreads/64 + 1 ints of LDS.
__device__ __forceinline__ int block_exclusive_scan(int x, int* scratch, int* total) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int incl = x;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int y = __shfl_up(incl, off);
    if (lane >= off) incl += y;
  }
  if (lane == 63) scratch[wave] = incl;
  __syncthreads();
  if (threadIdx.x == 0) {
    int run = 0;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) {
      const int t = scratch[w];
      scratch[w] = run;
      run += t;
    }
    scratch[blockDim.x >> 6] = run;
  }
  __syncthreads();
  const int res = scratch[wave] + incl - x;
  *total = scratch[blockDim.x >> 6];
  __syncthreads();
  return res;
}

template <typename coord_t, bool ZEROS, bool STAGE>
__global__ __launch_bounds__(kSortThreads) void msda_bwd_sort_kernel(
    const coord_t* __restrict__ loc, const coord_t* __restrict__ aw, int2* __restrict__ rowinfo,
    Entry<coord_t>* __restrict__ entries, const Levels lv, const int L, const int P, const int S,
    const int M, const int Lq, const int sort_rows) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  const unsigned blk = xcd_block(blockIdx.x, gridDim.x);
  const int l = (int)(blk % (unsigned)L);
  const long long bm = blk / (unsigned)L;
  const int m = (int)(bm % M);
  const long long b = bm / M;
  const int T = lv.T[l];
  // LDS: [stage entries (STAGE)][cursor T ints][scan scratch 16 ints]
  const int ncap = 2 * Lq * P;
  Entry<coord_t>* stage = reinterpret_cast<Entry<coord_t>*>(smem_raw);
  int* cur = reinterpret_cast<int*>(smem_raw + (STAGE ? (size_t)ncap * sizeof(Entry<coord_t>) : 0));
  int* scratch = cur + T;

  for (int i = threadIdx.x; i < T; i += kSortThreads) cur[i] = 0;
  __syncthreads();

  const int LP = L * P;
  const long long qs = (long long)M * LP;
  const coord_t* __restrict__ locb = loc + (b * Lq * M + m) * LP + l * P;
  const coord_t* __restrict__ awb = aw + (b * Lq * M + m) * LP + l * P;
  const int nsamp = Lq * P;

  // pass 1: taps per row
  for (int s = threadIdx.x; s < nsamp; s += kSortThreads) {
    const int q = s / P, p = s - (s / P) * P;
    const Taps<coord_t> t = make_taps<coord_t, ZEROS>(locb[q * qs + p], T);
    if (t.ok0) atomicAdd(&cur[t.i0], 1);
    if (t.ok1) atomicAdd(&cur[t.i1], 1);
  }
  __syncthreads();

  // exclusive scan over rows: thread i owns rows [i*chunk, (i+1)*chunk)
  const int chunk = (T + kSortThreads - 1) / kSortThreads;
  const int lo = min((int)threadIdx.x * chunk, T), hi = min(lo + chunk, T);
  int mine = 0;
  for (int i = lo; i < hi; ++i) mine += cur[i];
  int total = 0;
  int run = block_exclusive_scan(mine, scratch, &total);
  const long long base = (bm * L + l) * (long long)ncap;  // this (b, m, level)'s entry region
  int2* __restrict__ rinfo = rowinfo + bm * S + lv.start[l];
  for (int i = lo; i < hi; ++i) {
    const int c = cur[i];
    rinfo[i] = make_int2((int)(base + run), c);  // base + run < 2^31 (checked on the host)
    cur[i] = run;
    run += c;
  }
  __syncthreads();

  // pass 2: place the entries
  for (int s = threadIdx.x; s < nsamp; s += kSortThreads) {
    const int q = s / P, p = s - (s / P) * P;
    const coord_t a = awb[q * qs + p];
    const Taps<coord_t> t = make_taps<coord_t, ZEROS>(locb[q * qs + p], T);
    if (t.ok0) {
      const int pos = atomicAdd(&cur[t.i0], 1);
      Entry<coord_t> e{q, a * t.w0};
      if constexpr (STAGE) stage[pos] = e; else entries[base + pos] = e;
    }
    if (t.ok1) {
      const int pos = atomicAdd(&cur[t.i1], 1);
      Entry<coord_t> e{q, a * t.w1};
      if constexpr (STAGE) stage[pos] = e; else entries[base + pos] = e;
    }
  }
  __syncthreads();
  // cur[i] now = end of row i.  In deterministic mode each row's list is sorted by tap id
  // (insertion sort by the row's owner thread: O(n^2) in the row length, so off by
  // default) so the pull kernel sums in a fixed order; then write out.
  if constexpr (STAGE) {
    for (int i = lo; i < hi && sort_rows; ++i) {
      const int e1 = cur[i], e0 = (i == 0 ? 0 : cur[i - 1]);
      for (int x = e0 + 1; x < e1; ++x) {
        const Entry<coord_t> key = stage[x];
        int y = x - 1;
        while (y >= e0 && entry_after(stage[y], key)) {
          stage[y + 1] = stage[y];
          --y;
        }
        stage[y + 1] = key;
      }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < total; i += kSortThreads) entries[base + i] = stage[i];
  } else {
    __threadfence_block();
    for (int i = lo; i < hi && sort_rows; ++i) {
      const int e1 = cur[i], e0 = (i == 0 ? 0 : cur[i - 1]);
      for (int x = e0 + 1; x < e1; ++x) {
        const Entry<coord_t> key = entries[base + x];
        int y = x - 1;
        while (y >= e0 && entry_after(entries[base + y], key)) {
          entries[base + y + 1] = entries[base + y];
          --y;
        }
        entries[base + y + 1] = key;
      }
    }
  }
}

// Sum of x over aligned groups of N lanes (N = 2..64), result in every lane of the group.
// Up to 16 lanes with DPP (quad_perm / row_half_mirror / row_mirror: VALU only, no LDS
// crossbar); beyond that ds_bpermute.
template <int N>
__device__ __forceinline__ float group_sum(float x) {
  if constexpr (N >= 2) x += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0xB1, 0xF, 0xF, false));
  if constexpr (N >= 4) x += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0x4E, 0xF, 0xF, false));
  if constexpr (N >= 8) x += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0x141, 0xF, 0xF, false));
  if constexpr (N >= 16) x += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0x140, 0xF, 0xF, false));
  if constexpr (N >= 32) x += __shfl_xor(x, 16);
  if constexpr (N >= 64) x += __shfl_xor(x, 32);
  return x;
}
template <int N>
__device__ __forceinline__ double group_sum(double x) {
#pragma unroll
  for (int off = N >> 1; off > 0; off >>= 1) x += __shfl_xor(x, off);
  return x;
}

constexpr int kPullThreads = 256;

// Row order of the pull: clip-major (with the XCD block order, a clip's grad_out rows stay in
// one L2), then levels by decreasing taps per row (T ascending: a level's rows all receive
// ~2*Lq*P/T_l taps), so the longest-running waves start first instead of forming the tail.
// Inside a clip, rows of level lvl[i] occupy [cum[i], cum[i+1]) as (m, s).
struct PullOrder {
  int lvl[MSDA_MAX_LEVELS];
  long long cum[MSDA_MAX_LEVELS + 1];
};

// NSLOT rows per wave, LPR = 64/NSLOT lanes per row, CPL = 16 B / sizeof(scalar_t) channels
// per lane (one 16-byte load per lane per row, as the forward); NSLOT = 0: generic path,
// one row per wave, lane = channel, D in passes of 64.
template <typename scalar_t, typename coord_t, int NSLOT>
__global__ __launch_bounds__(kPullThreads) void msda_bwd_pull_kernel(
    const scalar_t* __restrict__ gout, const int2* __restrict__ rowinfo,
    const Entry<coord_t>* __restrict__ entries, scalar_t* __restrict__ gval, const int S,
    const int M, const int D, const int Lq, const int P, const long long nrows, const Levels lv,
    const PullOrder po) {
  using acc_t = typename AccOf<scalar_t>::type;
  constexpr int CPL = NSLOT > 0 ? 16 / (int)sizeof(scalar_t) : 1;
  constexpr int NS = NSLOT > 0 ? NSLOT : 1;
  constexpr int LPR = 64 / NS;                            // lanes per row
  constexpr int U = NSLOT > 0 ? (64 / CPL < LPR ? 64 / CPL : LPR) : 16;  // loads in flight
  const int lane = threadIdx.x & 63;
  const int slot = lane / LPR;
  const int cl = lane - slot * LPR;
  const long long wave_id = ((long long)xcd_block(blockIdx.x, gridDim.x) * kPullThreads + threadIdx.x) >> 6;
  const long long row = wave_id * NS + slot;  // (b, m, s) flattened as (b*M + m)*S + s
  const bool valid = row < nrows;
  const long long ro = valid ? row : 0;
  const long long ms = (long long)M * S;
  const long long bq = ro / ms;
  const long long rem = ro - bq * ms;
  int i = 0;
  while (rem >= po.cum[i + 1]) ++i;
  const int l = po.lvl[i];
  const long long off = rem - po.cum[i];
  const long long mq = off / lv.T[l];
  const int s = lv.start[l] + (int)(off - mq * lv.T[l]);
  const long long bm = bq * M + mq;
  const long long rr = bm * S + s;
  const int m = (int)(bm % M);
  const long long b = bm / M;
  const int2 info = valid ? rowinfo[rr] : make_int2(0, 0);
  const int start = info.x, count = valid ? info.y : 0;
  const long long vrow = ((b * S + s) * M + m) * (long long)D;
  const long long gq = (long long)M * D;
  const scalar_t* __restrict__ gb = gout + (b * Lq * M + m) * (long long)D;

  const int npass = NSLOT > 0 ? 1 : (D + 63) / 64;
  for (int pass = 0; pass < npass; ++pass) {
    const int c0 = NSLOT > 0 ? cl * CPL : pass * 64 + lane;
    const bool on = valid && c0 < D;
    acc_t acc[CPL];
#pragma unroll
    for (int e = 0; e < CPL; ++e) acc[e] = (acc_t)0;
    // entries in chunks of LPR: lane cl of a row loads entry j0 + cl (coalesced), the next
    // chunk is prefetched, each entry is broadcast to the row's lanes with a shuffle, and U
    // grad_out row loads are in flight at once.
    Entry<coord_t> nxt = (cl < count) ? entries[start + cl] : Entry<coord_t>{0, (coord_t)0};
    for (int j0 = 0; __ballot(j0 < count) != 0ull; j0 += LPR) {
      const Entry<coord_t> cur = nxt;
      nxt = (j0 + LPR + cl < count) ? entries[start + j0 + LPR + cl] : Entry<coord_t>{0, (coord_t)0};
      const int nchunk = min(LPR, count - j0);  // <= 0 for a finished row
      for (int u0 = 0; __ballot(u0 < nchunk) != 0ull; u0 += U) {
        int qq[U];
        acc_t w[U], g[U][CPL];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int src = slot * LPR + u0 + u;
          qq[u] = __shfl(cur.q, src);
          w[u] = (acc_t)__shfl(cur.w, src);
          const bool have = u0 + u < nchunk;
          if (have && on) load_vec<scalar_t, CPL>(gb + qq[u] * gq + c0, g[u]);
          else {
#pragma unroll
            for (int e = 0; e < CPL; ++e) g[u][e] = (acc_t)0;
          }
          if (!have) w[u] = (acc_t)0;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
#pragma unroll
          for (int e = 0; e < CPL; ++e) acc[e] += w[u] * g[u][e];
        }
      }
    }
    if (on) {
      if constexpr (NSLOT > 0) store_vec<scalar_t, CPL>(gval + vrow + c0, acc);
      else from_acc(acc[0], gval + vrow + c0);
    }
  }
}

// Fused sort + pull: one 1024-thread workgroup per (b, m, level) builds the level's per-row
// entry lists in LDS exactly as msda_bwd_sort_kernel does, then pulls every value row of the
// level from them (the pull kernel's lane layout: NS rows per wave, 16 B per lane).  The entry
// lists never leave LDS, there is no row table, and a single launch replaces two.  Used when
// the lists fit in LDS (2*Lq*P entries + T_l cursors <= kGvLdsMax) and there are enough
// (b, m, level) workgroups to fill the chip; otherwise sort + pull.
constexpr int kGvThreads = 1024;
constexpr long long kGvLdsMax = 160 * 1024;
constexpr int kGvCache = 8;  // samples per thread whose loc / aw stay in registers between passes

template <typename scalar_t, typename coord_t, int NSLOT, bool ZEROS>
__global__ __launch_bounds__(kGvThreads) void msda_bwd_gvalue_kernel(
    const coord_t* __restrict__ loc, const coord_t* __restrict__ aw,
    const scalar_t* __restrict__ gout, scalar_t* __restrict__ gval, const Levels lv,
    const int L, const int P, const int S, const int M, const int D, const int Lq,
    const int sort_rows) {
  using acc_t = typename AccOf<scalar_t>::type;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  const unsigned blk = xcd_block(blockIdx.x, gridDim.x);
  const int l = (int)(blk % (unsigned)L);
  const long long bm = blk / (unsigned)L;
  const int m = (int)(bm % M);
  const long long b = bm / M;
  const int T = lv.T[l];
  const int ncap = 2 * Lq * P;
#ifdef MSDA_PHASE_TIMING  // debug build only: per-phase wall clock of two workgroups
  unsigned long long tph[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  tph[0] = wall_clock64();
#define MSDA_PH(i) do { __syncthreads(); tph[i] = wall_clock64(); } while (0)
#else
#define MSDA_PH(i) do { } while (0)
#endif
  Entry<coord_t>* ent = reinterpret_cast<Entry<coord_t>*>(smem_raw);
  int* cur = reinterpret_cast<int*>(smem_raw + (size_t)ncap * sizeof(Entry<coord_t>));
  int* scratch = cur + T;

  for (int i = threadIdx.x; i < T; i += kGvThreads) cur[i] = 0;
  __syncthreads();
  MSDA_PH(1);

  const int LP = L * P;
  const long long qs = (long long)M * LP;
  const coord_t* __restrict__ locb = loc + (b * Lq * M + m) * LP + l * P;
  const coord_t* __restrict__ awb = aw + (b * Lq * M + m) * LP + l * P;
  const int nsamp = Lq * P;

  // pass 1: taps per row; the first kGvCache samples of every thread keep loc / aw in registers
  coord_t cl[kGvCache], ca[kGvCache];
#pragma unroll
  for (int k = 0; k < kGvCache; ++k) {
    const int s = threadIdx.x + k * kGvThreads;
    if (s < nsamp) {
      const int q = s / P, p = s - (s / P) * P;
      cl[k] = locb[q * qs + p];
      ca[k] = awb[q * qs + p];
    }
  }
#pragma unroll
  for (int k = 0; k < kGvCache; ++k) {
    const int s = threadIdx.x + k * kGvThreads;
    if (s < nsamp) {
      const Taps<coord_t> t = make_taps<coord_t, ZEROS>(cl[k], T);
      if (t.ok0) atomicAdd(&cur[t.i0], 1);
      if (t.ok1) atomicAdd(&cur[t.i1], 1);
    }
  }
  for (int s = threadIdx.x + kGvCache * kGvThreads; s < nsamp; s += kGvThreads) {
    const int q = s / P, p = s - (s / P) * P;
    const Taps<coord_t> t = make_taps<coord_t, ZEROS>(locb[q * qs + p], T);
    if (t.ok0) atomicAdd(&cur[t.i0], 1);
    if (t.ok1) atomicAdd(&cur[t.i1], 1);
  }
  __syncthreads();
  MSDA_PH(2);

  // exclusive scan over rows: thread i owns rows [i*chunk, (i+1)*chunk)
  const int chunk = (T + kGvThreads - 1) / kGvThreads;
  const int lo = min((int)threadIdx.x * chunk, T), hi = min(lo + chunk, T);
  int mine = 0;
  for (int i = lo; i < hi; ++i) mine += cur[i];
  int total = 0;
  int run = block_exclusive_scan(mine, scratch, &total);
  for (int i = lo; i < hi; ++i) {
    const int c = cur[i];
    cur[i] = run;
    run += c;
  }
  __syncthreads();
  MSDA_PH(3);

  // pass 2: place the entries (cur[i] ends at the end of row i)
#pragma unroll
  for (int k = 0; k < kGvCache; ++k) {
    const int s = threadIdx.x + k * kGvThreads;
    if (s < nsamp) {
      const Taps<coord_t> t = make_taps<coord_t, ZEROS>(cl[k], T);
      const int q = s / P;
      if (t.ok0) ent[atomicAdd(&cur[t.i0], 1)] = Entry<coord_t>{q, ca[k] * t.w0};
      if (t.ok1) ent[atomicAdd(&cur[t.i1], 1)] = Entry<coord_t>{q, ca[k] * t.w1};
    }
  }
  for (int s = threadIdx.x + kGvCache * kGvThreads; s < nsamp; s += kGvThreads) {
    const int q = s / P, p = s - (s / P) * P;
    const coord_t a = awb[q * qs + p];
    const Taps<coord_t> t = make_taps<coord_t, ZEROS>(locb[q * qs + p], T);
    if (t.ok0) ent[atomicAdd(&cur[t.i0], 1)] = Entry<coord_t>{q, a * t.w0};
    if (t.ok1) ent[atomicAdd(&cur[t.i1], 1)] = Entry<coord_t>{q, a * t.w1};
  }
  __syncthreads();
  MSDA_PH(4);
  if (sort_rows) {  // deterministic mode: each row's list in tap order (insertion sort)
    for (int i = lo; i < hi; ++i) {
      const int e1 = cur[i], e0 = (i == 0 ? 0 : cur[i - 1]);
      for (int x = e0 + 1; x < e1; ++x) {
        const Entry<coord_t> key = ent[x];
        int y = x - 1;
        while (y >= e0 && entry_after(ent[y], key)) {
          ent[y + 1] = ent[y];
          --y;
        }
        ent[y + 1] = key;
      }
    }
    __syncthreads();
  }

  // pull: NS rows per wave-iteration, LPR lanes x CPL channels per row
  constexpr int CPL = NSLOT > 0 ? 16 / (int)sizeof(scalar_t) : 1;
  constexpr int NS = NSLOT > 0 ? NSLOT : 1;
  constexpr int LPR = 64 / NS;
  constexpr int U = 8;  // grad_out loads in flight per lane
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int slot = lane / LPR;
  const int c_l = lane - slot * LPR;
  const long long gq = (long long)M * D;
  const scalar_t* __restrict__ gb = gout + (b * Lq * M + m) * (long long)D;
  scalar_t* __restrict__ gvl = gval + ((b * S + lv.start[l]) * M + m) * (long long)D;
  const int npass = NSLOT > 0 ? 1 : (D + 63) / 64;
  for (int r0 = wave * NS; r0 < T; r0 += (kGvThreads / 64) * NS) {
    const int row = r0 + slot;
    const bool valid = row < T;
    const int e0 = valid ? (row == 0 ? 0 : cur[row - 1]) : 0;
    const int count = valid ? cur[row] - e0 : 0;
    for (int pass = 0; pass < npass; ++pass) {
      const int c0 = NSLOT > 0 ? c_l * CPL : pass * 64 + lane;
      const bool on = valid && c0 < D;
      acc_t acc[CPL];
#pragma unroll
      for (int e = 0; e < CPL; ++e) acc[e] = (acc_t)0;
      for (int j0 = 0; __ballot(j0 < count) != 0ull; j0 += U) {
        acc_t w[U], g[U][CPL];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const bool have = j0 + u < count;
          const Entry<coord_t> e = have ? ent[e0 + j0 + u] : Entry<coord_t>{0, (coord_t)0};
          w[u] = (acc_t)e.w;
          if (have && on) load_vec<scalar_t, CPL>(gb + e.q * gq + c0, g[u]);
          else {
#pragma unroll
            for (int x = 0; x < CPL; ++x) g[u][x] = (acc_t)0;
          }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
#pragma unroll
          for (int x = 0; x < CPL; ++x) acc[x] += w[u] * g[u][x];
        }
      }
      if (on) {
        if constexpr (NSLOT > 0) store_vec<scalar_t, CPL>(gvl + (long long)row * gq + c0, acc);
        else from_acc(acc[0], gvl + (long long)row * gq + c0);
      }
    }
  }
#ifdef MSDA_PHASE_TIMING
  MSDA_PH(5);
  if (threadIdx.x == 0 && bm == 0)
    printf("gvalue l=%d T=%d ncap=%d zero=%llu pass1=%llu scan=%llu pass2=%llu pull=%llu (x10ns)\n", l, T,
           ncap, tph[1] - tph[0], tph[2] - tph[1], tph[3] - tph[2], tph[4] - tph[3], tph[5] - tph[4]);
#endif
#undef MSDA_PH
}

// Fused backward: grad_value, grad_loc and grad_attn in ONE launch, one 1024-thread workgroup
// per (b, m, level).  Both taps of a sample lie in the same level, so everything a sample's
// coordinate gradients need is produced inside its level's workgroup:
//   1-3. histogram / scan / place (as msda_bwd_gvalue_kernel): per-row lists of the level's
//        in-map taps, key = q << 8 | (2p + k), in LDS; wd[tap] = aw * w_k (0 off the map);
//   4.   pull: the owner lanes of a value row hold that row of `value` in registers and walk
//        its list; every gathered grad_out row is used twice — accumulated into grad_value
//        (aw * w_k * g) and dotted with the value row, d_k = <g, v_row> (DPP reduction over the
//        row's lanes), which overwrites wd[tap] (each tap has exactly one entry);
//   5.   epilogue: per sample, grad_attn = w0 d0 + w1 d1, grad_loc = aw dy/dloc (d1 - d0).
// So the backward gathers grad_out once per tap and never gathers value rows — half the row
// fragments of the sort/pull + coordinate-kernel pair (tools/msda_microbench.py).
// LDS: 8 B per tap (key, wd) + 4 B per row.  COORDS=false: grad_value only.
template <typename scalar_t, int NSLOT, bool ZEROS, bool COORDS, int U>
__global__ __launch_bounds__(kGvThreads) void msda_bwd_fused_kernel(
    const scalar_t* __restrict__ value, const float* __restrict__ loc, const float* __restrict__ aw,
    const scalar_t* __restrict__ gout, scalar_t* __restrict__ gval, float* __restrict__ gloc,
    float* __restrict__ gaw, const Levels lv, const int L, const int P, const int S, const int M,
    const int D, const int Lq, const int sort_rows, const int gv_rs) {
  static_assert(NSLOT > 0, "fused backward needs whole 16-byte chunks per lane");
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  const unsigned blk = xcd_block(blockIdx.x, gridDim.x);
  const int l = (int)(blk % (unsigned)L);
  const long long bm = blk / (unsigned)L;
  const int m = (int)(bm % M);
  const long long b = bm / M;
  const int T = lv.T[l];
  const int nsamp = Lq * P;
  const int ncap = 2 * nsamp;
  unsigned* ent = reinterpret_cast<unsigned*>(smem_raw);
  float* wd = reinterpret_cast<float*>(smem_raw + (size_t)ncap * 4);
  int* cur = reinterpret_cast<int*>(smem_raw + (size_t)ncap * 8);
  int* scratch = cur + T;
#ifdef MSDA_PHASE_TIMING  // debug build only: per-phase wall clock of the (b=0, m=0) workgroups
  unsigned long long tph[7];
  tph[0] = wall_clock64();
#define MSDA_PH(i) do { __syncthreads(); tph[i] = wall_clock64(); } while (0)
#else
#define MSDA_PH(i) do { } while (0)
#endif

  for (int i = threadIdx.x; i < T; i += kGvThreads) cur[i] = 0;
  __syncthreads();
  MSDA_PH(1);

  const int LP = L * P;
  const long long qs = (long long)M * LP;
  const float* __restrict__ locb = loc + (b * Lq * M + m) * LP + l * P;
  const float* __restrict__ awb = aw + (b * Lq * M + m) * LP + l * P;

  // 1. taps per row; the first kGvCache samples of every thread keep loc / aw in registers
  float cl[kGvCache], ca[kGvCache];
#pragma unroll
  for (int k = 0; k < kGvCache; ++k) {
    const int s = threadIdx.x + k * kGvThreads;
    if (s < nsamp) {
      const int q = s / P, p = s - (s / P) * P;
      cl[k] = locb[q * qs + p];
      ca[k] = awb[q * qs + p];
    }
  }
#pragma unroll
  for (int k = 0; k < kGvCache; ++k) {
    const int s = threadIdx.x + k * kGvThreads;
    if (s < nsamp) {
      const Taps<float> t = make_taps<float, ZEROS>(cl[k], T);
      if (t.ok0) atomicAdd(&cur[t.i0], 1);
      if (t.ok1) atomicAdd(&cur[t.i1], 1);
    }
  }
  for (int s = threadIdx.x + kGvCache * kGvThreads; s < nsamp; s += kGvThreads) {
    const int q = s / P, p = s - (s / P) * P;
    const Taps<float> t = make_taps<float, ZEROS>(locb[q * qs + p], T);
    if (t.ok0) atomicAdd(&cur[t.i0], 1);
    if (t.ok1) atomicAdd(&cur[t.i1], 1);
  }
  __syncthreads();
  MSDA_PH(2);

  // 2. exclusive scan over rows: thread i owns rows [i*chunk, (i+1)*chunk)
  const int chunk = (T + kGvThreads - 1) / kGvThreads;
  const int lo = min((int)threadIdx.x * chunk, T), hi = min(lo + chunk, T);
  {
    int mine = 0;
    for (int i = lo; i < hi; ++i) mine += cur[i];
    int total = 0;
    int run = block_exclusive_scan(mine, scratch, &total);
    for (int i = lo; i < hi; ++i) {
      const int c = cur[i];
      cur[i] = run;
      run += c;
    }
  }
  __syncthreads();
  MSDA_PH(3);

  // 3. place the keys (cur[i] ends at the end of row i) and the tap weights
  auto place = [&](int s, float lc, float a) {
    const Taps<float> t = make_taps<float, ZEROS>(lc, T);
    const int q = s / P, p = s - q * P;
    const unsigned key = ((unsigned)q << 8) | (unsigned)(2 * p);
    if (t.ok0) ent[atomicAdd(&cur[t.i0], 1)] = key;
    if (t.ok1) ent[atomicAdd(&cur[t.i1], 1)] = key | 1u;
    wd[2 * s] = t.ok0 ? a * t.w0 : 0.f;
    wd[2 * s + 1] = t.ok1 ? a * t.w1 : 0.f;
  };
#pragma unroll
  for (int k = 0; k < kGvCache; ++k) {
    const int s = threadIdx.x + k * kGvThreads;
    if (s < nsamp) place(s, cl[k], ca[k]);
  }
  for (int s = threadIdx.x + kGvCache * kGvThreads; s < nsamp; s += kGvThreads) {
    const int q = s / P, p = s - q * P;
    place(s, locb[q * qs + p], awb[q * qs + p]);
  }
  __syncthreads();
  if (sort_rows) {  // deterministic mode: each row's list in tap order (insertion sort)
    for (int i = lo; i < hi; ++i) {
      const int e1 = cur[i], e0 = (i == 0 ? 0 : cur[i - 1]);
      for (int x = e0 + 1; x < e1; ++x) {
        const unsigned key = ent[x];
        int y = x - 1;
        while (y >= e0 && ent[y] > key) {
          ent[y + 1] = ent[y];
          --y;
        }
        ent[y + 1] = key;
      }
    }
    __syncthreads();
  }
  MSDA_PH(4);

  // 4. pull: NS rows per wave-iteration, LPR lanes x CPL channels (16 bytes) per row
  constexpr int CPL = 16 / (int)sizeof(scalar_t);
  constexpr int NS = NSLOT;
  constexpr int LPR = 64 / NS;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int slot = lane / LPR;
  const int c_l = lane - slot * LPR;
  const int rs = M * D;  // row stride; offsets inside one clip fit 32 bits
  const int twoP = 2 * P;
  const scalar_t* __restrict__ gb = gout + (b * Lq * M + m) * (long long)D + c_l * CPL;
  const long long vofs = ((b * S + lv.start[l]) * M + m) * (long long)D + c_l * CPL;
  const scalar_t* __restrict__ vl = value + vofs;
  // grad_value rows gv_rs elements apart (M * D, or a caller's strided slot: the decoder layers'
  // stacked value gradients, models/modules/value_proj.py)
  scalar_t* __restrict__ gvl = gval + ((b * S + lv.start[l]) * gv_rs + (long long)m * D + c_l * CPL);
  // Per wave iteration NS slots of LPR lanes; SPR consecutive slots share one value row
  // (slots-per-row, from the level's average taps per row: 1 for the fine levels, up to NS for
  // the coarsest), each taking every SPR-th entry of the row's list, so a long row is not walked
  // by one slot while the others idle; the SPR partial sums meet through lane shuffles.  Per
  // batch U grad_out fragments in flight.  (A software-pipelined variant that kept the next batch
  // in flight while consuming this one measured slower: 93 vs 81 us at the encoder shape.)
  const int avg_taps = ncap / T;
  int SPR = avg_taps >= 96 ? 8 : avg_taps >= 48 ? 4 : avg_taps >= 24 ? 2 : 1;
  SPR = SPR > NS ? NS : SPR;
#ifdef MSDA_NO_SPR  // A/B builds only
  SPR = 1;
#endif
  const int rpi = NS / SPR;  // value rows per wave iteration
  const int sub = slot % SPR;
  for (int r0 = wave * rpi; r0 < T; r0 += (kGvThreads / 64) * rpi) {
    const int row = r0 + slot / SPR;
    const bool valid = row < T;
    const int e0 = valid ? (row == 0 ? 0 : cur[row - 1]) : 0;
    const int count = valid ? cur[row] - e0 : 0;
    const int csub = count > sub ? (count - sub + SPR - 1) / SPR : 0;  // entries sub, sub+SPR, ...
    uint4 vr = make_uint4(0u, 0u, 0u, 0u);
    if constexpr (COORDS) vr = load16_if_nt(csub > 0, vl + row * rs);
    f32x2 acc[CPL / 2];
#pragma unroll
    for (int e = 0; e < CPL / 2; ++e) acc[e] = f32x2{0.f, 0.f};
    for (int j0 = 0; __ballot(j0 < csub) != 0ull; j0 += U) {
      // registers hold only the U gathered fragments; the keys and tap weights are read
      // from LDS again when consumed (a ds_read is ~50 cycles, a gather thousands)
      uint4 g[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const bool have = j0 + u < csub;
        const unsigned key = have ? ent[e0 + sub + (j0 + u) * SPR] : 0u;
        g[u] = load16_if(have, gb + (int)(key >> 8) * rs);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const bool have = j0 + u < csub;
        const unsigned key = have ? ent[e0 + sub + (j0 + u) * SPR] : 0u;
        const int tt = (int)(key >> 8) * twoP + (int)(key & 0xffu);
        const float w = have ? wd[tt] : 0.f;
        f32x2 x[CPL / 2];
        cvt16x2<scalar_t, CPL>(g[u], x);
        const f32x2 k2{w, w};
#pragma unroll
        for (int e = 0; e < CPL / 2; ++e) acc[e] = pk_fma(x[e], k2, acc[e]);
        if constexpr (COORDS) {
          const float d = group_sum<LPR>(dot16<scalar_t>(g[u], vr));
          if (have && c_l == 0) wd[tt] = d;
        }
      }
    }
    for (int o = LPR; o < LPR * SPR; o <<= 1) {  // sum the row's SPR partials (wave-uniform)
#pragma unroll
      for (int e = 0; e < CPL / 2; ++e) {
        acc[e].x += __shfl_xor(acc[e].x, o);
        acc[e].y += __shfl_xor(acc[e].y, o);
      }
    }
    if (valid && sub == 0) {
      float a[CPL];
#pragma unroll
      for (int e = 0; e < CPL / 2; ++e) {
        a[2 * e] = acc[e].x;
        a[2 * e + 1] = acc[e].y;
      }
      store_vec_nt<scalar_t, CPL>(gvl + row * gv_rs, a);
    }
  }
  MSDA_PH(5);
  if constexpr (COORDS) {
    __syncthreads();
    // 5. coordinate gradients of the level's samples: d_k = wd[2s + k] (0 off the map)
    float* __restrict__ gab = gaw == nullptr ? nullptr : gaw + (b * Lq * M + m) * LP + l * P;
    float* __restrict__ glb = gloc == nullptr ? nullptr : gloc + (b * Lq * M + m) * LP + l * P;
    // the first kGvCache samples of every thread still have loc / aw in registers (pass 1)
#pragma unroll
    for (int k = 0; k < kGvCache; ++k) {
      const int s = threadIdx.x + k * kGvThreads;
      if (s < nsamp) {
        const int q = s / P, p = s - q * P;
        const long long o = q * qs + p;
        const Taps<float> t = make_taps<float, ZEROS>(cl[k], T);
        const float d0 = wd[2 * s], d1 = wd[2 * s + 1];
        if (gab != nullptr) gab[o] = d0 * t.w0 + d1 * t.w1;
        if (glb != nullptr) glb[o] = ((d1 - d0) * ca[k]) * t.gmul;
      }
    }
    for (int s0 = kGvThreads * kGvCache; s0 < nsamp; s0 += kGvThreads * kGvCache) {
      float lc[kGvCache], ac[kGvCache];  // all loads of the batch in flight together
#pragma unroll
      for (int k = 0; k < kGvCache; ++k) {
        const int s = s0 + threadIdx.x + k * kGvThreads;
        if (s < nsamp) {
          const int q = s / P, p = s - q * P;
          lc[k] = locb[q * qs + p];
          ac[k] = awb[q * qs + p];
        }
      }
#pragma unroll
      for (int k = 0; k < kGvCache; ++k) {
        const int s = s0 + threadIdx.x + k * kGvThreads;
        if (s < nsamp) {
          const int q = s / P, p = s - q * P;
          const long long o = q * qs + p;
          const Taps<float> t = make_taps<float, ZEROS>(lc[k], T);
          const float d0 = wd[2 * s], d1 = wd[2 * s + 1];
          if (gab != nullptr) gab[o] = d0 * t.w0 + d1 * t.w1;
          if (glb != nullptr) glb[o] = ((d1 - d0) * ac[k]) * t.gmul;
        }
      }
    }
  }
#ifdef MSDA_PHASE_TIMING
  MSDA_PH(6);
  if (threadIdx.x == 0 && bm == 0)
    printf("fused l=%d T=%d ncap=%d zero=%llu pass1=%llu scan=%llu place=%llu pull=%llu coords=%llu (x10ns)\n", l, T,
           ncap, tph[1] - tph[0], tph[2] - tph[1], tph[3] - tph[2], tph[4] - tph[3], tph[5] - tph[4],
           tph[6] - tph[5]);
#endif
#undef MSDA_PH
}

// ---------------------------------------------------------------------------------
// Pair-pull fused backward (the default backward).
// ---------------------------------------------------------------------------------
// A sample's two taps always sit on consecutive rows i0, i0 + 1 of its level.  The per-tap
// lists of msda_bwd_fused_kernel gather the sample's grad_out row once per tap; here a sample
// is listed ONCE, under its base row r = i0 (r = -1 when only the upper tap is on the map, ZEROS
// mode), and one gathered grad_out row g serves both taps:
//   grad_value[r] = sum_{s in list r} c0_s g_s  +  sum_{s in list r-1} c1_s g_s,   c_k = aw w_k,
// and the same g gives both dots d0 = <g, v_r>, d1 = <g, v_{r+1}>.  Half the gathers of the
// per-tap kernel.  The lists are laid out by base row (list index r + 1) with, per entry, the key
// q << 8 | p and (c0, c1) computed once at placement (12 B of LDS per sample); the pull overwrites
// (c0, c1) with (d0, d1) and a per-entry epilogue turns them into grad_attn = w0 d0 + w1 d1 and
// grad_loc = aw dy/dloc (d1 - d0).  Walking a list r, a slot (LPR lanes x 16 B) keeps two fp32 row
// accumulators (rows r, r+1) and the two value rows; when list r is done row r is final.
//
// Work split.  One (or RS) workgroup(s) per (b, m, level); RS > 1 splits the level's list
// positions at list boundaries, each workgroup re-reading the list just before its window (the
// "pre-list", whose c1 halves complete its first row; nothing else of it is written).  Inside a
// workgroup, by level:
//   * row mode (sparse levels, N <= 4 (T + 1): decoder-like calls): every slot builds whole rows r
//     from lists r-1 (c1) and r (c0), so an entry is gathered by both its rows, but rows are
//     independent: no hand-over, no list walk;
//   * striped mode (T + 1 < 2 x slots: short pyramids, a few rows with tens to thousands of taps
//     each, as cross-modal calls onto the audio pyramid): every wave takes an even share of the
//     positions and its slots stripe through each list together; a finished row is summed over
//     the slots with lane shuffles, stored when all its taps lay in the wave's share, else kept as
//     one of the wave's (at most 4) partial rows, which are summed in wave order at the end;
//   * run mode (otherwise): every slot walks a run of whole lists, slot bounds snapped to list
//     starts at even shares of the positions; the one row two slots share (c1 part of the earlier
//     slot's last list | c0 part of the later slot's first list) is handed over through LDS after
//     the pull, the later slot holding that row in registers meanwhile.
// Rows with no listed tap on either side are written as zeros by a sweep.  No float atomics.
// Deterministic mode (MSDA_HIP_DETERMINISTIC=1): lists sorted by key, so every sum has a fixed
// order.  When 12 B per sample does not fit LDS (T = 4096: 30,720 samples a level, !STG) only the
// keys are kept, loc / aw are loaded beside the gather, the taps recomputed in the pull and the
// coordinate gradients stored from it (run mode only).
struct PairLayout {
  int off_cc, off_pos, off_xb, off_cur, off_pb, off_scr;
};

constexpr int kPairParts = 4;  // partial rows per wave (striped mode)

// STG: 1 = (c0, c1) and sample positions staged in LDS; 2 = staged in a global workspace slice
// of the workgroup (when they do not fit LDS beside the keys); 0 = keys only.
template <typename scalar_t, int NSLOT, bool ZEROS, int STG, int U>
__global__ __launch_bounds__(kGvThreads) void msda_bwd_pair_kernel(
    const scalar_t* __restrict__ value, const float* __restrict__ loc, const float* __restrict__ aw,
    const scalar_t* __restrict__ gout, scalar_t* __restrict__ gval, float* __restrict__ gloc,
    float* __restrict__ gaw, const Levels lv, const int L, const int P, const int S, const int M,
    const int D, const int Lq, const int RS, const unsigned striped_mask, const int sort_rows,
    const PairLayout lay, unsigned char* __restrict__ gstage) {
  static_assert(NSLOT > 0, "pair backward needs whole 16-byte chunks per lane");
  constexpr int CPL = 16 / (int)sizeof(scalar_t);
  constexpr int H = CPL / 2;
  constexpr int LPR = 64 / NSLOT;
  constexpr int NW = kGvThreads / 64;  // waves
  constexpr int W = NW * NSLOT;        // slots per workgroup
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  const unsigned blk = xcd_block(blockIdx.x, gridDim.x);
  const int part = (int)(blk % (unsigned)RS);
  const unsigned lblk = blk / (unsigned)RS;
  const int l = (int)(lblk % (unsigned)L);
  const long long bm = lblk / (unsigned)L;
  const int m = (int)(bm % M);
  const long long b = bm / M;
  const int T = lv.T[l];
  const int NL = T + 1;  // lists by base row r = -1 .. T-1 at list index r + 1
  const int nsamp = Lq * P;
  const bool striped = STG == 1 && ((striped_mask >> l) & 1u) != 0u;
  unsigned* ekey = reinterpret_cast<unsigned*>(smem_raw);
  // an entry's (c0, c1), then (d0, d1); a sample's list position.  STG == 2: in this workgroup's
  // slice of the workspace, [(c0, c1) x Lq*P | position x Lq*P].  Accessors (not one pointer
  // chosen by a condition) so that every access keeps its address space: ds_* for LDS.
  unsigned char* gsl = STG == 2 ? gstage + (size_t)blk * ((size_t)Lq * P * 12) : nullptr;
  auto ECC = [&](int i) -> f32x2& {
    if constexpr (STG == 2) return reinterpret_cast<f32x2*>(gsl)[i];
    else return reinterpret_cast<f32x2*>(smem_raw + lay.off_cc)[i];
  };
  auto POS = [&](int i) -> int& {
    if constexpr (STG == 2) return reinterpret_cast<int*>(gsl + (size_t)Lq * P * 8)[i];
    else return reinterpret_cast<int*>(smem_raw + lay.off_pos)[i];
  };
  // STG == 2: global stores of other waves become visible to this CU's loads only after they
  // completed (a barrier does not wait for them) and L1 holds no stale copy (agent acquire)
  auto gstage_sync = [&]() {
    if constexpr (STG == 2) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if constexpr (STG == 2) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  };
  float* xb = reinterpret_cast<float*>(smem_raw + lay.off_xb);    // hand-overs / wave partials
  int* cur = reinterpret_cast<int*>(smem_raw + lay.off_cur);
  int* pb = reinterpret_cast<int*>(smem_raw + lay.off_pb);
  int* scratch = reinterpret_cast<int*>(smem_raw + lay.off_scr);
#ifdef MSDA_PHASE_TIMING  // debug build only: per-phase wall clock of the (b=0, m=0) workgroups
  unsigned long long tph[6];
  tph[0] = wall_clock64();
#define MSDA_PH(i) do { __syncthreads(); tph[i] = wall_clock64(); } while (0)
#else
#define MSDA_PH(i) do { } while (0)
#endif

  for (int i = threadIdx.x; i < NL; i += kGvThreads) cur[i] = 0;
  __syncthreads();

  const int LP = L * P;
  const long long qs = (long long)M * LP;
  const float* __restrict__ locb = loc + (b * Lq * M + m) * LP + l * P;
  const float* __restrict__ awb = aw + (b * Lq * M + m) * LP + l * P;
  float* __restrict__ gab = gaw == nullptr ? nullptr : gaw + (b * Lq * M + m) * LP + l * P;
  float* __restrict__ glb = gloc == nullptr ? nullptr : gloc + (b * Lq * M + m) * LP + l * P;
  const bool coords = gab != nullptr || glb != nullptr;
  // list index of a sample (base row + 1); -1 when neither tap is on the map (ZEROS)
  auto list_index = [&](const Taps<float>& t) -> int {
    if constexpr (ZEROS) return t.ok0 ? t.i0 + 1 : (t.ok1 ? 0 : -1);
    else return t.i0 + 1;
  };

  // 1. samples per list; the first kGvCache samples of every thread keep loc in registers
  float cl[kGvCache];
#pragma unroll
  for (int k = 0; k < kGvCache; ++k) {
    const int s = threadIdx.x + k * kGvThreads;
    if (s < nsamp) {
      const int q = s / P, p = s - q * P;
      cl[k] = locb[q * qs + p];
    }
  }
#pragma unroll
  for (int k = 0; k < kGvCache; ++k) {
    const int s = threadIdx.x + k * kGvThreads;
    if (s < nsamp) {
      const int li = list_index(make_taps<float, ZEROS>(cl[k], T));
      if (li >= 0) atomicAdd(&cur[li], 1);
    }
  }
  for (int s = threadIdx.x + kGvCache * kGvThreads; s < nsamp; s += kGvThreads) {
    const int q = s / P, p = s - q * P;
    const int li = list_index(make_taps<float, ZEROS>(locb[q * qs + p], T));
    if (li >= 0) atomicAdd(&cur[li], 1);
  }
  __syncthreads();
  MSDA_PH(1);

  // 2. exclusive scan over the lists: thread i owns lists [i*chunk, (i+1)*chunk)
  const int chunk = (NL + kGvThreads - 1) / kGvThreads;
  const int clo = min((int)threadIdx.x * chunk, NL), chi = min(clo + chunk, NL);
  int N = 0;  // listed samples of the level
  {
    int mine = 0;
    for (int i = clo; i < chi; ++i) mine += cur[i];
    int run = block_exclusive_scan(mine, scratch, &N);
    for (int i = clo; i < chi; ++i) {
      const int c = cur[i];
      cur[i] = run;
      run += c;
    }
  }
  __syncthreads();
  // this workgroup's window of positions: snapped to list starts at even shares (cur = starts now)
  auto snap = [&](long long t) -> int {  // first list start >= t (N if none)
    if (t <= 0) return 0;
    if (t >= N || cur[NL - 1] < t) return N;
    int lo = 0, hi = NL - 1;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (cur[mid] >= t) hi = mid; else lo = mid + 1;
    }
    return cur[lo];
  };
  const int wlo = part == 0 ? 0 : snap((long long)N * part / RS);
  const int whi = part == RS - 1 ? N : snap((long long)N * (part + 1) / RS);
  if (RS > 1) __syncthreads();  // every thread has read the starts before placement moves them

  // 3. place key and (c0, c1) in list order (cur[li] ends at the end of list li); STG: the
  // sample's position, for the coordinate epilogue
  auto place = [&](int s, float lc) {
    const Taps<float> t = make_taps<float, ZEROS>(lc, T);
    const int li = list_index(t);
    const int q = s / P, p = s - q * P;
    if (li >= 0) {
      const int pos = atomicAdd(&cur[li], 1);
      ekey[pos] = ((unsigned)q << 8) | (unsigned)p;
      if constexpr (STG) {
        const float a = awb[q * qs + p];
        ECC(pos) = f32x2{t.ok0 ? a * t.w0 : 0.f, t.ok1 ? a * t.w1 : 0.f};
        POS(s) = pos;
      }
    } else if (part == 0) {  // no tap on the map: zero coordinate gradients
      const long long o = q * qs + p;
      if (gab != nullptr) gab[o] = 0.f;
      if (glb != nullptr) glb[o] = 0.f;
    }
  };
#pragma unroll
  for (int k = 0; k < kGvCache; ++k) {
    const int s = threadIdx.x + k * kGvThreads;
    if (s < nsamp) place(s, cl[k]);
  }
  for (int s = threadIdx.x + kGvCache * kGvThreads; s < nsamp; s += kGvThreads) {
    const int q = s / P, p = s - q * P;
    place(s, locb[q * qs + p]);
  }
  gstage_sync();
  if (sort_rows) {  // deterministic mode: every list in key order (insertion sort)
    for (int i = clo; i < chi; ++i) {
      const int e1 = cur[i], e0 = (i == 0 ? 0 : cur[i - 1]);
      for (int x = e0 + 1; x < e1; ++x) {
        const unsigned key = ekey[x];
        f32x2 kc = f32x2{0.f, 0.f};
        if constexpr (STG) kc = ECC(x);
        int y = x - 1;
        while (y >= e0 && ekey[y] > key) {
          ekey[y + 1] = ekey[y];
          if constexpr (STG) ECC(y + 1) = ECC(y);
          --y;
        }
        ekey[y + 1] = key;
        if constexpr (STG) ECC(y + 1) = kc;
      }
    }
    gstage_sync();
    if (STG)  // the sorted positions
      for (int e = (int)threadIdx.x; e < N; e += kGvThreads) {
        const unsigned key = ekey[e];
        POS((int)(key >> 8) * P + (int)(key & 0xffu)) = e;
      }
    gstage_sync();
  }
  MSDA_PH(2);

  // 4. the window's rows and pre-list, then slots (run mode); cur[li] = end of list li now
  auto en = [&](int r) -> int { return cur[r + 1]; };          // end of list r   (r >= -1)
  auto st = [&](int r) -> int { return r >= 0 ? cur[r] : 0; };  // start of list r
  auto snap_e = [&](long long t) -> int {  // first list start >= t (N if none)
    if (t <= 0) return 0;
    if (t >= N || st(T - 1) < t) return N;
    int lo = 0, hi = T - 1;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (st(mid) >= t) hi = mid; else lo = mid + 1;
    }
    return st(lo);
  };
  auto row_of = [&](int pos) -> int {  // base row of the list holding position pos < N
    int lo = -1, hi = T - 1;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;  // arithmetic shift: floor, also for lo = -1
      if (en(mid) > pos) hi = mid; else lo = mid + 1;
    }
    return lo;
  };
  int rlo = 0, rhi = 0, pre = wlo;  // rows [rlo, rhi) are this workgroup's to write from the pull
  if (wlo < whi) {
    const int bf = row_of(wlo), bl = row_of(whi - 1);
    rlo = bf;
    rhi = bl + 1 >= T ? T : (st(bl + 1) == en(bl + 1) ? bl + 2 : bl + 1);
    if (part > 0 && st(bf - 1) < en(bf - 1)) pre = st(bf - 1);
  }
  // row mode (sparse levels: decoder-like calls, a few samples a row): every slot builds whole
  // rows r from the entries of lists r-1 (c1) and r (c0) — each entry gathered by both of its rows,
  // but rows need no hand-over and every slot runs independently
  const bool rowmode = STG == 1 && (long long)N <= 4LL * NL;
  if (!striped && !rowmode && (int)threadIdx.x <= W) {
    const int j = threadIdx.x;
    pb[j] = j == 0 ? pre : (j == W ? whi : snap_e(wlo + (long long)(whi - wlo) * j / W));
  }
  __syncthreads();

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int slot = lane / LPR;
  const int c_l = lane - slot * LPR;
  const int rs = M * D;  // row stride; offsets inside one clip fit 32 bits
  // wave-uniform bases + 32-bit lane offsets
  const scalar_t* __restrict__ gb = gout + (b * Lq * M + m) * (long long)D;
  const long long vofs = ((b * S + lv.start[l]) * M + m) * (long long)D;
  const scalar_t* __restrict__ vl = value + vofs;
  scalar_t* __restrict__ gvl = gval + vofs;
  const int co = c_l * CPL;

  // rows with no listed tap on either side (lists r-1 and r empty) are zero
  {
    const int zlo = (int)((long long)T * part / RS), zhi = (int)((long long)T * (part + 1) / RS);
#ifndef MSDA_PAIR_NO_ZERO  // A/B timing builds only
    for (int x = zlo + wave * NSLOT + slot; x < zhi; x += W)
      if (st(x - 1) == en(x)) *reinterpret_cast<uint4*>(gvl + (x * rs + co)) = make_uint4(0u, 0u, 0u, 0u);
#endif
  }

  // 5. pull
  auto vload = [&](int x) -> uint4 {  // value row x (zeros off the level)
    if (!coords || x < 0 || x >= T) return make_uint4(0u, 0u, 0u, 0u);
    return load16_if_nt(true, vl + (x * rs + co));
  };
  auto store_row = [&](int x, const f32x2 (&a)[H]) {
#ifdef MSDA_PAIR_CHECK
    if (x < 0 || x >= T) {
      printf("pair check: store row %d of T=%d l=%d part=%d striped=%d row=%d\n", x, T, l, part, (int)striped,
             (int)rowmode);
      return;
    }
#endif
    float o[CPL];
#pragma unroll
    for (int e = 0; e < H; ++e) {
      o[2 * e] = a[e].x;
      o[2 * e + 1] = a[e].y;
    }
#ifndef MSDA_PAIR_NO_STORE  // A/B timing builds only
    store_vec_nt<scalar_t, CPL>(gvl + (x * rs + co), o);
#endif
  };
  f32x2 a0[H], a1[H];
#pragma unroll
  for (int e = 0; e < H; ++e) a0[e] = a1[e] = f32x2{0.f, 0.f};
  uint4 v0, v1;
  // one batch: the slot's entries ebase + u * STR below lim, all of list rb (rows rb, rb + 1)
  auto batch = [&](int ebase, int STR, int lim) {
    uint4 g[U];
    f32x2 cc[U];
    float lcv[U], acv[U];
    // steps u that no slot of the wave has an entry for (a list or a share ending inside the
    // batch) are skipped, gather and arithmetic: the pull is VALU-bound (one step is ~40 wave64
    // VALU instructions), and a cut batch computed all U steps before
    int nu = U;
#pragma unroll
    for (int u = 1; u < U; ++u)
      if (nu == U && __ballot(ebase + u * STR < lim) == 0ull) nu = u;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (u >= nu) break;
      const int e = ebase + u * STR;
      const bool have = e < lim;
      unsigned key = ekey[have ? e : 0];
#ifdef MSDA_PAIR_CHECK  // debug builds: report (instead of gathering through) an impossible key
      if ((int)(key >> 8) >= Lq || (int)(key & 0xffu) >= P || (have && (e < 0 || e >= N))) {
        printf("pair check: l=%d part=%d b=%lld m=%d e=%d lim=%d N=%d key=%u Lq=%d striped=%d row=%d\n", l, part,
               b, m, e, lim, N, key, Lq, (int)striped, (int)rowmode);
        key = 0;
      }
#endif
      g[u] = *reinterpret_cast<const uint4*>(gb + (__umul24(key >> 8, (unsigned)rs) + co));
      if constexpr (STG) {
        cc[u] = have ? ECC(e) : f32x2{0.f, 0.f};
      } else {
        const long long o = (long long)(key >> 8) * qs + (key & 0xffu);
        lcv[u] = locb[o];
        acv[u] = have ? awb[o] : 0.f;
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (u >= nu) break;
      const int e = ebase + u * STR;
      const bool have = e < lim;
      Taps<float> t{};
      if constexpr (!STG) {
        t = make_taps<float, ZEROS>(lcv[u], T);
        cc[u] = f32x2{t.ok0 ? acv[u] * t.w0 : 0.f, t.ok1 ? acv[u] * t.w1 : 0.f};
      }
      f32x2 x[H];
      cvt16x2<scalar_t, CPL>(g[u], x);
      const f32x2 k0{cc[u].x, cc[u].x}, k1{cc[u].y, cc[u].y};
#pragma unroll
      for (int e2 = 0; e2 < H; ++e2) {
        a0[e2] = pk_fma(x[e2], k0, a0[e2]);
        a1[e2] = pk_fma(x[e2], k1, a1[e2]);
      }
      if (coords) {
        const float d0 = group_sum<LPR>(dot16<scalar_t>(g[u], v0));
        const float d1 = group_sum<LPR>(dot16<scalar_t>(g[u], v1));
        if (have && c_l == 0) {
          if constexpr (STG) {
            ECC(e) = f32x2{d0, d1};
          } else if (e >= wlo) {  // pre-list samples belong to the previous workgroup
            const unsigned key = ekey[e];
            const long long o = (long long)(key >> 8) * qs + (key & 0xffu);
            if (gab != nullptr) gab[o] = d0 * t.w0 + d1 * t.w1;
            if (glb != nullptr) glb[o] = ((d1 - d0) * acv[u]) * t.gmul;
          }
        }
      }
    }
  };

  if (rowmode) {
    const int j = wave * NSLOT + slot;
    // entry e: [2e] = c0 -> d0, [2e + 1] = c1 -> d1 (row mode: STG == 1 only, LDS)
    float* ed = reinterpret_cast<float*>(smem_raw + lay.off_cc);
    const int rend = min(rhi, T - 1);  // row rhi: the dots of the window's last list only
    for (int rr = max(rlo, 0); rr <= rend; rr += W) {
      const int r = rr + j;
      const bool rv = r <= rend;
      int pos = rv ? st(r - 1) : 0;
      const int mid = rv ? en(r - 1) : 0, hi = rv ? en(r) : 0;
      v0 = vload(rv ? r : -1);
#pragma unroll
      for (int e = 0; e < H; ++e) a0[e] = f32x2{0.f, 0.f};
      while (__ballot(pos < hi) != 0ull) {
        const int lim = min(pos + U, hi);
        uint4 g[U];
        float k[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int e = pos + u;
          const bool have = e < lim;
          const unsigned key = ekey[have ? e : 0];
          g[u] = *reinterpret_cast<const uint4*>(gb + (__umul24(key >> 8, (unsigned)rs) + co));
          k[u] = have ? ed[2 * e + (e < mid ? 1 : 0)] : 0.f;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int e = pos + u;
          f32x2 x[H];
          cvt16x2<scalar_t, CPL>(g[u], x);
          const f32x2 kk{k[u], k[u]};
#pragma unroll
          for (int e2 = 0; e2 < H; ++e2) a0[e2] = pk_fma(x[e2], kk, a0[e2]);
          if (coords) {
            const float d = group_sum<LPR>(dot16<scalar_t>(g[u], v0));
            if (e < lim && c_l == 0) ed[2 * e + (e < mid ? 1 : 0)] = d;
          }
        }
        pos = max(pos, lim);
      }
      if (rv && r < rhi) store_row(r, a0);
    }
    MSDA_PH(3);
  } else if (!striped) {
    const int j = wave * NSLOT + slot;
    const int lo = pb[j], hi = pb[j + 1];
    int rb = lo < hi ? row_of(lo) : 0;
    // the slot's first row also takes the c1 part of list rb-1 from the slot before
    const int hold_row = (j > 0 && lo < hi && rb >= 0 && st(rb - 1) < en(rb - 1)) ? rb : -2;
    f32x2 hold[H];
#pragma unroll
    for (int e = 0; e < H; ++e) hold[e] = f32x2{0.f, 0.f};
    auto flush = [&](int x, const f32x2 (&a)[H]) {
      if (x < rlo || x >= rhi || x < 0) return;  // another workgroup's row
      if (x == hold_row) {
#pragma unroll
        for (int e = 0; e < H; ++e) hold[e] = a[e];
      } else {
        store_row(x, a);
      }
    };
    // (a software-pipelined variant — next batch's loads issued before this one is consumed, row
    // stores after them — measured slower: pull 42 vs 37 us at the encoder shape, U = 4 + 4;
    // its batch buffers, passed between lambdas, also went to scratch)
    int eo = lo < hi ? en(rb) : 0;  // end of list rb
    v0 = vload(rb);
    v1 = vload(rb + 1);
    int pos = lo;
    while (__ballot(pos < hi) != 0ull) {
      const bool act = pos < hi;
      const int lim = act ? min(pos + U, eo) : pos;
      batch(pos, 1, lim);
      pos = lim;
      if (act && pos < hi && pos == eo) {  // list rb done: row rb is final
        int nb = rb + 1;
        while (en(nb) == pos) ++nb;  // next list with entries
        flush(rb, a0);
        if (nb == rb + 1) {
#pragma unroll
          for (int e = 0; e < H; ++e) {
            a0[e] = a1[e];
            a1[e] = f32x2{0.f, 0.f};
          }
          v0 = v1;
          v1 = vload(nb + 1);
        } else {  // list rb+1 empty: row rb+1 holds only list rb's c1 part
          flush(rb + 1, a1);
#pragma unroll
          for (int e = 0; e < H; ++e) a0[e] = a1[e] = f32x2{0.f, 0.f};
          v0 = vload(nb);
          v1 = vload(nb + 1);
        }
        rb = nb;
        eo = en(nb);
      }
    }
    bool send = false;
    if (lo < hi) {
      flush(rb, a0);
      const int x = rb + 1;
      if (x < T) {
        if (st(x) < en(x)) send = x < rhi;  // list x goes on in the next slot: hand its row over
        else flush(x, a1);
      }
    }
    MSDA_PH(3);
    // hand-overs: a slot's c1 part goes to the next slot with entries; inside the wave by lane
    // shuffles (empty slots pass on what they got), across waves through LDS
    const bool busy = lo < hi;
    f32x2 fwd[H], inc[H];
#pragma unroll
    for (int e = 0; e < H; ++e) fwd[e] = send ? a1[e] : f32x2{0.f, 0.f};
    auto up = [&](const f32x2 (&x)[H], f32x2 (&y)[H]) {
#pragma unroll
      for (int e = 0; e < H; ++e) {
        y[e].x = __shfl_up(x[e].x, LPR);
        y[e].y = __shfl_up(x[e].y, LPR);
      }
    };
    for (int step = 0; step < NSLOT - 1; ++step) {
      up(fwd, inc);
      if (!busy && slot > 0)
#pragma unroll
        for (int e = 0; e < H; ++e) fwd[e] = inc[e];
    }
    up(fwd, inc);
    const unsigned long long busy_lanes = __ballot(busy && c_l == 0);
    int* wflag = reinterpret_cast<int*>(xb + NW * D);
    if (slot == NSLOT - 1) {  // the wave's carry-out: the c1 part of its last slot with entries
      float* cb = xb + (wave * D + co);
#pragma unroll
      for (int e = 0; e < H; ++e) {
        cb[2 * e] = fwd[e].x;
        cb[2 * e + 1] = fwd[e].y;
      }
      if (c_l == 0) wflag[wave] = busy_lanes != 0ull;
    }
    __syncthreads();
    if (hold_row >= 0) {
      const unsigned long long below = busy_lanes & ((1ull << (slot * LPR)) - 1ull);
      if (below != 0ull) {  // a slot of this wave sent it
#pragma unroll
        for (int e = 0; e < H; ++e) {
          hold[e].x += inc[e].x;
          hold[e].y += inc[e].y;
        }
      } else if (wave > 0) {  // the last slot with entries of the nearest earlier wave that has any
        int w = wave - 1;
        while (w > 0 && wflag[w] == 0) --w;
        const float* cb = xb + (w * D + co);
#pragma unroll
        for (int e = 0; e < H; ++e) {
          hold[e].x += cb[2 * e];
          hold[e].y += cb[2 * e + 1];
        }
      }
      store_row(hold_row, hold);
    }
  } else {
    // striped: wave w owns positions [qlo, qhi); its slots take every NSLOT-th entry of a list
    const int qlo = wave == 0 ? pre : wlo + (int)((long long)(whi - wlo) * wave / NW);
    const int qhi = wlo + (int)((long long)(whi - wlo) * (wave + 1) / NW);
    int* ptag = reinterpret_cast<int*>(xb + NW * kPairParts * D);  // [NW][kPairParts] rows, -1 = unused
    int npart = 0;
    auto flush = [&](int x, f32x2 (&a)[H]) {  // wave-uniform
      if (x < rlo || x >= rhi || x < 0) return;
      const int c_lo = st(x - 1), c_hi = en(x);
      if (c_lo >= c_hi) return;  // a zero row (the sweep wrote it)
      for (int o = LPR; o < 64; o <<= 1) {
#pragma unroll
        for (int e = 0; e < H; ++e) {
          a[e].x += __shfl_xor(a[e].x, o);
          a[e].y += __shfl_xor(a[e].y, o);
        }
      }
      if (c_lo >= qlo && c_hi <= qhi) {  // every tap of the row is in this wave's share
        if (slot == 0) store_row(x, a);
      } else {
        if (slot == 0) {
          float* pr = xb + ((wave * kPairParts + npart) * D + co);
#pragma unroll
          for (int e = 0; e < H; ++e) {
            pr[2 * e] = a[e].x;
            pr[2 * e + 1] = a[e].y;
          }
          if (c_l == 0) ptag[wave * kPairParts + npart] = x;
        }
        ++npart;
      }
    };
    if (lane < kPairParts) ptag[wave * kPairParts + lane] = -1;
    if (qlo < qhi) {
      int rb = row_of(qlo);
      int eo = en(rb);
      v0 = vload(rb);
      v1 = vload(rb + 1);
      int pos = qlo;
      while (pos < qhi) {
        const int lim = min(min(pos + NSLOT * U, eo), qhi);
        batch(pos + slot, NSLOT, lim);
        pos = lim;
        if (pos < qhi && pos == eo) {
          int nb = rb + 1;
          while (en(nb) == pos) ++nb;
          flush(rb, a0);
          if (nb == rb + 1) {
#pragma unroll
            for (int e = 0; e < H; ++e) {
              a0[e] = a1[e];
              a1[e] = f32x2{0.f, 0.f};
            }
            v0 = v1;
            v1 = vload(nb + 1);
          } else {
            flush(rb + 1, a1);
#pragma unroll
            for (int e = 0; e < H; ++e) a0[e] = a1[e] = f32x2{0.f, 0.f};
            v0 = vload(nb);
            v1 = vload(nb + 1);
          }
          rb = nb;
          eo = en(nb);
        }
      }
      flush(rb, a0);
      flush(rb + 1, a1);
    }
    MSDA_PH(3);
    __syncthreads();
    // partial rows: the first wave holding row x sums the partials of x over the waves in order
    {
      const int j = wave * NSLOT + slot;
      if (j < NW * kPairParts) {
        const int w = j / kPairParts;
        const int x = ptag[j];
        bool first = x >= 0;  // no earlier wave holds row x (waves with empty shares hold none)
        for (int k = 0; first && k < w * kPairParts; ++k) first = ptag[k] != x;
        if (first) {
          float o[CPL];
          const float* p0 = xb + (j * D + co);
#pragma unroll
          for (int e = 0; e < CPL; ++e) o[e] = p0[e];
          for (int k = (w + 1) * kPairParts; k < NW * kPairParts; ++k) {
            if (ptag[k] != x) continue;
            const float* p2 = xb + (k * D + co);
#pragma unroll
            for (int e = 0; e < CPL; ++e) o[e] += p2[e];
          }
#ifdef MSDA_PAIR_CHECK
          if (x >= T) printf("pair check: merged row %d of T=%d l=%d\n", x, T, l); else
#endif
          store_vec_nt<scalar_t, CPL>(gvl + (x * rs + co), o);
        }
      }
    }
  }

  // 6. coordinate gradients from the dots, in sample order (coalesced loc / aw / output): a
  // sample of this workgroup's window finds its list position parked in its output slot
  if constexpr (STG) {
    if (coords) {
      gstage_sync();  // every dot written
      MSDA_PH(5);
      const int li_lo = wlo < whi ? row_of(wlo) + 1 : 1, li_hi = wlo < whi ? row_of(whi - 1) + 1 : 0;
      for (int s0 = threadIdx.x; s0 < nsamp; s0 += kGvThreads * kGvCache) {
        float lcv[kGvCache], acv[kGvCache];
        int psv[kGvCache];
#pragma unroll
        for (int k = 0; k < kGvCache; ++k) {  // unconditional loads (clamped index): all in flight
          const int s = min(s0 + k * kGvThreads, nsamp - 1);
          const int q = s / P, p = s - q * P;
          const long long o = q * qs + p;
          lcv[k] = locb[o];
          acv[k] = awb[o];
          psv[k] = POS(s);  // beside loc / aw: the dot gather below then waits on one load, not two
        }
#pragma unroll
        for (int k = 0; k < kGvCache; ++k) {
          const int s = s0 + k * kGvThreads;
          if (s < nsamp) {
            const Taps<float> t = make_taps<float, ZEROS>(lcv[k], T);
            const int li = list_index(t);
            if (li >= li_lo && li <= li_hi) {
              const int q = s / P, p = s - q * P;
              const long long o = q * qs + p;
              const f32x2 d = ECC(psv[k]);
              if (gab != nullptr) gab[o] = d.x * t.w0 + d.y * t.w1;
              if (glb != nullptr) glb[o] = ((d.y - d.x) * acv[k]) * t.gmul;
            }
          }
        }
      }
    }
  }
#ifdef MSDA_PHASE_TIMING
  MSDA_PH(4);
  if (threadIdx.x == 0 && bm == 0 && part == 0)
    printf("pair l=%d T=%d N=%d striped=%d row=%d hist=%llu scan+place=%llu pull=%llu handover=%llu coords=%llu (x10ns)\n",
           l, T, N, (int)striped, (int)rowmode, tph[1] - tph[0], tph[2] - tph[1], tph[3] - tph[2], tph[5] - tph[3],
           tph[4] - tph[5]);
#endif
#undef MSDA_PH
}

// grad_aw / grad_loc fast path (conditions of msda_fwd16_kernel): coordinates and the
// item's grad_out chunk loaded once, 4 samples' fragments in flight, DPP reductions.
template <typename scalar_t, int VEC, int G, bool ZEROS>
__global__ __launch_bounds__(256) void msda_bwd_coord16_kernel(
    const scalar_t* __restrict__ value, const float* __restrict__ loc, const float* __restrict__ aw,
    const scalar_t* __restrict__ gout, float* __restrict__ gloc, float* __restrict__ gaw,
    const Levels lv, const int L, const int P, const int S, const int M, const int D, const int Lq,
    const long long n_items) {
  const long long tid = (long long)xcd_block(blockIdx.x, gridDim.x) * blockDim.x + threadIdx.x;
  const long long item_raw = tid / G;
  const bool active = item_raw < n_items;  // every lane stays for the reductions
  const long long item = active ? item_raw : 0;
  const int lg = (int)(tid % G);
  const int m = (int)(item % M);
  const long long b = item / M / Lq;
  const long long rowstride = (long long)M * D;
  const int LP = L * P;
  float lr[kLPMax], ar[kLPMax];
  load_coords16(loc + item * LP, LP, lr);
  load_coords16(aw + item * LP, LP, ar);
  f32x2 g2[VEC / 2];
  cvt16x2<scalar_t, VEC>(load16_if(active, gout + item * D + lg * VEC), g2);
  const scalar_t* __restrict__ vb = value + (b * S * M + m) * (long long)D + lg * VEC;
  const int rs = M * D;
#pragma unroll
  for (int j0 = 0; j0 < kLPMax; j0 += 4) {
    if (j0 < LP) {
      uint4 r0[4], r1[4];
      Taps<float> t[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int l = (j0 + u) / P;
        t[u] = make_taps<float, ZEROS>(lr[j0 + u], lv.T[l]);
        const scalar_t* __restrict__ vl = vb + (long long)lv.start[l] * rs;
        r0[u] = load16_if(active && t[u].ok0, vl + t[u].i0 * rs);
        r1[u] = load16_if(active && t[u].ok1, vl + t[u].i1 * rs);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        // d_k = <grad_out, tap k row>: grad_aw = w0 d0 + w1 d1, grad_loc = aw dy/dloc (d1 - d0)
        f32x2 x0[VEC / 2], x1[VEC / 2];
        cvt16x2<scalar_t, VEC>(r0[u], x0);
        cvt16x2<scalar_t, VEC>(r1[u], x1);
        f32x2 s0{0.f, 0.f}, s1{0.f, 0.f};
#pragma unroll
        for (int e = 0; e < VEC / 2; ++e) {
          s0 = pk_fma(g2[e], x0[e], s0);
          s1 = pk_fma(g2[e], x1[e], s1);
        }
        const float d0 = group_sum<G>(s0.x + s0.y);
        const float d1 = group_sum<G>(s1.x + s1.y);
        const int j = j0 + u;
        if (active && lg == j % G) {
          const long long o = item * LP + j;
          if (gaw != nullptr) gaw[o] = d0 * t[u].w0 + d1 * t[u].w1;
          if (gloc != nullptr) gloc[o] = ((d1 - d0) * ar[j]) * t[u].gmul;
        }
      }
    }
  }
}

// grad_aw / grad_loc: the forward's item decomposition (G lanes x VEC channels own one
// (b, q, m) row).  grad_out of the item is loaded once; per sample the two taps are
// gathered like the forward, the two partial dot products are reduced over the G lanes with
// DPP, and lane j % G writes sample j, so each item's 2*L*P outputs leave as coalesced
// stores.  ONE: D/VEC <= G (every lane owns exactly one chunk; the common case).
template <typename scalar_t, typename coord_t, int VEC, int G, bool ZEROS, bool ONE>
__global__ __launch_bounds__(256) void msda_bwd_coord_kernel(
    const scalar_t* __restrict__ value, const coord_t* __restrict__ loc,
    const coord_t* __restrict__ aw, const scalar_t* __restrict__ gout,
    coord_t* __restrict__ gloc, coord_t* __restrict__ gaw, const Levels lv, const int L,
    const int P, const int S, const int M, const int D, const int Lq, const long long n_items) {
  using acc_t = typename AccOf<scalar_t>::type;
  const long long tid = (long long)xcd_block(blockIdx.x, gridDim.x) * blockDim.x + threadIdx.x;
  const long long item_raw = tid / G;
  const bool active = item_raw < n_items;  // every lane stays for the reductions
  const long long item = active ? item_raw : 0;
  const int lg = (int)(tid % G);
  const int m = (int)(item % M);
  const long long b = item / M / Lq;
  const long long rowstride = (long long)M * D;
  const coord_t* __restrict__ locp = loc + item * (L * P);
  const coord_t* __restrict__ awp = aw + item * (L * P);
  const scalar_t* __restrict__ vb = value + (b * S * M + m) * (long long)D;
  const scalar_t* __restrict__ gp = gout + item * D;
  const int nchunk = D / VEC;
  const bool on = active && lg < nchunk;
  acc_t g1[VEC];
  if constexpr (ONE) {
    if (on) load_vec<scalar_t, VEC>(gp + lg * VEC, g1);
    else {
#pragma unroll
      for (int e = 0; e < VEC; ++e) g1[e] = (acc_t)0;
    }
  }
  for (int l = 0; l < L; ++l) {
    const int T = lv.T[l];
    const scalar_t* __restrict__ vl = vb + (long long)lv.start[l] * rowstride;
    for (int p = 0; p < P; ++p) {
      const int j = l * P + p;
      const coord_t a = awp[j];
      const Taps<coord_t> t = make_taps<coord_t, ZEROS>(locp[j], T);
      const acc_t w0 = (acc_t)t.w0, w1 = (acc_t)t.w1;
      acc_t pa = (acc_t)0, pl = (acc_t)0;
      if constexpr (ONE) {
        if (on) {
          acc_t v0[VEC], v1[VEC];
          load_vec<scalar_t, VEC>(vl + t.i0 * rowstride + lg * VEC, v0);
          load_vec<scalar_t, VEC>(vl + t.i1 * rowstride + lg * VEC, v1);
#pragma unroll
          for (int e = 0; e < VEC; ++e) {
            const acc_t x0 = t.ok0 ? v0[e] : (acc_t)0;
            const acc_t x1 = t.ok1 ? v1[e] : (acc_t)0;
            pa += g1[e] * (x0 * w0 + x1 * w1);
            pl += g1[e] * (x1 - x0);
          }
        }
      } else {
        if (active) {
          for (int ck = lg; ck < nchunk; ck += G) {
            acc_t g[VEC], v0[VEC], v1[VEC];
            load_vec<scalar_t, VEC>(gp + ck * VEC, g);
            load_vec<scalar_t, VEC>(vl + t.i0 * rowstride + ck * VEC, v0);
            load_vec<scalar_t, VEC>(vl + t.i1 * rowstride + ck * VEC, v1);
#pragma unroll
            for (int e = 0; e < VEC; ++e) {
              const acc_t x0 = t.ok0 ? v0[e] : (acc_t)0;
              const acc_t x1 = t.ok1 ? v1[e] : (acc_t)0;
              pa += g[e] * (x0 * w0 + x1 * w1);
              pl += g[e] * (x1 - x0);
            }
          }
        }
      }
      pa = group_sum<G>(pa);
      pl = group_sum<G>(pl);
      if (active && lg == j % G) {
        const long long o = item * (L * P) + j;
        if (gaw != nullptr) gaw[o] = (coord_t)pa;
        if (gloc != nullptr) gloc[o] = (coord_t)(pl * (acc_t)a) * t.gmul;
      }
    }
  }
}

// ---------------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------------

struct Problem {
  long long B, S, M, D, Lq, L, P;
  Levels lv;
  long long gv_rs = 0;  // grad_value row stride in elements (0: M * D, the contiguous layout)
};

int check_problem(const int64_t* shapes, const int64_t* starts, int64_t L, int64_t B,
                  int64_t S, int64_t M, int64_t D, int64_t Lq, int64_t P, Problem* pr) {
  if (L < 1 || L > MSDA_MAX_LEVELS) {
    set_error("msda: num_levels=%lld must be in [1, %d]", (long long)L, MSDA_MAX_LEVELS);
    return MSDA_ERR_ARG;
  }
  if (B < 0 || S < 0 || M < 1 || D < 1 || Lq < 0 || P < 1) {
    set_error("msda: bad sizes (B=%lld S=%lld M=%lld D=%lld Lq=%lld P=%lld)", (long long)B, (long long)S, (long long)M, (long long)D, (long long)Lq, (long long)P);
    return MSDA_ERR_ARG;
  }
  if (shapes == nullptr || starts == nullptr) {
    set_error("msda: spatial_shapes / level_start must be host arrays");
    return MSDA_ERR_ARG;
  }
  for (int64_t l = 0; l < L; ++l) {
    if (shapes[l] < 1 || starts[l] < 0 || starts[l] + shapes[l] > S) {
      set_error("msda: level %lld (T=%lld, start=%lld) does not fit spatial_size=%lld", (long long)l,
                (long long)shapes[l], (long long)starts[l], (long long)S);
      return MSDA_ERR_ARG;
    }
    pr->lv.T[l] = (int)shapes[l];
    pr->lv.start[l] = (int)starts[l];
  }
  if (S > (1LL << 30) || D > (1LL << 20) || M * D * S > (1LL << 40)) {
    set_error("msda: problem too large");
    return MSDA_ERR_ARG;
  }
  pr->B = B; pr->S = S; pr->M = M; pr->D = D; pr->Lq = Lq; pr->L = L; pr->P = P;
  return MSDA_OK;
}

int pick_vec(int dtype, long long D) {
  const int elt = dtype == MSDA_DTYPE_F64 ? 8 : (dtype == MSDA_DTYPE_F32 ? 4 : 2);
  const int v = 16 / elt;
  return (D % v == 0) ? v : 1;
}

int group_shift_for(long long nchunk) {
  int s = 0;
  while ((1LL << s) < nchunk && s < 6) ++s;
  return s;
}

int launch_status(const char* what) {
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("msda: %s launch failed: %s", what, hipGetErrorString(e));
    return MSDA_ERR_LAUNCH;
  }
  return MSDA_OK;
}

// Lanes per item of the fast (fwd16 / coord16) kernels, or 0 when they do not apply: fp32
// coordinates, L*P <= 16 and a multiple of 4, D an exact power-of-two number of 16-byte chunks.
template <typename scalar_t>
int fast16_group(const Problem& pr) {
  constexpr int VEC = 16 / (int)sizeof(scalar_t);
  const long long LP = pr.L * pr.P;
  if (LP > kLPMax || LP % 4 != 0 || pr.D % VEC != 0) return 0;
  const long long g = pr.D / VEC;
  if (g < 1 || g > 64 || (g & (g - 1)) != 0) return 0;
  return (int)g;
}

int env_int(const char* name, int dflt);
bool dense_takes(const Problem& pr, int value_dtype);
WinShape dense_win_shape(const Problem& pr);

template <typename scalar_t, typename coord_t, int VEC>
int run_forward(const Problem& pr, const void* value, const void* loc, const void* aw, void* out,
                int pad, hipStream_t st, void* tiles = nullptr, int layout = MSDA_COORD_API) {
  const bool lm = layout == MSDA_COORD_LEVEL_MAJOR;
  const long long n_items = pr.B * pr.Lq * pr.M;
  if (n_items == 0) return MSDA_OK;
  const int gshift = group_shift_for(pr.D / VEC);
  const long long threads = n_items << gshift;
  const unsigned blocks = (unsigned)((threads + 255) / 256);
  auto* v = static_cast<const scalar_t*>(value);
  auto* lc = static_cast<const coord_t*>(loc);
  auto* a = static_cast<const coord_t*>(aw);
  auto* o = static_cast<scalar_t*>(out);
  if constexpr (!std::is_same<coord_t, double>::value && VEC * sizeof(scalar_t) == 16) {
    const int G = fast16_group<scalar_t>(pr);
    if constexpr (std::is_same<scalar_t, bf16_t>::value) {
      if (dense_takes(pr, MSDA_DTYPE_BF16)) {  // (tiles, when handed over, written as the tiles forward does)
        const WinShape sh = dense_win_shape(pr);
        if (msda_dense_forward(value, loc, aw, out, tiles, &sh, pad == MSDA_PAD_ZEROS, lm ? 1 : 0, st) != 0) {
          set_error("msda forward: the dense small-pyramid kernel could not be launched");
          return MSDA_ERR_LAUNCH;
        }
        return launch_status("forward (dense)");
      }
    }
    if constexpr (sizeof(scalar_t) == 2) {
    if (tiles != nullptr) {  // the caller checked forward_tiles_ok: 16-bit values, D = 64 (G = 8)
      const int ntile = (int)((pr.Lq + kWinQT - 1) / kWinQT);
      const unsigned tblocks = (unsigned)(pr.B * pr.M * ntile);
      // MSDA_HIP_FWD_LDS=1: value rows staged in LDS per workgroup (msda_fwd16_lds_kernel) — measured
      // slower at the bench's encoder call (53.9 vs 33.6 us: the gathers' neighbouring rows hit in
      // L1 and the barrier-free gather kernel hides their latency), so the gathers stay the default
      const bool fwd_lds = env_int("MSDA_HIP_FWD_LDS", 0) != 0;
      // per-wave staged rows (msda_fwd16_stage_kernel; MSDA_HIP_FWD_STAGE=0: the gathering kernel)
      // (measured slower at the bench's encoder call: 76 / 66 us against 33.5, tools/win_exp.py, r05e)
      const int fwd_stage = fwd_lds ? 0 : env_int("MSDA_HIP_FWD_STAGE", 0);  // 1: 48 rows a wave, 2: 32
      auto* tl = static_cast<int2*>(tiles);
      const QOrder qo = make_qorder(pr.Lq, pr.S, (int)pr.L, pr.lv.T, pr.lv.start);
#define MSDA_FT(Z, PP)                                                                              \
  do {                                                                                            \
    if (fwd_lds && lm)                                                                            \
      hipLaunchKernelGGL((msda_fwd16_lds_kernel<scalar_t, Z, PP, true>), dim3(tblocks), dim3(256), 0, st, v, lc, \
                         a, o, tl, pr.lv, (int)pr.L, (int)pr.S, (int)pr.M, (int)pr.Lq, ntile, qo);   \
    else if (fwd_lds)                                                                             \
      hipLaunchKernelGGL((msda_fwd16_lds_kernel<scalar_t, Z, PP, false>), dim3(tblocks), dim3(256), 0, st, v, lc, \
                         a, o, tl, pr.lv, (int)pr.L, (int)pr.S, (int)pr.M, (int)pr.Lq, ntile, qo);   \
    else if (fwd_stage == 2 && lm && PP <= 4)                                                     \
      hipLaunchKernelGGL((msda_fwd16_stage_kernel<scalar_t, Z, PP, true, 32>), dim3(tblocks), dim3(256), 0, st, v, \
                         lc, a, o, tl, pr.lv, (int)pr.L, (int)pr.S, (int)pr.M, (int)pr.Lq, ntile, qo); \
    else if (fwd_stage && lm && PP <= 4)                                                          \
      hipLaunchKernelGGL((msda_fwd16_stage_kernel<scalar_t, Z, PP, true, 48>), dim3(tblocks), dim3(256), 0, st, v, \
                         lc, a, o, tl, pr.lv, (int)pr.L, (int)pr.S, (int)pr.M, (int)pr.Lq, ntile, qo); \
    else if (fwd_stage && PP <= 4)                                                                \
      hipLaunchKernelGGL((msda_fwd16_stage_kernel<scalar_t, Z, PP, false, 48>), dim3(tblocks), dim3(256), 0, st, v, \
                         lc, a, o, tl, pr.lv, (int)pr.L, (int)pr.S, (int)pr.M, (int)pr.Lq, ntile, qo); \
    else if (lm)                                                                                  \
      hipLaunchKernelGGL((msda_fwd16_tiles_kernel<scalar_t, Z, PP, true>), dim3(tblocks), dim3(256), 0, st, v, lc, \
                         a, o, tl, pr.lv, (int)pr.L, (int)pr.S, (int)pr.M, (int)pr.Lq, ntile, qo);   \
    else                                                                                          \
      hipLaunchKernelGGL((msda_fwd16_tiles_kernel<scalar_t, Z, PP, false>), dim3(tblocks), dim3(256), 0, st, v, lc, \
                         a, o, tl, pr.lv, (int)pr.L, (int)pr.S, (int)pr.M, (int)pr.Lq, ntile, qo);   \
  } while (0)
#define MSDA_FT_P(Z)                                                                                \
  switch (pr.P) {                                                                                 \
    case 1: MSDA_FT(Z, 1); break;                                                                 \
    case 2: MSDA_FT(Z, 2); break;                                                                 \
    case 4: MSDA_FT(Z, 4); break;                                                                 \
    default: MSDA_FT(Z, 8); break;                                                                \
  }
      if (tblocks > 0) {
        if (pad == MSDA_PAD_ZEROS) { MSDA_FT_P(true) } else { MSDA_FT_P(false) }
      }
#undef MSDA_FT_P
#undef MSDA_FT
      return launch_status("forward (tiles)");
    }
    }
    if (G > 0) {
      const unsigned fblocks = (unsigned)((n_items * G + 255) / 256);
#define MSDA_F16(GG, Z)                                                                            \
  do {                                                                                           \
    if (lm)                                                                                      \
      hipLaunchKernelGGL((msda_fwd16_kernel<scalar_t, VEC, GG, Z, true>), dim3(fblocks), dim3(256), 0, st, v, \
                         lc, a, o, pr.lv, (int)pr.L, (int)pr.P, (int)pr.S, (int)pr.M, (int)pr.D,    \
                         (int)pr.Lq, n_items);                                                   \
    else                                                                                         \
      hipLaunchKernelGGL((msda_fwd16_kernel<scalar_t, VEC, GG, Z, false>), dim3(fblocks), dim3(256), 0, st, v, \
                         lc, a, o, pr.lv, (int)pr.L, (int)pr.P, (int)pr.S, (int)pr.M, (int)pr.D,    \
                         (int)pr.Lq, n_items);                                                   \
  } while (0)
#define MSDA_F16_G(Z)                                                                              \
  switch (G) {                                                                                   \
    case 1: MSDA_F16(1, Z); break;                                                               \
    case 2: MSDA_F16(2, Z); break;                                                               \
    case 4: MSDA_F16(4, Z); break;                                                               \
    case 8: MSDA_F16(8, Z); break;                                                               \
    case 16: MSDA_F16(16, Z); break;                                                             \
    case 32: MSDA_F16(32, Z); break;                                                             \
    default: MSDA_F16(64, Z); break;                                                             \
  }
      if (pad == MSDA_PAD_ZEROS) { MSDA_F16_G(true) } else { MSDA_F16_G(false) }
#undef MSDA_F16_G
#undef MSDA_F16
      return launch_status("forward");
    }
  }
  if (lm) {
    set_error("msda forward: the level-major coordinate layout needs fp32 coordinates, L*P <= 16 with L*P %% 4 == 0 "
              "and D a power-of-two number of 16-byte chunks");
    return MSDA_ERR_ARG;
  }
  if (pad == MSDA_PAD_ZEROS)
    hipLaunchKernelGGL((msda_fwd_kernel<scalar_t, coord_t, VEC, true>), dim3(blocks), dim3(256), 0,
                       st, v, lc, a, o, pr.lv, (int)pr.L, (int)pr.P, (int)pr.S, (int)pr.M,
                       (int)pr.D, (int)pr.Lq, n_items, gshift);
  else
    hipLaunchKernelGGL((msda_fwd_kernel<scalar_t, coord_t, VEC, false>), dim3(blocks), dim3(256),
                       0, st, v, lc, a, o, pr.lv, (int)pr.L, (int)pr.P, (int)pr.S, (int)pr.M,
                       (int)pr.D, (int)pr.Lq, n_items, gshift);
  return launch_status("forward");
}

// backward workspace: [rowinfo int2 x B*M*S][entries Entry x B*M*L*2*Lq*P]
struct BwdLayout {
  size_t rowinfo, entries, total;
};

size_t align_up(size_t x) { return (x + 255) & ~(size_t)255; }

BwdLayout bwd_layout(int value_dtype, long long B, long long S, long long M, long long Lq,
                     long long L, long long P) {
  const size_t cs = value_dtype == MSDA_DTYPE_F64 ? 8 : 4;
  const size_t es = value_dtype == MSDA_DTYPE_F64 ? sizeof(Entry<double>) : sizeof(Entry<float>);
  BwdLayout w;
  w.rowinfo = 0;
  w.entries = align_up((size_t)B * M * S * sizeof(int2));
  w.total = w.entries + align_up((size_t)B * M * L * 2 * Lq * P * es);
  (void)cs;
  return w;
}

// Backward path choice, shared by the workspace query and the launcher: the fused gvalue kernel
// needs no workspace.  MSDA_HIP_BWD_PATH=split forces sort + pull (A/B measurements).
bool use_fused_gvalue(int value_dtype, long long B, long long S, long long M, long long Lq,
                      long long L, long long P) {
  static const int force_split = [] {
    const char* e = getenv("MSDA_HIP_BWD_PATH");
    return (e != nullptr && strcmp(e, "split") == 0) ? 1 : 0;
  }();
  if (force_split || value_dtype == MSDA_DTYPE_F64) return false;
  const long long lds = 2 * Lq * P * (long long)sizeof(Entry<float>) + (S + 32) * 4;
  return lds <= kGvLdsMax && B * M * L >= 256;
}

template <typename K>
int allow_lds(K kernel, size_t bytes) {
  if (bytes <= 64 * 1024) return MSDA_OK;
  if (hipFuncSetAttribute(reinterpret_cast<const void*>(kernel),
                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes) != hipSuccess) {
    set_error("msda: cannot raise dynamic LDS to %zu bytes", bytes);
    return MSDA_ERR_LAUNCH;
  }
  return MSDA_OK;
}

template <typename scalar_t, typename coord_t>
int run_backward_impl(const Problem& pr, const void* value, const void* loc, const void* aw,
                      const void* gout, void* gval, void* gloc, void* gaw, void* workspace,
                      int value_dtype, int pad, hipStream_t st, hipStream_t cst) {
  using acc_t = typename AccOf<scalar_t>::type;
  const long long nrows = pr.B * pr.M * pr.S;
  if (nrows == 0) return MSDA_OK;
  const BwdLayout wl = bwd_layout(value_dtype, pr.B, pr.S, pr.M, pr.Lq, pr.L, pr.P);
  auto* ws = static_cast<unsigned char*>(workspace);
  auto* rowinfo = reinterpret_cast<int2*>(ws + wl.rowinfo);
  auto* entries = reinterpret_cast<Entry<coord_t>*>(ws + wl.entries);
  auto* lc = static_cast<const coord_t*>(loc);
  auto* a = static_cast<const coord_t*>(aw);
  const bool z = pad == MSDA_PAD_ZEROS;
  int rc;

  // grad_loc / grad_attn: item kernel (independent of the sort / pull pair)
  bool coords_done = gloc == nullptr && gaw == nullptr;
  if constexpr (!std::is_same<coord_t, double>::value) {
    const int G = coords_done ? 0 : fast16_group<scalar_t>(pr);
    const long long n_items = pr.B * pr.Lq * pr.M;
    if (G > 0 && n_items > 0) {
      constexpr int VEC = 16 / (int)sizeof(scalar_t);
      const unsigned cblocks = (unsigned)((n_items * G + 255) / 256);
      auto* v = static_cast<const scalar_t*>(value);
      auto* g = static_cast<const scalar_t*>(gout);
      auto* gl = static_cast<float*>(gloc);
      auto* ga = static_cast<float*>(gaw);
#define MSDA_C16(GG, Z)                                                                            \
  hipLaunchKernelGGL((msda_bwd_coord16_kernel<scalar_t, VEC, GG, Z>), dim3(cblocks), dim3(256), 0,  \
                     cst, v, lc, a, g, gl, ga, pr.lv, (int)pr.L, (int)pr.P, (int)pr.S, (int)pr.M,    \
                     (int)pr.D, (int)pr.Lq, n_items)
#define MSDA_C16_G(Z)                                                                              \
  switch (G) {                                                                                   \
    case 1: MSDA_C16(1, Z); break;                                                               \
    case 2: MSDA_C16(2, Z); break;                                                               \
    case 4: MSDA_C16(4, Z); break;                                                               \
    case 8: MSDA_C16(8, Z); break;                                                               \
    case 16: MSDA_C16(16, Z); break;                                                             \
    case 32: MSDA_C16(32, Z); break;                                                             \
    default: MSDA_C16(64, Z); break;                                                             \
  }
      if (z) { MSDA_C16_G(true) } else { MSDA_C16_G(false) }
#undef MSDA_C16_G
#undef MSDA_C16
      if ((rc = launch_status("backward coords"))) return rc;
      coords_done = true;
    }
  }
  if (!coords_done) {
    const long long n_items = pr.B * pr.Lq * pr.M;
    if (n_items > 0) {
      constexpr int VEC = 16 / (int)sizeof(scalar_t);
      const bool vec_ok = pr.D % VEC == 0;
      const long long nchunk = vec_ok ? pr.D / VEC : pr.D;
      int G = 1;
      while (G < nchunk && G < 64) G <<= 1;
      const bool one = nchunk <= G;
      const long long threads = n_items * G;
      const unsigned blocks = (unsigned)((threads + 255) / 256);
      auto* v = static_cast<const scalar_t*>(value);
      auto* g = static_cast<const scalar_t*>(gout);
      auto* gl = static_cast<coord_t*>(gloc);
      auto* ga = static_cast<coord_t*>(gaw);
#define MSDA_CO(V, GG, Z, ONE)                                                                     \
  hipLaunchKernelGGL((msda_bwd_coord_kernel<scalar_t, coord_t, V, GG, Z, ONE>), dim3(blocks),        \
                     dim3(256), 0, cst, v, lc, a, g, gl, ga, pr.lv, (int)pr.L, (int)pr.P, (int)pr.S, \
                     (int)pr.M, (int)pr.D, (int)pr.Lq, n_items)
#define MSDA_CO_G(V, Z, ONE)                                                                       \
  switch (G) {                                                                                   \
    case 1: MSDA_CO(V, 1, Z, ONE); break;                                                        \
    case 2: MSDA_CO(V, 2, Z, ONE); break;                                                        \
    case 4: MSDA_CO(V, 4, Z, ONE); break;                                                        \
    case 8: MSDA_CO(V, 8, Z, ONE); break;                                                        \
    case 16: MSDA_CO(V, 16, Z, ONE); break;                                                      \
    case 32: MSDA_CO(V, 32, Z, ONE); break;                                                      \
    default: MSDA_CO(V, 64, Z, ONE); break;                                                      \
  }
      if (vec_ok) {
        if (z) { if (one) { MSDA_CO_G(VEC, true, true) } else { MSDA_CO_G(VEC, true, false) } }
        else { if (one) { MSDA_CO_G(VEC, false, true) } else { MSDA_CO_G(VEC, false, false) } }
      } else {
        if (z) { if (one) { MSDA_CO_G(1, true, true) } else { MSDA_CO_G(1, true, false) } }
        else { if (one) { MSDA_CO_G(1, false, true) } else { MSDA_CO_G(1, false, false) } }
      }
#undef MSDA_CO_G
#undef MSDA_CO
      if ((rc = launch_status("backward coords"))) return rc;
    }
  }
  if (gval == nullptr) return MSDA_OK;

  static const int deterministic_rows = [] {
    const char* e = getenv("MSDA_HIP_DETERMINISTIC");
    return (e != nullptr && e[0] == '1') ? 1 : 0;
  }();
  if (use_fused_gvalue(value_dtype, pr.B, pr.S, pr.M, pr.Lq, pr.L, pr.P)) {
    int maxT = 1;
    for (int l = 0; l < pr.L; ++l) maxT = max(maxT, pr.lv.T[l]);
    const size_t lds = (size_t)2 * pr.Lq * pr.P * sizeof(Entry<coord_t>) + (size_t)(maxT + 32) * 4;
    constexpr int CPL = 16 / (int)sizeof(scalar_t);
    int ns = 0;
    if (pr.D % CPL == 0) {
      const long long lpr = pr.D / CPL;
      if (lpr == 8) ns = 8;
      else if (lpr == 16) ns = 4;
      else if (lpr == 32) ns = 2;
      else if (lpr == 64) ns = 1;
    }
    const unsigned blocks = (unsigned)(pr.B * pr.M * pr.L);
    auto* g = static_cast<const scalar_t*>(gout);
    auto* gv = static_cast<scalar_t*>(gval);
#define MSDA_GV(NSL, Z)                                                                             \
  do {                                                                                            \
    if ((rc = allow_lds(msda_bwd_gvalue_kernel<scalar_t, coord_t, NSL, Z>, lds))) return rc;      \
    hipLaunchKernelGGL((msda_bwd_gvalue_kernel<scalar_t, coord_t, NSL, Z>), dim3(blocks),          \
                       dim3(kGvThreads), lds, st, lc, a, g, gv, pr.lv, (int)pr.L, (int)pr.P,        \
                       (int)pr.S, (int)pr.M, (int)pr.D, (int)pr.Lq, deterministic_rows);          \
  } while (0)
#define MSDA_GV_NS(Z)                                                                               \
  switch (ns) {                                                                                   \
    case 8: MSDA_GV(8, Z); break;                                                                 \
    case 4: MSDA_GV(4, Z); break;                                                                 \
    case 2: MSDA_GV(2, Z); break;                                                                 \
    case 1: MSDA_GV(1, Z); break;                                                                 \
    default: MSDA_GV(0, Z); break;                                                                \
  }
    if (z) { MSDA_GV_NS(true) } else { MSDA_GV_NS(false) }
#undef MSDA_GV_NS
#undef MSDA_GV
    return launch_status("backward gvalue");
  }

  // 1. sort: one workgroup per (b, m, level)
  if (workspace == nullptr) {  // the workspace query promised this call none: refuse, never fault
    set_error("msda_hip_backward: the sort / pull path needs a workspace of %zu bytes (none given)", wl.total);
    return MSDA_ERR_ARG;
  }
  {
    static const int deterministic = [] {
      const char* e = getenv("MSDA_HIP_DETERMINISTIC");
      return (e != nullptr && e[0] == '1') ? 1 : 0;
    }();
    int maxT = 1;
    for (int l = 0; l < pr.L; ++l) maxT = max(maxT, pr.lv.T[l]);
    const size_t tail = (size_t)(maxT + 16) * sizeof(int);
    const size_t stage = (size_t)2 * pr.Lq * pr.P * sizeof(Entry<coord_t>);
    const bool use_stage = stage + tail <= (size_t)kSortLdsMax;
    const size_t lds = (use_stage ? stage : 0) + tail;
    if (lds > (size_t)kSortLdsMax + tail) {
      set_error("msda_hip_backward: level of %d rows too long for the sort kernel", maxT);
      return MSDA_ERR_ARG;
    }
    const unsigned blocks = (unsigned)(pr.B * pr.M * pr.L);
#define MSDA_SORT(Z, STG)                                                                         \
  do {                                                                                          \
    if ((rc = allow_lds(msda_bwd_sort_kernel<coord_t, Z, STG>, lds))) return rc;               \
    hipLaunchKernelGGL((msda_bwd_sort_kernel<coord_t, Z, STG>), dim3(blocks), dim3(kSortThreads), \
                       lds, st, lc, a, rowinfo, entries, pr.lv, (int)pr.L, (int)pr.P, (int)pr.S, \
                       (int)pr.M, (int)pr.Lq, deterministic);                                   \
  } while (0)
    if (z) { if (use_stage) MSDA_SORT(true, true); else MSDA_SORT(true, false); }
    else { if (use_stage) MSDA_SORT(false, true); else MSDA_SORT(false, false); }
#undef MSDA_SORT
    if ((rc = launch_status("backward sort"))) return rc;
  }

  // 2. pull: NS rows per wave, 64/NS lanes x 16 bytes per row
  {
    constexpr int CPL = 16 / (int)sizeof(scalar_t);
    int ns = 0;
    if (pr.D % CPL == 0) {
      const long long lpr = pr.D / CPL;
      if (lpr == 8) ns = 8;
      else if (lpr == 16) ns = 4;
      else if (lpr == 32) ns = 2;
      else if (lpr == 64) ns = 1;
      else if (lpr < 8) ns = 0;  // narrow heads: generic
    }
    PullOrder po;
    for (int l = 0; l < pr.L; ++l) po.lvl[l] = l;
    std::stable_sort(po.lvl, po.lvl + pr.L, [&](int x, int y) { return pr.lv.T[x] < pr.lv.T[y]; });
    po.cum[0] = 0;
    for (int i = 0; i < pr.L; ++i) po.cum[i + 1] = po.cum[i] + pr.M * pr.lv.T[po.lvl[i]];
    for (int i = pr.L; i < MSDA_MAX_LEVELS; ++i) po.cum[i + 1] = 0x7fffffffffffffffll;
    const int nse = ns > 0 ? ns : 1;
    const long long waves = (nrows + nse - 1) / nse;
    const unsigned blocks = (unsigned)((waves + 3) / 4);
    auto* g = static_cast<const scalar_t*>(gout);
    auto* gv = static_cast<scalar_t*>(gval);
#define MSDA_PULL(NSL)                                                                          \
  hipLaunchKernelGGL((msda_bwd_pull_kernel<scalar_t, coord_t, NSL>), dim3(blocks),               \
                     dim3(kPullThreads), 0, st, g, rowinfo, entries, gv, (int)pr.S, (int)pr.M,     \
                     (int)pr.D, (int)pr.Lq, (int)pr.P, nrows, pr.lv, po)
    switch (ns) {
      case 8: MSDA_PULL(8); break;
      case 4: MSDA_PULL(4); break;
      case 2: MSDA_PULL(2); break;
      case 1: MSDA_PULL(1); break;
      default: MSDA_PULL(0); break;
    }
#undef MSDA_PULL
    if ((rc = launch_status("backward pull"))) return rc;
  }

  return MSDA_OK;
}

// Side stream of the calling device: grad_loc / grad_attn (coordinate kernel) and grad_value
// (sort / pull) read the same inputs and write disjoint outputs, so with all three requested
// the coordinate kernel runs beside the grad_value kernel, forked from and joined back into
// the caller's stream with events (both capture into a HIP graph as parallel branches).
// MSDA_HIP_SIDE_STREAM=0 serialises them on the caller's stream.
struct SideStream {
  hipStream_t s = nullptr;
  hipEvent_t fork = nullptr, join = nullptr;
  bool ok = false;
};

SideStream* side_stream() {
  static const int enabled = [] {
    const char* e = getenv("MSDA_HIP_SIDE_STREAM");
    return (e != nullptr && e[0] == '0') ? 0 : 1;
  }();
  if (!enabled) return nullptr;
  constexpr int kMaxDev = 64;
  static std::mutex mu;
  static SideStream per_dev[kMaxDev];
  static bool tried[kMaxDev] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDev) return nullptr;
  std::lock_guard<std::mutex> lock(mu);
  SideStream& ss = per_dev[dev];
  if (!tried[dev]) {
    tried[dev] = true;
    ss.ok = hipStreamCreateWithFlags(&ss.s, hipStreamNonBlocking) == hipSuccess &&
            hipEventCreateWithFlags(&ss.fork, hipEventDisableTiming) == hipSuccess &&
            hipEventCreateWithFlags(&ss.join, hipEventDisableTiming) == hipSuccess;
  }
  return ss.ok ? &ss : nullptr;
}

// Rows per wave of the fused backward (msda_bwd_fused_kernel), or 0 when it does not apply:
// fp32 coordinates, grad_value requested, the level's lists fit in LDS with enough
// (b, m, level) workgroups to fill the chip (use_fused_gvalue), D a power-of-two number of
// 16-byte chunks of at least 8 lanes, 2P <= 256 (key layout) and Lq < 2^23.
// MSDA_HIP_BWD_PATH=unfused forces the gvalue + coordinate kernel pair (A/B measurements).
template <typename scalar_t, typename coord_t>
int fused_bwd_rows(const Problem& pr, int value_dtype, const void* gval) {
  static const int force_unfused = [] {
    const char* e = getenv("MSDA_HIP_BWD_PATH");
    return (e != nullptr && strcmp(e, "unfused") == 0) ? 1 : 0;
  }();
  if (force_unfused || gval == nullptr || !std::is_same<coord_t, float>::value) return 0;
  if (2 * pr.P > 256 || pr.Lq >= (1LL << 23)) return 0;
  if (!use_fused_gvalue(value_dtype, pr.B, pr.S, pr.M, pr.Lq, pr.L, pr.P)) return 0;
  constexpr int CPL = 16 / (int)sizeof(scalar_t);
  if (pr.D % CPL != 0) return 0;
  const long long lpr = pr.D / CPL;
  if (lpr == 8) return 8;
  if (lpr == 16) return 4;
  if (lpr == 32) return 2;
  if (lpr == 64) return 1;
  return 0;
}

template <typename scalar_t>
int run_backward_fused(const Problem& pr, int ns, const void* value, const void* loc, const void* aw,
                       const void* gout, void* gval, void* gloc, void* gaw, int pad, hipStream_t st) {
  static const int deterministic_rows = [] {
    const char* e = getenv("MSDA_HIP_DETERMINISTIC");
    return (e != nullptr && e[0] == '1') ? 1 : 0;
  }();
  int maxT = 1;
  for (int l = 0; l < pr.L; ++l) maxT = max(maxT, pr.lv.T[l]);
  const size_t lds = (size_t)2 * pr.Lq * pr.P * 8 + (size_t)(maxT + 32) * 4;
  const unsigned blocks = (unsigned)(pr.B * pr.M * pr.L);
  const bool coords = gloc != nullptr || gaw != nullptr;
  const bool z = pad == MSDA_PAD_ZEROS;
  auto* v = static_cast<const scalar_t*>(value);
  auto* lc = static_cast<const float*>(loc);
  auto* a = static_cast<const float*>(aw);
  auto* g = static_cast<const scalar_t*>(gout);
  auto* gv = static_cast<scalar_t*>(gval);
  auto* gl = static_cast<float*>(gloc);
  auto* ga = static_cast<float*>(gaw);
  int rc;
  // gathers per batch: 8 when the finest level's rows average >= 8 taps (encoder-like
  // calls), 4 for sparse levels (decoder-like: few taps per row, row-set changes dominate)
  const bool wide = (long long)2 * pr.Lq * pr.P >= 8LL * maxT;
  const int gv_rs = (int)(pr.gv_rs > 0 ? pr.gv_rs : pr.M * pr.D);
#ifndef MSDA_FUSED_UW
#define MSDA_FUSED_UW 8
#endif
#define MSDA_FU_U(NSL, Z, C, UU)                                                                  \
  do {                                                                                          \
    if ((rc = allow_lds(msda_bwd_fused_kernel<scalar_t, NSL, Z, C, UU>, lds))) return rc;       \
    hipLaunchKernelGGL((msda_bwd_fused_kernel<scalar_t, NSL, Z, C, UU>), dim3(blocks),          \
                       dim3(kGvThreads), lds, st, v, lc, a, g, gv, gl, ga, pr.lv, (int)pr.L,      \
                       (int)pr.P, (int)pr.S, (int)pr.M, (int)pr.D, (int)pr.Lq,                  \
                       deterministic_rows, gv_rs);                                              \
  } while (0)
#define MSDA_FU(NSL, Z, C)                                                                        \
  do {                                                                                          \
    if (wide) MSDA_FU_U(NSL, Z, C, MSDA_FUSED_UW); else MSDA_FU_U(NSL, Z, C, 4);                            \
  } while (0)
#define MSDA_FU_NS(Z, C)                                                                          \
  switch (ns) {                                                                                 \
    case 8: MSDA_FU(8, Z, C); break;                                                            \
    case 4: MSDA_FU(4, Z, C); break;                                                            \
    case 2: MSDA_FU(2, Z, C); break;                                                            \
    default: MSDA_FU(1, Z, C); break;                                                           \
  }
  if (z) {
    if (coords) { MSDA_FU_NS(true, true) } else { MSDA_FU_NS(true, false) }
  } else {
    if (coords) { MSDA_FU_NS(false, true) } else { MSDA_FU_NS(false, false) }
  }
#undef MSDA_FU_NS
#undef MSDA_FU
#undef MSDA_FU_U
  return launch_status("backward fused");
}

// ---- pair-pull backward: path choice and LDS plan ----
// MSDA_HIP_BWD_PATH: unset = pair kernel where it applies; "fused1" = per-tap fused kernel,
// "unfused" = gvalue + coordinate kernels, "split" = sort + pull + coordinates (A/B builds).
int bwd_env_path() {
  static const int path = [] {
    const char* e = getenv("MSDA_HIP_BWD_PATH");
    if (e == nullptr || e[0] == 0) return 0;
    if (strcmp(e, "fused1") == 0) return 1;
    if (strcmp(e, "unfused") == 0) return 2;
    if (strcmp(e, "split") == 0) return 3;
    return 0;
  }();
  return path;
}

int env_int(const char* name, int dflt) {
  const char* e = getenv(name);
  return (e != nullptr && e[0] != 0) ? atoi(e) : dflt;
}

constexpr size_t kPairLdsMax = 160 * 1024;

struct PairPlan {
  PairLayout lay;
  size_t lds;
  unsigned striped_mask;
  int stg;          // staging of the entries' (c0, c1) / positions: 1 LDS, 2 workspace, 0 none
  int rs;           // workgroups per (b, m, level)
  size_t ws_bytes;  // workspace of stg 2
};

// workgroups per (b, m, level): enough to fill the chip's 256 CUs (MSDA_HIP_PAIR_RS overrides;
// read per call so tests can switch it)
int pair_rs(long long wgs) {
  const int rs = env_int("MSDA_HIP_PAIR_RS", 0);
  if (rs > 0) return rs;
  return wgs >= 256 ? 1 : (int)std::min<long long>(8, (256 + std::max<long long>(wgs, 1) - 1) / std::max<long long>(wgs, 1));
}

size_t a16(size_t x) { return (x + 15) & ~(size_t)15; }

// LDS bytes of the pair kernel: keys | (c0, c1), sample positions (STG) | wave carry-outs or wave
// partials | T+1 list cursors | W+1 slot bounds | scan scratch.
size_t pair_layout(long long N, long long D, int ns, long long maxT, bool stg, bool any_striped,
                   PairLayout* lay) {
  const size_t W = (size_t)(kGvThreads / 64) * ns;
  const size_t keys = a16((size_t)N * 4);
  const size_t hand = (size_t)(kGvThreads / 64) * (D * 4 + 4);  // per-wave carry-out + flag
  const size_t parts = any_striped ? (size_t)(kGvThreads / 64) * kPairParts * (D * 4 + 4) : 0;
  lay->off_cc = (int)keys;
  lay->off_pos = (int)(keys + (stg ? a16((size_t)N * 8) : 0));
  lay->off_xb = lay->off_pos + (int)(stg ? a16((size_t)N * 4) : 0);
  const size_t end = (size_t)lay->off_xb + a16(std::max(hand, parts));
  lay->off_cur = (int)a16(end);
  lay->off_pb = lay->off_cur + (int)a16((size_t)(maxT + 2) * 4);
  lay->off_scr = lay->off_pb + (int)a16((W + 1) * 4);
  return (size_t)lay->off_scr + 32 * 4;
}

// Slots per wave of the pair kernel (16-byte chunks: D/CPL lanes per row), or 0.
int pair_slots(int value_dtype, long long D) {
  if (value_dtype == MSDA_DTYPE_F64) return 0;
  const long long cpl = value_dtype == MSDA_DTYPE_F32 ? 4 : 8;
  if (D % cpl != 0) return 0;
  const long long lpr = D / cpl;
  return lpr == 8 ? 8 : lpr == 16 ? 4 : lpr == 32 ? 2 : lpr == 64 ? 1 : 0;
}

// The plan for a call (levels known) or, with T == nullptr, the bound used by the workspace
// query (every level taken as S rows long, no striped level): if the bound fits, the call does.
// Striped levels: fewer lists than twice the slots (T + 1 < 2 W), at least 4 slots a wave (the partial-row
// merge uses one slot per partial), STG only.  MSDA_HIP_STRIPED_ROWS caps T (A/B builds; read per
// call so tests can switch it).
// stg 2 (workspace staging) only when allow_ws: the query's bound sets it, and a launch with a
// workspace (the query asked for one) may take it.
bool pair_plan(int value_dtype, long long B, long long M, long long Lq, long long P, long long D, long long L,
               const int* T, long long S, bool allow_ws, PairPlan* pp) {
  if (bwd_env_path() != 0) return false;
  const int ns = pair_slots(value_dtype, D);
  if (ns == 0 || P > 256 || Lq >= (1LL << 24) || Lq * P >= (1LL << 30)) return false;
  const long long N = Lq * P;
  const long long W = (kGvThreads / 64) * ns;
  const int striped_rows = env_int("MSDA_HIP_STRIPED_ROWS", 1 << 30);
  long long maxT = 1;
  unsigned mask = 0;
  if (T == nullptr) {
    maxT = S;
  } else {
    for (int l = 0; l < L; ++l) {
      maxT = std::max(maxT, (long long)T[l]);
      if (ns >= 4 && T[l] + 1 < 2 * W && T[l] <= striped_rows) mask |= 1u << l;
    }
  }
  // the query's bound reserves the striped levels' wave-partial rows whenever a level could be
  // striped (ns >= 4): the call's plan then never needs more LDS than the bound, so a call whose
  // bound fitted stg 1 (no workspace handed over) fits stg 1 too
  const bool any_striped = T == nullptr ? ns >= 4 : mask != 0;
  pp->rs = pair_rs(B * M * L);
  for (int stg : {1, 2}) {  // (stg 0 — keys only, coordinates from the pull — is not launched)
    if (stg == 2 && !allow_ws) continue;
    PairLayout lay;
    const size_t lds = pair_layout(N, D, ns, maxT, stg == 1, stg == 1 && any_striped, &lay);
    if (lds <= kPairLdsMax) {
      pp->lay = lay;
      pp->lds = lds;
      pp->striped_mask = stg == 1 ? mask : 0u;
      pp->stg = stg;
      pp->ws_bytes = stg == 2 ? (size_t)(B * M * L * pp->rs) * (size_t)N * 12 : 0;
      return true;
    }
  }
  return false;
}

template <typename scalar_t>
int run_backward_pair(const Problem& pr, const PairPlan& pp, const void* value, const void* loc,
                      const void* aw, const void* gout, void* gval, void* gloc, void* gaw, void* workspace,
                      int pad, hipStream_t st) {
  static const int det = env_int("MSDA_HIP_DETERMINISTIC", 0);
  const int ns = pair_slots(std::is_same<scalar_t, float>::value ? MSDA_DTYPE_F32 : MSDA_DTYPE_BF16, pr.D);
  const long long wgs = pr.B * pr.M * pr.L;
  const int rs = pp.rs;
  const unsigned blocks = (unsigned)(wgs * rs);
  auto* gsg = static_cast<unsigned char*>(workspace);
  const bool z = pad == MSDA_PAD_ZEROS;
  auto* v = static_cast<const scalar_t*>(value);
  auto* lc = static_cast<const float*>(loc);
  auto* a = static_cast<const float*>(aw);
  auto* g = static_cast<const scalar_t*>(gout);
  auto* gv = static_cast<scalar_t*>(gval);
  auto* gl = static_cast<float*>(gloc);
  auto* ga = static_cast<float*>(gaw);
  int rc;
#define MSDA_PA_(NSL, Z, STGV, UU)                                                                  \
  do {                                                                                          \
    if ((rc = allow_lds(msda_bwd_pair_kernel<scalar_t, NSL, Z, STGV, UU>, pp.lds))) return rc;   \
    hipLaunchKernelGGL((msda_bwd_pair_kernel<scalar_t, NSL, Z, STGV, UU>), dim3(blocks),         \
                       dim3(kGvThreads), pp.lds, st, v, lc, a, g, gv, gl, ga, pr.lv, (int)pr.L,   \
                       (int)pr.P, (int)pr.S, (int)pr.M, (int)pr.D, (int)pr.Lq, rs, pp.striped_mask, \
                       det, pp.lay, gsg);                                                       \
  } while (0)
#ifndef MSDA_PAIR_U
#define MSDA_PAIR_U 8  // gathers in flight per slot
#endif
#define MSDA_PA(NSL, Z)                                                                           \
  do {                                                                                          \
    if (pp.stg == 1) MSDA_PA_(NSL, Z, 1, MSDA_PAIR_U);                                          \
    else MSDA_PA_(NSL, Z, 2, MSDA_PAIR_U);                                                      \
  } while (0)
#define MSDA_PA_NS(Z)                                                                             \
  switch (ns) {                                                                                 \
    case 8: MSDA_PA(8, Z); break;                                                               \
    case 4: MSDA_PA(4, Z); break;                                                               \
    case 2: MSDA_PA(2, Z); break;                                                               \
    default: MSDA_PA(1, Z); break;                                                              \
  }
  if (z) { MSDA_PA_NS(true) } else { MSDA_PA_NS(false) }
#undef MSDA_PA_NS
#undef MSDA_PA
#undef MSDA_PA_
  return launch_status("backward pair");
}

// Row-block MFMA backward (msda_win.hip): bf16 values, D = 64, P <= 8, a call with more than 512
// samples a level.  MSDA_HIP_BWD_WIN (read per call): "0" never, "1" wherever it applies; unset:
//  * where a level's samples do not fit the pair kernel's LDS lists (16 B a sample: key, (c0, c1),
//    position), i.e. where the pair kernel would stage them through a workspace — the configs[3]
//    per-rank call (T = 4096: 237-263 us against 421-511, tools/win_ab.py);
//  * self-attention-like calls — queries covering the value pyramid (2 Lq >= S) and every level at
//    least 64 rows: the encoder (T = 1024: 68-77 us against 69-82);
//  * queries far outnumbering the rows (Lq >= 4 S): the cross-modal call onto the audio pyramid,
//    where every query tile meets every row block — with several waves a block (msda_win.hip).
int win_env() { return env_int("MSDA_HIP_BWD_WIN", -1); }

bool win_supported_call(int value_dtype, long long D, long long Lq, long long P, long long M, long long L) {
  return value_dtype == MSDA_DTYPE_BF16 && msda_win_supported(1, D, P, Lq, M * L * P) && Lq * P > 512 &&
         win_env() != 0 && bwd_env_path() == 0;  // (a forced MSDA_HIP_BWD_PATH keeps its path)
}

bool win_overflow(long long Lq, long long P) { return (size_t)(Lq * P) * 16 > kPairLdsMax; }

// the decision for a call (levels known)
bool win_applies(int value_dtype, long long D, long long Lq, long long P, long long M, long long L, const int* T,
                 long long S) {
  if (!win_supported_call(value_dtype, D, Lq, P, M, L)) return false;
  if (win_env() == 1 || win_overflow(Lq, P)) return true;
  int minT = 1 << 30;
  for (int l = 0; l < L; ++l) minT = min(minT, T[l]);
  // encoder-like calls, or queries far outnumbering the rows (configs[2]'s video queries on the
  // 95-row audio pyramid: 8 waves a row block, 51.6 us against the pair kernel's 63.3), or the
  // Sparse-DETR encoder's position-sorted top-k queries (a third of the pyramid's tokens, each
  // sampling around its own position: 577 queries over the T = 1024 pyramid)
  return (minT >= 64 && 2 * Lq >= S) || Lq >= 4 * S || (minT >= 64 && Lq * P >= 2048);
}

// The backward of this call takes the row-block MFMA path (msda_win.hip) when handed a workspace
// or the forward's tile intervals (run_backward below)
bool win_takes(const Problem& pr, int value_dtype) {
  if (pr.B * pr.M * pr.S <= 0) return false;
  int minT = 1 << 30;
  for (int l = 0; l < pr.L; ++l) minT = min(minT, pr.lv.T[l]);
  const bool sparse = pr.Lq * pr.P <= 4LL * (minT + 1) || pr.Lq * pr.P <= 512;
  return !sparse && win_applies(value_dtype, pr.D, pr.Lq, pr.P, pr.M, pr.L, pr.lv.T, pr.S);
}

// The forward can write those intervals: the win_takes calls the tiles forward kernel covers
// (16-bit values with D = 64: 8 lanes an item, 32 items a workgroup; P of the win kernel)
bool forward_tiles_ok(const Problem& pr, int value_dtype) {
  if (value_dtype != MSDA_DTYPE_BF16 || pr.D != 64 || pr.L * pr.P > kLPMax || (pr.L * pr.P) % 4 != 0) return false;
  if (!(pr.P == 1 || pr.P == 2 || pr.P == 4 || pr.P == 8)) return false;
  return win_takes(pr, value_dtype);
}

// The dense small-pyramid kernels (msda_win.hip) take the call: bf16 values, D = 64, a pyramid of at
// most 128 rows (configs[2]'s audio pyramid: the video queries' cross-modal call and the audio
// self-attention), L <= 4, P <= 4; both coordinate layouts, the forward's tiles unused
bool dense_takes(const Problem& pr, int value_dtype) {
  return pr.B * pr.M * pr.S > 0 && pr.Lq > 0 &&
         msda_dense_supported(value_dtype == MSDA_DTYPE_BF16, pr.D, pr.S, pr.L, pr.P) != 0;
}

WinShape dense_win_shape(const Problem& pr) {
  WinShape sh{};
  sh.B = pr.B; sh.S = pr.S; sh.M = pr.M; sh.Lq = pr.Lq; sh.L = (int)pr.L; sh.P = (int)pr.P;
  for (int l = 0; l < pr.L; ++l) {
    sh.T[l] = pr.lv.T[l];
    sh.start[l] = pr.lv.start[l];
  }
  sh.gv_rs = pr.gv_rs;
  return sh;
}

template <typename scalar_t, typename coord_t>
int run_backward(const Problem& pr, const void* value, const void* loc, const void* aw,
                 const void* gout, void* gval, void* gloc, void* gaw, void* workspace,
                 int value_dtype, int pad, hipStream_t st, const void* tiles = nullptr,
                 int layout = MSDA_COORD_API) {
  if constexpr (std::is_same<coord_t, float>::value) {
    const int ns = pr.B * pr.M * pr.S > 0 ? fused_bwd_rows<scalar_t, coord_t>(pr, value_dtype, gval) : 0;
    // sparse or tiny calls (every level at most 4 samples a row: decoder-like; or at most 512
    // samples a level: the audio self / decoder calls of configs[2]) stay on the per-tap fused
    // kernel: its shorter phase chain wins where the pair kernel's halved gathers are few
    int minT = 1 << 30;
    for (int l = 0; l < pr.L; ++l) minT = min(minT, pr.lv.T[l]);
    const bool sparse = pr.Lq * pr.P <= 4LL * (minT + 1) || pr.Lq * pr.P <= 512;
    if constexpr (std::is_same<scalar_t, bf16_t>::value) {
      // the dense small-pyramid kernels (any of gval / gloc / gaw may be null; a strided grad_value too:
      // configs[2]'s decoder cross-attention into the audio memory writes layer_values' G in place)
      if (dense_takes(pr, value_dtype)) {
        const WinShape sh = dense_win_shape(pr);
        if (msda_dense_backward(value, loc, aw, gout, gval, gloc, gaw, workspace, &sh, pad == MSDA_PAD_ZEROS, layout,
                                st) != 0) {
          set_error("msda backward: the dense small-pyramid kernel could not be launched");
          return MSDA_ERR_LAUNCH;
        }
        return launch_status("backward (dense)");
      }
    }
    if (pr.gv_rs > 0 && pr.gv_rs != pr.M * pr.D) {
      // a strided grad_value: only the per-tap fused kernel writes it (the calls that ask for it,
      // the decoders' cross-attentions, take that path); others report it unsupported
      if (gval != nullptr && ns > 0 && sparse && layout == MSDA_COORD_API && tiles == nullptr)
        return run_backward_fused<scalar_t>(pr, ns, value, loc, aw, gout, gval, gloc, gaw, pad, st);
      set_error("msda backward: a strided grad_value needs the fused per-tap path");
      return MSDA_ERR_UNSUPPORTED;
    }
    if constexpr (std::is_same<scalar_t, bf16_t>::value) {
      // (gval may be null: the row-block kernel then writes the coordinate gradients only)
      if ((workspace != nullptr || tiles != nullptr) && win_takes(pr, value_dtype)) {
        WinShape sh{};
        sh.B = pr.B; sh.S = pr.S; sh.M = pr.M; sh.Lq = pr.Lq; sh.L = (int)pr.L; sh.P = (int)pr.P;
        for (int l = 0; l < pr.L; ++l) {
          sh.T[l] = pr.lv.T[l];
          sh.start[l] = pr.lv.start[l];
        }
        sh.qo = make_qorder(pr.Lq, pr.S, (int)pr.L, pr.lv.T, pr.lv.start);
        const int wrc = msda_win_backward(value, loc, aw, gout, gval, gloc, gaw, workspace, tiles, &sh,
                                          pad == MSDA_PAD_ZEROS, layout, st);
        if (wrc == -2) {
          set_error("msda backward: MSDA_HIP_WIN_EXP is a profiling switch that skips parts of the kernel (wrong "
                    "gradients); it needs MSDA_HIP_PROFILING=1");
          return MSDA_ERR_ARG;
        }
        if (wrc < 0) {
          set_error("msda backward: level-major coordinates need the forward's tile intervals");
          return MSDA_ERR_ARG;
        }
        return launch_status("backward rows (mfma)");
      }
    }
    if (layout != MSDA_COORD_API) {
      set_error("msda backward: the level-major coordinate layout needs the row-block path (bf16 values, D = 64, "
                "the forward's tile intervals)");
      return MSDA_ERR_ARG;
    }
    PairPlan pp;
    if (gval != nullptr && pr.B * pr.M * pr.S > 0 && !(sparse && ns > 0) &&
        pair_plan(value_dtype, pr.B, pr.M, pr.Lq, pr.P, pr.D, pr.L, pr.lv.T, pr.S, workspace != nullptr, &pp))
      return run_backward_pair<scalar_t>(pr, pp, value, loc, aw, gout, gval, gloc, gaw, workspace, pad, st);
    if (ns > 0)
      return run_backward_fused<scalar_t>(pr, ns, value, loc, aw, gout, gval, gloc, gaw, pad, st);
  }
  if (pr.gv_rs > 0 && pr.gv_rs != pr.M * pr.D) {
    set_error("msda backward: a strided grad_value needs the fused per-tap path");
    return MSDA_ERR_UNSUPPORTED;
  }
  SideStream* side = nullptr;
  // worth a fork / join (~5 us) only when the coordinate kernel is long (encoder-sized calls)
  if (gval != nullptr && (gloc != nullptr || gaw != nullptr) && pr.B * pr.M * pr.S > 0 &&
      pr.B * pr.Lq * pr.M >= 32768) {
    side = side_stream();
    if (side != nullptr && (hipEventRecord(side->fork, st) != hipSuccess ||
                            hipStreamWaitEvent(side->s, side->fork, 0) != hipSuccess))
      side = nullptr;
  }
  const int rc = run_backward_impl<scalar_t, coord_t>(pr, value, loc, aw, gout, gval, gloc, gaw,
                                                      workspace, value_dtype, pad, st,
                                                      side != nullptr ? side->s : st);
  if (side != nullptr) {
    if (hipEventRecord(side->join, side->s) != hipSuccess ||
        hipStreamWaitEvent(st, side->join, 0) != hipSuccess) {
      set_error("msda_hip_backward: side-stream join failed");
      return MSDA_ERR_LAUNCH;
    }
  }
  return rc;
}


// ---------------------------------------------------------------------------------
// MSDA prologue: the elementwise chain of MSDeformAttn.forward between
// the sampling_offsets / attention_weights projections and the core
// (reference models/modules/attention.py:468-483):
//   aw  = softmax(attention_weights(query).view(..., L*P))            (fp32 under autocast)
//   loc = ref[..., 0] + off / T_l                         (ref_dim 1)
//   loc = ref[..., 0] + off / P * ref[..., 1] * 0.5       (ref_dim 2, the box form)
// in ONE kernel per direction instead of ~5 PyTorch kernels each.  The 16-bit cases keep
// PyTorch's type promotion exactly: off / T_l and off / P are 16-bit tensors (computed in
// fp32, rounded once), everything after the promotion to the fp32 reference is fp32; the
// backward rounds where autograd casts back to the 16-bit inputs.
// ---------------------------------------------------------------------------------
template <typename scalar_t> struct Is16 { static constexpr bool value = false; };
template <> struct Is16<bf16_t> { static constexpr bool value = true; };
template <> struct Is16<f16_t> { static constexpr bool value = true; };

// value rounded to scalar_t and back (identity for fp32 / fp64)
template <typename scalar_t, typename coord_t>
__device__ __forceinline__ coord_t round_to(coord_t v) {
  if constexpr (Is16<scalar_t>::value) {
    scalar_t h;
    from_acc((float)v, &h);
    return (coord_t)to_acc(h);
  } else {
    return v;
  }
}

// One thread per sample (b, q, m, l, p): loads and stores are contiguous across the block.  A
// block holds G whole queries (G*M*L*P threads, M*L*P <= 1024); the 16-way softmax sums and the
// grad_ref sums over (m, p) go through LDS.
// Sum / max over the item's LP samples.  LP a power of two <= 64: the samples of one item are
// aligned lanes of one wave (QS = M*LP and blocks start at wave boundaries), so a butterfly of
// __shfl_xor does it without LDS or barriers; otherwise through LDS.
template <typename coord_t, bool MAXOP>
__device__ __forceinline__ coord_t item_reduce(coord_t v, int LP, bool pow2, coord_t* sx, int t, int t0) {
  if (pow2) {
    for (int o = 1; o < LP; o <<= 1) {
      const coord_t w = __shfl_xor(v, o);
      v = MAXOP ? (w > v ? w : v) : v + w;
    }
    return v;
  }
  __syncthreads();
  sx[t] = v;
  __syncthreads();
  coord_t r = MAXOP ? (coord_t)-INFINITY : (coord_t)0;
  for (int k = 0; k < LP; ++k) r = MAXOP ? (sx[t0 + k] > r ? sx[t0 + k] : r) : r + sx[t0 + k];
  return r;
}

// Thread -> (query in block, sample j, level l): shifts when P, L*P and M*L*P are powers of
// two (the reference's 4 x 4 x 8), integer division otherwise (runtime divisions cost ~40
// VALU each and made the kernel ALU-bound).
struct PrologueIdx {
  int g, r, j, l;
};
template <bool POW2>
__device__ __forceinline__ PrologueIdx prologue_idx(int t, int QS, int LP, int P, int sQS, int sLP, int sP) {
  PrologueIdx x;
  if constexpr (POW2) {
    x.g = t >> sQS;
    x.r = t & (QS - 1);
    x.j = x.r & (LP - 1);
    x.l = x.j >> sP;
  } else {
    x.g = t / QS;
    x.r = t - x.g * QS;
    x.j = x.r % LP;
    x.l = x.j / P;
  }
  (void)sLP;
  return x;
}

// T_l for a per-lane level index without a dynamically indexed kernel-argument load (which
// costs one extra dependent memory round trip): a select chain over the uniform table.
__device__ __forceinline__ int level_T(const Levels& lv, int l, int L) {
  int T = lv.T[0];
#pragma unroll
  for (int k = 1; k < MSDA_MAX_LEVELS; ++k)
    if (k < L && l == k) T = lv.T[k];
  return T;
}

template <typename scalar_t, typename coord_t, bool POW2>
__global__ __launch_bounds__(1024) void msda_prologue_fwd_kernel(
    const scalar_t* __restrict__ off, const scalar_t* __restrict__ logits,
    const coord_t* __restrict__ ref, const int ref_dim, coord_t* __restrict__ loc,
    coord_t* __restrict__ aw, const Levels lv, const int L, const int P, const int M,
    const long long n_queries, const int G, const int sQS, const int sLP, const int sP, const long long is) {
#pragma clang fp contract(off)  // PyTorch evaluates these as separate kernels: no FMA fusion
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  coord_t* sx = reinterpret_cast<coord_t*>(smem_raw);
  const int LP = L * P, QS = M * LP;
  const bool pow2 = POW2 || (LP & (LP - 1)) == 0;
  const int t = threadIdx.x;
  const PrologueIdx ix = prologue_idx<POW2>(t, QS, LP, P, sQS, sLP, sP);
  const long long bq_raw = (long long)blockIdx.x * G + ix.g;
  const bool active = bq_raw < n_queries;
  const long long bq = active ? bq_raw : 0;  // clamped: every load below is unconditional
  const int r = ix.r, j = ix.j, l = ix.l;
  const long long e = bq * QS + r;
  const long long ei = bq * is + r;  // offsets / logits rows: `is` elements apart
  // all global loads of the thread issued together: one round trip
  const coord_t x = (coord_t)to_acc(logits[ei]);
  const coord_t v = (coord_t)to_acc(off[ei]);
  const coord_t r0 = ref[(bq * L + l) * ref_dim];
  const coord_t r1 = ref[(bq * L + l) * ref_dim + (ref_dim - 1)];
  const coord_t T = (coord_t)level_T(lv, l, L);
  const int t0 = t - j;
  const coord_t mx = item_reduce<coord_t, true>(x, LP, pow2, sx, t, t0);
  const coord_t ex = exp(x - mx);  // one exp per sample
  const coord_t sum = item_reduce<coord_t, false>(ex, LP, pow2, sx, t, t0);
  if (!active) return;
  aw[e] = ex / sum;
  if (ref_dim == 1)
    loc[e] = r0 + round_to<scalar_t>(v / T);
  else
    loc[e] = r0 + (round_to<scalar_t>(v / (coord_t)P) * r1) * (coord_t)0.5;
}

template <typename scalar_t, typename coord_t, bool POW2>
__global__ __launch_bounds__(1024) void msda_prologue_bwd_kernel(
    const coord_t* __restrict__ grad_loc, const coord_t* __restrict__ grad_aw,
    const coord_t* __restrict__ aw, const scalar_t* __restrict__ off, const coord_t* __restrict__ ref,
    const int ref_dim, scalar_t* __restrict__ grad_off, scalar_t* __restrict__ grad_logits,
    coord_t* __restrict__ grad_ref, const Levels lv, const int L, const int P, const int M,
    const long long n_queries, const int G, const int sQS, const int sLP, const int sP, const long long is) {
#pragma clang fp contract(off)  // PyTorch evaluates these as separate kernels: no FMA fusion
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  coord_t* s0 = reinterpret_cast<coord_t*>(smem_raw);  // g*y, then grad_loc
  coord_t* s1 = s0 + blockDim.x;                        // box form: grad of ref[..., 1]
  const int LP = L * P, QS = M * LP;
  const int t = threadIdx.x;
  const PrologueIdx ix = prologue_idx<POW2>(t, QS, LP, P, sQS, sLP, sP);
  const long long bq_raw = (long long)blockIdx.x * G + ix.g;
  const bool active = bq_raw < n_queries;
  const long long bq = active ? bq_raw : 0;  // clamped: loads below are unconditional
  const int r = ix.r, j = ix.j, l = ix.l;
  const long long e = bq * QS + r;
  const long long ei = bq * is + r;  // offsets / logits (and their gradients) rows: `is` elements apart
  const bool pow2 = (LP & (LP - 1)) == 0;
  const bool loc_side = grad_off != nullptr || grad_ref != nullptr;
  const bool box = ref_dim == 2;
  const coord_t T = (coord_t)level_T(lv, l, L);
  const coord_t gl = loc_side ? (active ? grad_loc[e] : (coord_t)0) : (coord_t)0;
  const coord_t r1 = box ? ref[(bq * L + l) * 2 + 1] : (coord_t)0;
  const coord_t ov = box ? (coord_t)to_acc(off[ei]) : (coord_t)0;
  if (grad_logits != nullptr) {  // uniform
    const coord_t g = active ? grad_aw[e] : (coord_t)0;
    const coord_t y = active ? aw[e] : (coord_t)0;
    const coord_t dot = item_reduce<coord_t, false>(g * y, LP, pow2, s0, t, t - j);
    if (active) from_acc((typename AccOf<scalar_t>::type)(y * (g - dot)), &grad_logits[ei]);
  }
  if (!loc_side) return;
  coord_t gu = 0;  // box form: d loc / d ref1 contribution
  if (!box) {
    if (grad_off != nullptr && active)
      from_acc((typename AccOf<scalar_t>::type)(round_to<scalar_t>(gl) / T), &grad_off[ei]);
  } else if (active) {
    const coord_t gh = gl * (coord_t)0.5;
    if (grad_off != nullptr)
      from_acc((typename AccOf<scalar_t>::type)(round_to<scalar_t>(gh * r1) / (coord_t)P), &grad_off[ei]);
    gu = gh * round_to<scalar_t>(ov / (coord_t)P);
  }
  if (grad_ref == nullptr) return;  // uniform
  __syncthreads();
  s0[t] = gl;
  s1[t] = gu;
  __syncthreads();
  // grad_ref[bq, l, c]: sum over (m, p) of the block's G queries
  for (int o = t; o < G * L * ref_dim; o += blockDim.x) {
    const int c = o % ref_dim, ql = o / ref_dim;
    const int lq = ql % L, g = ql / L;
    const long long bqo = (long long)blockIdx.x * G + g;
    if (bqo >= n_queries) continue;
    const coord_t* src = c == 0 ? s0 : s1;
    coord_t acc = 0;
    for (int m = 0; m < M; ++m)
      for (int p = 0; p < P; ++p) acc += src[g * QS + m * LP + lq * P + p];
    grad_ref[(bqo * L + lq) * ref_dim + c] = acc;
  }
}

// Fast path for the reference's shape (L*P == 16, M a power of two <= 64, fp32 coordinates):
// one thread per (b, q, m) item, all of its 16 samples in registers, 16-byte loads and stores
// (the per-sample kernels above spend most of their time on per-lane address arithmetic).
template <typename scalar_t>
__device__ __forceinline__ void load16s(const scalar_t* __restrict__ p, float (&r)[16]) {
  constexpr int V = 16 / (int)sizeof(scalar_t);
#pragma unroll
  for (int c = 0; c < 16 / V; ++c) {
    float t[V];
    load_vec<scalar_t, V>(p + c * V, t);
#pragma unroll
    for (int i = 0; i < V; ++i) r[c * V + i] = t[i];
  }
}
template <typename scalar_t>
__device__ __forceinline__ void store16s(scalar_t* __restrict__ p, const float (&r)[16]) {
  constexpr int V = 16 / (int)sizeof(scalar_t);
#pragma unroll
  for (int c = 0; c < 16 / V; ++c) {
    float t[V];
#pragma unroll
    for (int i = 0; i < V; ++i) t[i] = r[c * V + i];
    store_vec<scalar_t, V>(p + c * V, t);
  }
}

template <typename scalar_t, int M, int P>
__global__ __launch_bounds__(256) void msda_prologue16_fwd_kernel(
    const scalar_t* __restrict__ off, const scalar_t* __restrict__ logits, const float* __restrict__ ref,
    const int ref_dim, float* __restrict__ loc, float* __restrict__ aw, const Levels lv,
    const long long n_items, const long long is) {
#pragma clang fp contract(off)  // PyTorch evaluates these as separate kernels: no FMA fusion
  constexpr int L = 16 / P;
  const long long item = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (item >= n_items) return;
  const long long bq = item / M;
  const long long ii = bq * is + (item % M) * 16;  // offsets / logits rows: `is` elements apart
  float x[16], v[16];
  load16s<scalar_t>(logits + ii, x);
  load16s<scalar_t>(off + ii, v);
  float mx = x[0];
#pragma unroll
  for (int j = 1; j < 16; ++j) mx = x[j] > mx ? x[j] : mx;
  float sum = 0.f;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    x[j] = expf(x[j] - mx);
    sum += x[j];
  }
#pragma unroll
  for (int j = 0; j < 16; ++j) x[j] = x[j] / sum;
  store16s<float>(aw + item * 16, x);
  const float* __restrict__ rb = ref + bq * L * ref_dim;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int l = j / P;
    const float r0 = rb[l * ref_dim];
    if (ref_dim == 1) {
      v[j] = r0 + round_to<scalar_t>(v[j] / (float)lv.T[l]);
    } else {
      v[j] = r0 + (round_to<scalar_t>(v[j] / (float)P) * rb[l * 2 + 1]) * 0.5f;
    }
  }
  store16s<float>(loc + item * 16, v);
}

template <typename scalar_t, int M, int P>
__global__ __launch_bounds__(256) void msda_prologue16_bwd_kernel(
    const float* __restrict__ grad_loc, const float* __restrict__ grad_aw, const float* __restrict__ aw,
    const scalar_t* __restrict__ off, const float* __restrict__ ref, const int ref_dim,
    scalar_t* __restrict__ grad_off, scalar_t* __restrict__ grad_logits, float* __restrict__ grad_ref,
    const Levels lv, const long long n_items, const long long is) {
#pragma clang fp contract(off)  // PyTorch evaluates these as separate kernels: no FMA fusion
  constexpr int L = 16 / P;
  const long long item_raw = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const bool active = item_raw < n_items;  // every lane stays for the grad_ref lane sums
  const long long item = active ? item_raw : 0;
  const long long bq = item / M;
  const int m = (int)(item % M);
  const long long ii = bq * is + m * 16;  // offsets / logits (and their gradients): rows `is` elements apart
  if (grad_logits != nullptr) {
    float g[16], y[16];
    load16s<float>(grad_aw + item * 16, g);
    load16s<float>(aw + item * 16, y);
    float dot = 0.f;
#pragma unroll
    for (int j = 0; j < 16; ++j) dot += g[j] * y[j];
#pragma unroll
    for (int j = 0; j < 16; ++j) g[j] = y[j] * (g[j] - dot);
    if (active) store16s<scalar_t>(grad_logits + ii, g);
  }
  if (grad_off == nullptr && grad_ref == nullptr) return;
  float gl[16], o[16];
  load16s<float>(grad_loc + item * 16, gl);
  const bool box = ref_dim == 2;
  if (box) load16s<scalar_t>(off + ii, o);
  const float* __restrict__ rb = ref + bq * L * ref_dim;
  float go[16], s1[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int l = j / P;
    if (!box) {
      go[j] = round_to<scalar_t>(gl[j]) / (float)lv.T[l];
      s1[j] = 0.f;
    } else {
      const float gh = gl[j] * 0.5f;
      go[j] = round_to<scalar_t>(gh * rb[l * 2 + 1]) / (float)P;
      s1[j] = gh * round_to<scalar_t>(o[j] / (float)P);
    }
  }
  if (grad_off != nullptr && active) store16s<scalar_t>(grad_off + ii, go);
  if (grad_ref != nullptr) {
#pragma unroll
    for (int l = 0; l < L; ++l) {
      float a0 = 0.f, a1 = 0.f;
#pragma unroll
      for (int p = 0; p < P; ++p) {
        a0 += active ? gl[l * P + p] : 0.f;
        a1 += active ? s1[l * P + p] : 0.f;
      }
      a0 = group_sum<M>(a0);
      if (box) a1 = group_sum<M>(a1);
      if (active && m == 0) {
        grad_ref[(bq * L + l) * ref_dim] = a0;
        if (box) grad_ref[(bq * L + l) * 2 + 1] = a1;
      }
    }
  }
}

// Level-major variants (MSDA_COORD_LEVEL_MAJOR, (B, M, L, Lq, P); num_point a multiple of 4, L*P == 16,
// M <= 8): one workgroup of 32 M threads per (b, tile of 32 queries), thread (m, i) the item
// (b, q0 + i, m), so level l's P coordinates of 32 consecutive queries are one contiguous store
// (the backward's row blocks then read and write whole lines).  Same arithmetic as
// msda_prologue16_*_kernel; grad_ref sums the heads through LDS in head order.
template <int P>
__device__ __forceinline__ void store_level_lm(float* __restrict__ dst, long long cl, const float (&r)[16]) {
#pragma unroll
  for (int l = 0; l < 16 / P; ++l)
#pragma unroll
    for (int c = 0; c < P / 4; ++c)
      *reinterpret_cast<float4*>(dst + l * cl + 4 * c) =
          make_float4(r[l * P + 4 * c], r[l * P + 4 * c + 1], r[l * P + 4 * c + 2], r[l * P + 4 * c + 3]);
}
template <int P>
__device__ __forceinline__ void load_level_lm(const float* __restrict__ src, long long cl, float (&r)[16]) {
#pragma unroll
  for (int l = 0; l < 16 / P; ++l)
#pragma unroll
    for (int c = 0; c < P / 4; ++c) {
      const float4 x = *reinterpret_cast<const float4*>(src + l * cl + 4 * c);
      r[l * P + 4 * c] = x.x; r[l * P + 4 * c + 1] = x.y; r[l * P + 4 * c + 2] = x.z; r[l * P + 4 * c + 3] = x.w;
    }
}

template <typename scalar_t, int P>
__global__ __launch_bounds__(256) void msda_prologue16lm_fwd_kernel(
    const scalar_t* __restrict__ off, const scalar_t* __restrict__ logits, const float* __restrict__ ref,
    const int ref_dim, float* __restrict__ loc, float* __restrict__ aw, const Levels lv, const int M,
    const long long Lq, const int ntile, const long long is) {
#pragma clang fp contract(off)  // PyTorch evaluates these as separate kernels: no FMA fusion
  static_assert(P % 4 == 0 && 16 % P == 0, "level-major prologue: P in {4, 8, 16}");
  constexpr int L = 16 / P;
  const long long b = blockIdx.x / ntile;
  const long long q = (long long)(blockIdx.x % ntile) * 32 + (threadIdx.x & 31);
  const int m = (int)(threadIdx.x >> 5);
  if (q >= Lq || m >= M) return;
  const long long bq = b * Lq + q;
  const long long ii = bq * is + m * 16;
  float x[16], v[16];
  load16s<scalar_t>(logits + ii, x);
  load16s<scalar_t>(off + ii, v);
  float mx = x[0];
#pragma unroll
  for (int j = 1; j < 16; ++j) mx = x[j] > mx ? x[j] : mx;
  float sum = 0.f;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    x[j] = expf(x[j] - mx);
    sum += x[j];
  }
#pragma unroll
  for (int j = 0; j < 16; ++j) x[j] = x[j] / sum;
  const long long cl = Lq * P;
  const long long c0 = (b * M + m) * L * cl + q * P;
  store_level_lm<P>(aw + c0, cl, x);
  const float* __restrict__ rb = ref + bq * L * ref_dim;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int l = j / P;
    const float r0 = rb[l * ref_dim];
    if (ref_dim == 1) {
      v[j] = r0 + round_to<scalar_t>(v[j] / (float)lv.T[l]);
    } else {
      v[j] = r0 + (round_to<scalar_t>(v[j] / (float)P) * rb[l * 2 + 1]) * 0.5f;
    }
  }
  store_level_lm<P>(loc + c0, cl, v);
}

template <typename scalar_t, int P>
__global__ __launch_bounds__(256) void msda_prologue16lm_bwd_kernel(
    const float* __restrict__ grad_loc, const float* __restrict__ grad_aw, const float* __restrict__ aw,
    const scalar_t* __restrict__ off, const float* __restrict__ ref, const int ref_dim,
    scalar_t* __restrict__ grad_off, scalar_t* __restrict__ grad_logits, float* __restrict__ grad_ref,
    const Levels lv, const int M, const long long Lq, const int ntile, const long long is) {
#pragma clang fp contract(off)  // PyTorch evaluates these as separate kernels: no FMA fusion
  static_assert(P % 4 == 0 && 16 % P == 0, "level-major prologue: P in {4, 8, 16}");
  constexpr int L = 16 / P;
  __shared__ float s_ref[2][L][8][32];
  const long long b = blockIdx.x / ntile;
  const int i = (int)(threadIdx.x & 31);
  const long long q = (long long)(blockIdx.x % ntile) * 32 + i;
  const int m = (int)(threadIdx.x >> 5);
  const bool active = q < Lq && m < M;  // every thread stays for the grad_ref sums
  const long long bq = b * Lq + (active ? q : 0);
  const int mm = active ? m : 0;
  const long long ii = bq * is + mm * 16;
  const long long cl = Lq * P;
  const long long c0 = (b * M + mm) * L * cl + (active ? q : 0) * P;
  if (grad_logits != nullptr) {
    float g[16], y[16];
    load_level_lm<P>(grad_aw + c0, cl, g);
    load_level_lm<P>(aw + c0, cl, y);
    float dot = 0.f;
#pragma unroll
    for (int j = 0; j < 16; ++j) dot += g[j] * y[j];
#pragma unroll
    for (int j = 0; j < 16; ++j) g[j] = y[j] * (g[j] - dot);
    if (active) store16s<scalar_t>(grad_logits + ii, g);
  }
  if (grad_off == nullptr && grad_ref == nullptr) return;  // uniform
  float gl[16], o[16];
  load_level_lm<P>(grad_loc + c0, cl, gl);
  const bool box = ref_dim == 2;
  if (box) load16s<scalar_t>(off + ii, o);
  const float* __restrict__ rb = ref + bq * L * ref_dim;
  float go[16], s1[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int l = j / P;
    if (!box) {
      go[j] = round_to<scalar_t>(gl[j]) / (float)lv.T[l];
      s1[j] = 0.f;
    } else {
      const float gh = gl[j] * 0.5f;
      go[j] = round_to<scalar_t>(gh * rb[l * 2 + 1]) / (float)P;
      s1[j] = gh * round_to<scalar_t>(o[j] / (float)P);
    }
  }
  if (grad_off != nullptr && active) store16s<scalar_t>(grad_off + ii, go);
  if (grad_ref == nullptr) return;  // uniform
#pragma unroll
  for (int l = 0; l < L; ++l) {
    float a0 = 0.f, a1 = 0.f;
#pragma unroll
    for (int p = 0; p < P; ++p) {
      a0 += active ? gl[l * P + p] : 0.f;
      a1 += active ? s1[l * P + p] : 0.f;
    }
    if (m < 8) {
      s_ref[0][l][m][i] = a0;
      s_ref[1][l][m][i] = a1;
    }
  }
  __syncthreads();
  if (m == 0 && q < Lq) {
#pragma unroll
    for (int l = 0; l < L; ++l) {
      float a0 = 0.f, a1 = 0.f;
      for (int h = 0; h < M; ++h) {
        a0 += s_ref[0][l][h][i];
        a1 += s_ref[1][l][h][i];
      }
      grad_ref[(bq * L + l) * ref_dim] = a0;
      if (box) grad_ref[(bq * L + l) * 2 + 1] = a1;
    }
  }
}

// the level-major prologue's coverage (msda_prologue16lm_*_kernel)
bool prologue_lm_ok(long long M, long long L, long long P) {
  return L * P == 16 && (P == 4 || P == 8 || P == 16) && M >= 1 && M <= 8;
}

template <typename scalar_t, typename coord_t>
int run_prologue(bool fwd, const Problem& pr, int ref_dim, const void* off, const void* logits,
                 const void* ref, void* loc, void* aw, const void* grad_loc, const void* grad_aw,
                 void* grad_off, void* grad_logits, void* grad_ref, long long is, hipStream_t st,
                 int layout = MSDA_COORD_API) {
  const long long n_queries = pr.B * pr.Lq;
  if (layout == MSDA_COORD_LEVEL_MAJOR) {
    if constexpr (std::is_same<coord_t, double>::value) {
      set_error("msda prologue: the level-major layout needs fp32 coordinates");
      return MSDA_ERR_ARG;
    } else {
      if (!prologue_lm_ok(pr.M, pr.L, pr.P)) {
        set_error("msda prologue: the level-major layout needs num_levels*num_point == 16, num_point in {4, 8, 16} "
                  "and num_heads <= 8");
        return MSDA_ERR_ARG;
      }
      if (n_queries == 0) return MSDA_OK;
      const int ntile = (int)((pr.Lq + 31) / 32);
      const unsigned blocks = (unsigned)(pr.B * ntile);
      const unsigned threads = (unsigned)(32 * pr.M);
      auto* o = static_cast<const scalar_t*>(off);
      auto* rf = static_cast<const float*>(ref);
#define MSDA_PLM(PP)                                                                                  \
  do {                                                                                              \
    if (fwd)                                                                                        \
      hipLaunchKernelGGL((msda_prologue16lm_fwd_kernel<scalar_t, PP>), dim3(blocks), dim3(threads), 0, st, o, \
                         static_cast<const scalar_t*>(logits), rf, ref_dim, static_cast<float*>(loc),     \
                         static_cast<float*>(aw), pr.lv, (int)pr.M, pr.Lq, ntile, is);               \
    else                                                                                            \
      hipLaunchKernelGGL((msda_prologue16lm_bwd_kernel<scalar_t, PP>), dim3(blocks), dim3(threads), 0, st, \
                         static_cast<const float*>(grad_loc), static_cast<const float*>(grad_aw),    \
                         static_cast<const float*>(aw), o, rf, ref_dim, static_cast<scalar_t*>(grad_off), \
                         static_cast<scalar_t*>(grad_logits), static_cast<float*>(grad_ref), pr.lv, (int)pr.M, \
                         pr.Lq, ntile, is);                                                          \
  } while (0)
      if (pr.P == 4) MSDA_PLM(4);
      else if (pr.P == 8) MSDA_PLM(8);
      else MSDA_PLM(16);
#undef MSDA_PLM
      return launch_status(fwd ? "prologue forward (level-major)" : "prologue backward (level-major)");
    }
  }
  if (n_queries == 0) return MSDA_OK;
  if constexpr (!std::is_same<coord_t, double>::value) {
    const int Mi = (int)pr.M;
    // item-per-thread kernels need enough items to fill the chip (encoder-sized calls: 10.6 / 7.2 us
    // vs 11.6 / 13.7 us per-sample at B=8, Lq=1920); small calls (decoder queries) take the
    // per-sample kernels (3.2 / 4.8 us vs 5.5 / 5.0 us at Lq=100)
    if (pr.L * pr.P == 16 && 16 % pr.P == 0 && Mi <= 64 && (Mi & (Mi - 1)) == 0 &&
        n_queries * pr.M >= 65536) {
      const long long n_items = n_queries * pr.M;
      const unsigned blocks = (unsigned)((n_items + 255) / 256);
      auto* o = static_cast<const scalar_t*>(off);
      auto* rf = static_cast<const float*>(ref);
#define MSDA_P16_(MM, PP)                                                                          \
  do {                                                                                           \
    if (fwd)                                                                                     \
      hipLaunchKernelGGL((msda_prologue16_fwd_kernel<scalar_t, MM, PP>), dim3(blocks), dim3(256), 0, st, o, \
                         static_cast<const scalar_t*>(logits), rf, ref_dim, static_cast<float*>(loc), \
                         static_cast<float*>(aw), pr.lv, n_items, is);                           \
    else                                                                                         \
      hipLaunchKernelGGL((msda_prologue16_bwd_kernel<scalar_t, MM, PP>), dim3(blocks), dim3(256), 0, st, \
                         static_cast<const float*>(grad_loc), static_cast<const float*>(grad_aw), \
                         static_cast<const float*>(aw), o, rf, ref_dim, static_cast<scalar_t*>(grad_off), \
                         static_cast<scalar_t*>(grad_logits), static_cast<float*>(grad_ref), pr.lv, n_items, is); \
  } while (0)
#define MSDA_P16(MM)                                                                               \
  do {                                                                                           \
    switch (pr.P) {                                                                              \
      case 1: MSDA_P16_(MM, 1); break;                                                           \
      case 2: MSDA_P16_(MM, 2); break;                                                           \
      case 4: MSDA_P16_(MM, 4); break;                                                           \
      case 8: MSDA_P16_(MM, 8); break;                                                           \
      default: MSDA_P16_(MM, 16); break;                                                         \
    }                                                                                            \
  } while (0)
      switch (Mi) {
        case 1: MSDA_P16(1); break;
        case 2: MSDA_P16(2); break;
        case 4: MSDA_P16(4); break;
        case 8: MSDA_P16(8); break;
        case 16: MSDA_P16(16); break;
        case 32: MSDA_P16(32); break;
        default: MSDA_P16(64); break;
      }
#undef MSDA_P16
#undef MSDA_P16_
      return launch_status(fwd ? "prologue forward" : "prologue backward");
    }
  }
  const int QS = (int)(pr.M * pr.L * pr.P);
  const int G = max(1, 256 / QS);
  const int threads = G * QS;
  const unsigned blocks = (unsigned)((n_queries + G - 1) / G);
  const size_t lds = (size_t)threads * sizeof(coord_t) * (fwd ? 1 : 2);
  auto* o = static_cast<const scalar_t*>(off);
  auto* r = static_cast<const coord_t*>(ref);
  auto lg2 = [](long long v) { int k = 0; while ((1LL << k) < v) ++k; return (1LL << k) == v ? k : -1; };
  const int sQS = lg2(QS), sLP = lg2(pr.L * pr.P), sP = lg2(pr.P);
  const bool pow2 = sQS >= 0 && sLP >= 0 && sP >= 0;
#define MSDA_PRO(PW)                                                                                  \
  do {                                                                                              \
    if (fwd)                                                                                        \
      hipLaunchKernelGGL((msda_prologue_fwd_kernel<scalar_t, coord_t, PW>), dim3(blocks), dim3(threads), lds, \
                         st, o, static_cast<const scalar_t*>(logits), r, ref_dim, static_cast<coord_t*>(loc), \
                         static_cast<coord_t*>(aw), pr.lv, (int)pr.L, (int)pr.P, (int)pr.M, n_queries, G, \
                         sQS, sLP, sP, is);                                                          \
    else                                                                                            \
      hipLaunchKernelGGL((msda_prologue_bwd_kernel<scalar_t, coord_t, PW>), dim3(blocks), dim3(threads), lds, \
                         st, static_cast<const coord_t*>(grad_loc), static_cast<const coord_t*>(grad_aw), \
                         static_cast<const coord_t*>(aw), o, r, ref_dim, static_cast<scalar_t*>(grad_off), \
                         static_cast<scalar_t*>(grad_logits), static_cast<coord_t*>(grad_ref), pr.lv,   \
                         (int)pr.L, (int)pr.P, (int)pr.M, n_queries, G, sQS, sLP, sP, is);          \
  } while (0)
  if (pow2) MSDA_PRO(true);
  else MSDA_PRO(false);
#undef MSDA_PRO
  return launch_status(fwd ? "prologue forward" : "prologue backward");
}

int check_prologue(const int64_t* shapes, int64_t L, int64_t B, int64_t Lq, int64_t M, int64_t P,
                   int ref_dim, Problem* pr) {
  if (L < 1 || L > MSDA_MAX_LEVELS || B < 0 || Lq < 0 || M < 1 || P < 1 || M * L * P > 1024 ||
      (ref_dim != 1 && ref_dim != 2) || shapes == nullptr) {
    set_error("msda prologue: bad arguments (L=%lld M=%lld P=%lld ref_dim=%d; M*L*P must be <= 1024)",
              (long long)L, (long long)M, (long long)P, ref_dim);
    return MSDA_ERR_ARG;
  }
  for (int64_t l = 0; l < L; ++l) {
    if (shapes[l] < 1) {
      set_error("msda prologue: level %lld has T=%lld", (long long)l, (long long)shapes[l]);
      return MSDA_ERR_ARG;
    }
    pr->lv.T[l] = (int)shapes[l];
    pr->lv.start[l] = 0;
  }
  pr->B = B; pr->S = 0; pr->M = M; pr->D = 1; pr->Lq = Lq; pr->L = L; pr->P = P;
  return MSDA_OK;
}

int dispatch_prologue(bool fwd, int dtype, const Problem& pr, int ref_dim, const void* off,
                      const void* logits, const void* ref, void* loc, void* aw, const void* grad_loc,
                      const void* grad_aw, void* grad_off, void* grad_logits, void* grad_ref,
                      long long is, hipStream_t st, int layout = MSDA_COORD_API) {
  if (layout != MSDA_COORD_API && layout != MSDA_COORD_LEVEL_MAJOR) {
    set_error("msda prologue: unknown coordinate layout %d", layout);
    return MSDA_ERR_ARG;
  }
  switch (dtype) {
    case MSDA_DTYPE_F32:
      return run_prologue<float, float>(fwd, pr, ref_dim, off, logits, ref, loc, aw, grad_loc, grad_aw, grad_off,
                                        grad_logits, grad_ref, is, st, layout);
    case MSDA_DTYPE_F64:
      return run_prologue<double, double>(fwd, pr, ref_dim, off, logits, ref, loc, aw, grad_loc, grad_aw,
                                          grad_off, grad_logits, grad_ref, is, st, layout);
    case MSDA_DTYPE_BF16:
      return run_prologue<bf16_t, float>(fwd, pr, ref_dim, off, logits, ref, loc, aw, grad_loc, grad_aw,
                                         grad_off, grad_logits, grad_ref, is, st, layout);
    case MSDA_DTYPE_F16:
      return run_prologue<f16_t, float>(fwd, pr, ref_dim, off, logits, ref, loc, aw, grad_loc, grad_aw,
                                        grad_off, grad_logits, grad_ref, is, st, layout);
    default:
      set_error("msda prologue: unknown dtype %d", dtype);
      return MSDA_ERR_ARG;
  }
}


// ---------------------------------------------------------------------------------
// Sparse-DETR decoder attention map (reference utils/dam.py:20-73,
// attn_map_to_flat_grid): for every (batch*layer, head) row, scatter-add each sample's
// attention weight onto the two tokens around x = loc * T_l of its level:
//   token start_l + floor(x)     += aw * (x - floor(x) - 1)   (the reference's margin_end, <= 0)
//   token start_l + floor(x) + 1 += aw * (x - floor(x))
// each only if the token lies inside the level.  One workgroup per row accumulates the row in
// LDS (S fp32 words) and writes it once; rows too long for LDS accumulate with global atomics
// into the zeroed output.
// ---------------------------------------------------------------------------------
constexpr int kDamThreads = 256;
constexpr long long kDamLdsMax = 128 * 1024;

template <bool LDS>
__global__ __launch_bounds__(kDamThreads) void msda_dam_kernel(
    const float* __restrict__ loc, const float* __restrict__ aw, float* __restrict__ out, const Levels lv,
    const int L, const int P, const int M, const int Lq, const int S) {
#pragma clang fp contract(off)  // the reference's separate mul / sub kernels
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  float* acc = reinterpret_cast<float*>(smem_raw);
  const long long row = blockIdx.x;  // (batch*layer) * M + m
  const int m = (int)(row % M);
  const long long bn = row / M;
  float* __restrict__ orow = out + row * S;
  if constexpr (LDS) {
    for (int i = threadIdx.x; i < S; i += kDamThreads) acc[i] = 0.f;
    __syncthreads();
  }
  const int LP = L * P;
  const long long nsamp = (long long)Lq * LP;
  for (long long s = threadIdx.x; s < nsamp; s += kDamThreads) {
    const int q = (int)(s / LP), j = (int)(s - (long long)q * LP);
    const int l = j / P;
    const long long e = ((bn * Lq + q) * M + m) * LP + j;
    const int T = level_T(lv, l, L);
    int st = lv.start[0];
#pragma unroll
    for (int k = 1; k < MSDA_MAX_LEVELS; ++k)
      if (k < L && l == k) st = lv.start[k];
    const float x = loc[e] * (float)T;
    const float a = aw[e];
    const float f = floorf(x);
    const long long i0 = (long long)f;
    const float m_start = x - (float)i0;
    const float m_end = x - (float)(i0 + 1);
    if (i0 >= 0 && i0 < T) {
      if constexpr (LDS) atomicAdd(&acc[st + (int)i0], a * m_end);
      else atomicAdd(&orow[st + (int)i0], a * m_end);
    }
    if (i0 + 1 >= 0 && i0 + 1 < T) {
      if constexpr (LDS) atomicAdd(&acc[st + (int)i0 + 1], a * m_start);
      else atomicAdd(&orow[st + (int)i0 + 1], a * m_start);
    }
  }
  if constexpr (LDS) {
    __syncthreads();
    for (int i = threadIdx.x; i < S; i += kDamThreads) orow[i] = acc[i];
  }
}

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

int msda_hip_abi_version(void) { return 8; }

const char* msda_hip_last_error(void) { return g_last_error; }

int msda_hip_dam_flat_grid(const void* sampling_loc, const void* attn_weight, const int64_t* spatial_shapes,
                           const int64_t* level_start, int64_t num_levels, int64_t rows, int64_t num_query,
                           int64_t num_heads, int64_t num_point, void* flat_grid, void* stream) {
  g_last_error[0] = 0;
  Problem pr;
  long long S = 0;
  if (spatial_shapes != nullptr && num_levels >= 1 && num_levels <= MSDA_MAX_LEVELS)
    for (int64_t l = 0; l < num_levels; ++l) S += spatial_shapes[l];
  int rc = check_problem(spatial_shapes, level_start, num_levels, rows, S, num_heads, 1, num_query, num_point, &pr);
  if (rc) return rc;
  const long long nrows = rows * num_heads;
  if (nrows == 0 || S == 0) return MSDA_OK;
  if (flat_grid == nullptr || (num_query > 0 && (sampling_loc == nullptr || attn_weight == nullptr))) {
    set_error("msda_hip_dam_flat_grid: null pointer");
    return MSDA_ERR_ARG;
  }
  hipStream_t st = static_cast<hipStream_t>(stream);
  auto* lc = static_cast<const float*>(sampling_loc);
  auto* a = static_cast<const float*>(attn_weight);
  auto* out = static_cast<float*>(flat_grid);
  const size_t lds = (size_t)S * 4;
  if ((long long)lds <= kDamLdsMax) {
    if ((rc = allow_lds(msda_dam_kernel<true>, lds))) return rc;
    hipLaunchKernelGGL((msda_dam_kernel<true>), dim3((unsigned)nrows), dim3(kDamThreads), lds, st, lc, a, out,
                       pr.lv, (int)pr.L, (int)pr.P, (int)pr.M, (int)pr.Lq, (int)S);
  } else {
    if (zero_f32(out, nrows * S, st) != hipSuccess) {
      set_error("msda_hip_dam_flat_grid: zero fill failed");
      return MSDA_ERR_LAUNCH;
    }
    hipLaunchKernelGGL((msda_dam_kernel<false>), dim3((unsigned)nrows), dim3(kDamThreads), 0, st, lc, a, out, pr.lv,
                       (int)pr.L, (int)pr.P, (int)pr.M, (int)pr.Lq, (int)S);
  }
  return launch_status("dam flat grid");
}

int msda_hip_prologue_forward_ex(const void* sampling_offsets, const void* attn_logits, int dtype,
                                 const void* reference_points, int ref_dim, const int64_t* spatial_shapes,
                                 int64_t num_levels, int64_t batch, int64_t num_query, int64_t num_heads,
                                 int64_t num_point, int64_t in_stride, void* sampling_loc, void* attn_weight,
                                 void* stream) {
  g_last_error[0] = 0;
  Problem pr;
  int rc = check_prologue(spatial_shapes, num_levels, batch, num_query, num_heads, num_point, ref_dim, &pr);
  if (rc) return rc;
  if (in_stride < num_heads * num_levels * num_point) {
    set_error("msda_hip_prologue_forward: in_stride %lld < num_heads * num_levels * num_point", (long long)in_stride);
    return MSDA_ERR_ARG;
  }
  if (batch * num_query > 0 && (sampling_offsets == nullptr || attn_logits == nullptr ||
                                reference_points == nullptr || sampling_loc == nullptr || attn_weight == nullptr)) {
    set_error("msda_hip_prologue_forward: null pointer");
    return MSDA_ERR_ARG;
  }
  return dispatch_prologue(true, dtype, pr, ref_dim, sampling_offsets, attn_logits, reference_points,
                           sampling_loc, attn_weight, nullptr, nullptr, nullptr, nullptr, nullptr, in_stride,
                           static_cast<hipStream_t>(stream));
}

int msda_hip_prologue_forward(const void* sampling_offsets, const void* attn_logits, int dtype,
                              const void* reference_points, int ref_dim, const int64_t* spatial_shapes,
                              int64_t num_levels, int64_t batch, int64_t num_query, int64_t num_heads,
                              int64_t num_point, void* sampling_loc, void* attn_weight, void* stream) {
  return msda_hip_prologue_forward_ex(sampling_offsets, attn_logits, dtype, reference_points, ref_dim, spatial_shapes,
                                      num_levels, batch, num_query, num_heads, num_point,
                                      num_heads * num_levels * num_point, sampling_loc, attn_weight, stream);
}

int msda_hip_prologue_backward_ex(const void* grad_loc, const void* grad_attn, const void* attn_weight,
                                  const void* sampling_offsets, int dtype, const void* reference_points,
                                  int ref_dim, const int64_t* spatial_shapes, int64_t num_levels,
                                  int64_t batch, int64_t num_query, int64_t num_heads, int64_t num_point,
                                  int64_t in_stride, void* grad_offsets, void* grad_logits, void* grad_ref,
                                  void* stream) {
  g_last_error[0] = 0;
  Problem pr;
  int rc = check_prologue(spatial_shapes, num_levels, batch, num_query, num_heads, num_point, ref_dim, &pr);
  if (rc) return rc;
  if (in_stride < num_heads * num_levels * num_point) {
    set_error("msda_hip_prologue_backward: in_stride %lld < num_heads * num_levels * num_point", (long long)in_stride);
    return MSDA_ERR_ARG;
  }
  const bool need_loc_side = grad_offsets != nullptr || grad_ref != nullptr;
  if (batch * num_query > 0 &&
      ((need_loc_side && grad_loc == nullptr) || (grad_logits != nullptr && (grad_attn == nullptr || attn_weight == nullptr)) ||
       (ref_dim == 2 && need_loc_side && (reference_points == nullptr || sampling_offsets == nullptr)))) {
    set_error("msda_hip_prologue_backward: null pointer");
    return MSDA_ERR_ARG;
  }
  return dispatch_prologue(false, dtype, pr, ref_dim, sampling_offsets, nullptr, reference_points, nullptr,
                           const_cast<void*>(attn_weight), grad_loc, grad_attn, grad_offsets, grad_logits,
                           grad_ref, in_stride, static_cast<hipStream_t>(stream));
}

int msda_hip_prologue_backward(const void* grad_loc, const void* grad_attn, const void* attn_weight,
                               const void* sampling_offsets, int dtype, const void* reference_points,
                               int ref_dim, const int64_t* spatial_shapes, int64_t num_levels,
                               int64_t batch, int64_t num_query, int64_t num_heads, int64_t num_point,
                               void* grad_offsets, void* grad_logits, void* grad_ref, void* stream) {
  return msda_hip_prologue_backward_ex(grad_loc, grad_attn, attn_weight, sampling_offsets, dtype, reference_points,
                                       ref_dim, spatial_shapes, num_levels, batch, num_query, num_heads, num_point,
                                       num_heads * num_levels * num_point, grad_offsets, grad_logits, grad_ref,
                                       stream);
}

size_t msda_hip_backward_workspace_bytes(int value_dtype, int64_t batch, int64_t spatial_size,
                                         int64_t num_heads, int64_t channels, int64_t num_query,
                                         int64_t num_levels, int64_t num_point) {
  (void)channels;
  if (batch <= 0 || spatial_size <= 0 || num_heads <= 0) return 0;
  if (value_dtype == MSDA_DTYPE_BF16 && num_query > 0 &&
      msda_dense_supported(1, channels, spatial_size, num_levels, num_point) != 0)
    return msda_dense_workspace_bytes(batch, spatial_size, num_heads, num_query);  // (dense_takes: its partial sums)
  PairPlan pp;
  // the row-block MFMA path's tile intervals (when it may run: the levels are not known here)
  const bool may_win = win_supported_call(value_dtype, channels, num_query, num_point, num_heads, num_levels);
  const size_t win = may_win ? msda_win_workspace_bytes(batch, num_heads, num_levels, num_query) : 0;
  if (may_win && (win_env() == 1 || win_overflow(num_query, num_point)))
    return win;  // the call takes the row-block path whatever its levels (run_backward)
  if (value_dtype != MSDA_DTYPE_F64 && pair_plan(value_dtype, batch, num_heads, num_query, num_point, channels,
                                                  num_levels, nullptr, spatial_size, true, &pp))
    return std::max(pp.ws_bytes, win);
  if (win > 0) return win;
  if (use_fused_gvalue(value_dtype, batch, spatial_size, num_heads, num_query, num_levels, num_point))
    return 0;
  return bwd_layout(value_dtype, batch, spatial_size, num_heads, num_query, num_levels, num_point).total;
}

static int forward_entry(const void* value, int value_dtype, const int64_t* spatial_shapes,
                         const int64_t* level_start, int64_t num_levels, const void* sampling_loc,
                         const void* attn_weight, void* output, void* tiles, int64_t batch, int64_t spatial_size,
                         int64_t num_heads, int64_t channels, int64_t num_query, int64_t num_point,
                         int padding_mode, void* stream, int layout = MSDA_COORD_API) {
  g_last_error[0] = 0;
  Problem pr;
  int rc = check_problem(spatial_shapes, level_start, num_levels, batch, spatial_size, num_heads,
                         channels, num_query, num_point, &pr);
  if (rc) return rc;
  if (padding_mode != MSDA_PAD_BORDER && padding_mode != MSDA_PAD_ZEROS) {
    set_error("msda: unknown padding_mode %d", padding_mode);
    return MSDA_ERR_ARG;
  }
  const long long n_out = pr.B * pr.Lq * pr.M * pr.D;
  if (n_out > 0 && (output == nullptr || sampling_loc == nullptr || attn_weight == nullptr ||
                    (pr.S > 0 && value == nullptr))) {
    set_error("msda_hip_forward: null pointer");
    return MSDA_ERR_ARG;
  }
  if (pr.S == 0 && n_out > 0) {
    set_error("msda_hip_forward: empty value with non-empty query");
    return MSDA_ERR_ARG;
  }
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (layout != MSDA_COORD_API && layout != MSDA_COORD_LEVEL_MAJOR) {
    set_error("msda_hip_forward: unknown coordinate layout %d", layout);
    return MSDA_ERR_ARG;
  }
  if (tiles != nullptr) {
    if (!forward_tiles_ok(pr, value_dtype)) {
      set_error("msda_hip_forward_tiles: the call's backward does not take the row-block path "
                "(msda_hip_forward_tiles_bytes is 0)");
      return MSDA_ERR_ARG;
    }
    return run_forward<bf16_t, float, 8>(pr, value, sampling_loc, attn_weight, output, padding_mode, st, tiles,
                                         layout);
  }
  if (layout != MSDA_COORD_API) {
    set_error("msda_hip_forward: the level-major coordinate layout goes with the tiles forward");
    return MSDA_ERR_ARG;
  }
  const int vec = pick_vec(value_dtype, pr.D);
  switch (value_dtype) {
    case MSDA_DTYPE_F32:
      return vec == 4 ? run_forward<float, float, 4>(pr, value, sampling_loc, attn_weight, output, padding_mode, st)
                      : run_forward<float, float, 1>(pr, value, sampling_loc, attn_weight, output, padding_mode, st);
    case MSDA_DTYPE_F64:
      return vec == 2 ? run_forward<double, double, 2>(pr, value, sampling_loc, attn_weight, output, padding_mode, st)
                      : run_forward<double, double, 1>(pr, value, sampling_loc, attn_weight, output, padding_mode, st);
    case MSDA_DTYPE_BF16:
      return vec == 8 ? run_forward<bf16_t, float, 8>(pr, value, sampling_loc, attn_weight, output, padding_mode, st)
                      : run_forward<bf16_t, float, 1>(pr, value, sampling_loc, attn_weight, output, padding_mode, st);
    case MSDA_DTYPE_F16:
      return vec == 8 ? run_forward<f16_t, float, 8>(pr, value, sampling_loc, attn_weight, output, padding_mode, st)
                      : run_forward<f16_t, float, 1>(pr, value, sampling_loc, attn_weight, output, padding_mode, st);
    default:
      set_error("msda_hip_forward: unknown value dtype %d", value_dtype);
      return MSDA_ERR_ARG;
  }
}

int msda_hip_forward(const void* value, int value_dtype, const int64_t* spatial_shapes,
                     const int64_t* level_start, int64_t num_levels, const void* sampling_loc,
                     const void* attn_weight, void* output, int64_t batch, int64_t spatial_size,
                     int64_t num_heads, int64_t channels, int64_t num_query, int64_t num_point,
                     int padding_mode, void* stream) {
  return forward_entry(value, value_dtype, spatial_shapes, level_start, num_levels, sampling_loc, attn_weight,
                       output, nullptr, batch, spatial_size, num_heads, channels, num_query, num_point,
                       padding_mode, stream);
}

size_t msda_hip_forward_tiles_bytes(int value_dtype, const int64_t* spatial_shapes, int64_t num_levels,
                                    int64_t batch, int64_t spatial_size, int64_t num_heads, int64_t channels,
                                    int64_t num_query, int64_t num_point) {
  if (spatial_shapes == nullptr || num_levels < 1 || num_levels > MSDA_MAX_LEVELS) return 0;
  Problem pr{};
  pr.B = batch; pr.S = spatial_size; pr.M = num_heads; pr.D = channels; pr.Lq = num_query;
  pr.L = num_levels; pr.P = num_point;
  for (int l = 0; l < num_levels; ++l) {
    if (spatial_shapes[l] < 1 || spatial_shapes[l] > (1 << 24)) return 0;
    pr.lv.T[l] = (int)spatial_shapes[l];
  }
  if (batch <= 0 || num_query <= 0 || !forward_tiles_ok(pr, value_dtype)) return 0;
  return msda_win_workspace_bytes(batch, num_heads, num_levels, num_query);
}

int msda_hip_forward_tiles(const void* value, int value_dtype, const int64_t* spatial_shapes,
                           const int64_t* level_start, int64_t num_levels, const void* sampling_loc,
                           const void* attn_weight, void* output, void* tiles, int64_t batch, int64_t spatial_size,
                           int64_t num_heads, int64_t channels, int64_t num_query, int64_t num_point,
                           int padding_mode, void* stream) {
  if (tiles == nullptr) {
    g_last_error[0] = 0;
    set_error("msda_hip_forward_tiles: null tiles");
    return MSDA_ERR_ARG;
  }
  return forward_entry(value, value_dtype, spatial_shapes, level_start, num_levels, sampling_loc, attn_weight,
                       output, tiles, batch, spatial_size, num_heads, channels, num_query, num_point,
                       padding_mode, stream);
}

static int backward_entry(const void* value, int value_dtype, const int64_t* spatial_shapes,
                          const int64_t* level_start, int64_t num_levels, const void* sampling_loc,
                          const void* attn_weight, const void* grad_output, void* grad_value,
                          void* grad_loc, void* grad_attn, void* workspace, const void* tiles, int64_t batch,
                          int64_t spatial_size, int64_t num_heads, int64_t channels,
                          int64_t num_query, int64_t num_point, int padding_mode, void* stream,
                          int layout = MSDA_COORD_API, int64_t gval_row_stride = 0) {
  g_last_error[0] = 0;
  Problem pr;
  int rc = check_problem(spatial_shapes, level_start, num_levels, batch, spatial_size, num_heads,
                         channels, num_query, num_point, &pr);
  if (rc) return rc;
  if (gval_row_stride != 0 && (gval_row_stride < pr.M * pr.D || gval_row_stride % 8 != 0 ||
                               pr.B * pr.S * gval_row_stride >= (1LL << 31))) {
    set_error("msda_hip_backward_ex: grad_value row stride must be >= num_heads * channels, a multiple of 8, "
              "and the strided grad_value under 2^31 elements");
    return MSDA_ERR_ARG;
  }
  pr.gv_rs = gval_row_stride;
  if (padding_mode != MSDA_PAD_BORDER && padding_mode != MSDA_PAD_ZEROS) {
    set_error("msda: unknown padding_mode %d", padding_mode);
    return MSDA_ERR_ARG;
  }
  const long long n_items = pr.B * pr.Lq * pr.M;
  if (n_items > 0 && (sampling_loc == nullptr || attn_weight == nullptr ||
                      grad_output == nullptr || (pr.S > 0 && value == nullptr))) {
    set_error("msda_hip_backward: null input pointer");
    return MSDA_ERR_ARG;
  }
  if (pr.S == 0 && n_items > 0) {
    set_error("msda_hip_backward: empty value with non-empty query");
    return MSDA_ERR_ARG;
  }
  // the backward's row table covers [0, S) level by level: levels must tile it in order
  // (as the reference's level_start_index = cumsum of the shapes does)
  for (int l = 0, run = 0; l < pr.L; ++l) {
    if (pr.lv.start[l] != run) {
      set_error("msda_hip_backward: level_start must be the running sum of spatial_shapes");
      return MSDA_ERR_ARG;
    }
    run += pr.lv.T[l];
    if (l == pr.L - 1 && run != pr.S) {
      set_error("msda_hip_backward: spatial_shapes must sum to spatial_size (%lld != %lld)",
                (long long)run, pr.S);
      return MSDA_ERR_ARG;
    }
  }
  if (2 * pr.Lq * pr.P >= (1LL << 30) || pr.B * pr.M * pr.L * 2 * pr.Lq * pr.P >= (1LL << 31)) {
    set_error("msda_hip_backward: too many taps for 32-bit entry indices");
    return MSDA_ERR_ARG;
  }
  if (value_dtype < MSDA_DTYPE_F32 || value_dtype > MSDA_DTYPE_F16) {
    set_error("msda_hip_backward: unknown value dtype %d", value_dtype);
    return MSDA_ERR_ARG;
  }
  const size_t need = msda_hip_backward_workspace_bytes(value_dtype, batch, spatial_size, num_heads,
                                                        channels, num_query, num_levels, num_point);
  // (the forward's tile intervals are all the row-block path needs)
  const bool tiles_do = tiles != nullptr && forward_tiles_ok(pr, value_dtype);
  if (need > 0 && workspace == nullptr &&
      !(tiles_do && need == msda_win_workspace_bytes(batch, num_heads, num_levels, num_query))) {
    set_error("msda_hip_backward: workspace of %zu bytes required", need);
    return MSDA_ERR_ARG;
  }
  if (tiles != nullptr && !tiles_do) {
    set_error("msda_hip_backward_tiles: the call does not take the row-block path (no tiles forward)");
    return MSDA_ERR_ARG;
  }
  if (layout != MSDA_COORD_API && (layout != MSDA_COORD_LEVEL_MAJOR || !tiles_do)) {
    set_error("msda_hip_backward: coordinate layout %d needs the forward's tile intervals of a row-block call", layout);
    return MSDA_ERR_ARG;
  }
  if (grad_value == nullptr && grad_loc == nullptr && grad_attn == nullptr) return MSDA_OK;
  hipStream_t st = static_cast<hipStream_t>(stream);
  switch (value_dtype) {
    case MSDA_DTYPE_F32:
      return run_backward<float, float>(pr, value, sampling_loc, attn_weight, grad_output, grad_value,
                                        grad_loc, grad_attn, workspace, value_dtype, padding_mode, st);
    case MSDA_DTYPE_F64:
      return run_backward<double, double>(pr, value, sampling_loc, attn_weight, grad_output, grad_value,
                                          grad_loc, grad_attn, workspace, value_dtype, padding_mode, st);
    case MSDA_DTYPE_BF16:
      return run_backward<bf16_t, float>(pr, value, sampling_loc, attn_weight, grad_output, grad_value,
                                         grad_loc, grad_attn, workspace, value_dtype, padding_mode, st, tiles, layout);
    default:
      return run_backward<f16_t, float>(pr, value, sampling_loc, attn_weight, grad_output, grad_value,
                                        grad_loc, grad_attn, workspace, value_dtype, padding_mode, st);
  }
}

int msda_hip_backward(const void* value, int value_dtype, const int64_t* spatial_shapes,
                      const int64_t* level_start, int64_t num_levels, const void* sampling_loc,
                      const void* attn_weight, const void* grad_output, void* grad_value,
                      void* grad_loc, void* grad_attn, void* workspace, int64_t batch,
                      int64_t spatial_size, int64_t num_heads, int64_t channels,
                      int64_t num_query, int64_t num_point, int padding_mode, void* stream) {
  return backward_entry(value, value_dtype, spatial_shapes, level_start, num_levels, sampling_loc, attn_weight,
                        grad_output, grad_value, grad_loc, grad_attn, workspace, nullptr, batch, spatial_size,
                        num_heads, channels, num_query, num_point, padding_mode, stream);
}

int msda_hip_backward_ex(const void* value, int value_dtype, const int64_t* spatial_shapes,
                         const int64_t* level_start, int64_t num_levels, const void* sampling_loc,
                         const void* attn_weight, const void* grad_output, void* grad_value,
                         void* grad_loc, void* grad_attn, void* workspace, int64_t batch,
                         int64_t spatial_size, int64_t num_heads, int64_t channels,
                         int64_t num_query, int64_t num_point, int padding_mode, int64_t grad_value_row_stride,
                         void* stream) {
  return backward_entry(value, value_dtype, spatial_shapes, level_start, num_levels, sampling_loc, attn_weight,
                        grad_output, grad_value, grad_loc, grad_attn, workspace, nullptr, batch, spatial_size,
                        num_heads, channels, num_query, num_point, padding_mode, stream, MSDA_COORD_API,
                        grad_value_row_stride);
}

int msda_hip_backward_tiles(const void* value, int value_dtype, const int64_t* spatial_shapes,
                            const int64_t* level_start, int64_t num_levels, const void* sampling_loc,
                            const void* attn_weight, const void* grad_output, void* grad_value,
                            void* grad_loc, void* grad_attn, void* workspace, const void* tiles, int64_t batch,
                            int64_t spatial_size, int64_t num_heads, int64_t channels,
                            int64_t num_query, int64_t num_point, int padding_mode, void* stream) {
  if (tiles == nullptr) {
    g_last_error[0] = 0;
    set_error("msda_hip_backward_tiles: null tiles");
    return MSDA_ERR_ARG;
  }
  return backward_entry(value, value_dtype, spatial_shapes, level_start, num_levels, sampling_loc, attn_weight,
                        grad_output, grad_value, grad_loc, grad_attn, workspace, tiles, batch, spatial_size,
                        num_heads, channels, num_query, num_point, padding_mode, stream);
}

int msda_hip_level_major_ok(int value_dtype, const int64_t* spatial_shapes, int64_t num_levels, int64_t batch,
                            int64_t spatial_size, int64_t num_heads, int64_t channels, int64_t num_query,
                            int64_t num_point) {
  return prologue_lm_ok(num_heads, num_levels, num_point) &&
         msda_hip_forward_tiles_bytes(value_dtype, spatial_shapes, num_levels, batch, spatial_size, num_heads,
                                      channels, num_query, num_point) > 0;
}

int msda_hip_forward_tiles_layout(const void* value, int value_dtype, const int64_t* spatial_shapes,
                                  const int64_t* level_start, int64_t num_levels, const void* sampling_loc,
                                  const void* attn_weight, void* output, void* tiles, int64_t batch,
                                  int64_t spatial_size, int64_t num_heads, int64_t channels, int64_t num_query,
                                  int64_t num_point, int padding_mode, int coord_layout, void* stream) {
  if (tiles == nullptr) {
    g_last_error[0] = 0;
    set_error("msda_hip_forward_tiles_layout: null tiles");
    return MSDA_ERR_ARG;
  }
  return forward_entry(value, value_dtype, spatial_shapes, level_start, num_levels, sampling_loc, attn_weight,
                       output, tiles, batch, spatial_size, num_heads, channels, num_query, num_point,
                       padding_mode, stream, coord_layout);
}

int msda_hip_backward_tiles_layout(const void* value, int value_dtype, const int64_t* spatial_shapes,
                                   const int64_t* level_start, int64_t num_levels, const void* sampling_loc,
                                   const void* attn_weight, const void* grad_output, void* grad_value,
                                   void* grad_loc, void* grad_attn, void* workspace, const void* tiles,
                                   int64_t batch, int64_t spatial_size, int64_t num_heads, int64_t channels,
                                   int64_t num_query, int64_t num_point, int padding_mode, int coord_layout,
                                   void* stream) {
  if (tiles == nullptr) {
    g_last_error[0] = 0;
    set_error("msda_hip_backward_tiles_layout: null tiles");
    return MSDA_ERR_ARG;
  }
  return backward_entry(value, value_dtype, spatial_shapes, level_start, num_levels, sampling_loc, attn_weight,
                        grad_output, grad_value, grad_loc, grad_attn, workspace, tiles, batch, spatial_size,
                        num_heads, channels, num_query, num_point, padding_mode, stream, coord_layout);
}

int msda_hip_prologue_forward_layout(const void* sampling_offsets, const void* attn_logits, int dtype,
                                     const void* reference_points, int ref_dim, const int64_t* spatial_shapes,
                                     int64_t num_levels, int64_t batch, int64_t num_query, int64_t num_heads,
                                     int64_t num_point, int64_t in_stride, int coord_layout, void* sampling_loc,
                                     void* attn_weight, void* stream) {
  g_last_error[0] = 0;
  Problem pr;
  int rc = check_prologue(spatial_shapes, num_levels, batch, num_query, num_heads, num_point, ref_dim, &pr);
  if (rc) return rc;
  if (in_stride < num_heads * num_levels * num_point) {
    set_error("msda_hip_prologue_forward: in_stride %lld < num_heads * num_levels * num_point", (long long)in_stride);
    return MSDA_ERR_ARG;
  }
  if (batch * num_query > 0 && (sampling_offsets == nullptr || attn_logits == nullptr ||
                                reference_points == nullptr || sampling_loc == nullptr || attn_weight == nullptr)) {
    set_error("msda_hip_prologue_forward: null pointer");
    return MSDA_ERR_ARG;
  }
  return dispatch_prologue(true, dtype, pr, ref_dim, sampling_offsets, attn_logits, reference_points,
                           sampling_loc, attn_weight, nullptr, nullptr, nullptr, nullptr, nullptr, in_stride,
                           static_cast<hipStream_t>(stream), coord_layout);
}

int msda_hip_prologue_backward_layout(const void* grad_loc, const void* grad_attn, const void* attn_weight,
                                      const void* sampling_offsets, int dtype, const void* reference_points,
                                      int ref_dim, const int64_t* spatial_shapes, int64_t num_levels,
                                      int64_t batch, int64_t num_query, int64_t num_heads, int64_t num_point,
                                      int64_t in_stride, int coord_layout, void* grad_offsets, void* grad_logits,
                                      void* grad_ref, void* stream) {
  g_last_error[0] = 0;
  Problem pr;
  int rc = check_prologue(spatial_shapes, num_levels, batch, num_query, num_heads, num_point, ref_dim, &pr);
  if (rc) return rc;
  if (in_stride < num_heads * num_levels * num_point) {
    set_error("msda_hip_prologue_backward: in_stride %lld < num_heads * num_levels * num_point", (long long)in_stride);
    return MSDA_ERR_ARG;
  }
  const bool need_loc_side = grad_offsets != nullptr || grad_ref != nullptr;
  if (batch * num_query > 0 &&
      ((need_loc_side && grad_loc == nullptr) || (grad_logits != nullptr && (grad_attn == nullptr || attn_weight == nullptr)) ||
       (ref_dim == 2 && need_loc_side && (reference_points == nullptr || sampling_offsets == nullptr)))) {
    set_error("msda_hip_prologue_backward: null pointer");
    return MSDA_ERR_ARG;
  }
  return dispatch_prologue(false, dtype, pr, ref_dim, sampling_offsets, nullptr, reference_points, nullptr,
                           const_cast<void*>(attn_weight), grad_loc, grad_attn, grad_offsets, grad_logits,
                           grad_ref, in_stride, static_cast<hipStream_t>(stream), coord_layout);
}

}  // extern "C"
