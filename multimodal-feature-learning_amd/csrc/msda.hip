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
#include <hip/hip_bf16.h>
#include <hip/hip_fp16.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "msda_hip.h"

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
  const long long tid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
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

// ---------------------------------------------------------------------------------
// backward
// ---------------------------------------------------------------------------------
template <typename scalar_t, typename coord_t, int VEC, bool ZEROS>
__global__ __launch_bounds__(256) void msda_bwd_kernel(
    const scalar_t* __restrict__ value, const coord_t* __restrict__ loc,
    const coord_t* __restrict__ aw, const scalar_t* __restrict__ gout,
    coord_t* __restrict__ gloc, coord_t* __restrict__ gaw,
    const Levels lv, const int L, const int P, const int S, const int M, const int D,
    const int Lq, const long long n_items, const int gshift) {
  using acc_t = typename AccOf<scalar_t>::type;
  const long long tid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long item_raw = tid >> gshift;
  // every lane stays alive for the butterfly reductions below
  const bool active = item_raw < n_items;
  const long long item = active ? item_raw : 0;
  const int G = 1 << gshift;
  const int lg = (int)(tid & (G - 1));
  const int m = (int)(item % M);
  const long long b = item / M / Lq;
  const long long rowstride = (long long)M * D;
  const coord_t* __restrict__ locp = loc + item * (L * P);
  const coord_t* __restrict__ awp = aw + item * (L * P);
  const long long vrow0 = (b * S * M + m) * (long long)D;
  const scalar_t* __restrict__ vb = value + vrow0;
  const scalar_t* __restrict__ gp = gout + item * D;
  const int nchunk = D / VEC;
  for (int l = 0; l < L; ++l) {
    const int T = lv.T[l];
    const long long lbase = (long long)lv.start[l] * rowstride;
    for (int p = 0; p < P; ++p) {
      const coord_t a = awp[l * P + p];
      const Taps<coord_t> t = make_taps<coord_t, ZEROS>(locp[l * P + p], T);
      const acc_t w0 = (acc_t)t.w0, w1 = (acc_t)t.w1, aa = (acc_t)a;
      acc_t pa = (acc_t)0;  // d out / d aw
      acc_t pl = (acc_t)0;  // sum_c g * (v1 - v0)
      if (active) {
        for (int ck = lg; ck < nchunk; ck += G) {
          acc_t g[VEC], v0[VEC], v1[VEC];
          load_vec<scalar_t, VEC>(gp + ck * VEC, g);
          load_vec<scalar_t, VEC>(vb + lbase + t.i0 * rowstride + ck * VEC, v0);
          load_vec<scalar_t, VEC>(vb + lbase + t.i1 * rowstride + ck * VEC, v1);
#pragma unroll
          for (int e = 0; e < VEC; ++e) {
            const acc_t x0 = t.ok0 ? v0[e] : (acc_t)0;
            const acc_t x1 = t.ok1 ? v1[e] : (acc_t)0;
            pa += g[e] * (x0 * w0 + x1 * w1);
            pl += g[e] * (x1 - x0);
          }
        }
      }
      // butterfly over the G lanes of this item (G divides 64, groups are aligned)
      for (int off = G >> 1; off > 0; off >>= 1) {
        pa += __shfl_xor(pa, off);
        pl += __shfl_xor(pl, off);
      }
      if (active && lg == 0) {
        const long long o = item * (L * P) + l * P + p;
        if (gaw != nullptr) gaw[o] = (coord_t)pa;
        if (gloc != nullptr) gloc[o] = (coord_t)(pl * aa) * t.gmul;
      }
    }
  }
}

// ---------------------------------------------------------------------------------
// backward, grad_value: scatter through LDS with plain (non-atomic) read-modify-write
// ---------------------------------------------------------------------------------
// One workgroup owns rows [r0, r1) of one (b, head m, level l) slab of grad_value and keeps
// them in LDS as fp32 (fp64 for fp64 values).  It scans every sample (q, p) of level l for
// (b, m), recomputes the two taps and adds aw*w*grad_out[b,q,m,:] to each tap row it owns.
// Every grad_value row has exactly one owner workgroup, so the slab is written once with
// plain stores: no global atomics, no memset, no fp32 staging buffer for bf16/fp16.
//
// No LDS atomics either: ds_add_f32 measured ~81 ns per wave-op per CU on gfx950 against
// ~7 ns for a ds_read + ds_write pair (tools/lds_probe.hip).  Races are avoided by
// ownership instead:
//   * wave w of the workgroup owns the rows with (row - r0) % 4 == w (both taps of a sample
//     are adjacent rows, so they always belong to different waves);
//   * inside a wave, NSLOT contributions are applied per instruction, one per "slot" of
//     64/NSLOT lanes (CPL channels per lane = one 16-byte ds_read/ds_write); slot =
//     ((row - r0) / 4) % NSLOT, so the rows of one instruction are always distinct, and
//     later rounds of the same slot are ordered by the wave's in-order LDS pipe.
// NSLOT (1, 2 or 4) needs D % CPL == 0 and D <= 64/NSLOT*CPL; NSLOT = 0 is the generic
// path (any channel count): one contribution per round, lane = channel, 4/8-byte RMW.
struct RangePlan {
  int rows;                      // rows per workgroup
  int cum[MSDA_MAX_LEVELS + 1];  // prefix sum over levels of ceil(T_l / rows)
};

template <typename acc_t, int N>
struct alignas(16) AccN {
  acc_t v[N];
};

constexpr int kGvThreads = 256;
constexpr int kGvSampPerThread = 4;                             // samples per thread per step
constexpr int kGvStep = kGvThreads * kGvSampPerThread;          // samples scanned per step
constexpr int kGvQueue = 2 * kGvStep;                           // <= 2 taps per sample
constexpr int kGvSlotCap = 64;                                  // entries per (wave, slot) table

template <typename scalar_t, typename coord_t, bool ZEROS, int NSLOT>
__global__ __launch_bounds__(kGvThreads) void msda_gvalue_kernel(
    const coord_t* __restrict__ loc, const coord_t* __restrict__ aw,
    const scalar_t* __restrict__ gout, scalar_t* __restrict__ gval, const Levels lv,
    const RangePlan rp, const int L, const int P, const int S, const int M, const int D,
    const int Lq) {
  using acc_t = typename AccOf<scalar_t>::type;
  constexpr int CPL = NSLOT > 0 ? 16 / (int)sizeof(acc_t) : 1;  // channels per lane
  constexpr int NS = NSLOT > 0 ? NSLOT : 1;
  constexpr int LPR = 64 / NS;                                   // lanes per slot
  constexpr int ROUNDS = 16;  // slot-rounds whose grad_out loads are in flight together

  // LDS: [slab rows*D acc_t][queue w acc_t][queue q int][queue row int]
  //      [per-wave slot tables: w acc_t x 4*NS*cap][q|row int x 4*NS*cap][queue counter]
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  const int rows_cap = rp.rows;
  acc_t* slab = reinterpret_cast<acc_t*>(smem_raw);
  acc_t* q_w = slab + (size_t)rows_cap * D;
  acc_t* t_w = q_w + kGvQueue;
  int* q_q = reinterpret_cast<int*>(t_w + 4 * NS * kGvSlotCap);
  int* q_row = q_q + kGvQueue;
  int* t_qr = q_row + kGvQueue;
  int* q_cnt = t_qr + 4 * NS * kGvSlotCap;

  const int nr = rp.cum[L];
  const int r = (int)(blockIdx.x % (unsigned)nr);
  const long long bm = blockIdx.x / (unsigned)nr;
  const int m = (int)(bm % M);
  const long long b = bm / M;
  int l = 0;
  while (r >= rp.cum[l + 1]) ++l;
  const int T = lv.T[l];
  const int r0 = (r - rp.cum[l]) * rp.rows;
  const int r1 = min(r0 + rp.rows, T);
  const int nrows = r1 - r0;

  for (int i = threadIdx.x * CPL; i < nrows * D; i += kGvThreads * CPL) {
#pragma unroll
    for (int e = 0; e < CPL; ++e) slab[i + e] = (acc_t)0;
  }
  if (threadIdx.x == 0) *q_cnt = 0;
  __syncthreads();

  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int LP = L * P;
  const long long qstride_c = (long long)M * LP;  // loc/aw stride between queries
  const long long qstride_g = (long long)M * D;   // grad_out stride between queries
  const coord_t* __restrict__ locb = loc + (b * Lq * M + m) * LP + l * P;
  const coord_t* __restrict__ awb = aw + (b * Lq * M + m) * LP + l * P;
  const scalar_t* __restrict__ gb = gout + (b * Lq * M + m) * (long long)D;
  const int nsamp = Lq * P;
  const int slot = lane / LPR;
  const int cl = lane - slot * LPR;

  // per-wave slot tables: tw / tqr [NS][kGvSlotCap]; counts are wave-uniform
  int* tqr = t_qr + wave * (NS * kGvSlotCap);
  acc_t* tw = t_w + wave * (NS * kGvSlotCap);
  int tcnt[NS];
#pragma unroll
  for (int sl = 0; sl < NS; ++sl) tcnt[sl] = 0;
  auto flush = [&]() {
    int nr = 0, my_cnt = 0;
#pragma unroll
    for (int sl = 0; sl < NS; ++sl) {
      nr = tcnt[sl] > nr ? tcnt[sl] : nr;
      if (slot == sl) my_cnt = tcnt[sl];
    }
    for (int k0 = 0; k0 < nr; k0 += ROUNDS) {
      int srow[ROUNDS], sq[ROUNDS];
      acc_t sw[ROUNDS];
#pragma unroll
      for (int k = 0; k < ROUNDS; ++k) {
        const bool v = k0 + k < my_cnt;
        const int idx = slot * kGvSlotCap + (v ? k0 + k : 0);
        const int qr = tqr[idx];
        const acc_t w = tw[idx];
        sq[k] = v ? (qr >> 12) : 0;
        srow[k] = v ? (qr & 4095) : -1;
        sw[k] = v ? w : (acc_t)0;
      }
      if constexpr (NSLOT > 0) {
        const bool lane_on = cl * CPL < D;  // narrow heads leave the slot's upper lanes idle
        acc_t g[ROUNDS][CPL];
#pragma unroll
        for (int k = 0; k < ROUNDS; ++k) {
          if (lane_on) load_vec<scalar_t, CPL>(gb + sq[k] * qstride_g + cl * CPL, g[k]);
        }
#pragma unroll
        for (int k = 0; k < ROUNDS; ++k) {
          if (srow[k] >= 0 && lane_on) {
            AccN<acc_t, CPL>* dst = reinterpret_cast<AccN<acc_t, CPL>*>(slab + srow[k] * D + cl * CPL);
            AccN<acc_t, CPL> v = *dst;
#pragma unroll
            for (int c = 0; c < CPL; ++c) v.v[c] += sw[k] * g[k][c];
            *dst = v;
          }
        }
      } else {
        for (int c = lane; c < D; c += 64) {
          acc_t g[ROUNDS];
#pragma unroll
          for (int k = 0; k < ROUNDS; ++k) g[k] = to_acc(gb[sq[k] * qstride_g + c]);
#pragma unroll
          for (int k = 0; k < ROUNDS; ++k)
            if (srow[k] >= 0) slab[srow[k] * D + c] += sw[k] * g[k];
        }
      }
    }
#pragma unroll
    for (int sl = 0; sl < NS; ++sl) tcnt[sl] = 0;
  };

  for (int base = 0; base < nsamp; base += kGvStep) {
    // ---- phase A: the whole workgroup scans kGvStep samples (loads issued together) ----
    coord_t lc[kGvSampPerThread], av[kGvSampPerThread];
#pragma unroll
    for (int u = 0; u < kGvSampPerThread; ++u) {
      const int sidx = base + u * kGvThreads + threadIdx.x;
      const int qq = sidx / P, pp = sidx - (sidx / P) * P;
      const bool live = sidx < nsamp;
      lc[u] = live ? locb[qq * qstride_c + pp] : (coord_t)-1e30;
      av[u] = live ? awb[qq * qstride_c + pp] : (coord_t)0;
    }
#pragma unroll
    for (int u = 0; u < kGvSampPerThread; ++u) {
      const int sidx = base + u * kGvThreads + threadIdx.x;
      const int qq = sidx / P;
      bool c[2] = {false, false};
      int rw[2] = {0, 0};
      acc_t wv[2] = {(acc_t)0, (acc_t)0};
      if (sidx < nsamp) {
        const Taps<coord_t> t = make_taps<coord_t, ZEROS>(lc[u], T);
        c[0] = t.ok0 && t.w0 != (coord_t)0 && t.i0 >= r0 && t.i0 < r1;
        c[1] = t.ok1 && t.w1 != (coord_t)0 && t.i1 >= r0 && t.i1 < r1;
        rw[0] = t.i0 - r0;
        rw[1] = t.i1 - r0;
        wv[0] = (acc_t)av[u] * (acc_t)t.w0;
        wv[1] = (acc_t)av[u] * (acc_t)t.w1;
      }
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        // wave-level compaction, one LDS counter bump per wave
        const unsigned long long mk = __ballot(c[k]);
        if (mk == 0ull) continue;
        const int before = __builtin_amdgcn_mbcnt_hi((unsigned)(mk >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)mk, 0u));
        int start = 0;
        if (lane == 0) start = atomicAdd(q_cnt, __popcll(mk));
        start = __shfl(start, 0);
        if (c[k]) {
          q_q[start + before] = qq;
          q_row[start + before] = rw[k];
          q_w[start + before] = wv[k];
        }
      }
    }
    __syncthreads();
    const int n = *q_cnt;
    // ---- phase B: wave w moves the entries whose row it owns ((row & 3) == w) into its
    // per-slot tables (slot = (row/4) % NS, kGvSlotCap entries each); a table that would
    // overflow is first drained by flush().  Tables persist across steps (the slab rows are
    // private to the wave), so drains run in long batches with ROUNDS loads in flight.
    for (int e0 = 0; e0 < n; e0 += 64) {
      const int e = e0 + lane;
      int er = 0, eq = 0;
      acc_t ew = (acc_t)0;
      bool mine = false;
      if (e < n) {
        er = q_row[e];
        mine = (er & 3) == wave;
        eq = q_q[e];
        ew = q_w[e];
      }
      const int es = (er >> 2) % NS;
      unsigned long long mk[NS];
      bool full = false;
#pragma unroll
      for (int sl = 0; sl < NS; ++sl) {
        mk[sl] = __ballot(mine && es == sl);
        full |= tcnt[sl] + __popcll(mk[sl]) > kGvSlotCap;
      }
      if (full) flush();
      if (mine) {
        int pos = 0;
#pragma unroll
        for (int sl = 0; sl < NS; ++sl)
          if (es == sl)
            pos = sl * kGvSlotCap + tcnt[sl] +
                  __builtin_amdgcn_mbcnt_hi((unsigned)(mk[sl] >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)mk[sl], 0u));
        tqr[pos] = (eq << 12) | er;  // row < 4096, q < 2^19 (checked on the host)
        tw[pos] = ew;
      }
#pragma unroll
      for (int sl = 0; sl < NS; ++sl) tcnt[sl] += __popcll(mk[sl]);
    }
    __syncthreads();
    if (threadIdx.x == 0) *q_cnt = 0;
    __syncthreads();
  }
  flush();
  __syncthreads();

  scalar_t* __restrict__ dst = gval + ((b * S + lv.start[l] + r0) * M + m) * (long long)D;
  const long long rowstride = (long long)M * D;
  for (int i = threadIdx.x * CPL; i < nrows * D; i += kGvThreads * CPL) {
    const int row = i / D, c = i - row * D;
    if constexpr (CPL > 1) {
      acc_t v[CPL];
#pragma unroll
      for (int e = 0; e < CPL; ++e) v[e] = slab[i + e];
      store_vec<scalar_t, CPL>(dst + row * rowstride + c, v);
    } else {
      from_acc(slab[i], dst + row * rowstride + c);
    }
  }
}

// ---------------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------------
constexpr long long kSlabBytes = 32 * 1024;  // grad_value LDS slab per workgroup (+ queue: ~58 KB, 2 per CU)
constexpr long long kLdsLimit = 64 * 1024;   // dynamic LDS per workgroup we allow ourselves

struct Problem {
  long long B, S, M, D, Lq, L, P;
  Levels lv;
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

template <typename scalar_t, typename coord_t, int VEC>
int run_forward(const Problem& pr, const void* value, const void* loc, const void* aw, void* out,
                int pad, hipStream_t st) {
  const long long n_items = pr.B * pr.Lq * pr.M;
  if (n_items == 0) return MSDA_OK;
  const int gshift = group_shift_for(pr.D / VEC);
  const long long threads = n_items << gshift;
  const unsigned blocks = (unsigned)((threads + 255) / 256);
  auto* v = static_cast<const scalar_t*>(value);
  auto* lc = static_cast<const coord_t*>(loc);
  auto* a = static_cast<const coord_t*>(aw);
  auto* o = static_cast<scalar_t*>(out);
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

template <typename scalar_t, typename coord_t, int VEC>
int run_backward(const Problem& pr, const void* value, const void* loc, const void* aw,
                 const void* gout, void* gloc, void* gaw, int pad, hipStream_t st) {
  const long long n_items = pr.B * pr.Lq * pr.M;
  if (n_items == 0) return MSDA_OK;
  const int gshift = group_shift_for(pr.D / VEC);
  const long long threads = n_items << gshift;
  const unsigned blocks = (unsigned)((threads + 255) / 256);
  auto* v = static_cast<const scalar_t*>(value);
  auto* lc = static_cast<const coord_t*>(loc);
  auto* a = static_cast<const coord_t*>(aw);
  auto* g = static_cast<const scalar_t*>(gout);
  auto* gl = static_cast<coord_t*>(gloc);
  auto* ga = static_cast<coord_t*>(gaw);
  if (pad == MSDA_PAD_ZEROS)
    hipLaunchKernelGGL((msda_bwd_kernel<scalar_t, coord_t, VEC, true>), dim3(blocks),
                       dim3(256), 0, st, v, lc, a, g, gl, ga, pr.lv, (int)pr.L, (int)pr.P,
                       (int)pr.S, (int)pr.M, (int)pr.D, (int)pr.Lq, n_items, gshift);
  else
    hipLaunchKernelGGL((msda_bwd_kernel<scalar_t, coord_t, VEC, false>), dim3(blocks),
                       dim3(256), 0, st, v, lc, a, g, gl, ga, pr.lv, (int)pr.L, (int)pr.P,
                       (int)pr.S, (int)pr.M, (int)pr.D, (int)pr.Lq, n_items, gshift);
  return launch_status("backward");
}

template <typename scalar_t, typename coord_t>
int run_grad_value(const Problem& pr, const void* loc, const void* aw, const void* gout, void* gval,
                   int pad, hipStream_t st) {
  using acc_t = typename AccOf<scalar_t>::type;
  if (pr.B * pr.M * pr.S * pr.D == 0) return MSDA_OK;
  // slots per instruction for 16-byte lanes: NSLOT = 64 / (D / CPL) when that is a power of 2
  constexpr int CPL = 16 / (int)sizeof(acc_t);
  // (at most 4 slots: a slot's table must hold a whole 64-entry group; lanes whose chunk
  //  is past D idle for narrow heads)
  int ns = 0;
  if (pr.D % CPL == 0) {
    if (pr.D <= 16 * CPL) ns = 4;
    else if (pr.D <= 32 * CPL) ns = 2;
    else if (pr.D <= 64 * CPL) ns = 1;
  }
  const int ns_eff = ns > 0 ? ns : 1;
  // LDS = slab (rows x D acc) + queue + slot tables; stay within 64 KB per workgroup
  const long long row_bytes = pr.D * (long long)sizeof(acc_t);
  const long long table = 4LL * ns_eff * kGvSlotCap;
  const long long overhead = (long long)(kGvQueue + table) * (sizeof(int) + sizeof(acc_t)) +
                             (long long)kGvQueue * sizeof(int) + 16;
  const long long slab_budget = min(kSlabBytes, kLdsLimit - overhead);
  if (row_bytes > slab_budget) {
    set_error("msda_hip_backward: channels=%lld too large for the LDS grad_value slab", pr.D);
    return MSDA_ERR_ARG;
  }
  int maxT = 1;
  for (int l = 0; l < pr.L; ++l) maxT = max(maxT, pr.lv.T[l]);
  RangePlan rp;
  rp.rows = (int)min((long long)maxT, slab_budget / row_bytes);
  rp.cum[0] = 0;
  for (int l = 0; l < pr.L; ++l) rp.cum[l + 1] = rp.cum[l] + (pr.lv.T[l] + rp.rows - 1) / rp.rows;
  const long long blocks = pr.B * pr.M * rp.cum[pr.L];
  const size_t lds = (size_t)(rp.rows * row_bytes + overhead);
  if (rp.rows > 4096 || pr.Lq >= (1 << 19)) {  // packing of (q, row) in the slot tables
    set_error("msda_hip_backward: num_query=%lld too large for the grad_value kernel", pr.Lq);
    return MSDA_ERR_ARG;
  }
  auto* lc = static_cast<const coord_t*>(loc);
  auto* a = static_cast<const coord_t*>(aw);
  auto* g = static_cast<const scalar_t*>(gout);
  auto* gv = static_cast<scalar_t*>(gval);
#define MSDA_GV(Z, NS)                                                                          \
  hipLaunchKernelGGL((msda_gvalue_kernel<scalar_t, coord_t, Z, NS>), dim3((unsigned)blocks),    \
                     dim3(kGvThreads), lds, st, lc, a, g, gv, pr.lv, rp, (int)pr.L, (int)pr.P,         \
                     (int)pr.S, (int)pr.M, (int)pr.D, (int)pr.Lq)
  const bool z = pad == MSDA_PAD_ZEROS;
  switch (ns) {
    case 1: if (z) MSDA_GV(true, 1); else MSDA_GV(false, 1); break;
    case 2: if (z) MSDA_GV(true, 2); else MSDA_GV(false, 2); break;
    case 4: if (z) MSDA_GV(true, 4); else MSDA_GV(false, 4); break;
    default: if (z) MSDA_GV(true, 0); else MSDA_GV(false, 0); break;
  }
#undef MSDA_GV
  return launch_status("grad_value");
}

}  // namespace

extern "C" {

int msda_hip_abi_version(void) { return 1; }

const char* msda_hip_last_error(void) { return g_last_error; }

size_t msda_hip_backward_workspace_bytes(int value_dtype, int64_t batch, int64_t spatial_size,
                                         int64_t num_heads, int64_t channels) {
  (void)value_dtype; (void)batch; (void)spatial_size; (void)num_heads; (void)channels;
  return 0;  // grad_value is accumulated in LDS slabs (msda_gvalue_kernel): no scratch
}

int msda_hip_forward(const void* value, int value_dtype, const int64_t* spatial_shapes,
                     const int64_t* level_start, int64_t num_levels, const void* sampling_loc,
                     const void* attn_weight, void* output, int64_t batch, int64_t spatial_size,
                     int64_t num_heads, int64_t channels, int64_t num_query, int64_t num_point,
                     int padding_mode, void* stream) {
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

int msda_hip_backward(const void* value, int value_dtype, const int64_t* spatial_shapes,
                      const int64_t* level_start, int64_t num_levels, const void* sampling_loc,
                      const void* attn_weight, const void* grad_output, void* grad_value,
                      void* grad_loc, void* grad_attn, void* workspace, int64_t batch,
                      int64_t spatial_size, int64_t num_heads, int64_t channels,
                      int64_t num_query, int64_t num_point, int padding_mode, void* stream) {
  g_last_error[0] = 0;
  Problem pr;
  int rc = check_problem(spatial_shapes, level_start, num_levels, batch, spatial_size, num_heads,
                         channels, num_query, num_point, &pr);
  if (rc) return rc;
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
  hipStream_t st = static_cast<hipStream_t>(stream);
  const int vec = pick_vec(value_dtype, pr.D);
  (void)workspace;  // ABI v1 slot; grad_value no longer needs scratch (see msda_gvalue_kernel)
  // grad_loc / grad_attn: per-item gathers + lane-group butterflies
  if (grad_loc != nullptr || grad_attn != nullptr) {
    switch (value_dtype) {
      case MSDA_DTYPE_F32:
        rc = vec == 4 ? run_backward<float, float, 4>(pr, value, sampling_loc, attn_weight, grad_output, grad_loc, grad_attn, padding_mode, st)
                      : run_backward<float, float, 1>(pr, value, sampling_loc, attn_weight, grad_output, grad_loc, grad_attn, padding_mode, st);
        break;
      case MSDA_DTYPE_F64:
        rc = vec == 2 ? run_backward<double, double, 2>(pr, value, sampling_loc, attn_weight, grad_output, grad_loc, grad_attn, padding_mode, st)
                      : run_backward<double, double, 1>(pr, value, sampling_loc, attn_weight, grad_output, grad_loc, grad_attn, padding_mode, st);
        break;
      case MSDA_DTYPE_BF16:
        rc = vec == 8 ? run_backward<bf16_t, float, 8>(pr, value, sampling_loc, attn_weight, grad_output, grad_loc, grad_attn, padding_mode, st)
                      : run_backward<bf16_t, float, 1>(pr, value, sampling_loc, attn_weight, grad_output, grad_loc, grad_attn, padding_mode, st);
        break;
      case MSDA_DTYPE_F16:
        rc = vec == 8 ? run_backward<f16_t, float, 8>(pr, value, sampling_loc, attn_weight, grad_output, grad_loc, grad_attn, padding_mode, st)
                      : run_backward<f16_t, float, 1>(pr, value, sampling_loc, attn_weight, grad_output, grad_loc, grad_attn, padding_mode, st);
        break;
      default:
        set_error("msda_hip_backward: unknown value dtype %d", value_dtype);
        return MSDA_ERR_ARG;
    }
    if (rc) return rc;
  }
  if (grad_value == nullptr) return MSDA_OK;
  switch (value_dtype) {
    case MSDA_DTYPE_F32:
      return run_grad_value<float, float>(pr, sampling_loc, attn_weight, grad_output, grad_value, padding_mode, st);
    case MSDA_DTYPE_F64:
      return run_grad_value<double, double>(pr, sampling_loc, attn_weight, grad_output, grad_value, padding_mode, st);
    case MSDA_DTYPE_BF16:
      return run_grad_value<bf16_t, float>(pr, sampling_loc, attn_weight, grad_output, grad_value, padding_mode, st);
    case MSDA_DTYPE_F16:
      return run_grad_value<f16_t, float>(pr, sampling_loc, attn_weight, grad_output, grad_value, padding_mode, st);
    default:
      set_error("msda_hip_backward: unknown value dtype %d", value_dtype);
      return MSDA_ERR_ARG;
  }
}

}  // extern "C"
