// msda_win.hip — MSDA backward for 16-bit values with D = 64: output-stationary row blocks on
// the matrix cores (gfx950).
//
// Same result as the pair-pull backward of msda.hip (reference semantics: the autograd
// backward of models/modules/attention.py:331-383, grid_sample bilinear / border,
// align_corners=False; or the dormant extension's zero padding): for every sample
// (b, q, m, l, p) with taps base, base+1 and weights (w0, w1):
//   grad_value[b, start_l + base,   m, :] += aw * w0 * grad_out[b, q, m, :]
//   grad_value[b, start_l + base+1, m, :] += aw * w1 * grad_out[b, q, m, :]
//   grad_attn = w0 * d0 + w1 * d1,   grad_loc = aw * (d1 - d0) * dy/dloc,
//   d_k = <grad_out[b, q, m, :], value[b, start_l + base + k, m, :]>.
//
// Why a second kernel: the pair kernel sorts every (b, m, level)'s samples into per-row lists
// (one 1024-thread workgroup per CU, LDS full) and then gathers one grad_out row per sample on
// the vector ALUs; its phases are latency-bound and the ALUs do ~40 instructions per sample.
// Here nothing is sorted.  A workgroup owns 64 consecutive rows of one (b, m, level) and visits
// the query tiles (32 consecutive queries) whose samples touch those rows — in the encoder a
// query samples around its own position, so a row block meets a handful of tiles (a prepass
// stores each tile's row interval).  Per visit:
//   * the tile's grad_out rows are ONE contiguous 4 KB load (32 queries x 128 B), not gathers;
//   * grad_value (16 rows x 64 channels per wave) += C (16 rows x 32 samples) . G (32 samples
//     x 64 channels) on v_mfma_f32_16x16x32_bf16, C holding the samples' aw*w coefficients
//     (a bf16 hi + lo split: ~2^-17 relative, below the bf16 output rounding), G read
//     transposed from LDS with ds_read_b64_tr_b16; only samples whose taps fall in the wave's
//     16 rows enter C (compacted with a ballot);
//   * the dots d_k of every sample of the tile with every row of the block are one more MFMA
//     product, G (32 q x 64 ch) . V^T (64 ch x 80 rows), the block's value rows staged once;
//   * each sample's grad_attn / grad_loc is written by the block holding its base row.
// Every grad_value row is written once (zeros where no tap lands), every coordinate gradient
// once: no atomics, deterministic by construction.
//
// Workspace: one int2 row interval per (b, m, level, query tile).

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "msda_win.h"

namespace {

constexpr int kQT = 32;       // queries per tile
constexpr int kRB = 64;       // value rows per workgroup (4 waves x 16)
constexpr int kThreads = 256;
constexpr int kDotRows = 80;  // rows r0 .. r0+79 in the dot products (r0+64 is the last needed)
constexpr int kGS = 144;      // LDS row stride (bytes) of grad_out / value rows: 16-B aligned, spreads banks
constexpr int kDS = kDotRows + 1;  // floats per dot row (padded)
constexpr int kMaxSamp = 256;      // samples per tile (32 x P, P <= 8)
constexpr int kNone = 1 << 29;     // base of an absent sample

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

__device__ __forceinline__ unsigned xcd_block(unsigned orig, unsigned nwg) {
  const unsigned xcd = orig % 8u, q = nwg / 8u, r = nwg % 8u;
  return (xcd < r ? xcd * (q + 1u) : r * (q + 1u) + (xcd - r) * q) + orig / 8u;
}

struct Taps {
  int base;      // floor of the sample position (-1 .. T-1); taps base, base + 1
  float w0, w1;  // 0 for a tap outside the map
  bool ok0, ok1, live;
  float gmul;
};

// The coordinate arithmetic of msda.hip (taps_border / taps_zeros), FP contraction off: the
// same tap rows and weights bit for bit.
template <bool ZEROS>
__device__ __forceinline__ Taps make_taps(float loc, int T) {
#pragma clang fp contract(off)
  Taps t;
  if constexpr (ZEROS) {
    const float x = loc * (float)T - 0.5f;
    const bool live = (x > -1.f) && (x < (float)T);
    const float x0 = floorf(live ? x : 0.f);
    const float lw = (live ? x : 0.f) - x0;
    const int lo = (int)x0;
    t.live = live;
    t.ok0 = live && lo >= 0;
    t.ok1 = live && lo + 1 <= T - 1;
    t.base = lo;
    t.w0 = t.ok0 ? 1.f - lw : 0.f;
    t.w1 = t.ok1 ? lw : 0.f;
    t.gmul = live ? (float)T : 0.f;
  } else {
    const float g = loc * 2.f - 1.f;
    const float y = fmaf(g + 1.f, (float)T * 0.5f, -0.5f);
    const float ymax = (float)(T - 1);
    const bool inb = (y > 0.f) && (y < ymax);
    const float yc = y > 0.f ? (y < ymax ? y : ymax) : 0.f;
    const float y0 = floorf(yc);
    const float n = yc - y0;
    t.base = (int)y0;
    t.live = true;
    t.ok0 = true;
    t.ok1 = t.base + 1 <= T - 1;
    t.w0 = 1.f - n;
    t.w1 = n;
    t.gmul = inb ? (float)T : 0.f;
  }
  return t;
}

// rows a sample writes or owns: [lo, hi] (base / base + 1 for a live sample; row 0 otherwise:
// samples with no tap on the map are owned by the level's first block, which writes their zeros)
template <bool ZEROS>
__device__ __forceinline__ int2 sample_rows(const Taps& t) {
  if (!t.live) return make_int2(0, 0);
  return make_int2(t.base < 0 ? 0 : t.base, t.base + 1);
}

__device__ __forceinline__ int wave_min(int x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x = min(x, __shfl_xor(x, o));
  return x;
}
__device__ __forceinline__ int wave_max(int x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x = max(x, __shfl_xor(x, o));
  return x;
}

// One wave per (b, m, level, tile): the interval of rows its samples touch or own.
template <bool ZEROS>
__global__ __launch_bounds__(kThreads) void win_tiles_kernel(const float* __restrict__ loc, int2* __restrict__ tiles,
                                                             const WinShape sh, const long long n_waves) {
  const long long wv = (long long)blockIdx.x * (kThreads / 64) + (threadIdx.x >> 6);
  if (wv >= n_waves) return;  // wave-uniform
  const int lane = threadIdx.x & 63;
  const int tile = (int)(wv % sh.ntile);
  const long long bml = wv / sh.ntile;
  const int l = (int)(bml % sh.L);
  const long long bm = bml / sh.L;
  const int m = (int)(bm % sh.M);
  const long long b = bm / sh.M;
  const int T = sh.T[l];
  const int P = sh.P, LP = sh.L * sh.P;
  int lo = kNone, hi = -kNone;
  for (int s = lane; s < kQT * P; s += 64) {
    const int q = tile * kQT + s / P;
    if (q < sh.Lq) {
      const Taps t = make_taps<ZEROS>(loc[((b * sh.Lq + q) * sh.M + m) * LP + l * P + s % P], T);
      const int2 r = sample_rows<ZEROS>(t);
      lo = min(lo, r.x);
      hi = max(hi, r.y);
    }
  }
  lo = wave_min(lo);
  hi = wave_max(hi);
  if (lane == 0) tiles[wv] = make_int2(lo, hi);
}

__device__ __forceinline__ short bf16_bits(float x) {  // round to nearest even (finite inputs)
  const uint32_t u = __float_as_uint(x);
  return (short)((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
}
__device__ __forceinline__ float bf16_val(short h) { return __uint_as_float(((uint32_t)(uint16_t)h) << 16); }

template <bool ZEROS, bool COORDS>
__global__ __launch_bounds__(kThreads) void win_bwd_kernel(
    const uint16_t* __restrict__ value, const float* __restrict__ loc, const float* __restrict__ aw,
    const uint16_t* __restrict__ gout, uint16_t* __restrict__ gval, float* __restrict__ gloc,
    float* __restrict__ gaw, const int2* __restrict__ tiles, const WinShape sh) {
  __shared__ __attribute__((aligned(16))) unsigned char s_g[kQT * kGS];        // grad_out rows of the tile
  __shared__ __attribute__((aligned(16))) unsigned char s_v[kDotRows * kGS];   // the block's value rows
  __shared__ float s_d[kQT * kDS];                                             // dots [q][row - r0]
  __shared__ int s_base[kMaxSamp + 1];
  __shared__ float s_c0[kMaxSamp + 1], s_c1[kMaxSamp + 1];
  __shared__ unsigned short s_list[4][kMaxSamp + kQT];                         // per-wave compacted samples
  __shared__ unsigned short s_visit[kThreads];
  __shared__ int s_nvisit[kThreads / 64];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, li = lane & 15;
  // workgroup -> (b, m, level, block): (b, m) major, so a clip-head's workgroups share one XCD's L2
  const unsigned id = xcd_block(blockIdx.x, gridDim.x);
  const unsigned bm = id / (unsigned)sh.nblk;
  unsigned rem = id % (unsigned)sh.nblk;
  int l = 0;
  while (l + 1 < sh.L && rem >= (unsigned)sh.blk0[l + 1]) ++l;
  const int k = (int)rem - sh.blk0[l];
  const int m = (int)(bm % (unsigned)sh.M);
  const long long b = bm / (unsigned)sh.M;
  const int T = sh.T[l], P = sh.P, LP = sh.L * sh.P, nsamp = kQT * P;
  const int r0 = k * kRB, rw0 = r0 + 16 * wave;
  const int rs = sh.M * 64;  // value / grad_out row stride (elements)
  const uint16_t* __restrict__ vl = value + ((b * sh.S + sh.start[l]) * sh.M + m) * 64;
  const uint16_t* __restrict__ gb = gout + (b * sh.Lq * sh.M + m) * 64;
  const long long cbase = (b * sh.Lq * sh.M + m) * (long long)LP + l * P;  // + q * M * LP + p

  // the block's value rows r0 .. r0+79 (zeros outside the level), staged once
  for (int c = tid; c < kDotRows * 8; c += kThreads) {
    const int row = c >> 3, ch = c & 7, x = r0 + row;
    uint4 v = make_uint4(0u, 0u, 0u, 0u);
    if (x < T) v = *reinterpret_cast<const uint4*>(vl + (long long)x * rs + ch * 8);
    *reinterpret_cast<uint4*>(s_v + row * kGS + ch * 16) = v;
  }
  if (tid == 0) {  // the padding sample of the compacted lists: no tap anywhere
    s_base[kMaxSamp] = kNone;
    s_c0[kMaxSamp] = 0.f;
    s_c1[kMaxSamp] = 0.f;
  }

  f32x4 acc[4];
#pragma unroll
  for (int cb = 0; cb < 4; ++cb) acc[cb] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int2* __restrict__ tl = tiles + ((long long)bm * sh.L + l) * sh.ntile;
  for (int t0 = 0; t0 < sh.ntile; t0 += kThreads) {
    // the tiles of this chunk whose row interval meets [r0, r0 + 63]
    {
      const int t = t0 + tid;
      bool hit = false;
      if (t < sh.ntile) {
        const int2 iv = tl[t];
        hit = iv.x <= r0 + kRB - 1 && iv.y >= r0;
      }
      const unsigned long long bal = __ballot(hit);
      if (lane == 0) s_nvisit[wave] = __popcll(bal);
      __syncthreads();
      int before = 0;
      for (int w = 0; w < wave; ++w) before += s_nvisit[w];
      if (hit) s_visit[before + __popcll(bal & ((1ull << lane) - 1ull))] = (unsigned short)(t - t0);
      __syncthreads();
    }
    const int nvisit = s_nvisit[0] + s_nvisit[1] + s_nvisit[2] + s_nvisit[3];

    for (int vi = 0; vi < nvisit; ++vi) {
      const int tile = t0 + s_visit[vi];
      const int q0 = tile * kQT;
      // 1. the tile's samples (one per thread) and its grad_out rows (one 16-B piece per thread)
      Taps tp;
      float a = 0.f;
      int q = 0, p = 0;
      bool have = false;
      if (tid < nsamp) {
        q = q0 + tid / P;
        p = tid % P;
        have = q < sh.Lq;
        if (have) {
          const long long o = cbase + (long long)q * sh.M * LP + p;
          a = aw[o];
          tp = make_taps<ZEROS>(loc[o], T);
        }
        s_base[tid] = have && tp.live ? tp.base : kNone;
        s_c0[tid] = have && tp.ok0 ? a * tp.w0 : 0.f;
        s_c1[tid] = have && tp.ok1 ? a * tp.w1 : 0.f;
      }
      {
        const int row = tid >> 3, ch = tid & 7;
        uint4 v = make_uint4(0u, 0u, 0u, 0u);
        if (q0 + row < sh.Lq) v = *reinterpret_cast<const uint4*>(gb + (long long)(q0 + row) * rs + ch * 8);
        *reinterpret_cast<uint4*>(s_g + row * kGS + ch * 16) = v;
      }
      __syncthreads();

      // 2a. grad_value of the wave's 16 rows: the samples with a tap in them, 32 per MFMA step
      if (rw0 < T) {
        int n = 0;
        for (int s0 = 0; s0 < nsamp; s0 += 64) {
          const int s = s0 + lane;
          const int bs = s < nsamp ? s_base[s] : kNone;
          const bool sel = bs >= rw0 - 1 && bs <= rw0 + 15;
          const unsigned long long bal = __ballot(sel);
          if (sel) s_list[wave][n + __popcll(bal & ((1ull << lane) - 1ull))] = (unsigned short)s;
          n += __popcll(bal);
        }
        if (n > 0) {
          const int nk = (n + 31) >> 5;
          if (lane < nk * 32 - n) s_list[wave][n + lane] = (unsigned short)kMaxSamp;  // pad to whole steps
          for (int ks = 0; ks < nk; ++ks) {
            const unsigned short* lst = &s_list[wave][ks * 32 + 8 * g];
            bf16x8 ahi, alo;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
              const int s = lst[j];
              const int dr = s_base[s] - rw0;
              const float c = (dr == li ? s_c0[s] : 0.f) + (dr + 1 == li ? s_c1[s] : 0.f);
              const short h = bf16_bits(c);
              ahi[j] = __builtin_bit_cast(__bf16, h);
              alo[j] = __builtin_bit_cast(__bf16, bf16_bits(c - bf16_val(h)));
            }
            // rows of the transposed reads: lane 4q'+pp of the group names sample 8g + 4h + q'
            const int qq = (li >> 2), pp = li & 3;
            const int sa = lst[qq], sb = lst[4 + qq];
            const int ra = sa < kMaxSamp ? sa / P : 0, rb = sb < kMaxSamp ? sb / P : 0;
#pragma unroll
            for (int cb = 0; cb < 4; ++cb) {
              const int col = (cb * 16 + 4 * pp) * 2;
              const s16x4 x0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(s_g + ra * kGS + col));
              const s16x4 x1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(s_g + rb * kGS + col));
              bf16x8 bv;
#pragma unroll
              for (int j = 0; j < 4; ++j) {
                bv[j] = __builtin_bit_cast(__bf16, x0[j]);
                bv[4 + j] = __builtin_bit_cast(__bf16, x1[j]);
              }
              acc[cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ahi, bv, acc[cb], 0, 0, 0);
              acc[cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(alo, bv, acc[cb], 0, 0, 0);
            }
          }
        }
      }
      // 2b. dots of the tile's 32 queries with rows r0 .. r0+79: 2 query halves x 5 row blocks
      if (COORDS) {
        for (int tt = wave; tt < 10; tt += 4) {
          const int qh = tt / 5, cb = tt % 5;
          f32x4 d = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int ks = 0; ks < 2; ++ks) {
            const int off = (ks * 32 + 8 * g) * 2;
            const bf16x8 av = *reinterpret_cast<const bf16x8*>(s_g + (qh * 16 + li) * kGS + off);
            const bf16x8 bv = *reinterpret_cast<const bf16x8*>(s_v + (cb * 16 + li) * kGS + off);
            d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bv, d, 0, 0, 0);
          }
#pragma unroll
          for (int j = 0; j < 4; ++j) s_d[(qh * 16 + 4 * g + j) * kDS + cb * 16 + li] = d[j];
        }
      }
      __syncthreads();

      // 3. coordinate gradients of the samples this block owns (base row in it; the level's first
      // block also owns the samples with no tap on the map)
      if (COORDS && tid < nsamp && have) {
        const bool own = tp.live ? (tp.base >= r0 && tp.base < r0 + kRB) || (tp.base < 0 && k == 0) : k == 0;
        if (own) {
          const int qi = tid / P;
          const float d0 = tp.ok0 ? s_d[qi * kDS + tp.base - r0] : 0.f;
          const float d1 = tp.ok1 ? s_d[qi * kDS + tp.base + 1 - r0] : 0.f;
          const long long o = cbase + (long long)q * sh.M * LP + p;
          if (gaw != nullptr) gaw[o] = d0 * tp.w0 + d1 * tp.w1;
          if (gloc != nullptr) gloc[o] = ((d1 - d0) * a) * tp.gmul;
        }
      }
      __syncthreads();  // the next visit overwrites the tile's LDS
    }
    __syncthreads();  // every wave has read this chunk's visit count before the next chunk writes it
  }

  // grad_value rows rw0 + 4g + j, channels 16 cb + li (every row of the block, zeros included)
  if (rw0 < T) {
    uint16_t* __restrict__ gvl = gval + ((b * sh.S + sh.start[l]) * sh.M + m) * 64;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int x = rw0 + 4 * g + j;
      if (x < T) {
#pragma unroll
        for (int cb = 0; cb < 4; ++cb) gvl[(long long)x * rs + cb * 16 + li] = (uint16_t)bf16_bits(acc[cb][j]);
      }
    }
  }
}

}  // namespace

size_t msda_win_workspace_bytes(long long B, long long M, long long L, long long Lq) {
  const long long ntile = (Lq + kQT - 1) / kQT;
  return (size_t)(B * M * L * ntile) * sizeof(int2);
}

int msda_win_supported(int value_dtype_is_bf16, long long D, long long P) {
  return value_dtype_is_bf16 && D == 64 && P >= 1 && P <= kMaxSamp / kQT;
}

int msda_win_backward(const void* value, const void* loc, const void* aw, const void* gout, void* gval,
                      void* gloc, void* gaw, void* workspace, const WinShape* shape, int zeros, hipStream_t st) {
  WinShape sh = *shape;
  sh.ntile = (int)((sh.Lq + kQT - 1) / kQT);
  int nb = 0;
  for (int l = 0; l < sh.L; ++l) {
    sh.blk0[l] = nb;
    nb += (sh.T[l] + kRB - 1) / kRB;
  }
  sh.blk0[sh.L] = nb;
  sh.nblk = nb;
  if (sh.B * sh.M == 0 || nb == 0) return 0;
  auto* tiles = static_cast<int2*>(workspace);
  const long long n_waves = sh.B * sh.M * sh.L * sh.ntile;
  if (n_waves > 0) {
    const unsigned blocks = (unsigned)((n_waves + 3) / 4);
    if (zeros)
      hipLaunchKernelGGL(win_tiles_kernel<true>, dim3(blocks), dim3(kThreads), 0, st,
                         static_cast<const float*>(loc), tiles, sh, n_waves);
    else
      hipLaunchKernelGGL(win_tiles_kernel<false>, dim3(blocks), dim3(kThreads), 0, st,
                         static_cast<const float*>(loc), tiles, sh, n_waves);
  }
  const unsigned grid = (unsigned)(sh.B * sh.M * nb);
  const bool coords = gloc != nullptr || gaw != nullptr;
  auto* v = static_cast<const uint16_t*>(value);
  auto* lc = static_cast<const float*>(loc);
  auto* a = static_cast<const float*>(aw);
  auto* g = static_cast<const uint16_t*>(gout);
  auto* gv = static_cast<uint16_t*>(gval);
  auto* gl = static_cast<float*>(gloc);
  auto* ga = static_cast<float*>(gaw);
#define WIN_LAUNCH(Z, C) \
  hipLaunchKernelGGL((win_bwd_kernel<Z, C>), dim3(grid), dim3(kThreads), 0, st, v, lc, a, g, gv, gl, ga, tiles, sh)
  if (zeros) {
    if (coords) WIN_LAUNCH(true, true); else WIN_LAUNCH(true, false);
  } else {
    if (coords) WIN_LAUNCH(false, true); else WIN_LAUNCH(false, false);
  }
#undef WIN_LAUNCH
  return 0;  // launch errors: the caller's hipGetLastError
}
