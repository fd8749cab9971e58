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
#include <stdlib.h>

#include "msda_win.h"

namespace {

constexpr int kQT = kWinQT;    // queries per tile
constexpr int kThreads = 256;
constexpr int kGS = 144;      // LDS row stride (bytes) of grad_out / value rows: 16-B aligned, spreads banks
constexpr int kMaxSamp = 256;      // samples per tile (32 x P, P <= 8)
constexpr int kNone = kWinNone;    // an empty interval is (kNone, -kNone)

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(4))) unsigned u32x4;
typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;
// (the v4i16 form of the transposed read with per-element bit casts into a bf16x8 was compiled
// into a splat of element 0 — tools/probes/mfma_tr_probe.hip; the v4bf16 form + shufflevector is exact)

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


// The row interval every (b, m, level, query tile) touches or owns.  One 256-thread workgroup per
// (b, tile): a query's coordinates of all heads and levels are one contiguous row of M * L * P
// floats, so each wave reads 8 of the tile's 32 rows coalesced (lane i: floats i + 64 j), every
// load issued before the first is used; each (m, level)'s P consecutive floats are reduced over P
// lanes, then the four waves' intervals through LDS.
constexpr int kRowRegs = 8;  // M * L * P <= 512 floats per query row
constexpr int kTileWaves = kThreads / 64;
constexpr int kQPW = kQT / kTileWaves;  // queries per wave
template <bool ZEROS, int NJ>
__global__ __launch_bounds__(kThreads) void win_tiles_kernel(const float* __restrict__ loc, int2* __restrict__ tiles,
                                                             const WinShape sh) {
  __shared__ int2 s_iv[kTileWaves][64 * NJ];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int tile = (int)(blockIdx.x % (unsigned)sh.ntile);
  const long long b = blockIdx.x / (unsigned)sh.ntile;
  const int P = sh.P, n = (int)sh.M * sh.L * P;
  const int q0 = tile * kQT + w * kQPW;
  const int nq = (int)max(0LL, min((long long)kQPW, sh.Lq - q0));
  float x[kQPW][NJ];
#pragma unroll
  for (int u = 0; u < kQPW; ++u) {
    const float* __restrict__ row = loc + (b * sh.Lq + (u < nq ? qo_query(sh.qo, q0 + u) : 0)) * (long long)n;
#pragma unroll
    for (int j = 0; j < NJ; ++j) x[u][j] = (u < nq && lane + 64 * j < n) ? row[lane + 64 * j] : 0.f;
  }
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int i = lane + 64 * j;
    const int T = sh.T[(i / P) % sh.L];
    int lo = kNone, hi = -kNone;
#pragma unroll
    for (int u = 0; u < kQPW; ++u) {
      if (u < nq && i < n) {
        const int2 r = win_sample_rows(x[u][j], T, ZEROS);  // msda_win.h: the rows make_taps gives
        lo = min(lo, r.x);
        hi = max(hi, r.y);
      }
    }
    for (int o = 1; o < P; o <<= 1) {
      lo = min(lo, __shfl_xor(lo, o));
      hi = max(hi, __shfl_xor(hi, o));
    }
    s_iv[w][i] = make_int2(lo, hi);
  }
  __syncthreads();
  for (int g = threadIdx.x; g * P < n; g += kThreads) {  // one (m, level) per thread
    int2 iv = s_iv[0][g * P];
#pragma unroll
    for (int v = 1; v < kTileWaves; ++v) {
      const int2 o = s_iv[v][g * P];
      iv.x = min(iv.x, o.x);
      iv.y = max(iv.y, o.y);
    }
    tiles[(b * sh.M * sh.L + g) * sh.ntile + tile] = iv;
  }
}

__device__ __forceinline__ short bf16_bits(float x) {  // round to nearest even (finite inputs)
  const uint32_t u = __float_as_uint(x);
  return (short)((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
}
// two values rounded to nearest even by one v_cvt_pk_bf16_f32 (bitwise bf16_bits for finite inputs),
// x in the low half
__device__ __forceinline__ uint32_t bf16_pair(float x, float y) {
  typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2;
  return __builtin_bit_cast(uint32_t, bf16x2{(__bf16)x, (__bf16)y});
}
__device__ __forceinline__ float bf16_val(short h) { return __uint_as_float(((uint32_t)(uint16_t)h) << 16); }

// One wave per 16-row block of one (b, m, level): barrier-free (every LDS exchange is inside the
// wave, ordered by the wave's own LDS queue), so many blocks per CU overlap their latencies, and
// a coarse level's block meets about as many query tiles as a fine level's (16 rows each).
// The next visit's coordinates and grad_out rows are loaded into registers while the current
// visit computes.
constexpr int kRW = 16;          // rows per block (one wave)
constexpr int kVRows = kRW + 1;  // value rows r0 .. r0+16 in the dot products
constexpr int kDQS = kQT + 4;    // dots row stride (floats): [row - r0][q], rows r0 .. r0+16, 16-B rows

// Orders one wave's LDS writes before its later LDS reads: the wave's LDS operations execute in
// issue order, so this only has to stop the compiler from moving LDS accesses across it (no
// wait on the global loads in flight).
__device__ __forceinline__ void wave_lds_fence() { asm volatile("" ::: "memory"); }

// W waves per row block (one workgroup of 64 W threads): the block's query-tile visits are dealt
// round-robin over the waves (each with its own LDS), and the waves' grad_value partial sums are
// added through LDS at the end — for calls with few row blocks (short pyramids: video queries on
// the audio pyramid), where one wave per block leaves the chip mostly idle.
template <bool ZEROS, bool COORDS, int P, int W>
__global__ __launch_bounds__(64 * W) __attribute__((amdgpu_waves_per_eu(P >= 8 ? 2 : 4))) void win_bwd_kernel(
    const uint16_t* __restrict__ value, const float* __restrict__ loc, const float* __restrict__ aw,
    const uint16_t* __restrict__ gout, uint16_t* __restrict__ gval, float* __restrict__ gloc,
    float* __restrict__ gaw, const int2* __restrict__ tiles, const WinShape sh) {
  constexpr int NS = kQT * P;                  // samples per tile
  constexpr int SPL = NS >= 64 ? NS / 64 : 1;  // samples per lane
  __shared__ __attribute__((aligned(16))) unsigned char s_g_w[W][kQT * kGS];     // grad_out rows of the tile
  // C of one MFMA step ([row][hi 32 | lo 32], step 2a) and the dots ([row - r0][q], 2b / 3)
  __shared__ __attribute__((aligned(16))) unsigned char s_c_w[W][kRW * kGS];
  __shared__ __attribute__((aligned(16))) float s_d_w[W][kVRows * kDQS];
  __shared__ int s_q_w[W][NS + kQT];  // query row (in the tile) of each compacted sample, padded
  const int wid = W > 1 ? (int)(threadIdx.x >> 6) : 0;
  unsigned char* const s_g = s_g_w[wid];
  unsigned char* const s_c = s_c_w[wid];
  float* const s_d = s_d_w[wid];
  int* const s_q = s_q_w[wid];

  const int lane = (int)(threadIdx.x & 63), g = lane >> 4, li = lane & 15;
  const unsigned x8 = blockIdx.x % 8u;  // block p runs on XCD p % 8 (round-robin dispatch)
  unsigned slot = blockIdx.x / 8u;
  int l = sh.L - 1, k;
  unsigned bm;
  if (sh.nchunk > 0) {
    // position-chunk order: XCD x takes (b, m) pairs [x ppx, (x+1) ppx) and walks the level
    // pyramid by position — chunk c of every level for each of its pairs, coarse level first,
    // then chunk c + 1.  The blocks that write one query's coordinate gradients (its (m, level)
    // pieces: 16 B each, one 64-B line per (q, m)) and read its loc / aw lines then run together
    // on one XCD, so those lines are merged / reused in its L2 instead of written back and
    // fetched once per level (row-block traffic: tools/pmc_win.sh)
    int c = 0;
    while (c + 1 < sh.nchunk && slot >= (unsigned)sh.ppx * sh.cs[c + 1]) ++c;
    const unsigned nc = sh.cs[c + 1] - sh.cs[c];
    const unsigned off = slot - (unsigned)sh.ppx * sh.cs[c];
    const unsigned pair = x8 * (unsigned)sh.ppx + off / nc;
    if (off / nc >= (unsigned)sh.ppx || pair >= (unsigned)(sh.B * sh.M)) return;  // grid padding (wave-uniform)
    const unsigned e = sh.seq[sh.cs[c] + off % nc];
    l = (int)(e >> 12);
    k = (int)(e & 4095u);
    bm = pair;
  } else {
    // the coarsest level's blocks first (a level-3 block meets ~12 query tiles, a level-0 block
    // ~5: longest first shortens the tail), each level split into 8 contiguous chunks, chunk x
    // on XCD x, so neighbouring blocks share that XCD's L2
    long long j = -1;
    for (; l >= 0; --l) {
      const long long nl = (long long)sh.B * sh.M * (sh.blk0[l + 1] - sh.blk0[l]);
      const unsigned cl = (unsigned)((nl + 7) / 8);
      if (slot < cl) {
        j = (long long)x8 * cl + slot;
        if (j >= nl) return;  // padding of the level's last chunk (wave-uniform, before any LDS use)
        break;
      }
      slot -= cl;
    }
    if (l < 0) return;
    const int nbl = sh.blk0[l + 1] - sh.blk0[l];
    bm = (unsigned)(j / nbl);
    k = (int)(j % nbl);
  }
  const int m = (int)(bm % (unsigned)sh.M);
  const long long b = bm / (unsigned)sh.M;
  const int T = sh.T[l];
  const int r0 = k * kRW;
  const int rs = sh.M * 64;                           // grad_out / value row stride (elements)
  // the query order of the tiles: the forward's (stored in the tiles tail) when it wrote them
  const QOrder qo = sh.qo_dev ? *reinterpret_cast<const QOrder*>(
                                    reinterpret_cast<const char*>(tiles + sh.B * sh.M * sh.L * sh.ntile) +
                                    kWinQOrderOffset)
                              : sh.qo;
  const int qstride = sh.cq;                          // coordinate stride of one query
  const uint16_t* __restrict__ vl = value + ((b * sh.S + sh.start[l]) * sh.M + m) * 64;
  const uint16_t* __restrict__ gb = gout + (b * sh.Lq * sh.M + m) * 64;
  const long long cbase = b * sh.cb + m * sh.cm + (long long)l * sh.cl;
  // coordinate offset of sample s of the tile at entry q0 of the query order (sh.qo; the caller
  // keeps q0 + s / P < Lq)
  auto coff = [&](int q0, int s) -> long long {
    return (long long)qo_query(qo, q0 + s / P) * qstride + s % P;
  };
  // The dots' B operands, constant over the block's visits, in registers: lane (li, g) holds
  // channels ks*32 + 8g .. +7 of value row r0 + li (vb[0][ks]) and of row r0 + 16 (vb[1][ks])
  // (zeros outside the level) — the dots then read no LDS
  bf16x8 vb[2][2];
#pragma unroll
  for (int cb = 0; cb < 2; ++cb) {
    const int x = r0 + (cb == 0 ? li : kRW);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      uint4 v = make_uint4(0u, 0u, 0u, 0u);
      if (x < T) v = *reinterpret_cast<const uint4*>(vl + (long long)x * rs + ks * 32 + 8 * g);
      vb[cb][ks] = __builtin_bit_cast(bf16x8, v);
    }
  }
  // the query tiles whose row interval meets [r0, r0 + 15]: 64 tiles per ballot mask, walked
  // bit by bit (wave-uniform); the next visit is known one visit ahead for the prefetch
  const int2* __restrict__ tl = tiles + ((long long)bm * sh.L + l) * sh.ntile;
  auto chunk_mask = [&](int t0) -> unsigned long long {
    const int t = min(t0 + lane, sh.ntile - 1);
    const int2 iv = tl[t];
    return __ballot(t0 + lane < sh.ntile && iv.x <= r0 + kRW - 1 && iv.y >= r0);
  };
  int cur_t0 = 0;
  unsigned long long mask = chunk_mask(0);
  auto pop_tile = [&]() -> int {  // pops the block's next visit (-1 when done)
    while (mask == 0ull) {
      cur_t0 += 64;
      if (cur_t0 >= sh.ntile) return -1;
      mask = chunk_mask(cur_t0);
    }
    const int t = cur_t0 + __builtin_ctzll(mask);
    mask &= mask - 1ull;
    return t;
  };
  bool first_pop = true;
  auto next_tile = [&]() -> int {  // this wave's next visit: visits wid, wid + W, wid + 2W, ...
    const int skip = first_pop ? wid : W - 1;
    first_pop = false;
    for (int i = 0; i < skip; ++i)
      if (pop_tile() < 0) return -1;
    return pop_tile();
  };

  f32x4 acc[4];
#pragma unroll
  for (int cb = 0; cb < 4; ++cb) acc[cb] = f32x4{0.f, 0.f, 0.f, 0.f};

  // a visit's inputs in registers: SPL samples and 4 grad_out pieces per lane (rows grow + 8 i,
  // 16-byte chunk gch: 8 lanes a 128-B row, coalesced)
  const int grow = lane >> 3, gch = lane & 7;
  float rl[SPL], ra[SPL];
  uint4 rg[4];
  auto fetch = [&](int tile) {
    const int q0 = tile * kQT;
    const float* __restrict__ lt = loc + cbase;
    const float* __restrict__ at = aw + cbase;
    if (sh.exp & 32) {  // (profiling: no coordinate loads)
#pragma unroll
      for (int j = 0; j < SPL; ++j) {
        rl[j] = ((float)(q0 + (lane + 64 * j) / P) + 0.5f) / (float)sh.Lq;
        ra[j] = 0.25f;
      }
    }
    if (sh.exp & 8) {  // (profiling: no grad_out loads)
#pragma unroll
      for (int i = 0; i < 4; ++i) rg[i] = make_uint4(0u, 0u, 0u, 0u);
    }
    if (sh.exp & 40) return;
    if (q0 + kQT <= sh.Lq) {  // a whole tile (wave-uniform)
#pragma unroll
      for (int j = 0; j < SPL; ++j) {
        const bool in = NS >= 64 || lane < NS;
        const long long o = coff(q0, in ? lane + 64 * j : 0);
        rl[j] = in ? lt[o] : 0.f;
        ra[j] = in ? at[o] : 0.f;
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
        rg[i] = *reinterpret_cast<const uint4*>(gb + (long long)qo_query(qo, q0 + grow + 8 * i) * rs + gch * 8);
    } else {
#pragma unroll
      for (int j = 0; j < SPL; ++j) {
        const int s = lane + 64 * j;
        const bool in = (NS >= 64 || lane < NS) && q0 + s / P < sh.Lq;
        const long long o = in ? coff(q0, s) : 0;
        rl[j] = in ? lt[o] : 0.f;
        ra[j] = in ? at[o] : 0.f;
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
        rg[i] = q0 + grow + 8 * i < sh.Lq
                    ? *reinterpret_cast<const uint4*>(gb + (long long)qo_query(qo, q0 + grow + 8 * i) * rs + gch * 8)
                    : make_uint4(0u, 0u, 0u, 0u);
    }
  };
  int tile = next_tile();
  if (tile >= 0) fetch(tile);

  while (tile >= 0) {
    const int q0 = tile * kQT;
    // 1. the visit's taps (kept in registers) and grad_out rows (into LDS); the samples with a tap
    // in the block's 16 rows are compacted (ballot): position kp, coefficients split into bf16 hi / lo
    Taps tp[SPL];
    float a[SPL];
    int kp[SPL], dr[SPL];
    uint32_t ch[SPL], cl[SPL];  // c0 | c1 << 16, hi and lo parts
    int n = 0;
#pragma unroll
    for (int j = 0; j < SPL; ++j) {
      const int s = lane + 64 * j;
      const bool in = (NS >= 64 || lane < NS) && q0 + s / P < sh.Lq;
      tp[j] = make_taps<ZEROS>(rl[j], T);
      tp[j].live = tp[j].live && in;
      a[j] = ra[j];
      dr[j] = tp[j].base - r0;
      const bool sel = tp[j].live && dr[j] >= -1 && dr[j] <= kRW - 1;
      const unsigned long long bal = __ballot(sel);
      kp[j] = sel ? n + __popcll(bal & ((1ull << lane) - 1ull)) : -1;
      const float c0 = tp[j].ok0 ? a[j] * tp[j].w0 : 0.f;
      const float c1 = tp[j].ok1 ? a[j] * tp[j].w1 : 0.f;
      // c = hi + lo: hi the truncated bf16 (exact remainder c - hi), lo that remainder rounded to
      // bf16 — |c - hi - lo| <= 2^-16 |c|, far below the bf16 rounding of grad_value
      const uint32_t u0 = __float_as_uint(c0) & 0xffff0000u, u1 = __float_as_uint(c1) & 0xffff0000u;
      ch[j] = __builtin_amdgcn_perm(u1, u0, 0x07060302u);  // hi halves: c0 low, c1 high
      cl[j] = bf16_pair(c0 - __uint_as_float(u0), c1 - __uint_as_float(u1));
      if (sel) s_q[kp[j]] = s / P;
      n += __popcll(bal);
    }
    const int nk = (n + 31) >> 5;
    if (lane < nk * 32 - n) s_q[n + lane] = 0;  // padding columns: C is zero there
#pragma unroll
    for (int i = 0; i < 4; ++i) *reinterpret_cast<uint4*>(s_g + (grow + 8 * i) * kGS + gch * 16) = rg[i];
    wave_lds_fence();
    // 2b. dots of the tile's 32 queries with rows r0 .. r0+16 (2 query halves x 2 row blocks; of
    // the second block only row r0+16 is kept, its other columns read row r0+16 again): the A
    // fragments (grad_out rows) read once from LDS, the B fragments (value rows) block-constant in
    // registers; into LDS at once (lane (g, li) holds queries qh*16 + 4g .. +3 of row li (cb 0) /
    // row 16 (cb 1), one 16-B store)
    if (COORDS && !(sh.exp & 4)) {
#pragma unroll
      for (int qh = 0; qh < 2; ++qh) {
        bf16x8 av[2];
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
          av[ks] = *reinterpret_cast<const bf16x8*>(s_g + (qh * 16 + li) * kGS + (ks * 32 + 8 * g) * 2);
#pragma unroll
        for (int cb = 0; cb < 2; ++cb) {
          f32x4 d = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int ks = 0; ks < 2; ++ks) d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[ks], vb[cb][ks], d, 0, 0, 0);
          if (cb == 0 || li == 0) *reinterpret_cast<f32x4*>(s_d + (cb * 16 + li) * kDQS + qh * 16 + 4 * g) = d;
        }
      }
    }
    const int next = next_tile();
    if (next >= 0) fetch(next);  // in flight during the compute below

    // 2a. grad_value of the 16 rows += C . G, 32 compacted samples per MFMA step: C built in LDS
    // (zeroed, then each sample writes c0 on its base row and c1 on the next, where in the block)
    for (int ks = 0; ks < ((sh.exp & 1) ? 0 : nk); ++ks) {
      {
        uint4* z = reinterpret_cast<uint4*>(s_c + (lane >> 2) * kGS + (lane & 3) * 32);
        z[0] = make_uint4(0u, 0u, 0u, 0u);
        z[1] = make_uint4(0u, 0u, 0u, 0u);
      }
      wave_lds_fence();
#pragma unroll
      for (int j = 0; j < SPL; ++j) {
        const int col = kp[j] - 32 * ks;
        if (col >= 0 && col < 32) {
          uint16_t* r = reinterpret_cast<uint16_t*>(s_c + dr[j] * kGS) + col;  // row dr (may be -1: not written)
          if (dr[j] >= 0) {
            r[0] = (uint16_t)ch[j];
            r[32] = (uint16_t)cl[j];
          }
          if (dr[j] + 1 < kRW) {
            r[kGS / 2] = (uint16_t)(ch[j] >> 16);
            r[kGS / 2 + 32] = (uint16_t)(cl[j] >> 16);
          }
        }
      }
      wave_lds_fence();
      const bf16x8 ahi = *reinterpret_cast<const bf16x8*>(s_c + li * kGS + 16 * g);
      const bf16x8 alo = *reinterpret_cast<const bf16x8*>(s_c + li * kGS + 64 + 16 * g);
      // rows of the transposed reads: lane 4q'+pp of the group names compacted sample 8g + 4h + q'
      const int qq = li >> 2, pp = li & 3;
      const int rowa = s_q[ks * 32 + 8 * g + qq], rowb = s_q[ks * 32 + 8 * g + 4 + qq];
#pragma unroll
      for (int cb = 0; cb < 4; ++cb) {
        const int col = (cb * 16 + 4 * pp) * 2;
        const bf16x4 x0 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(s_g + rowa * kGS + col));
        const bf16x4 x1 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(s_g + rowb * kGS + col));
        const bf16x8 bv = __builtin_shufflevector(x0, x1, 0, 1, 2, 3, 4, 5, 6, 7);
        acc[cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ahi, bv, acc[cb], 0, 0, 0);
        acc[cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(alo, bv, acc[cb], 0, 0, 0);
      }
      wave_lds_fence();  // this step's C reads before the next step's zeroing
    }
    if (COORDS && !(sh.exp & 4)) {
      wave_lds_fence();
      // 3. coordinate gradients of the samples this block owns (base row in it; the level's first
      // block also owns the samples with no tap on the map)
      const long long tb = cbase;
#pragma unroll
      for (int j = 0; j < SPL; ++j) {
        const int s = lane + 64 * j;
        const bool in = (NS >= 64 || lane < NS) && q0 + s / P < sh.Lq;
        const Taps& t = tp[j];
        const bool own = t.live ? (t.base >= r0 && t.base < r0 + kRW) || (t.base < 0 && k == 0) : k == 0;
        if (in && own && !(sh.exp & 2)) {
          const int qi = s / P;
          const long long o = coff(q0, s);
          const float d0 = t.ok0 ? s_d[(t.base - r0) * kDQS + qi] : 0.f;
          const float d1 = t.ok1 ? s_d[(t.base + 1 - r0) * kDQS + qi] : 0.f;
          if (gaw != nullptr) gaw[tb + o] = d0 * t.w0 + d1 * t.w1;
          if (gloc != nullptr) gloc[tb + o] = ((d1 - d0) * a[j]) * t.gmul;
        }
      }
    }
    wave_lds_fence();  // this visit's LDS reads before the next visit's writes
    tile = next;
  }

  // grad_value rows r0 + 4g + j, channels 16 cb + li (every row of the block, zeros included)
  if (gval == nullptr) return;
  if constexpr (W > 1) {  // the waves' partial sums through LDS (each wave's grad_out tile space)
    __syncthreads();
    float* red = reinterpret_cast<float*>(s_g);
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int cb = 0; cb < 4; ++cb) red[(4 * g + j) * 64 + cb * 16 + li] = acc[cb][j];
    __syncthreads();
    if (wid != 0) return;
#pragma unroll
    for (int v = 1; v < W; ++v) {
      const float* o = reinterpret_cast<const float*>(s_g_w[v]);
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int cb = 0; cb < 4; ++cb) acc[cb][j] += o[(4 * g + j) * 64 + cb * 16 + li];
    }
  }
  uint16_t* __restrict__ gvl = gval + ((b * sh.S + sh.start[l]) * sh.M + m) * 64;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int x = r0 + 4 * g + j;
    if (x < T) {
#pragma unroll
      for (int cb = 0; cb < 4; ++cb) gvl[(long long)x * rs + cb * 16 + li] = (uint16_t)bf16_bits(acc[cb][j]);
    }
  }
}


// ---------------------------------------------------------------------------------------------
// win_lm_kernel: the row-block backward for level-major coordinates with the forward's tile
// intervals (the encoder calls: MSDeformAttn's prologue writes level-major locations / weights),
// one wave per 16-row block as win_bwd_kernel (same dispatch order: coarsest level first, each
// level in 8 contiguous chunks, chunk x on XCD x), with the per-visit work restructured:
//  * 7.2 KB of LDS a wave instead of 10 KB: the grad_out tile in 128-B rows with an XOR swizzle of
//    the 16-B chunks (conflict-free for the row writes, the dots' A reads and the transposed B reads
//    of rows {0-3, 8-11} (+4, +16)) instead of 144-B padded rows, and the dots buffer reused for the
//    coefficient tile C (phases reordered: dots -> coordinate gradients -> grad_value);
//  * 32-bit offsets from per-block base pointers (level-major: a tile's coordinates of one level
//    are 32 P contiguous floats), the compaction rank from mbcnt;
//  * the next visit's coordinates and grad_out rows requested once the coordinate gradients are
//    stored (rg / rl free), before the grad_value steps.
// Measured at the bench's encoder call (tools/win_exp.py, r05g): 49.4 / 54.8 us (init / trained
// sampling) against 51.0 / 55.7 for win_bwd_kernel on level-major coordinates.  Persistent variants
// were slower or no better: waves popping blocks from per-XCD queues (a returning atomic per block)
// 202 us; a static round-robin of blocks over a resident grid 51.5 / 58.3 us.
// Same arithmetic per visit as win_bwd_kernel (the same taps, bf16 hi + lo coefficient split and
// MFMA products in the same order), so its outputs are win_bwd_kernel's bit for bit
// (tests/test_gpu_op.py::test_persistent_level_major_backward_equals_per_block_kernel).
// ---------------------------------------------------------------------------------------------
constexpr int kLmRow = 128;  // bytes per grad_out / coefficient row in LDS

// the swizzled byte offset of 16-B chunk c of row r: chunk c ^ f(r), f(r) in {0, 2, 4, 6} from
// bits 1 and 3 of r — rows {0,1,2,3,8,9,10,11} (a 32-lane half of a transposed read) land on 16
// distinct bank quads, and so do the row reads of the dots
__device__ __forceinline__ int lm_sw(int r, int c) {
  return r * kLmRow + ((c ^ ((((r >> 1) & 1) << 1) | (((r >> 3) & 1) << 2))) << 4);
}

// the coefficient tile C's layout: chunk c ^ (r & 7).  Its b16 stores bank on (a / 4) mod 32, where
// the 128-B row drops out: XOR-ing the chunk with all three low row bits spreads the stores of
// different rows; the A-operand reads (rows li, chunk g / 4 + g) still meet 16 distinct bank quads
__device__ __forceinline__ int lm_csw(int r, int c) { return r * kLmRow + ((c ^ (r & 7)) << 4); }

// NW (round 6): waves per workgroup.  NW = 1: one wave a 16-row block.  NW = 4 (split mode): a
// workgroup holds 4 / W_l blocks of level l with W_l = sh.wsplit[l] waves each (1, 2 or 4); the
// waves of one block take its visits round-robin (wave p: visits p, p + W_l, ...) and add their
// grad_value partials through LDS at the end in wave order.  The coarse levels' blocks meet the most
// query tiles (bench encoder call: ~12 visits a level-3 block against ~5 a level-0 block,
// tools/win_visits.py); with one wave each they are the kernel's longest waves.
template <bool ZEROS, bool COORDS, int P, int NW = 1>
__global__ __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(4))) void win_lm_kernel(
    const uint16_t* __restrict__ value, const float* __restrict__ loc, const float* __restrict__ aw,
    const uint16_t* __restrict__ gout, uint16_t* __restrict__ gval, float* __restrict__ gloc,
    float* __restrict__ gaw, const int2* __restrict__ tiles, const WinShape sh) {
  constexpr int NS = kQT * P;                  // samples per tile and level
  constexpr int SPL = NS >= 64 ? NS / 64 : 1;  // samples per lane
  __shared__ __attribute__((aligned(16))) unsigned char s_g_w[NW][kQT * kLmRow];  // the tile's grad_out rows
  // dots [row - r0][q] (kVRows x kDQS floats), then, once the coordinate gradients have read them,
  // the coefficient tile C [16 rows][hi 32 | lo 32] bf16 of each MFMA step
  __shared__ __attribute__((aligned(16))) float s_cd_w[NW][kVRows * kDQS];
  __shared__ int s_q_w[NW][NS + kQT];  // query (in the tile) of each compacted sample, padded
  const int wid = NW > 1 ? __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)) : 0;  // (wave-uniform)
  unsigned char* const s_g = s_g_w[wid];
  float* const s_cd = s_cd_w[wid];
  int* const s_q = s_q_w[wid];
  unsigned char* const s_c = reinterpret_cast<unsigned char*>(s_cd);
  const int lane = (int)(threadIdx.x & 63), g = lane >> 4, li = lane & 15;
  const int grow = lane >> 3, gch = lane & 7;
  // LDS offsets fixed per lane: grad_out row writes (rows grow, grow + 8), and the row reads of
  // chunks g / 4 + g of row li (the dots' A operand, rows li and 16 + li; the C tile's hi / lo)
  const int wg0 = lm_sw(grow, gch), wg1 = lm_sw(grow + 8, gch);
  const int wa0 = lm_sw(li, g), wa1 = lm_sw(li, 4 + g);
  const unsigned x8 = blockIdx.x & 7u;
  const long long ntiles_all = sh.B * sh.M * sh.L * (long long)sh.ntile;
  const QOrder qo = *reinterpret_cast<const QOrder*>(reinterpret_cast<const char*>(tiles + ntiles_all) +
                                                     kWinQOrderOffset);
  // the slots of XCD x8 (blocks p with p % 8 == x8 share one): level l (coarsest first) has
  // cl = ceil(B M nbl / 8) slots, slot i of it is block x8 cl + i of the level (none past its end)
  const int rs = sh.M * 64;  // grad_out / value row stride (elements)
  const int cq = qo.cs == 0 ? 1 : 0;  // (uniform) consecutive tiles

  const unsigned slot = blockIdx.x >> 3;
  f32x4 acc[4];
#pragma unroll
  for (int cb = 0; cb < 4; ++cb) acc[cb] = f32x4{0.f, 0.f, 0.f, 0.f};
  int Wl = 1, part = 0;  // waves of this wave's block and its rank among them
  int j = -1;            // (B M nblk < 2^31: checked by the host)
  int l = sh.L - 1;
  {
    {
      // the workgroups of XCD x8: level l (coarsest first) has cl = ceil(nu / 8) slots of its nu
      // workgroups (4 / W_l blocks each in split mode), slot i of it is workgroup x8 cl + i
      unsigned s = slot;
      for (; l >= 0; --l) {
        const int wl = NW > 1 ? sh.wsplit[l] : 1;
        const unsigned bpu = (unsigned)(NW / wl);
        const unsigned nl = (unsigned)sh.B * (unsigned)sh.M * (unsigned)(sh.blk0[l + 1] - sh.blk0[l]);
        const unsigned nu = (nl + bpu - 1u) / bpu;
        const unsigned cl = (nu + 7u) / 8u;
        if (s < cl) {
          const unsigned uu = x8 * cl + s;
          const unsigned jj = uu * bpu + (unsigned)(wid / wl);
          j = uu < nu && jj < nl ? (int)jj : -1;  // (past the level's end on this XCD: none)
          Wl = wl;
          part = wid % wl;
          break;
        }
        s -= cl;
      }
    }
    if (j >= 0) {
      const unsigned nbl = (unsigned)(sh.blk0[l + 1] - sh.blk0[l]);
      const unsigned bm = (unsigned)j / nbl;
      const int k = (int)((unsigned)j - bm * nbl);
      const int m = (int)(bm % (unsigned)sh.M);
      const long long b = bm / (unsigned)sh.M;
      const int T = sh.T[l];
      const int r0 = k * kRW;
      const uint16_t* __restrict__ vl = value + ((b * sh.S + sh.start[l]) * sh.M + m) * 64;
      const uint16_t* __restrict__ gb = gout + (b * sh.Lq * sh.M + m) * 64;
      const long long cbase = ((long long)bm * sh.L + l) * sh.Lq * P;  // level-major (b, m, l, q, p)
      const float* __restrict__ lt = loc + cbase;
      const float* __restrict__ at = aw + cbase;
      bf16x8 vb[2][2];  // the dots' B operands: value rows r0 + li and r0 + 16 (zeros past T)
#pragma unroll
      for (int cb = 0; cb < 2; ++cb) {
        const int x = r0 + (cb == 0 ? li : kRW);
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          uint4 v = make_uint4(0u, 0u, 0u, 0u);
          if (x < T) v = *reinterpret_cast<const uint4*>(vl + x * rs + ks * 32 + 8 * g);
          vb[cb][ks] = __builtin_bit_cast(bf16x8, v);
        }
      }
      const int2* __restrict__ tl = tiles + ((long long)bm * sh.L + l) * sh.ntile;
      auto chunk_mask = [&](int t0) -> unsigned long long {
        const int t = min(t0 + lane, sh.ntile - 1);
        const int2 iv = tl[t];
        return __ballot(t0 + lane < sh.ntile && iv.x <= r0 + kRW - 1 && iv.y >= r0);
      };
      int cur_t0 = 0;
      unsigned long long mask = chunk_mask(0);
      auto pop_tile = [&]() -> int {
        while (mask == 0ull) {
          cur_t0 += 64;
          if (cur_t0 >= sh.ntile) return -1;
          mask = chunk_mask(cur_t0);
        }
        const int t = cur_t0 + __builtin_ctzll(mask);
        mask &= mask - 1ull;
        return t;
      };
      bool first_pop = true;
      auto next_tile = [&]() -> int {  // this wave's visits: part, part + Wl, ... of the block's
        if constexpr (NW > 1) {
          const int skip = first_pop ? part : Wl - 1;
          first_pop = false;
          for (int i = 0; i < skip; ++i)
            if (pop_tile() < 0) return -1;
        }
        return pop_tile();
      };
      // the query of entry e of the tile order
      auto qry = [&](int e) -> int { return cq ? e : qo_query(qo, e); };

      float rl[SPL], ra[SPL];
      uint4 rg[4];
      auto fetch = [&](int tile) {
        const int q0 = tile * kQT;
        if (cq && q0 + kQT <= sh.Lq) {  // a whole tile of consecutive queries (uniform)
#pragma unroll
          for (int jj = 0; jj < SPL; ++jj) {
            const bool in = NS >= 64 || lane < NS;
            const int o = q0 * P + (in ? lane + 64 * jj : 0);
            rl[jj] = in ? lt[o] : 0.f;
            ra[jj] = in ? at[o] : 0.f;
          }
#pragma unroll
          for (int i = 0; i < 4; ++i)
            rg[i] = *reinterpret_cast<const uint4*>(gb + (q0 + grow + 8 * i) * rs + gch * 8);
        } else {
#pragma unroll
          for (int jj = 0; jj < SPL; ++jj) {
            const int s = lane + 64 * jj;
            const bool in = (NS >= 64 || lane < NS) && q0 + s / P < sh.Lq;
            const int o = in ? qry(q0 + s / P) * P + s % P : 0;
            rl[jj] = in ? lt[o] : 0.f;
            ra[jj] = in ? at[o] : 0.f;
          }
#pragma unroll
          for (int i = 0; i < 4; ++i)
            rg[i] = q0 + grow + 8 * i < sh.Lq
                        ? *reinterpret_cast<const uint4*>(gb + qry(q0 + grow + 8 * i) * rs + gch * 8)
                        : make_uint4(0u, 0u, 0u, 0u);
        }
      };
      int tile = next_tile();
      if (tile >= 0) fetch(tile);

      while (tile >= 0) {
        const int q0 = tile * kQT;
        // rows grow + 8 i: the swizzle of rows grow + 16 / grow + 24 is that of grow / grow + 8
        *reinterpret_cast<uint4*>(s_g + wg0) = rg[0];
        *reinterpret_cast<uint4*>(s_g + wg1) = rg[1];
        *reinterpret_cast<uint4*>(s_g + wg0 + 16 * kLmRow) = rg[2];
        *reinterpret_cast<uint4*>(s_g + wg1 + 16 * kLmRow) = rg[3];
        // 1. taps of the visit's samples (registers); the samples with a tap in the block's rows
        // compacted (ballot): position kp, coefficients split into bf16 hi / lo
        Taps tp[SPL];
        float a[SPL];
        int kp[SPL], dr[SPL];
        uint32_t ch[SPL], cl[SPL];
        int n = 0;
#pragma unroll
        for (int jj = 0; jj < SPL; ++jj) {
          const int s = lane + 64 * jj;
          const bool in = (NS >= 64 || lane < NS) && q0 + s / P < sh.Lq;
          tp[jj] = make_taps<ZEROS>(rl[jj], T);
          tp[jj].live = tp[jj].live && in;
          a[jj] = ra[jj];
          dr[jj] = tp[jj].base - r0;
          const bool sel = tp[jj].live && dr[jj] >= -1 && dr[jj] <= kRW - 1;
          const unsigned long long bal = __ballot(sel);
          const int below = (int)__builtin_amdgcn_mbcnt_hi((unsigned)(bal >> 32),
                                                           __builtin_amdgcn_mbcnt_lo((unsigned)bal, 0u));
          kp[jj] = sel ? n + below : -1;
          const float c0 = tp[jj].ok0 ? a[jj] * tp[jj].w0 : 0.f;
          const float c1 = tp[jj].ok1 ? a[jj] * tp[jj].w1 : 0.f;
          const uint32_t u0 = __float_as_uint(c0) & 0xffff0000u, u1 = __float_as_uint(c1) & 0xffff0000u;
          ch[jj] = __builtin_amdgcn_perm(u1, u0, 0x07060302u);
          cl[jj] = bf16_pair(c0 - __uint_as_float(u0), c1 - __uint_as_float(u1));
          if (sel) s_q[kp[jj]] = s / P;
          n += __popcll(bal);
        }
        const int nk = (n + 31) >> 5;
        if (lane < nk * 32 - n) s_q[n + lane] = 0;  // padding columns: C is zero there
        wave_lds_fence();
        if constexpr (COORDS) {
          // 2. dots of the tile's 32 queries with rows r0 .. r0+16 (MFMA, B operands in registers)
#pragma unroll
          for (int qh = 0; qh < 2; ++qh) {
            bf16x8 av[2];
#pragma unroll
            for (int ks = 0; ks < 2; ++ks)
              av[ks] = *reinterpret_cast<const bf16x8*>(s_g + (ks ? wa1 : wa0) + qh * 16 * kLmRow);
            f32x4 d[2];
#pragma unroll
            for (int cb = 0; cb < 2; ++cb) {
              d[cb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
              for (int ks = 0; ks < 2; ++ks)
                d[cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[ks], vb[cb][ks], d[cb], 0, 0, 0);
            }
            *reinterpret_cast<f32x4*>(s_cd + li * kDQS + qh * 16 + 4 * g) = d[0];
            if (li == 0) *reinterpret_cast<f32x4*>(s_cd + kRW * kDQS + qh * 16 + 4 * g) = d[1];
          }
          wave_lds_fence();
          // 3. coordinate gradients of the samples this block owns (base row in it; the level's
          // first block also owns the samples with no tap on the map)
#pragma unroll
          for (int jj = 0; jj < SPL; ++jj) {
            const int s = lane + 64 * jj;
            const bool in = (NS >= 64 || lane < NS) && q0 + s / P < sh.Lq;
            const Taps& t = tp[jj];
            const bool own = t.live ? (t.base >= r0 && t.base < r0 + kRW) || (t.base < 0 && k == 0) : k == 0;
            if (in && own) {
              const int qi = s / P;
              const int o = cq ? q0 * P + s : qry(q0 + qi) * P + s % P;
              const float d0 = t.ok0 ? s_cd[(t.base - r0) * kDQS + qi] : 0.f;
              const float d1 = t.ok1 ? s_cd[(t.base + 1 - r0) * kDQS + qi] : 0.f;
              if (gaw != nullptr) gaw[cbase + o] = d0 * t.w0 + d1 * t.w1;
              if (gloc != nullptr) gloc[cbase + o] = ((d1 - d0) * a[jj]) * t.gmul;
            }
          }
          wave_lds_fence();  // the dots' reads before C overwrites them
        }
        // the next visit's inputs, in flight during the grad_value steps
        const int next = next_tile();
        if (next >= 0) fetch(next);
        // 4. grad_value of the 16 rows += C . G, 32 compacted samples per MFMA step
        for (int ks = 0; ks < nk; ++ks) {
          {
            // 8 consecutive lanes zero one whole 128-B row (a ds_write_b128 bank group: 32 distinct
            // banks; two rows per group were a 2-way conflict in all 8 groups)
            uint4* z = reinterpret_cast<uint4*>(s_c + (lane >> 3) * kLmRow + (lane & 7) * 16);
            z[0] = make_uint4(0u, 0u, 0u, 0u);
            z[8 * kLmRow / 16] = make_uint4(0u, 0u, 0u, 0u);
          }
          wave_lds_fence();
#pragma unroll
          for (int jj = 0; jj < SPL; ++jj) {
            const int col = kp[jj] - 32 * ks;
            if (col >= 0 && col < 32) {
              const int cc = col >> 3, cw = (col & 7) * 2;
              if (dr[jj] >= 0) {
                *reinterpret_cast<uint16_t*>(s_c + lm_csw(dr[jj], cc) + cw) = (uint16_t)ch[jj];
                *reinterpret_cast<uint16_t*>(s_c + lm_csw(dr[jj], 4 + cc) + cw) = (uint16_t)cl[jj];
              }
              if (dr[jj] + 1 < kRW) {
                *reinterpret_cast<uint16_t*>(s_c + lm_csw(dr[jj] + 1, cc) + cw) = (uint16_t)(ch[jj] >> 16);
                *reinterpret_cast<uint16_t*>(s_c + lm_csw(dr[jj] + 1, 4 + cc) + cw) = (uint16_t)(cl[jj] >> 16);
              }
            }
          }
          wave_lds_fence();
          const bf16x8 ahi = *reinterpret_cast<const bf16x8*>(s_c + lm_csw(li, g));
          const bf16x8 alo = *reinterpret_cast<const bf16x8*>(s_c + lm_csw(li, 4 + g));
          const int qq = li >> 2, pp = li & 3;
          const int rowa = s_q[ks * 32 + 8 * g + qq], rowb = s_q[ks * 32 + 8 * g + 4 + qq];
#pragma unroll
          for (int cb = 0; cb < 4; ++cb) {
            const int c = 2 * cb + (pp >> 1), w8 = (pp & 1) * 8;
            const bf16x4 x0 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(s_g + lm_sw(rowa, c) + w8));
            const bf16x4 x1 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(s_g + lm_sw(rowb, c) + w8));
            const bf16x8 bv = __builtin_shufflevector(x0, x1, 0, 1, 2, 3, 4, 5, 6, 7);
            acc[cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ahi, bv, acc[cb], 0, 0, 0);
            acc[cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(alo, bv, acc[cb], 0, 0, 0);
          }
          wave_lds_fence();  // this step's C reads before the next step's zeroing
        }
        wave_lds_fence();  // this visit's LDS reads before the next visit's writes
        tile = next;
      }
    }
  }
  if constexpr (NW > 1) {
    // split blocks: waves 1 .. W_l - 1 of a block hand their partial sums to wave 0 through their own
    // (now idle) grad_out tile; the barriers are reached by every wave of the workgroup
    __syncthreads();
    if (j >= 0 && part > 0) {
#pragma unroll
      for (int cb = 0; cb < 4; ++cb) reinterpret_cast<f32x4*>(s_g)[cb * 64 + lane] = acc[cb];
    }
    __syncthreads();
    if (j >= 0 && part == 0) {
      for (int p = 1; p < Wl; ++p) {
#pragma unroll
        for (int cb = 0; cb < 4; ++cb) acc[cb] += reinterpret_cast<const f32x4*>(s_g_w[wid + p])[cb * 64 + lane];
      }
    }
  }
  // grad_value rows r0 + 4g + jj, channels 16 cb + li (every row of the block, zeros included)
  if (j >= 0 && part == 0 && gval != nullptr) {
    const int nbl = sh.blk0[l + 1] - sh.blk0[l];
    const unsigned bm = (unsigned)j / (unsigned)nbl;
    const int k = (int)((unsigned)j - bm * (unsigned)nbl);
    const int m = (int)(bm % (unsigned)sh.M);
    const long long b = bm / (unsigned)sh.M;
    const int T = sh.T[l];
    const int r0 = k * kRW;
    const int rs = sh.M * 64;
    uint16_t* __restrict__ gvl = gval + ((b * sh.S + sh.start[l]) * sh.M + m) * 64;
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
      const int x = r0 + 4 * g + jj;
      if (x < T) {
#pragma unroll
        for (int cb = 0; cb < 4; ++cb) gvl[x * rs + cb * 16 + li] = (uint16_t)bf16_bits(acc[cb][jj]);
      }
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Dense small-pyramid kernels (round 6): calls whose value pyramid has at most kDnMaxRows rows per
// (b, m) — configs[2]'s video queries on the audio pyramid (S = 95, Lq = 1920) and the audio
// self-attention (S = Lq = 95).  A 32-query tile's samples there touch about a third of the rows,
// so the sampling of a tile is a DENSE matrix C (queries x pyramid rows: each sample's aw * w at
// its two tap rows, the samples of one query on one row summed) and the call is small GEMMs on
// the matrix cores:
//   forward    out (q x 64) = C . V                    (V: the (b, m) pyramid, staged in LDS once)
//   backward   grad_value (rows x 64) += C^T . G       (G: the tile's grad_out rows)
//              dots D (rows x q) = V . G^T             grad_attn = w0 d0 + w1 d1,
//                                                      grad_loc = aw (d1 - d0) dy/dloc (two rows of D)
// instead of the row-block kernel's 8 waves per 16-row block that each stage every tile (all 60
// tiles meet each of the 8 blocks of the 95-row pyramid: 44 us, 1.49x its algorithmic bytes) and
// the gathering forward's 2 x 16 row fragments per query from L2 (34 us).
// C is built without atomics: thread (q, l) owns query q's coefficients on level l's rows (levels'
// rows never coincide), sums its 2P taps' coefficients per row in registers in sample order and
// stores each distinct row once as a bf16 hi + lo pair (|c - hi - lo| <= 2^-16 |c|, as
// win_lm_kernel), then clears what it stored once the products have read it.  Taps and weights
// are make_taps' (the other kernels' bit for bit); every grad_value row is written once, every
// coordinate gradient once: deterministic, no atomics.
// ---------------------------------------------------------------------------------------------
constexpr int kDnMaxRows = 128;  // pyramid rows per (b, m)
constexpr int kDnMaxL = 4;
constexpr int kDnSub = 2;        // backward: query tiles in flight per workgroup (4 waves each)
constexpr int kDnDQ = kQT + 4;   // backward dots: [row][q] floats, 16-B rows

struct DenseShape {
  long long B, S, M, Lq;
  int L, P;
  int R;  // rows rounded up to 32 (the MFMA K steps of the forward)
  int T[kDnMaxL], start[kDnMaxL];
  long long cb, cm;  // coordinate strides (coord_strides)
  int cq, cl;
  int ntile;         // backward: 32-query tiles
  int ngroup;        // backward: workgroups per (b, m) (query tiles dealt over them; > 1: partial sums)
  int nchunk;        // forward: query chunks per (b, m) of 64 wt queries (4 waves x wt 16-query tiles)
  int wt;            // forward: 16-query tiles a wave takes
  long long gvs;     // grad_value row stride (elements): M * 64, or a caller's strided slot
};

// the thread's P samples on one level: tap rows (row, row + 1) in the flattened pyramid and weights
template <int P>
struct DnTaps {
  int row[P];
  float w0[P], w1[P], a[P], gmul[P];
  bool ok0[P], ok1[P];
  int ivlo, ivhi;  // the rows the samples touch or own on their level (win_sample_rows: the tile intervals)
};

template <int P>
__device__ __forceinline__ void dn_load4(const float* __restrict__ p, float (&x)[P]) {
  if constexpr (P == 4) {
    const float4 v = *reinterpret_cast<const float4*>(p);
    x[0] = v.x; x[1] = v.y; x[2] = v.z; x[3] = v.w;
  } else if constexpr (P == 2) {
    const float2 v = *reinterpret_cast<const float2*>(p);
    x[0] = v.x; x[1] = v.y;
  } else {
    x[0] = p[0];
  }
}

template <int P>
__device__ __forceinline__ void dn_store4(float* __restrict__ p, const float (&x)[P]) {
  if constexpr (P == 4) {
    *reinterpret_cast<float4*>(p) = make_float4(x[0], x[1], x[2], x[3]);
  } else if constexpr (P == 2) {
    *reinterpret_cast<float2*>(p) = make_float2(x[0], x[1]);
  } else {
    p[0] = x[0];
  }
}

template <bool ZEROS, int P>
__device__ __forceinline__ void dn_taps(const float* __restrict__ lp, const float* __restrict__ ap, int T, int st,
                                        DnTaps<P>& tp) {
  float lc[P], ac[P];
  dn_load4<P>(lp, lc);
  dn_load4<P>(ap, ac);
  tp.ivlo = kNone;
  tp.ivhi = -kNone;
#pragma unroll
  for (int p = 0; p < P; ++p) {
    const int2 iv = win_sample_rows(lc[p], T, ZEROS);
    tp.ivlo = min(tp.ivlo, iv.x);
    tp.ivhi = max(tp.ivhi, iv.y);
    const Taps t = make_taps<ZEROS>(lc[p], T);
    tp.row[p] = st + t.base;
    tp.w0[p] = t.w0;
    tp.w1[p] = t.w1;
    tp.ok0[p] = t.ok0;
    tp.ok1[p] = t.ok1;
    tp.a[p] = ac[p];
    tp.gmul[p] = t.gmul;
  }
}

// the distinct rows of the thread's 2P taps with their summed coefficients (sample order), each
// handed to f(row, coefficient) once; clear(row) variants hand the same rows only
template <int P, typename F>
__device__ __forceinline__ void dn_rows(const DnTaps<P>& tp, F f) {
  int r[2 * P];
  float c[2 * P];
#pragma unroll
  for (int p = 0; p < P; ++p) {
    r[2 * p] = tp.ok0[p] ? tp.row[p] : -1;
    c[2 * p] = tp.ok0[p] ? tp.a[p] * tp.w0[p] : 0.f;
    r[2 * p + 1] = tp.ok1[p] ? tp.row[p] + 1 : -1;
    c[2 * p + 1] = tp.ok1[p] ? tp.a[p] * tp.w1[p] : 0.f;
  }
#pragma unroll
  for (int j = 0; j < 2 * P; ++j) {
    bool first = r[j] >= 0;
#pragma unroll
    for (int k = 0; k < j; ++k) first = first && r[k] != r[j];
    if (first) {
      float s = c[j];
#pragma unroll
      for (int k = j + 1; k < 2 * P; ++k) s += r[k] == r[j] ? c[k] : 0.f;
      f(r[j], s);
    }
  }
}

__device__ __forceinline__ uint16_t dn_hi(float c) { return (uint16_t)(__float_as_uint(c) >> 16); }
__device__ __forceinline__ uint16_t dn_lo(float c) {
  return __builtin_bit_cast(uint16_t, (__bf16)(c - __uint_as_float(__float_as_uint(c) & 0xffff0000u)));
}

// backward C tile: [row][32 queries] bf16, 64-B rows, 16-B chunk (8 queries) c at c ^ ((row >> 1) & 3):
// the A-operand reads (16 rows, one chunk) meet 16 distinct bank quads
__device__ __forceinline__ int dn_bc(int row, int q) {
  return row * 64 + ((((q >> 3) ^ (row >> 1)) & 3) << 4) + (q & 7) * 2;
}
// forward C tile: [16 queries][128 rows] bf16, 256-B rows, chunk (8 rows) c at c ^ (q & 7)
__device__ __forceinline__ int dn_fc(int q, int row) { return q * 256 + ((((row >> 3) ^ q) & 15) << 4) + (row & 7) * 2; }

// sh.ngroup workgroups per (b, m), kDnSub x 4 waves each: sub-group s of group r takes query tiles
// (r kDnSub + s) + i ngroup kDnSub; in a tile, threads (q, l) of the sub-group build C, wave w then owns
// row blocks w and w + 4 (16 rows each: grad_value += C^T G, dots D = V G^T), threads (q, l) write
// their coordinate gradients from D; at the end the sub-groups' grad_value partials meet in LDS in a
// fixed order, and with several groups each group's sum goes to `part` (fp32, group-major) for
// dense_sum_kernel to add in group order.
template <bool ZEROS, bool COORDS, int P>
__global__ __launch_bounds__(256 * kDnSub) void dense_bwd_kernel(
    const uint16_t* __restrict__ value, const float* __restrict__ loc, const float* __restrict__ aw,
    const uint16_t* __restrict__ gout, uint16_t* __restrict__ gval, float* __restrict__ gloc,
    float* __restrict__ gaw, float* __restrict__ gpart, const DenseShape sh) {
  extern __shared__ __attribute__((aligned(16))) unsigned char s_dyn[];
  const int R = sh.R, nrb = (int)((sh.S + 15) / 16);
  const int sub_bytes = kQT * kLmRow + 128 * R + 4 * kDnDQ * R;  // G | C hi, lo | D
  const int tid = (int)threadIdx.x, sub = tid >> 8, t = tid & 255, wave = t >> 6, lane = t & 63;
  const int g = lane >> 4, li = lane & 15;
  unsigned char* const s_g = s_dyn + sub * sub_bytes;
  unsigned char* const s_chi = s_g + kQT * kLmRow;
  unsigned char* const s_clo = s_chi + 64 * R;
  float* const s_d = reinterpret_cast<float*>(s_clo + 64 * R);
  const int grp = (int)(blockIdx.x % (unsigned)sh.ngroup);
  const unsigned bm = blockIdx.x / (unsigned)sh.ngroup;
  const int m = (int)(bm % (unsigned)sh.M);
  const long long b = bm / (unsigned)sh.M;
  const int rs = (int)sh.M * 64;  // value / grad_out row stride (elements)
  const uint16_t* __restrict__ vb = value + (b * sh.S * sh.M + m) * 64;
  const uint16_t* __restrict__ gb = gout + (b * sh.Lq * sh.M + m) * 64;
  const long long cbase = b * sh.cb + m * sh.cm;
  // the dots' B operands: value rows r0 + li of the wave's blocks (zeros past S)
  bf16x8 vr[2][2];
#pragma unroll
  for (int o = 0; o < 2; ++o) {
    const int x = (wave + 4 * o) * 16 + li;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      uint4 v = make_uint4(0u, 0u, 0u, 0u);
      if (x < sh.S) v = *reinterpret_cast<const uint4*>(vb + x * rs + ks * 32 + 8 * g);
      vr[o][ks] = __builtin_bit_cast(bf16x8, v);
    }
  }
  f32x4 acc[2][4];
#pragma unroll
  for (int o = 0; o < 2; ++o)
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) acc[o][cb] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int i = t; i < 128 * R / 16; i += 256) reinterpret_cast<uint4*>(s_chi)[i] = make_uint4(0u, 0u, 0u, 0u);
  __syncthreads();
  const int cqi = t >> 2, cli = t & 3;  // the C / coordinate thread's query in the tile and level
  const int span = kDnSub * sh.ngroup;  // tiles a round of every group's sub-groups takes
  const int nit = (sh.ntile + span - 1) / span;
  const int qq = li >> 2, pp = li & 3;
  for (int it = 0; it < nit; ++it) {
    const int tile = it * span + grp * kDnSub + sub;
    const int q0 = tile * kQT;
    {  // the tile's grad_out rows: one 16-B chunk a thread
      const int row = t >> 3, ch = t & 7, q = q0 + row;
      uint4 v = make_uint4(0u, 0u, 0u, 0u);
      if (tile < sh.ntile && q < sh.Lq) v = *reinterpret_cast<const uint4*>(gb + (long long)q * rs + ch * 8);
      *reinterpret_cast<uint4*>(s_g + lm_sw(row, ch)) = v;
    }
    const bool own = tile < sh.ntile && t < 4 * kQT && cli < sh.L && q0 + cqi < sh.Lq;
    const long long co = cbase + (long long)(q0 + cqi) * sh.cq + (long long)cli * sh.cl;
    if (own) {
      DnTaps<P> tp;
      dn_taps<ZEROS, P>(loc + co, aw + co, sh.T[cli], sh.start[cli], tp);
      dn_rows<P>(tp, [&](int r, float c) {
        *reinterpret_cast<uint16_t*>(s_chi + dn_bc(r, cqi)) = dn_hi(c);
        *reinterpret_cast<uint16_t*>(s_clo + dn_bc(r, cqi)) = dn_lo(c);
      });
    }
    __syncthreads();
#pragma unroll
    for (int o = 0; o < 2; ++o) {
      const int rb = wave + 4 * o;
      if (rb < nrb) {
        const int r0 = rb * 16;
        const bf16x8 ahi = *reinterpret_cast<const bf16x8*>(s_chi + dn_bc(r0 + li, 8 * g));
        const bf16x8 alo = *reinterpret_cast<const bf16x8*>(s_clo + dn_bc(r0 + li, 8 * g));
#pragma unroll
        for (int cb = 0; cb < 4; ++cb) {
          const int c = 2 * cb + (pp >> 1), w8 = (pp & 1) * 8;
          const bf16x4 x0 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(s_g + lm_sw(8 * g + qq, c) + w8));
          const bf16x4 x1 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(s_g + lm_sw(8 * g + 4 + qq, c) + w8));
          const bf16x8 bv = __builtin_shufflevector(x0, x1, 0, 1, 2, 3, 4, 5, 6, 7);
          acc[o][cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ahi, bv, acc[o][cb], 0, 0, 0);
          acc[o][cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(alo, bv, acc[o][cb], 0, 0, 0);
        }
        if constexpr (COORDS) {
#pragma unroll
          for (int qh = 0; qh < 2; ++qh) {
            const bf16x8 a0 = *reinterpret_cast<const bf16x8*>(s_g + lm_sw(li, g) + qh * 16 * kLmRow);
            const bf16x8 a1 = *reinterpret_cast<const bf16x8*>(s_g + lm_sw(li, 4 + g) + qh * 16 * kLmRow);
            f32x4 d = f32x4{0.f, 0.f, 0.f, 0.f};
            d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, vr[o][0], d, 0, 0, 0);
            d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, vr[o][1], d, 0, 0, 0);
            *reinterpret_cast<f32x4*>(s_d + (r0 + li) * kDnDQ + qh * 16 + 4 * g) = d;  // rows r0 + li, queries 4g..
          }
        }
      }
    }
    __syncthreads();
    if (own) {
      DnTaps<P> tp;  // (re-read: not held in registers across the products)
      dn_taps<ZEROS, P>(loc + co, aw + co, sh.T[cli], sh.start[cli], tp);
      if constexpr (COORDS) {
        float ga[P], gl[P];
#pragma unroll
        for (int p = 0; p < P; ++p) {
          const float d0 = tp.ok0[p] ? s_d[tp.row[p] * kDnDQ + cqi] : 0.f;
          const float d1 = tp.ok1[p] ? s_d[(tp.row[p] + 1) * kDnDQ + cqi] : 0.f;
          ga[p] = d0 * tp.w0[p] + d1 * tp.w1[p];
          gl[p] = ((d1 - d0) * tp.a[p]) * tp.gmul[p];
        }
        if (gaw != nullptr) dn_store4<P>(gaw + co, ga);
        if (gloc != nullptr) dn_store4<P>(gloc + co, gl);
      }
      // clear this tile's coefficients (the next tile's threads write other entries)
      dn_rows<P>(tp, [&](int r, float) {
        *reinterpret_cast<uint16_t*>(s_chi + dn_bc(r, cqi)) = 0;
        *reinterpret_cast<uint16_t*>(s_clo + dn_bc(r, cqi)) = 0;
      });
    }
    __syncthreads();
  }
  // the sub-groups' partial sums: 1..kDnSub-1 through LDS, added to sub-group 0's in order
  f32x4* const part = reinterpret_cast<f32x4*>(s_dyn);
  if (sub > 0) {
#pragma unroll
    for (int o = 0; o < 2; ++o)
#pragma unroll
      for (int cb = 0; cb < 4; ++cb) part[((((sub - 1) * 4 + wave) * 2 + o) * 4 + cb) * 64 + lane] = acc[o][cb];
  }
  __syncthreads();
  if (sub == 0 && gval != nullptr) {
    uint16_t* __restrict__ gv = gval + b * sh.S * sh.gvs + m * 64;
    // (several groups: this group's fp32 sum, rows [0, R) x 64 channels)
    float* __restrict__ gp = gpart + ((long long)bm * sh.ngroup + grp) * sh.R * 64;
#pragma unroll
    for (int o = 0; o < 2; ++o) {
      const int rb = wave + 4 * o;
      if (rb >= nrb) continue;
#pragma unroll
      for (int cb = 0; cb < 4; ++cb) {
        f32x4 s = acc[o][cb];
        for (int u = 1; u < kDnSub; ++u) s += part[((((u - 1) * 4 + wave) * 2 + o) * 4 + cb) * 64 + lane];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int x = rb * 16 + 4 * g + j;
          if (x < sh.S) {
            if (sh.ngroup > 1) gp[x * 64 + cb * 16 + li] = s[j];
            else gv[(long long)x * sh.gvs + cb * 16 + li] = (uint16_t)bf16_bits(s[j]);
          }
        }
      }
    }
  }
}

// grad_value rows of the (b, m) pairs as the sum of their groups' fp32 partials in group order (one
// thread a 4-channel piece of a row); bf16 out
__global__ __launch_bounds__(256) void dense_sum_kernel(const float* __restrict__ gpart, uint16_t* __restrict__ gval,
                                                        const DenseShape sh) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;  // (bm, row, 4-channel piece)
  const long long n = sh.B * sh.M * sh.S * 16;
  if (i >= n) return;
  const int pc = (int)(i & 15);
  const long long br = i >> 4;
  const int row = (int)(br % sh.S);
  const long long bm = br / sh.S;
  const int m = (int)(bm % sh.M);
  const long long b = bm / sh.M;
  const float4* __restrict__ src = reinterpret_cast<const float4*>(gpart + bm * sh.ngroup * sh.R * 64 + row * 64) + pc;
  float4 s = src[0];
  // the groups 8 at a time: loads issued together (branch-free: an index past the end re-reads the
  // last group and is not added), added in group order — one dependent load a group cost ~5 us a call
  for (int r = 1; r < sh.ngroup; r += 8) {
    float4 t[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) t[u] = src[(long long)min(r + u, sh.ngroup - 1) * sh.R * 16];
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (r + u < sh.ngroup) {
        s.x += t[u].x; s.y += t[u].y; s.z += t[u].z; s.w += t[u].w;
      }
  }
  uint2 o;
  o.x = (uint32_t)(uint16_t)bf16_bits(s.x) | ((uint32_t)(uint16_t)bf16_bits(s.y) << 16);
  o.y = (uint32_t)(uint16_t)bf16_bits(s.z) | ((uint32_t)(uint16_t)bf16_bits(s.w) << 16);
  *reinterpret_cast<uint2*>(gval + (b * sh.S + row) * sh.gvs + m * 64 + pc * 4) = o;
}

// One workgroup per (b, m, 128-query chunk), 4 waves: the (b, m) pyramid staged in LDS once (128-B
// rows, lm_sw), then each wave takes 16-query tiles: threads (q, l) build the tile's C, then
// out = C . V over the pyramid's rows in 32-row MFMA steps (B operands read transposed).
// With `tiles` (the level-major calls' buffer, msda_hip_forward_tiles_bytes) it also writes the row
// intervals of every (b, m, level, 32-query tile) and the buffer's tail as msda_fwd16_tiles_kernel
// does for consecutive tiles (win_sample_rows, zero tail), so the buffer is defined whichever backward
// later reads it.
template <bool ZEROS, int P>
__global__ __launch_bounds__(256) void dense_fwd_kernel(const uint16_t* __restrict__ value,
                                                        const float* __restrict__ loc,
                                                        const float* __restrict__ aw, uint16_t* __restrict__ out,
                                                        int2* __restrict__ tiles, const DenseShape sh) {
  extern __shared__ __attribute__((aligned(16))) unsigned char s_dyn[];
  __shared__ int2 s_iv[4][kDnMaxL];
  const int R = sh.R;
  const int tid = (int)threadIdx.x, wave = tid >> 6, lane = tid & 63, g = lane >> 4, li = lane & 15;
  unsigned char* const s_v = s_dyn;
  unsigned char* const s_chi = s_dyn + R * kLmRow + wave * (2 * 16 * 256);
  unsigned char* const s_clo = s_chi + 16 * 256;
  const unsigned chunk = blockIdx.x % (unsigned)sh.nchunk;  // (of 64 sh.wt queries)
  const unsigned bm = blockIdx.x / (unsigned)sh.nchunk;
  const int m = (int)(bm % (unsigned)sh.M);
  const long long b = bm / (unsigned)sh.M;
  const int rs = (int)sh.M * 64;
  const uint16_t* __restrict__ vb = value + (b * sh.S * sh.M + m) * 64;
  if (tiles != nullptr && blockIdx.x == 0 && tid < (int)(kWinTailBytes / 16))  // the tail: zero (consecutive tiles)
    reinterpret_cast<uint4*>(tiles + sh.B * sh.M * sh.L * sh.ntile)[tid] = make_uint4(0u, 0u, 0u, 0u);
  for (int i = tid; i < R * 8; i += 256) {
    const int row = i >> 3, ch = i & 7;
    uint4 v = make_uint4(0u, 0u, 0u, 0u);
    if (row < sh.S) v = *reinterpret_cast<const uint4*>(vb + row * rs + ch * 8);
    *reinterpret_cast<uint4*>(s_v + lm_sw(row, ch)) = v;
  }
  for (int i = lane; i < 2 * 16 * 256 / 16; i += 64) reinterpret_cast<uint4*>(s_chi)[i] = make_uint4(0u, 0u, 0u, 0u);
  __syncthreads();
  const int cqi = lane >> 2, cli = lane & 3;
  const int qq = li >> 2, pp = li & 3;
  const long long cbase = b * sh.cb + m * sh.cm;
  for (int wt = 0; wt < sh.wt; ++wt) {
    const int q0 = ((int)chunk * sh.wt + wt) * 64 + wave * 16;
    const bool own = cli < sh.L && q0 + cqi < sh.Lq;
    DnTaps<P> tp;
    tp.ivlo = kNone;
    tp.ivhi = -kNone;
    if (own) {
      const long long co = cbase + (long long)(q0 + cqi) * sh.cq + (long long)cli * sh.cl;
      dn_taps<ZEROS, P>(loc + co, aw + co, sh.T[cli], sh.start[cli], tp);
      dn_rows<P>(tp, [&](int r, float c) {
        *reinterpret_cast<uint16_t*>(s_chi + dn_fc(cqi, r)) = dn_hi(c);
        *reinterpret_cast<uint16_t*>(s_clo + dn_fc(cqi, r)) = dn_lo(c);
      });
    }
    if (tiles != nullptr) {
      // the wave's 16 queries' intervals per level (lanes q * 4 + l), then the two waves of a 32-query
      // tile combined through LDS (the barriers: every wave runs every wt)
      int lo = tp.ivlo, hi = tp.ivhi;
#pragma unroll
      for (int o = 4; o < 64; o <<= 1) {
        lo = min(lo, __shfl_xor(lo, o));
        hi = max(hi, __shfl_xor(hi, o));
      }
      if (lane < kDnMaxL) s_iv[wave][lane] = make_int2(lo, hi);
      __syncthreads();
      const int tile = q0 / kQT;
      if ((wave & 1) == 0 && lane < sh.L && tile < sh.ntile) {
        const int2 o = s_iv[wave + 1][lane];
        tiles[((long long)bm * sh.L + lane) * sh.ntile + tile] = make_int2(min(lo, o.x), max(hi, o.y));
      }
      __syncthreads();
    }
    if (q0 >= sh.Lq) continue;  // (wave-uniform: no products for a tile past the queries)
    wave_lds_fence();
    f32x4 acc[4];
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) acc[cb] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int ks = 0; ks < R / 32; ++ks) {
      const bf16x8 ahi = *reinterpret_cast<const bf16x8*>(s_chi + dn_fc(li, ks * 32 + 8 * g));
      const bf16x8 alo = *reinterpret_cast<const bf16x8*>(s_clo + dn_fc(li, ks * 32 + 8 * g));
#pragma unroll
      for (int cb = 0; cb < 4; ++cb) {
        const int c = 2 * cb + (pp >> 1), w8 = (pp & 1) * 8;
        const bf16x4 x0 =
            __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(s_v + lm_sw(ks * 32 + 8 * g + qq, c) + w8));
        const bf16x4 x1 =
            __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(s_v + lm_sw(ks * 32 + 8 * g + 4 + qq, c) + w8));
        const bf16x8 bv = __builtin_shufflevector(x0, x1, 0, 1, 2, 3, 4, 5, 6, 7);
        acc[cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ahi, bv, acc[cb], 0, 0, 0);
        acc[cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(alo, bv, acc[cb], 0, 0, 0);
      }
    }
    wave_lds_fence();  // the products' C reads before the clears
    if (own) {
      dn_rows<P>(tp, [&](int r, float) {
        *reinterpret_cast<uint16_t*>(s_chi + dn_fc(cqi, r)) = 0;
        *reinterpret_cast<uint16_t*>(s_clo + dn_fc(cqi, r)) = 0;
      });
    }
    // out rows q0 + 4g + j, channels 16 cb + li
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int q = q0 + 4 * g + j;
      if (q < sh.Lq) {
        uint16_t* __restrict__ op = out + ((b * sh.Lq + q) * sh.M + m) * 64;
#pragma unroll
        for (int cb = 0; cb < 4; ++cb) op[cb * 16 + li] = (uint16_t)bf16_bits(acc[cb][j]);
      }
    }
    wave_lds_fence();  // the clears before the next tile's stores
  }
}
}  // namespace

// the dense kernels' LDS (bytes): backward per workgroup, forward per workgroup
// (backward: the sub-groups' tiles, or the partial sums they add at the end, whichever is larger)
static size_t dense_bwd_lds(int R) {
  const size_t tiles = (size_t)kDnSub * (kQT * kLmRow + 128 * R + 4 * kDnDQ * R);
  const size_t parts = (size_t)(kDnSub - 1) * 4 * 2 * 4 * 64 * 16;
  return tiles > parts ? tiles : parts;
}
static size_t dense_fwd_lds(int R) { return (size_t)R * kLmRow + 4 * 2 * 16 * 256; }

int msda_dense_supported(int value_dtype_is_bf16, long long D, long long S, long long L, long long P) {
  const char* e = getenv("MSDA_HIP_DENSE");
  if (e != nullptr && atoi(e) == 0) return 0;
  return value_dtype_is_bf16 && D == 64 && S >= 1 && S <= kDnMaxRows && L >= 1 && L <= kDnMaxL &&
         (P == 1 || P == 2 || P == 4);
}

static bool dense_shape(const WinShape* in, int coord_layout, DenseShape& sh) {
  sh.B = in->B; sh.S = in->S; sh.M = in->M; sh.Lq = in->Lq;
  sh.L = in->L; sh.P = in->P;
  if (sh.L < 1 || sh.L > kDnMaxL || sh.S > kDnMaxRows || sh.S * sh.M * 64 >= (1LL << 31) ||
      sh.Lq * sh.M * 64 >= (1LL << 31))
    return false;
  for (int l = 0; l < sh.L; ++l) {
    sh.T[l] = in->T[l];
    sh.start[l] = in->start[l];
  }
  sh.R = (int)((sh.S + 31) / 32) * 32;
  const CoordStrides cs = coord_strides(coord_layout, sh.Lq, sh.M, sh.L, sh.P);
  sh.cb = cs.cb; sh.cm = cs.cm; sh.cq = cs.cq; sh.cl = cs.cl;
  sh.ntile = (int)((sh.Lq + kQT - 1) / kQT);
  sh.ngroup = 1;
  // forward chunks: 128 queries a workgroup on long query sets, 64 on short ones (the audio self-
  // attention's 95 queries: 2 workgroups a (b, m) instead of one)
  sh.wt = sh.Lq >= 1024 ? 2 : 1;
  sh.nchunk = (int)((sh.Lq + 64 * sh.wt - 1) / (64 * sh.wt));
  sh.gvs = in->gv_rs > 0 ? in->gv_rs : sh.M * 64;
  return true;
}

// workgroups per (b, m) of the dense backward: about 512 workgroups over the chip, at least one
// tile a sub-group
static int dense_groups(long long B, long long M, long long Lq) {
  const long long ntile = (Lq + kQT - 1) / kQT;
  long long ng = (512 + B * M - 1) / max(1LL, B * M);
  ng = min(ng, (ntile + kDnSub - 1) / kDnSub);
  return (int)max(1LL, min(ng, 64LL));
}

size_t msda_dense_workspace_bytes(long long B, long long S, long long M, long long Lq) {
  const int ng = dense_groups(B, M, Lq);
  if (ng <= 1) return 0;
  const long long R = (S + 31) / 32 * 32;
  return (size_t)(B * M * ng * R * 64) * sizeof(float);
}

template <typename K>
static int dense_lds_attr(K kernel, size_t bytes) {
  if (bytes <= 64 * 1024) return 0;
  return hipFuncSetAttribute(reinterpret_cast<const void*>(kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                             (int)bytes) == hipSuccess
             ? 0
             : -1;
}

int msda_dense_forward(const void* value, const void* loc, const void* aw, void* out, void* tiles,
                       const WinShape* shape, int zeros, int coord_layout, hipStream_t st) {
  DenseShape sh{};
  if (!dense_shape(shape, coord_layout, sh)) return -1;
  if (sh.B * sh.M == 0 || sh.Lq == 0) return 0;
  const unsigned grid = (unsigned)(sh.B * sh.M * sh.nchunk);
  const size_t lds = dense_fwd_lds(sh.R);
  auto* v = static_cast<const uint16_t*>(value);
  auto* lc = static_cast<const float*>(loc);
  auto* a = static_cast<const float*>(aw);
  auto* o = static_cast<uint16_t*>(out);
  auto* tl = static_cast<int2*>(tiles);
#define DN_FWD(Z, PP)                                                                                   \
  do {                                                                                                  \
    if (dense_lds_attr(dense_fwd_kernel<Z, PP>, lds)) return -1;                                        \
    hipLaunchKernelGGL((dense_fwd_kernel<Z, PP>), dim3(grid), dim3(256), lds, st, v, lc, a, o, tl, sh);  \
  } while (0)
#define DN_FWD_P(Z)                     \
  switch (sh.P) {                       \
    case 1: DN_FWD(Z, 1); break;        \
    case 2: DN_FWD(Z, 2); break;        \
    default: DN_FWD(Z, 4); break;       \
  }
  if (zeros) { DN_FWD_P(true) } else { DN_FWD_P(false) }
#undef DN_FWD_P
#undef DN_FWD
  return 0;
}

int msda_dense_backward(const void* value, const void* loc, const void* aw, const void* gout, void* gval, void* gloc,
                        void* gaw, void* workspace, const WinShape* shape, int zeros, int coord_layout,
                        hipStream_t st) {
  DenseShape sh{};
  if (!dense_shape(shape, coord_layout, sh)) return -1;
  if (sh.B * sh.M == 0) return 0;
  // several workgroups per (b, m) when the caller handed the partial sums' workspace
  // (msda_dense_workspace_bytes; one workgroup a (b, m) writes grad_value directly otherwise)
  if (workspace != nullptr && gval != nullptr) sh.ngroup = dense_groups(sh.B, sh.M, sh.Lq);
  auto* gp = static_cast<float*>(workspace);
  const unsigned grid = (unsigned)(sh.B * sh.M * sh.ngroup);
  const size_t lds = dense_bwd_lds(sh.R);
  const bool coords = gloc != nullptr || gaw != nullptr;
  auto* v = static_cast<const uint16_t*>(value);
  auto* lc = static_cast<const float*>(loc);
  auto* a = static_cast<const float*>(aw);
  auto* g = static_cast<const uint16_t*>(gout);
  auto* gv = static_cast<uint16_t*>(gval);
  auto* gl = static_cast<float*>(gloc);
  auto* ga = static_cast<float*>(gaw);
#define DN_BWD(Z, C, PP)                                                                                 \
  do {                                                                                                   \
    if (dense_lds_attr(dense_bwd_kernel<Z, C, PP>, lds)) return -1;                                      \
    hipLaunchKernelGGL((dense_bwd_kernel<Z, C, PP>), dim3(grid), dim3(256 * kDnSub), lds, st, v, lc, a, g, gv, gl, \
                       ga, gp, sh);                                                                      \
  } while (0)
#define DN_BWD_P(Z, C)                  \
  switch (sh.P) {                       \
    case 1: DN_BWD(Z, C, 1); break;     \
    case 2: DN_BWD(Z, C, 2); break;     \
    default: DN_BWD(Z, C, 4); break;    \
  }
  if (zeros) {
    if (coords) { DN_BWD_P(true, true) } else { DN_BWD_P(true, false) }
  } else {
    if (coords) { DN_BWD_P(false, true) } else { DN_BWD_P(false, false) }
  }
#undef DN_BWD_P
#undef DN_BWD
  if (sh.ngroup > 1) {
    const long long n = sh.B * sh.M * sh.S * 16;
    hipLaunchKernelGGL(dense_sum_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, gp, gv, sh);
  }
  return 0;
}

size_t msda_win_workspace_bytes(long long B, long long M, long long L, long long Lq) {
  const long long ntile = (Lq + kQT - 1) / kQT;
  return (size_t)(B * M * L * ntile) * sizeof(int2) + kWinTailBytes;
}

int msda_win_supported(int value_dtype_is_bf16, long long D, long long P, long long Lq, long long row_floats) {
  // row_floats = M * L * P: one query's coordinates, read by the prepass in kRowRegs x 64 lanes
  return value_dtype_is_bf16 && D == 64 && (P == 1 || P == 2 || P == 4 || P == 8) && Lq < (1LL << 24) &&
         row_floats <= 64 * kRowRegs;
}

// The position-chunk dispatch order of win_bwd_kernel: chunks of the level with the fewest
// blocks (one of its blocks each), every level's blocks split evenly over them.  Returns false
// (coarsest-level-first order) when the table does not fit WinShape.
static bool win_chunk_order(WinShape& sh) {
  sh.nchunk = 0;
  int C = 1 << 30;
  for (int l = 0; l < sh.L; ++l) C = min(C, sh.blk0[l + 1] - sh.blk0[l]);
  if (C < 1 || C > kWinMaxChunks || sh.nblk > kWinMaxSeq) return false;
  int n = 0;
  for (int c = 0; c < C; ++c) {
    sh.cs[c] = (unsigned short)n;
    for (int l = sh.L - 1; l >= 0; --l) {
      const int nb = sh.blk0[l + 1] - sh.blk0[l];
      if (nb > 4096) return false;
      for (int k = (int)((long long)c * nb / C); k < (int)((long long)(c + 1) * nb / C); ++k)
        sh.seq[n++] = (unsigned short)(l << 12 | k);
    }
  }
  sh.cs[C] = (unsigned short)n;
  sh.nchunk = C;
  sh.ppx = (int)((sh.B * sh.M + 7) / 8);
  return n == sh.nblk;
}

int msda_win_backward(const void* value, const void* loc, const void* aw, const void* gout, void* gval,
                      void* gloc, void* gaw, void* workspace, const void* tiles_ready, const WinShape* shape,
                      int zeros, int coord_layout, hipStream_t st) {
  WinShape sh = *shape;
  // profiling only: MSDA_HIP_WIN_EXP skips parts of the kernel (the results are WRONG), so it is
  // honoured only together with MSDA_HIP_PROFILING=1 (tools/win_exp.py); alone it is an error, never
  // silently wrong gradients in training
  const char* xe = getenv("MSDA_HIP_WIN_EXP");
  sh.exp = xe ? atoi(xe) : 0;
  if (sh.exp != 0) {
    const char* pe = getenv("MSDA_HIP_PROFILING");
    if (pe == nullptr || atoi(pe) != 1) return -2;
  }
  sh.qo_dev = tiles_ready != nullptr ? 1 : 0;
  // (the interval prepass reads whole query rows: the reference layout; level-major calls bring
  // the forward's intervals)
  if (coord_layout != 0 && tiles_ready == nullptr) return -1;
  const CoordStrides cs = coord_strides(coord_layout, sh.Lq, sh.M, sh.L, sh.P);
  sh.cb = cs.cb; sh.cm = cs.cm; sh.cq = cs.cq; sh.cl = cs.cl;
  sh.ntile = (int)((sh.Lq + kQT - 1) / kQT);
  int nb = 0;
  for (int l = 0; l < sh.L; ++l) {
    sh.blk0[l] = nb;
    nb += (sh.T[l] + kRW - 1) / kRW;
  }
  sh.blk0[sh.L] = nb;
  sh.nblk = nb;
  if (sh.B * sh.M == 0 || nb == 0) return 0;
  const long long nblocks = sh.B * sh.M * (long long)nb;
  // the level-major row kernel (win_lm_kernel): the forward's tiles (and their tail: the query
  // order), many blocks (one wave each), 32-bit element offsets within a clip
  // (MSDA_HIP_WIN_LM=0: the per-block kernel, for A/B)
  const char* lme = getenv("MSDA_HIP_WIN_LM");
  const bool lm_kernel = coord_layout == 1 && tiles_ready != nullptr && nblocks > 4096 && sh.P <= 4 &&
                         (lme == nullptr || atoi(lme) != 0) && sh.Lq * sh.M * 64 < (1LL << 31) &&
                         sh.S * sh.M * 64 < (1LL << 31) && sh.L * sh.Lq * sh.P < (1LL << 31) && nblocks < (1LL << 31) &&
                         sh.exp == 0 && getenv("MSDA_HIP_WIN_SPLIT") == nullptr;
  // position-chunk order where the blocks are many (T = 4096: 3,840 an XCD; 245 -> 219 us at the
  // configs[3] call), coarsest-level-first where they are few and the longest blocks set the tail
  // (T = 1024: 960 an XCD; 55 against 64 us, tools/win_tiles_ab.py).  MSDA_HIP_WIN_ORDER: 0 / 1 forces.
  const char* oe = getenv("MSDA_HIP_WIN_ORDER");
  const int order_env = oe ? atoi(oe) : -1;
  if (lm_kernel) {
    sh.qo_dev = 1;
    sh.exp = 0;
    // split mode (4-wave workgroups, MSDA_HIP_WIN_LM_SPLIT=1; measured slower, so opt-in): a level
    // with a quarter / an eighth of the finest level's rows gets 2 / 4 waves a block (its blocks meet
    // 2-3x the query tiles).  Bench encoder call (tools/msda_microbench.py, r06l): 56.4 / 61.2 us
    // (init / trained sampling) against 49.4 / 54.8 with one wave a block — the coarse blocks are not
    // the kernel's critical path; the split adds waves, barriers and the partial-sum exchange
    const char* spe = getenv("MSDA_HIP_WIN_LM_SPLIT");
    int tmax = 1;
    for (int l = 0; l < sh.L; ++l) tmax = max(tmax, sh.T[l]);
    bool split = false;
    for (int l = 0; l < sh.L; ++l) {
      const int ratio = tmax / max(1, sh.T[l]);
      sh.wsplit[l] = ratio >= 8 ? 4 : ratio >= 4 ? 2 : 1;
      split = split || sh.wsplit[l] > 1;
    }
    if (spe == nullptr || atoi(spe) != 1) split = false;
    const int nw = split ? 4 : 1;
    unsigned nsx = 0;
    for (int l = 0; l < sh.L; ++l) {
      const long long bpu = split ? 4 / sh.wsplit[l] : 1;
      const long long nu = (sh.B * sh.M * (sh.blk0[l + 1] - sh.blk0[l]) + bpu - 1) / bpu;
      nsx += (unsigned)((nu + 7) / 8);
    }
    auto* tl = static_cast<const int2*>(tiles_ready);
    const bool coords = gloc != nullptr || gaw != nullptr;
    auto* v = static_cast<const uint16_t*>(value);
    auto* lc = static_cast<const float*>(loc);
    auto* a = static_cast<const float*>(aw);
    auto* g = static_cast<const uint16_t*>(gout);
    auto* gv = static_cast<uint16_t*>(gval);
    auto* gl = static_cast<float*>(gloc);
    auto* ga = static_cast<float*>(gaw);
#define WIN_LM(Z, C, N)                                                                                      \
  do {                                                                                                       \
    if (nw == 4)                                                                                             \
      hipLaunchKernelGGL((win_lm_kernel<Z, C, N, 4>), dim3(8u * nsx), dim3(256), 0, st, v, lc, a, g, gv, gl, ga, tl, sh); \
    else                                                                                                     \
      hipLaunchKernelGGL((win_lm_kernel<Z, C, N, 1>), dim3(8u * nsx), dim3(64), 0, st, v, lc, a, g, gv, gl, ga, tl, sh); \
  } while (0)
#define WIN_LM_P(Z, C)                                                  \
  do {                                                                  \
    switch (sh.P) {                                                     \
      case 1: WIN_LM(Z, C, 1); break;                                   \
      case 2: WIN_LM(Z, C, 2); break;                                   \
      default: WIN_LM(Z, C, 4); break;                                  \
    }                                                                   \
  } while (0)
    if (zeros) {
      if (coords) WIN_LM_P(true, true); else WIN_LM_P(true, false);
    } else {
      if (coords) WIN_LM_P(false, true); else WIN_LM_P(false, false);
    }
#undef WIN_LM_P
#undef WIN_LM
    return 0;
  }
  const bool chunked = win_chunk_order(sh) &&
                       (order_env == 1 || (order_env != 0 && (long long)sh.ppx * sh.nblk >= 2048));
  if (!chunked) sh.nchunk = 0;
  // tile intervals: written by the forward (msda_fwd16_tiles_kernel) or by the prepass below
  auto* tiles = static_cast<int2*>(tiles_ready != nullptr ? const_cast<void*>(tiles_ready) : workspace);
  const unsigned tile_wgs = tiles_ready != nullptr ? 0u : (unsigned)(sh.B * sh.ntile);
  const int nj = (int)((sh.M * sh.L * sh.P + 63) / 64);
  auto* lc0 = static_cast<const float*>(loc);
#define WIN_TILES(Z, NJ) hipLaunchKernelGGL((win_tiles_kernel<Z, NJ>), dim3(tile_wgs), dim3(kThreads), 0, st, lc0, tiles, sh)
#define WIN_TILES_NJ(Z)                                              \
  do {                                                               \
    if (nj <= 1) WIN_TILES(Z, 1);                                    \
    else if (nj <= 2) WIN_TILES(Z, 2);                               \
    else if (nj <= 4) WIN_TILES(Z, 4);                               \
    else WIN_TILES(Z, 8);                                            \
  } while (0)
  if (tile_wgs > 0) {
    if (zeros) WIN_TILES_NJ(true); else WIN_TILES_NJ(false);
  }
#undef WIN_TILES_NJ
#undef WIN_TILES
  unsigned grid = 0;  // 8 x per-XCD slots (see win_bwd_kernel's dispatch order)
  if (sh.nchunk > 0)
    grid = 8u * (unsigned)sh.ppx * (unsigned)sh.nblk;
  else
    for (int l = 0; l < sh.L; ++l) grid += 8u * (unsigned)((sh.B * sh.M * (sh.blk0[l + 1] - sh.blk0[l]) + 7) / 8);
  const bool coords = gloc != nullptr || gaw != nullptr;
  auto* v = static_cast<const uint16_t*>(value);
  auto* lc = static_cast<const float*>(loc);
  auto* a = static_cast<const float*>(aw);
  auto* g = static_cast<const uint16_t*>(gout);
  auto* gv = static_cast<uint16_t*>(gval);
  auto* gl = static_cast<float*>(gloc);
  auto* ga = static_cast<float*>(gaw);
  // waves per row block: enough waves for the chip when the blocks are few (MSDA_HIP_WIN_SPLIT
  // forces 1 / 4 / 8)
  int W = nblocks <= 1024 ? 8 : nblocks <= 4096 ? 4 : 1;
  if (const char* e = getenv("MSDA_HIP_WIN_SPLIT")) {
    const int f = atoi(e);
    if (f == 1 || f == 4 || f == 8) W = f;
  }
#define WIN_LAUNCH_W(Z, C, N, WW) \
  hipLaunchKernelGGL((win_bwd_kernel<Z, C, N, WW>), dim3(grid), dim3(64 * WW), 0, st, v, lc, a, g, gv, gl, ga, tiles, sh)
#define WIN_LAUNCH(Z, C, N)                                             \
  do {                                                                  \
    if (W == 8) WIN_LAUNCH_W(Z, C, N, 8);                               \
    else if (W == 4) WIN_LAUNCH_W(Z, C, N, 4);                          \
    else WIN_LAUNCH_W(Z, C, N, 1);                                      \
  } while (0)
#define WIN_SPL(Z, C)                                                   \
  do {                                                                  \
    switch (sh.P) {                                                     \
      case 1: WIN_LAUNCH(Z, C, 1); break;                               \
      case 2: WIN_LAUNCH(Z, C, 2); break;                               \
      case 4: WIN_LAUNCH(Z, C, 4); break;                               \
      default: WIN_LAUNCH(Z, C, 8); break;                              \
    }                                                                   \
  } while (0)
  if (zeros) {
    if (coords) WIN_SPL(true, true); else WIN_SPL(true, false);
  } else {
    if (coords) WIN_SPL(false, true); else WIN_SPL(false, false);
  }
#undef WIN_SPL
#undef WIN_LAUNCH
#undef WIN_LAUNCH_W
  return 0;  // launch errors: the caller's hipGetLastError
}
