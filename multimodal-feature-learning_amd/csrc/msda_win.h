// Internal interface between msda.hip (dispatch, workspace sizing) and msda_win.hip (the
// row-block MFMA backward for 16-bit values, D = 64).  Not part of the public C-ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdlib.h>

// Query order of the row-block backward's tiles.  A tile is 32 queries; by default 32 consecutive
// ones.  In an encoder self-attention call (Lq == S: the queries are the pyramid's tokens, level
// by level) a tile of consecutive queries of a coarse level spans a large stretch of every finer
// level (32 level-3 tokens of a 1024/512/256/128 pyramid: a quarter of level 0), so the row blocks
// there each meet many tiles holding few of their samples.  Position order instead: chunk c holds
// the tokens of every level covering the c-th T_{L-1}-th of the sequence (tokens c n_l .. c n_l +
// n_l - 1 of level l, n_l = T_l / T_{L-1}), chunks in order, and a tile is 32 consecutive
// entries of that order — every tile a short stretch of every level (bench encoder call: 720 ->
// 416 visits per (b, m), tools/win_visits.py).  Grouping only: every sample is still handled once
// per level by the blocks holding its taps — the forward output and the coordinate gradients are
// the same bit for bit; grad_value rows add the same terms in another order (fp32 accumulation,
// one bf16 rounding).
constexpr int kQOrderMaxL = 4;
struct QOrder {
  int cs;        // entries per chunk (sum of n); 0: consecutive queries
  float inv_cs;  // 1 / cs
  int L;
  int n[kQOrderMaxL], start[kQOrderMaxL];
};

// Measured (tools/win_exp.py, bench encoder call, one MI355X): fewer visits but SLOWER — backward
// 49.3 / 57.3 us (init / trained sampling) against 46.5 / 51.9 with consecutive tiles, the tiles
// forward 35.3 against 31.0: the grad_out loads of a visit (exp 8 in win_exp) cost 13.8 against
// 9.1 us — a tile's rows now come from four separate stretches of grad_out.  So consecutive tiles
// stay the default and MSDA_HIP_QORDER=1 opts in (A/B).  (The Sparse-DETR encoder instead hands
// its top-k queries over already sorted by position: models/sparse/.)
// Position order applies when the call is encoder-shaped (Lq == S, 2 <= L <= 4, every T_l a
// multiple of T_{L-1}, level starts the running sums, Lq < 2^22 so the float chunk division is
// exact).  The forward that writes the tile intervals and the backward that reads them both call
// this on the same shapes.
inline QOrder make_qorder(long long Lq, long long S, int L, const int* T, const int* start) {
  QOrder o{};
  const char* e = getenv("MSDA_HIP_QORDER");
  if (e == nullptr || atoi(e) != 1 || Lq != S || L < 2 || L > kQOrderMaxL || Lq >= (1LL << 22)) return o;
  const int tc = T[L - 1];
  if (tc < 1) return o;
  int cs = 0, run = 0;
  for (int l = 0; l < L; ++l) {
    if (T[l] % tc != 0 || start[l] != run) return o;
    o.n[l] = T[l] / tc;
    o.start[l] = start[l];
    cs += o.n[l];
    run += T[l];
  }
  o.cs = cs;
  o.inv_cs = 1.f / (float)cs;
  o.L = L;
  return o;
}

// The query at entry s (< Lq) of the tile order.
__device__ __forceinline__ int qo_query(const QOrder& o, int s) {
  if (o.cs == 0) return s;
  const int c = (int)(((float)s + 0.5f) * o.inv_cs);
  int j = s - c * o.cs, q = 0;
  bool found = false;
#pragma unroll
  for (int l = 0; l < kQOrderMaxL; ++l) {
    if (l < o.L && !found) {
      if (j < o.n[l]) {
        q = o.start[l] + c * o.n[l] + j;
        found = true;
      } else {
        j -= o.n[l];
      }
    }
  }
  return q;
}

constexpr int kWinMaxChunks = 64;  // position chunks of the dispatch order
constexpr int kWinMaxSeq = 512;    // row blocks of one (b, m) in the position-chunk order

struct WinShape {
  long long B, S, M, Lq;
  int L, P;
  int T[16], start[16];
  int blk0[17];  // first row block of each level (set by msda_win_backward)
  int nblk;      // row blocks over all levels (set by msda_win_backward)
  int ntile;     // query tiles (set by msda_win_backward)
  // dispatch order (set by msda_win_backward; nchunk == 0: coarsest level first): position
  // chunks c of every level, chunk c = level l's blocks [cs_l(c), cs_l(c+1)); the blocks of one
  // (b, m) in chunk order are seq[cs[c] .. cs[c+1]) as (level << 12 | block)
  int nchunk, ppx;
  // coordinate strides (floats): element (b, q, m, l, p) of loc / aw / grad_loc / grad_attn sits at
  // b cb + q cq + m cm + l cl + p (set by msda_win_backward from the layout tag)
  long long cb, cm;
  int cq, cl;
  QOrder qo;  // tile order of the queries (set by the caller: make_qorder; ignored when qo_dev)
  int qo_dev;  // 1: the tiles came from the forward, which stored its QOrder in the tiles tail
  int exp;  // profiling only (MSDA_HIP_WIN_EXP bitmask, 0 in production): skip parts of win_bwd_kernel
  long long gv_rs;  // dense kernels: grad_value row stride in elements (0: M * 64)
  int wsplit[16];  // win_lm_kernel split mode: waves per row block of each level (1, 2 or 4; set by msda_win_backward)
  unsigned short cs[kWinMaxChunks + 1];
  unsigned short seq[kWinMaxSeq];
};

constexpr int kWinQT = 32;          // queries per tile of the row-block backward
constexpr int kWinNone = 1 << 29;   // an empty interval is (kWinNone, -kWinNone)
// After the tile intervals, the tiles buffer holds a 128-B tail written by the tiles forward (every
// byte defined): 64 reserved bytes (zero), then the query order the forward grouped its tiles by (a
// QOrder): the backward reads it from there, so the two always agree whatever the environment does
// between them (MSDA_HIP_QORDER is read by the forward only).
constexpr int kWinQueueWords = 16;  // (reserved words)
constexpr size_t kWinQOrderOffset = kWinQueueWords * sizeof(unsigned);
constexpr size_t kWinTailBytes = 128;
static_assert(kWinQOrderOffset + sizeof(QOrder) <= kWinTailBytes, "tiles tail too small");

// The rows [lo, hi] a sample at normalised location `loc` on a T-row level touches or owns in
// the row-block backward: its taps base and base + 1 (base = floor of the sample position, as
// msda_win.hip's make_taps computes it); a zero-padding sample with no tap on the map is owned
// by row 0.  Shared by the backward's interval prepass and the forward that writes the same
// intervals (msda.hip, msda_fwd16_tiles_kernel), so both see the same rows bit for bit.
__device__ __forceinline__ int2 win_sample_rows(float loc, int T, bool zeros) {
#pragma clang fp contract(off)
  if (zeros) {
    const float x = loc * (float)T - 0.5f;
    if (!((x > -1.f) && (x < (float)T))) return make_int2(0, 0);
    const int lo = (int)floorf(x);
    return make_int2(lo < 0 ? 0 : lo, lo + 1);
  }
  const float g = loc * 2.f - 1.f;
  const float y = fmaf(g + 1.f, (float)T * 0.5f, -0.5f);
  const float ymax = (float)(T - 1);
  const float yc = y > 0.f ? (y < ymax ? y : ymax) : 0.f;
  const int base = (int)floorf(yc);
  return make_int2(base, base + 1);
}

__attribute__((visibility("hidden"))) size_t msda_win_workspace_bytes(long long B, long long M, long long L,
                                                                     long long Lq);
__attribute__((visibility("hidden"))) int msda_win_supported(int value_dtype_is_bf16, long long D, long long P, long long Lq,
                                                                  long long row_floats);
// Coordinate layouts of loc / aw and their gradients: the reference's (B, Lq, M, L, P), or
// level-major (B, M, L, Lq, P) — one (b, m, level)'s coordinates of consecutive queries contiguous
// (include/msda_hip.h, MSDA_COORD_*)
struct CoordStrides {
  long long cb, cm;
  int cq, cl;
};
__host__ __device__ inline CoordStrides coord_strides(int layout, long long Lq, long long M, long long L, long long P) {
  if (layout == 1) return CoordStrides{M * L * Lq * P, L * Lq * P, (int)P, (int)(Lq * P)};
  return CoordStrides{Lq * M * L * P, L * P, (int)(M * L * P), (int)P};
}

__attribute__((visibility("hidden"))) int msda_win_backward(const void* value, const void* loc, const void* aw,
                                                            const void* gout, void* gval, void* gloc, void* gaw,
                                                            void* workspace, const void* tiles_ready,
                                                            const WinShape* shape, int zeros, int coord_layout,
                                                            hipStream_t st);

// The dense small-pyramid kernels (msda_win.hip): 16-bit values, D = 64, at most 128 pyramid rows per
// (b, m), L <= 4, P in {1, 2, 4}; MSDA_HIP_DENSE=0 turns them off (A/B).  Shape fields used: B, S, M,
// Lq, L, P, T, start.  Return 0, or -1 when the shape does not fit (nothing launched).
__attribute__((visibility("hidden"))) int msda_dense_supported(int value_dtype_is_bf16, long long D, long long S,
                                                               long long L, long long P);
// tiles (may be null): the forward's tile buffer (msda_hip_forward_tiles_bytes), written as the tiles
// forward writes it (consecutive tiles)
__attribute__((visibility("hidden"))) int msda_dense_forward(const void* value, const void* loc, const void* aw,
                                                             void* out, void* tiles, const WinShape* shape, int zeros,
                                                             int coord_layout, hipStream_t st);
// workspace: msda_dense_workspace_bytes (the groups' fp32 partial sums of grad_value), or null (one
// workgroup a (b, m), slower)
__attribute__((visibility("hidden"))) int msda_dense_backward(const void* value, const void* loc, const void* aw,
                                                              const void* gout, void* gval, void* gloc, void* gaw,
                                                              void* workspace, const WinShape* shape, int zeros,
                                                              int coord_layout, hipStream_t st);
__attribute__((visibility("hidden"))) size_t msda_dense_workspace_bytes(long long B, long long S, long long M,
                                                                       long long Lq);
