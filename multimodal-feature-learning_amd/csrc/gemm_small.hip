// gemm_small.hip — short-M bf16 GEMM C = A . Bt^T (+ bias) on the matrix cores (include/gemm_small.h).
//
// The training step's GEMMs over the decoder's 800 query rows (and the caption decoder's segment
// tokens, the audio stream's 760) are latency-bound in the library: 0.4-1.7 GFLOP taking 9-15 us
// (profiles/r03_gemm_census.txt), because a large-tile kernel leaves most of the 256 CUs idle and
// walks K serially.  Here a workgroup owns one 32 x 32 output tile and its KS waves split K: each
// wave loads its MFMA fragments straight from global memory (both operands are K-contiguous, so a
// lane's 8 bf16 of a fragment are one 16-byte load; no LDS staging for operands read once per
// tile), runs 2 x 2 v_mfma_f32_16x16x32_bf16 accumulators, and the partial tiles are added in LDS.
// (800, 512) x (512, 512): 25 x 16 tiles = 400 workgroups of 4 waves, each wave 4 K-steps.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdarg.h>

#include "gemm_small.h"

namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;

thread_local char g_err[256];

void set_err(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

constexpr int kT = 32;  // output tile (rows and columns)
constexpr int kU = 4;   // K-steps (of 32) whose fragments are loaded together

__device__ __forceinline__ bf16x8 load_frag(const uint16_t* p) {
  return *reinterpret_cast<const bf16x8*>(p);
}

__device__ __forceinline__ uint16_t bf16_rne(float x) {  // finite inputs
  const uint32_t u = __float_as_uint(x);
  return (uint16_t)((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
}

template <int KS>
__global__ __launch_bounds__(64 * KS) void gemm_nt_small_kernel(const uint16_t* __restrict__ A,
                                                                 const uint16_t* __restrict__ Bt,
                                                                 const uint16_t* __restrict__ bias,
                                                                 uint16_t* __restrict__ C, int M, int K,
                                                                 long long lda, long long ldb, long long ldc,
                                                                 int tiles_n) {
  __shared__ __attribute__((aligned(16))) float red[KS > 1 ? KS : 1][4][64][4];
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));  // (scalar)
  const int tm = blockIdx.x / tiles_n, tn = blockIdx.x % tiles_n;
  const int m0 = tm * kT, n0 = tn * kT;
  // fragments: lane l reads row (l & 15) of a 16-row block, K offset 8 (l >> 4) of a 32-step
  const int r = lane & 15, kq = (lane >> 4) * 8;
  const uint16_t* __restrict__ a0 = A + (long long)min(m0 + r, M - 1) * lda + kq;  // rows past M: clamped
  const uint16_t* __restrict__ a1 = A + (long long)min(m0 + 16 + r, M - 1) * lda + kq;
  const uint16_t* __restrict__ b0 = Bt + (long long)(n0 + r) * ldb + kq;
  const uint16_t* __restrict__ b1 = Bt + (long long)(n0 + 16 + r) * ldb + kq;
  // this wave's K-steps [s0, s1)
  const int nsteps = K / 32, per = (nsteps + KS - 1) / KS;
  const int s0 = min(w * per, nsteps), s1 = min(s0 + per, nsteps);
  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  int s = s0;
  for (; s + kU <= s1; s += kU) {  // whole batches: every load issued before the first MFMA
    bf16x8 fa[kU][2], fb[kU][2];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int k = (s + u) * 32;
      fa[u][0] = load_frag(a0 + k);
      fa[u][1] = load_frag(a1 + k);
      fb[u][0] = load_frag(b0 + k);
      fb[u][1] = load_frag(b1 + k);
    }
#pragma unroll
    for (int u = 0; u < kU; ++u)
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[u][i], fb[u][j], acc[i][j], 0, 0, 0);
  }
  for (; s < s1; ++s) {  // the remainder, one step at a time
    const int k = s * 32;
    const bf16x8 x0 = load_frag(a0 + k), x1 = load_frag(a1 + k), y0 = load_frag(b0 + k), y1 = load_frag(b1 + k);
    acc[0][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x0, y0, acc[0][0], 0, 0, 0);
    acc[0][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x0, y1, acc[0][1], 0, 0, 0);
    acc[1][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x1, y0, acc[1][0], 0, 0, 0);
    acc[1][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x1, y1, acc[1][1], 0, 0, 0);
  }
  // the waves' partial tiles through LDS; wave w then finishes the 16 x 16 sub-tiles t = w, w + KS, ...
  if constexpr (KS > 1) {
#pragma unroll
    for (int t = 0; t < 4; ++t) *reinterpret_cast<f32x4*>(red[w][t][lane]) = acc[t >> 1][t & 1];
    __syncthreads();
  }
  // C/D of v_mfma_f32_16x16x32: column lane & 15, rows 4 (lane >> 4) + 0..3
  const int col_in = lane & 15, row_in = (lane >> 4) * 4;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    if (KS > 1 && t % KS != w) continue;
    if (KS == 1 && w != 0) continue;
    f32x4 v = acc[t >> 1][t & 1];
    if constexpr (KS > 1) {
      v = *reinterpret_cast<const f32x4*>(red[0][t][lane]);
#pragma unroll
      for (int o = 1; o < KS; ++o) {
        const f32x4 x = *reinterpret_cast<const f32x4*>(red[o][t][lane]);
        v += x;
      }
    }
    const int col = n0 + 16 * (t & 1) + col_in;
    const float bv = bias ? __uint_as_float((uint32_t)bias[col] << 16) : 0.f;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int row = m0 + 16 * (t >> 1) + row_in + q;
      if (row < M) C[(long long)row * ldc + col] = bf16_rne(v[q] + bv);
    }
  }
}

// C = A . B with B row-major (K, N): the input gradient of a Linear layer, dX = dY . W (W stored
// (out, in): the reduction runs over W's rows).  A's fragments load as above; B's are K-strided,
// so each wave stages its 32 K-rows x 32 columns of B in LDS (one 16-byte load per lane and half
// row) and reads them transposed with ds_read_b64_tr_b16 (the grad_out tiles of msda_win.hip use
// the same read).  Each wave's LDS is its own: its writes and reads are ordered by its LDS queue.
constexpr int kBS = 80;  // LDS row stride (bytes) of a staged 32-column B row: 16-B aligned, spreads banks
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;

template <int KS>
__global__ __launch_bounds__(64 * KS) void gemm_nn_small_kernel(const uint16_t* __restrict__ A,
                                                                 const uint16_t* __restrict__ B,
                                                                 const uint16_t* __restrict__ bias,
                                                                 uint16_t* __restrict__ C, int M, int K,
                                                                 long long lda, long long ldb, long long ldc,
                                                                 int tiles_n) {
  __shared__ __attribute__((aligned(16))) float red[KS > 1 ? KS : 1][4][64][4];
  __shared__ __attribute__((aligned(16))) unsigned char sb[KS][kU][32 * kBS];
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));  // (scalar)
  const int tm = blockIdx.x / tiles_n, tn = blockIdx.x % tiles_n;
  const int m0 = tm * kT, n0 = tn * kT;
  const int r = lane & 15, kq = (lane >> 4) * 8;
  const uint16_t* __restrict__ a0 = A + (long long)min(m0 + r, M - 1) * lda + kq;
  const uint16_t* __restrict__ a1 = A + (long long)min(m0 + 16 + r, M - 1) * lda + kq;
  // B staging: lane l copies row (l >> 1) of the step, columns n0 + 16 (l & 1) .. + 15
  const uint16_t* __restrict__ bsrc = B + (long long)(lane >> 1) * ldb + n0 + 16 * (lane & 1);
  const int bdst = (lane >> 1) * kBS + 32 * (lane & 1);
  // transposed reads: lane (g, li = 4 qq + pp) reads rows 8 g + qq and 8 g + 4 + qq, columns 4 pp + 16 cb
  const int g = lane >> 4, qq = (lane & 15) >> 2, pp = lane & 3;
  const int rowa = 8 * g + qq, rowb = 8 * g + 4 + qq;
  const int nsteps = K / 32, per = (nsteps + KS - 1) / KS;
  const int s0 = min(w * per, nsteps), s1 = min(s0 + per, nsteps);
  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  unsigned char* const my = sb[w][0];  // this wave's staging slots
  // one step: A fragments from global, the step's B rows through LDS (slot u), 4 MFMAs
  auto b_frags = [&](int u, bf16x8 (&fb)[2]) {
#pragma unroll
    for (int cb = 0; cb < 2; ++cb) {
      const int col = (cb * 16 + 4 * pp) * 2;
      const bf16x4 x0 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(my + u * 32 * kBS + rowa * kBS + col));
      const bf16x4 x1 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(my + u * 32 * kBS + rowb * kBS + col));
      fb[cb] = __builtin_shufflevector(x0, x1, 0, 1, 2, 3, 4, 5, 6, 7);
    }
  };
  int s = s0;
  for (; s + kU <= s1; s += kU) {  // whole batches: every load issued before the first LDS write
    bf16x8 fa[kU][2];
    uint4 rb[kU][2];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int k = (s + u) * 32;
      fa[u][0] = load_frag(a0 + k);
      fa[u][1] = load_frag(a1 + k);
      const uint16_t* src = bsrc + (long long)k * ldb;
      rb[u][0] = *reinterpret_cast<const uint4*>(src);
      rb[u][1] = *reinterpret_cast<const uint4*>(src + 8);
    }
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      *reinterpret_cast<uint4*>(my + u * 32 * kBS + bdst) = rb[u][0];
      *reinterpret_cast<uint4*>(my + u * 32 * kBS + bdst + 16) = rb[u][1];
    }
    asm volatile("" ::: "memory");  // this wave's LDS writes before its reads (same LDS queue)
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      bf16x8 fb[2];
      b_frags(u, fb);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[u][i], fb[j], acc[i][j], 0, 0, 0);
    }
    asm volatile("" ::: "memory");  // this batch's LDS reads before the next batch's writes
  }
  for (; s < s1; ++s) {  // the remainder, one step at a time (slot 0)
    const int k = s * 32;
    const bf16x8 x0 = load_frag(a0 + k), x1 = load_frag(a1 + k);
    const uint16_t* src = bsrc + (long long)k * ldb;
    const uint4 y0 = *reinterpret_cast<const uint4*>(src), y1 = *reinterpret_cast<const uint4*>(src + 8);
    *reinterpret_cast<uint4*>(my + bdst) = y0;
    *reinterpret_cast<uint4*>(my + bdst + 16) = y1;
    asm volatile("" ::: "memory");
    bf16x8 fb[2];
    b_frags(0, fb);
    acc[0][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x0, fb[0], acc[0][0], 0, 0, 0);
    acc[0][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x0, fb[1], acc[0][1], 0, 0, 0);
    acc[1][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x1, fb[0], acc[1][0], 0, 0, 0);
    acc[1][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x1, fb[1], acc[1][1], 0, 0, 0);
    asm volatile("" ::: "memory");
  }
  if constexpr (KS > 1) {
#pragma unroll
    for (int t = 0; t < 4; ++t) *reinterpret_cast<f32x4*>(red[w][t][lane]) = acc[t >> 1][t & 1];
    __syncthreads();
  }
  const int col_in = lane & 15, row_in = (lane >> 4) * 4;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    if (KS > 1 && t % KS != w) continue;
    if (KS == 1 && w != 0) continue;
    f32x4 v = acc[t >> 1][t & 1];
    if constexpr (KS > 1) {
      v = *reinterpret_cast<const f32x4*>(red[0][t][lane]);
#pragma unroll
      for (int o = 1; o < KS; ++o) {
        const f32x4 x = *reinterpret_cast<const f32x4*>(red[o][t][lane]);
        v += x;
      }
    }
    const int col = n0 + 16 * (t & 1) + col_in;
    const float bv = bias ? __uint_as_float((uint32_t)bias[col] << 16) : 0.f;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int row = m0 + 16 * (t >> 1) + row_in + q;
      if (row < M) C[(long long)row * ldc + col] = bf16_rne(v[q] + bv);
    }
  }
}

}  // namespace

extern "C" {

int mfl_gemm_nt_bf16(const void* A, const void* Bt, const void* bias, void* C, int64_t M, int64_t N, int64_t K,
                     int64_t lda, int64_t ldb, int64_t ldc, void* stream) {
  g_err[0] = 0;
  if (M < 0 || N < 0 || K < 0) {
    set_err("mfl_gemm_nt_bf16: negative sizes");
    return 1;
  }
  if (M == 0 || N == 0) return 0;
  const auto al16 = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; };
  if (N % kT || K % 32 || K == 0 || lda < K || ldb < K || ldc < N || lda % 8 || ldb % 8 || ldc % 8 || !al16(A) ||
      !al16(Bt) || !al16(C) || M > (1 << 20)) {
    set_err("mfl_gemm_nt_bf16: unsupported shape / layout (M=%lld N=%lld K=%lld)", (long long)M, (long long)N,
            (long long)K);
    return MFL_GEMM_UNSUPPORTED;
  }
  const int tiles_n = (int)(N / kT);
  const long long tiles = (M + kT - 1) / kT * tiles_n;
  hipStream_t st = static_cast<hipStream_t>(stream);
  auto* a = static_cast<const uint16_t*>(A);
  auto* b = static_cast<const uint16_t*>(Bt);
  auto* bi = static_cast<const uint16_t*>(bias);
  auto* c = static_cast<uint16_t*>(C);
  const int steps = (int)(K / 32);
  // waves a tile: at least kU K-steps each (every wave's loads in one batch when K <= 32 kU KS)
  const int ks = steps >= 8 * kU ? 8 : steps >= 4 * kU ? 4 : steps >= 2 * kU ? 2 : 1;
#define GEMM_L(KS)                                                                                       \
  hipLaunchKernelGGL((gemm_nt_small_kernel<KS>), dim3((unsigned)tiles), dim3(64 * KS), 0, st, a, b, bi, c, \
                     (int)M, (int)K, (long long)lda, (long long)ldb, (long long)ldc, tiles_n)
  switch (ks) {
    case 8: GEMM_L(8); break;
    case 4: GEMM_L(4); break;
    case 2: GEMM_L(2); break;
    default: GEMM_L(1); break;
  }
#undef GEMM_L
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_err("mfl_gemm_nt_bf16: launch failed: %s", hipGetErrorString(e));
    return 1;
  }
  return 0;
}

int mfl_gemm_nn_bf16(const void* A, const void* B, const void* bias, void* C, int64_t M, int64_t N, int64_t K,
                     int64_t lda, int64_t ldb, int64_t ldc, void* stream) {
  g_err[0] = 0;
  if (M < 0 || N < 0 || K < 0) {
    set_err("mfl_gemm_nn_bf16: negative sizes");
    return 1;
  }
  if (M == 0 || N == 0) return 0;
  const auto al16 = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; };
  if (N % kT || K % 32 || K == 0 || lda < K || ldb < N || ldc < N || lda % 8 || ldb % 8 || ldc % 8 || !al16(A) ||
      !al16(B) || !al16(C) || M > (1 << 20)) {
    set_err("mfl_gemm_nn_bf16: unsupported shape / layout (M=%lld N=%lld K=%lld)", (long long)M, (long long)N,
            (long long)K);
    return MFL_GEMM_UNSUPPORTED;
  }
  const int tiles_n = (int)(N / kT);
  const long long tiles = (M + kT - 1) / kT * tiles_n;
  hipStream_t st = static_cast<hipStream_t>(stream);
  auto* a = static_cast<const uint16_t*>(A);
  auto* b = static_cast<const uint16_t*>(B);
  auto* bi = static_cast<const uint16_t*>(bias);
  auto* c = static_cast<uint16_t*>(C);
  const int steps = (int)(K / 32);
  const int ks = steps >= 8 * kU ? 8 : steps >= 4 * kU ? 4 : steps >= 2 * kU ? 2 : 1;
#define GEMM_L(KS)                                                                                       \
  hipLaunchKernelGGL((gemm_nn_small_kernel<KS>), dim3((unsigned)tiles), dim3(64 * KS), 0, st, a, b, bi, c, \
                     (int)M, (int)K, (long long)lda, (long long)ldb, (long long)ldc, tiles_n)
  switch (ks) {
    case 8: GEMM_L(8); break;
    case 4: GEMM_L(4); break;
    case 2: GEMM_L(2); break;
    default: GEMM_L(1); break;
  }
#undef GEMM_L
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_err("mfl_gemm_nn_bf16: launch failed: %s", hipGetErrorString(e));
    return 1;
  }
  return 0;
}

const char* mfl_gemm_last_error(void) { return g_err; }

}  // extern "C"
