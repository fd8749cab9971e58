// flat_adamw.hip — the training step's optimizer on ONE flat fp32 parameter buffer (gfx950).
//
// Replaces, for the flat-buffer trainer (train_step.py), the reference step's
//   torch.nn.utils.clip_grad_norm_(params, max_norm)   (engine.py:125-126)
//   torch.optim.AdamW(...).step()                        (main.py:113, engine.py:127)
// plus the trainer's bf16 weight shadow refresh.  torch's foreach AdamW on 260 parameter tensors
// launches ~40 multi-tensor kernels and, with capturable step counters, ~520 per-tensor division
// kernels (its tensor-list division falls off the fused path for 0-d operands): ~3.5 ms of a
// 21 ms step.  Here: three kernels over the flat buffers, graph-capturable (step counter and
// clip coefficient live in device memory):
//   1. flat_sq_partials   per-block sums of g^2 (fp32 lanes, fp64 block sum)
//   2. flat_adamw_prepare one workgroup: total norm -> clip coefficient, step += 1, the bias
//                         corrections (fp64), written to a small device state block
//   3. flat_adamw_update  p = p*(1-lr*wd); m = lerp(m, g*c, 1-b1); v = b2*v + (1-b2)*(g*c)^2;
//                         p -= lr/bc1 * m / (sqrt(v)/sqrt(bc2) + eps); bf16 shadow of p.
// All three are HBM-streaming: update moves 7 x 4 B + 2 B per parameter (1.29 GB at 42.8 M).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <math.h>
#include <algorithm>
#include <stdio.h>

#include "flat_adamw.h"

namespace {

thread_local char g_err[256] = {0};

constexpr int kThreads = 256;
constexpr int kPartials = 2048;  // blocks of the norm pass (grid-stride)

struct State {  // device-resident, FLAT_ADAMW_STATE_BYTES
  double sq;        // sum of g^2
  double coef;      // clip coefficient (<= 1)
  double step;      // step count after this update
  double step_size; // lr / bc1
  double bc2_sqrt;  // sqrt(1 - b2^step)
  double decay;     // 1 - lr * weight_decay
  double pad[2];
};

__global__ __launch_bounds__(kThreads) void flat_sq_partials(const float* __restrict__ g, long long n,
                                                            double* __restrict__ partials) {
  float acc = 0.f;
  const long long n4 = n / 4;
  const float4* __restrict__ g4 = reinterpret_cast<const float4*>(g);
  for (long long i = (long long)blockIdx.x * kThreads + threadIdx.x; i < n4; i += (long long)gridDim.x * kThreads) {
    const float4 v = g4[i];
    acc = fmaf(v.x, v.x, acc);
    acc = fmaf(v.y, v.y, acc);
    acc = fmaf(v.z, v.z, acc);
    acc = fmaf(v.w, v.w, acc);
  }
  if (blockIdx.x == 0)
    for (long long i = n4 * 4 + threadIdx.x; i < n; i += kThreads) acc = fmaf(g[i], g[i], acc);
  double d = acc;
  for (int o = 32; o > 0; o >>= 1) d += __shfl_xor(d, o);
  __shared__ double wsum[kThreads / 64];
  if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = d;
  __syncthreads();
  if (threadIdx.x == 0) {
    double s = 0;
    for (int w = 0; w < kThreads / 64; ++w) s += wsum[w];
    partials[blockIdx.x] = s;
  }
}

__global__ __launch_bounds__(kThreads) void flat_adamw_prepare(const double* __restrict__ partials, int nparts,
                                                              State* __restrict__ st, float* __restrict__ step_io,
                                                              double max_norm, double beta1, double beta2, double lr,
                                                              double wd, const float* __restrict__ lr_wd) {
  double d = 0;
  for (int i = threadIdx.x; i < nparts; i += kThreads) d += partials[i];
  for (int o = 32; o > 0; o >>= 1) d += __shfl_xor(d, o);
  __shared__ double wsum[kThreads / 64];
  if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = d;
  __syncthreads();
  if (threadIdx.x == 0) {
    double s = 0;
    for (int w = 0; w < kThreads / 64; ++w) s += wsum[w];
    st->sq = s;
    // clip_grad_norm_: coef = max_norm / (total_norm + 1e-6), clamped to 1; max_norm <= 0: no clip
    const double norm = sqrt(s);
    double c = max_norm > 0 ? max_norm / (norm + 1e-6) : 1.0;
    st->coef = c < 1.0 ? c : 1.0;
    const double step = (double)step_io[0] + 1.0;
    step_io[0] = (float)step;
    st->step = step;
    // lr / weight_decay from device memory when given: a graph replays the values of the step,
    // not those of the capture (a StepLR schedule changes them between replays)
    const float lr_f = lr_wd != nullptr ? lr_wd[0] : (float)lr;
    const float wd_f = lr_wd != nullptr ? lr_wd[1] : (float)wd;
    st->step_size = (double)lr_f / (1.0 - pow(beta1, step));
    st->bc2_sqrt = sqrt(1.0 - pow(beta2, step));
    st->decay = (double)(1.f - lr_f * wd_f);  // fp32 as torch's p.mul_(1 - lr * wd)
  }
}

__device__ __forceinline__ void adamw_one(float& p, float g, float& m, float& v, float c, float b1, float b2,
                                          float decay, float step_size, float bc2_sqrt, float eps) {
  const float gc = g * c;
  p = p * decay;
  m = m + (1.f - b1) * (gc - m);  // torch: exp_avg.lerp_(grad, 1 - beta1)
  v = v * b2 + (1.f - b2) * gc * gc;
  const float denom = sqrtf(v) / bc2_sqrt + eps;
  p = p - step_size * (m / denom);
}

__device__ __forceinline__ uint16_t to_bf16(float x) {
  uint32_t u = __float_as_uint(x);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40);  // NaN stays NaN
  u += 0x7fffu + ((u >> 16) & 1u);                                           // round to nearest even
  return (uint16_t)(u >> 16);
}

__global__ __launch_bounds__(kThreads) void flat_adamw_update(float* __restrict__ p, const float* __restrict__ g,
                                                             float* __restrict__ m, float* __restrict__ v,
                                                             uint16_t* __restrict__ shadow, long long n,
                                                             const State* __restrict__ st, float b1, float b2,
                                                             float eps) {
  const float c = (float)st->coef;
  const float step_size = (float)st->step_size;
  const float bc2 = (float)st->bc2_sqrt;
  const float decay = (float)st->decay;
  const long long n4 = n / 4;
  for (long long i = (long long)blockIdx.x * kThreads + threadIdx.x; i < n4; i += (long long)gridDim.x * kThreads) {
    float4 pp = reinterpret_cast<float4*>(p)[i];
    const float4 gg = reinterpret_cast<const float4*>(g)[i];
    float4 mm = reinterpret_cast<float4*>(m)[i];
    float4 vv = reinterpret_cast<float4*>(v)[i];
    adamw_one(pp.x, gg.x, mm.x, vv.x, c, b1, b2, decay, step_size, bc2, eps);
    adamw_one(pp.y, gg.y, mm.y, vv.y, c, b1, b2, decay, step_size, bc2, eps);
    adamw_one(pp.z, gg.z, mm.z, vv.z, c, b1, b2, decay, step_size, bc2, eps);
    adamw_one(pp.w, gg.w, mm.w, vv.w, c, b1, b2, decay, step_size, bc2, eps);
    reinterpret_cast<float4*>(p)[i] = pp;
    reinterpret_cast<float4*>(m)[i] = mm;
    reinterpret_cast<float4*>(v)[i] = vv;
    if (shadow != nullptr) {
      uint2 sh;
      sh.x = (uint32_t)to_bf16(pp.x) | ((uint32_t)to_bf16(pp.y) << 16);
      sh.y = (uint32_t)to_bf16(pp.z) | ((uint32_t)to_bf16(pp.w) << 16);
      reinterpret_cast<uint2*>(shadow)[i] = sh;
    }
  }
  if (blockIdx.x == 0) {
    for (long long i = n4 * 4 + threadIdx.x; i < n; i += kThreads) {
      adamw_one(p[i], g[i], m[i], v[i], c, b1, b2, decay, step_size, bc2, eps);
      if (shadow != nullptr) shadow[i] = to_bf16(p[i]);
    }
  }
}


// ---------------------------------------------------------------------------------
// Bias gradient of the autocast Linear (models/modules/linear.py): db = sum over the K token
// rows of dY (K x N, 16-bit or fp32) in fp32.  torch's column reduction of a (15360, 512) bf16
// tensor takes ~14 us; here one pass of 16-byte loads: block (column strip of 32x16 B, row
// chunk) partial sums in LDS -> partials[chunk][N], then a fixed-order sum over chunks
// (deterministic).
// ---------------------------------------------------------------------------------
constexpr int kColRows = 8;    // row lanes per block
constexpr int kColLanes = 32;  // 16-byte column lanes per block

template <typename T>
__device__ __forceinline__ void cvt16(const uint4& raw, float (&f)[16 / sizeof(T)]);
template <>
__device__ __forceinline__ void cvt16<uint16_t>(const uint4& raw, float (&f)[8]) {  // bf16
  const uint32_t d[4] = {raw.x, raw.y, raw.z, raw.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = __uint_as_float(d[i] << 16);
    f[2 * i + 1] = __uint_as_float(d[i] & 0xffff0000u);
  }
}
template <>
__device__ __forceinline__ void cvt16<_Float16>(const uint4& raw, float (&f)[8]) {
  const _Float16* h = reinterpret_cast<const _Float16*>(&raw);
#pragma unroll
  for (int i = 0; i < 8; ++i) f[i] = (float)h[i];
}
template <>
__device__ __forceinline__ void cvt16<float>(const uint4& raw, float (&f)[4]) {
  f[0] = __uint_as_float(raw.x); f[1] = __uint_as_float(raw.y);
  f[2] = __uint_as_float(raw.z); f[3] = __uint_as_float(raw.w);
}

template <typename T>
__global__ __launch_bounds__(kColRows * kColLanes) void colsum_partial(const T* __restrict__ x, long long K, int N,
                                                                      int rows_per_chunk, float* __restrict__ part) {
  constexpr int V = 16 / sizeof(T);
  __shared__ float red[kColRows][kColLanes * V];
  const int cl = threadIdx.x % kColLanes, rl = threadIdx.x / kColLanes;
  const int c0 = (blockIdx.x * kColLanes + cl) * V;
  const long long r_begin = (long long)blockIdx.y * rows_per_chunk;
  const long long r_end = min(K, r_begin + rows_per_chunk);
  float acc[V];
#pragma unroll
  for (int i = 0; i < V; ++i) acc[i] = 0.f;
  if (c0 < N) {
    for (long long r = r_begin + rl; r < r_end; r += kColRows) {
      float f[V];
      cvt16<T>(*reinterpret_cast<const uint4*>(x + r * N + c0), f);
#pragma unroll
      for (int i = 0; i < V; ++i) acc[i] += f[i];
    }
  }
#pragma unroll
  for (int i = 0; i < V; ++i) red[rl][cl * V + i] = acc[i];
  __syncthreads();
  for (int c = threadIdx.x; c < kColLanes * V; c += kColRows * kColLanes) {
    float s = 0.f;
#pragma unroll
    for (int r = 0; r < kColRows; ++r) s += red[r][c];
    const int col = blockIdx.x * kColLanes * V + c;
    if (col < N) part[(long long)blockIdx.y * N + col] = s;
  }
}

// Short K (the decoder's 800-token Linear layers): one pass, no partials.  A 256-thread block owns
// a strip of 2 x 16-byte column lanes and all K rows (128 row lanes stride through them); the row
// lanes are then summed in LDS in two fixed-order stages (deterministic).  Narrow strips give
// N / 16 workgroups for bf16 (32 at N = 512): wide ones left this latency-bound on 8 CUs.
constexpr int kSmallCL = 2;     // 16-byte column lanes per block
constexpr int kSmallRL = 128;   // row lanes per block
template <typename T>
__global__ __launch_bounds__(kSmallCL * kSmallRL) void colsum_small(const T* __restrict__ x, long long K, int N,
                                                                   float* __restrict__ out, int accumulate) {
  constexpr int V = 16 / sizeof(T);
  constexpr int C = kSmallCL * V;                 // columns per block
  constexpr int G = kSmallCL * kSmallRL / C;      // row groups of stage 2
  __shared__ float red[kSmallRL][C];
  __shared__ float red2[G][C];
  const int cl = threadIdx.x % kSmallCL, rl = threadIdx.x / kSmallCL;
  const int c0 = (blockIdx.x * kSmallCL + cl) * V;
  float acc[V];
#pragma unroll
  for (int i = 0; i < V; ++i) acc[i] = 0.f;
  if (c0 < N) {
    for (long long r = rl; r < K; r += kSmallRL) {
      float f[V];
      cvt16<T>(*reinterpret_cast<const uint4*>(x + r * N + c0), f);
#pragma unroll
      for (int i = 0; i < V; ++i) acc[i] += f[i];
    }
  }
#pragma unroll
  for (int i = 0; i < V; ++i) red[rl][cl * V + i] = acc[i];
  __syncthreads();
  {
    const int c = threadIdx.x % C, g = threadIdx.x / C;
    float t = 0.f;
#pragma unroll
    for (int r = 0; r < kSmallRL / G; ++r) t += red[g * (kSmallRL / G) + r][c];
    red2[g][c] = t;
  }
  __syncthreads();
  if (threadIdx.x < C) {
    float t = 0.f;
#pragma unroll
    for (int g = 0; g < G; ++g) t += red2[g][threadIdx.x];
    const int col = blockIdx.x * C + threadIdx.x;
    if (col < N) out[col] = accumulate ? out[col] + t : t;
  }
}

// out[c] = sum over chunks of part[k][c]: 16 chunk groups x 64 columns per 1024-thread block,
// each thread a strided run over its chunks in eight independent chains, then an LDS reduction over the
// groups (fixed order: deterministic).
constexpr int kFinGroups = 16;
__global__ __launch_bounds__(kFinGroups * 64) void colsum_final(const float* __restrict__ part, int nchunks, int N,
                                                               float* __restrict__ out, int accumulate) {
  __shared__ float red[kFinGroups][64];
  const int c_l = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + c_l;
  float sc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};  // eight independent chains, fixed order
  if (c < N) {
    int k = g;
    for (; k + 7 * kFinGroups < nchunks; k += 8 * kFinGroups) {
#pragma unroll
      for (int u = 0; u < 8; ++u) sc[u] += part[(long long)(k + u * kFinGroups) * N + c];
    }
    for (; k < nchunks; k += kFinGroups) sc[0] += part[(long long)k * N + c];
  }
  red[g][c_l] = ((sc[0] + sc[1]) + (sc[2] + sc[3])) + ((sc[4] + sc[5]) + (sc[6] + sc[7]));
  __syncthreads();
  if (g == 0 && c < N) {
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < kFinGroups; ++i) t += red[i][c_l];
    out[c] = accumulate ? out[c] + t : t;
  }
}

// Split-K weight gradient of the autocast Linear (models/modules/linear.py): the fp32 partial
// products of the K chunks, (s, n) row-major, summed over the chunks in chunk order — one read of
// the partials and one write, 16 bytes a lane (torch's dim-0 sum of the (8, 512, 512) partials:
// ~10 us).  G groups of s slabs each (group g's sum into out + g n), and with `accumulate` the sum
// is added to out (out + sum, the sum formed first: autograd's accumulation of a finished
// gradient, bit for bit).
__global__ __launch_bounds__(256) void sum_slabs_kernel(const float4* __restrict__ part, int s, long long n4,
                                                        float4* __restrict__ out, int accumulate) {
  const float4* __restrict__ pg = part + (long long)blockIdx.y * s * n4;  // group blockIdx.y
  out += (long long)blockIdx.y * n4;
  for (long long j = (long long)blockIdx.x * 256 + threadIdx.x; j < n4; j += (long long)gridDim.x * 256) {
    const long long i = j;
    float4 a = pg[i];
    // slabs 8 at a time: the 8 loads issued together (branch-free: a slab index past the end re-reads
    // the last slab and is not added), then added in slab order — bitwise the sequential sum.  One
    // dependent load per slab made a 512 x 512 sum of 8 slabs take ~5 us for 9 MB
    for (int k = 1; k < s; k += 8) {
      float4 b[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) b[u] = pg[(long long)min(k + u, s - 1) * n4 + i];
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (k + u < s) {
          a.x += b[u].x; a.y += b[u].y; a.z += b[u].z; a.w += b[u].w;
        }
    }
    if (accumulate) {
      const float4 o = out[j];
      a.x = o.x + a.x; a.y = o.y + a.y; a.z = o.z + a.z; a.w = o.w + a.w;
    }
    out[j] = a;
  }
}

int status(const char* what) {
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    snprintf(g_err, sizeof(g_err), "flat_adamw: %s launch failed: %s", what, hipGetErrorString(e));
    return 2;
  }
  return 0;
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

size_t flat_adamw_workspace_bytes(void) { return sizeof(State) + kPartials * sizeof(double); }

int flat_adamw_step(float* params, const float* grads, float* exp_avg, float* exp_avg_sq, uint16_t* bf16_shadow,
                    int64_t n, float* step, void* workspace, float lr, float beta1, float beta2, float eps,
                    float weight_decay, float max_norm, const float* lr_wd, void* stream) {
  g_err[0] = 0;
  if (n < 0 || (n > 0 && (params == nullptr || grads == nullptr || exp_avg == nullptr || exp_avg_sq == nullptr)) ||
      step == nullptr || workspace == nullptr) {
    snprintf(g_err, sizeof(g_err), "flat_adamw_step: bad arguments");
    return 1;
  }
  for (const void* ptr : {(const void*)params, (const void*)grads, (const void*)exp_avg, (const void*)exp_avg_sq})
    if (reinterpret_cast<uintptr_t>(ptr) % 16 != 0) {
      snprintf(g_err, sizeof(g_err), "flat_adamw_step: buffers must be 16-byte aligned");
      return 1;
    }
  if (bf16_shadow != nullptr && reinterpret_cast<uintptr_t>(bf16_shadow) % 8 != 0) {
    snprintf(g_err, sizeof(g_err), "flat_adamw_step: the bf16 shadow must be 8-byte aligned");
    return 1;
  }
  hipStream_t st = static_cast<hipStream_t>(stream);
  auto* state = static_cast<State*>(workspace);
  auto* partials = reinterpret_cast<double*>(static_cast<unsigned char*>(workspace) + sizeof(State));
  const long long n4 = n / 4;
  const int nparts = (int)std::min<long long>(kPartials, std::max<long long>(1, (n4 + kThreads - 1) / kThreads));
  int rc;
  hipLaunchKernelGGL(flat_sq_partials, dim3(nparts), dim3(kThreads), 0, st, grads, (long long)n, partials);
  if ((rc = status("norm"))) return rc;
  hipLaunchKernelGGL(flat_adamw_prepare, dim3(1), dim3(kThreads), 0, st, partials, nparts, state, step,
                     (double)max_norm, (double)beta1, (double)beta2, (double)lr, (double)weight_decay, lr_wd);
  if ((rc = status("prepare"))) return rc;
  const unsigned blocks = (unsigned)std::min<long long>(8192, std::max<long long>(1, (n4 + kThreads - 1) / kThreads));
  hipLaunchKernelGGL(flat_adamw_update, dim3(blocks), dim3(kThreads), 0, st, params, grads, exp_avg, exp_avg_sq,
                     bf16_shadow, (long long)n, state, beta1, beta2, eps);
  return status("update");
}


size_t mfl_colsum_workspace_bytes(int64_t K, int64_t N) {
  const long long chunks = std::min<long long>(256, std::max<long long>(1, (K + 63) / 64));
  return (size_t)chunks * (size_t)std::max<int64_t>(N, 1) * sizeof(float);
}

int mfl_colsum(const void* x, int dtype, int64_t K, int64_t N, float* out, void* workspace, void* stream) {
  return mfl_colsum_ex(x, dtype, K, N, out, 0, workspace, stream);
}

int mfl_colsum_ex(const void* x, int dtype, int64_t K, int64_t N, float* out, int accumulate, void* workspace,
                  void* stream) {
  g_err[0] = 0;
  const int elt = dtype == 0 ? 4 : 2;
  if (K < 0 || N <= 0 || out == nullptr || (K > 0 && (x == nullptr || workspace == nullptr)) ||
      (dtype != 0 && dtype != 2 && dtype != 3) || (N * elt) % 16 != 0 || reinterpret_cast<uintptr_t>(x) % 16 != 0) {
    snprintf(g_err, sizeof(g_err), "mfl_colsum: bad arguments (N*elt must be a multiple of 16 B, x 16-B aligned)");
    return 1;
  }
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (K == 0) {
    if (accumulate) return 0;
    return zero_f32(out, N, st) == hipSuccess ? 0 : 2;
  }
  const int V = 16 / elt;
  if (K <= 4096) {  // one pass: at most 128 rows per row lane
    const dim3 g1((unsigned)((N / V + kSmallCL - 1) / kSmallCL));
    if (dtype == 0)
      hipLaunchKernelGGL(colsum_small<float>, g1, dim3(kSmallCL * kSmallRL), 0, st, static_cast<const float*>(x),
                         (long long)K, (int)N, out, accumulate);
    else if (dtype == 2)
      hipLaunchKernelGGL(colsum_small<uint16_t>, g1, dim3(kSmallCL * kSmallRL), 0, st,
                         static_cast<const uint16_t*>(x), (long long)K, (int)N, out, accumulate);
    else
      hipLaunchKernelGGL(colsum_small<_Float16>, g1, dim3(kSmallCL * kSmallRL), 0, st,
                         static_cast<const _Float16*>(x), (long long)K, (int)N, out, accumulate);
    return status("colsum small");
  }
  const long long chunks = std::min<long long>(256, std::max<long long>(1, (K + 63) / 64));
  const int rows_per_chunk = (int)((K + chunks - 1) / chunks);
  const dim3 grid((unsigned)((N / V + kColLanes - 1) / kColLanes), (unsigned)chunks);
  auto* part = static_cast<float*>(workspace);
  if (dtype == 0)
    hipLaunchKernelGGL(colsum_partial<float>, grid, dim3(kColRows * kColLanes), 0, st, static_cast<const float*>(x),
                       (long long)K, (int)N, rows_per_chunk, part);
  else if (dtype == 2)
    hipLaunchKernelGGL(colsum_partial<uint16_t>, grid, dim3(kColRows * kColLanes), 0, st,
                       static_cast<const uint16_t*>(x), (long long)K, (int)N, rows_per_chunk, part);
  else
    hipLaunchKernelGGL(colsum_partial<_Float16>, grid, dim3(kColRows * kColLanes), 0, st,
                       static_cast<const _Float16*>(x), (long long)K, (int)N, rows_per_chunk, part);
  int rc;
  if ((rc = status("colsum partial"))) return rc;
  hipLaunchKernelGGL(colsum_final, dim3((unsigned)((N + 63) / 64)), dim3(kFinGroups * 64), 0, st, part, (int)chunks,
                     (int)N, out, accumulate);
  return status("colsum final");
}

int mfl_sum_slabs(const float* part, int64_t s, int64_t n, float* out, void* stream) {
  return mfl_sum_slabs_ex(part, 1, s, n, out, 0, stream);
}

int mfl_sum_slabs_ex(const float* part, int64_t groups, int64_t s, int64_t n, float* out, int accumulate,
                     void* stream) {
  g_err[0] = 0;
  if (s <= 0 || s > (1 << 20) || groups <= 0 || groups > 65535 || n < 0 || n % 4 != 0 || groups * n > (1LL << 40) ||
      (n > 0 && (part == nullptr || out == nullptr)) ||
      ((reinterpret_cast<uintptr_t>(part) | reinterpret_cast<uintptr_t>(out)) & 15u)) {
    snprintf(g_err, sizeof(g_err),
             "mfl_sum_slabs: bad arguments (s > 0, groups > 0, n %% 4 == 0, 16-B aligned pointers)");
    return 1;
  }
  if (n == 0) return 0;
  const long long n4 = n / 4;
  const unsigned blocks = (unsigned)std::max<long long>(1, std::min<long long>((n4 + 255) / 256, 8192 / groups));
  hipLaunchKernelGGL(sum_slabs_kernel, dim3(blocks, (unsigned)groups), dim3(256), 0, static_cast<hipStream_t>(stream),
                     reinterpret_cast<const float4*>(part), (int)s, n4, reinterpret_cast<float4*>(out), accumulate);
  return status("sum slabs");
}

int mfl_stream_create(int device, void** stream) {
  g_err[0] = 0;
  if (stream == nullptr) {
    snprintf(g_err, sizeof(g_err), "mfl_stream_create: stream is NULL");
    return 1;
  }
  int prev = 0;
  if (hipGetDevice(&prev) != hipSuccess || hipSetDevice(device) != hipSuccess) {
    snprintf(g_err, sizeof(g_err), "mfl_stream_create: bad device %d", device);
    return 1;
  }
  hipStream_t s = nullptr;
  const hipError_t e = hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  (void)hipSetDevice(prev);
  if (e != hipSuccess) {
    snprintf(g_err, sizeof(g_err), "mfl_stream_create: %s", hipGetErrorString(e));
    return 1;
  }
  *stream = s;
  return 0;
}

const char* flat_adamw_last_error(void) { return g_err; }

}  // extern "C"
