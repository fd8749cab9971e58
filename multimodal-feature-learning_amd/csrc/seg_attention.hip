// Segment cross-attention of the caption decoder (include/seg_attention.h) for gfx950.
//
// Reference: models/modules/attention.py:278-300 (CrossAttention: q @ k^T, masked_fill(-1e20), * scale,
// softmax, dropout, @ v) over the cropped memory of crop_segments (models/deformable/
// unimodal_deformable_dvc.py:457-493).  The stock form gathers every segment's (K, d) key and value
// rows (n copies of ~2,000 x 512), permutes them to heads and runs two batched GEMMs and a softmax
// over (n, H, Lq, K) scores: 36 such calls a DVC step cost ~25 ms, almost all of it copies.  Here a
// segment reads its clip's projected rows (index[s]) in place and the scores never leave registers:
//
//   seg_attn_fwd      one workgroup per (segment, head), 4 waves dealing 32-key blocks round-robin,
//                     flash-style running max / sum per query, O = P V on MFMA; the waves' partial
//                     (m, l, O) meet in LDS.  Key blocks with no unmasked key are skipped (their
//                     softmax weight is exactly 0 in the reference too: exp(-1.25e19 - m) = 0).
//   seg_attn_bwd_dq   one workgroup per (segment, head): D = rowsum(dO * O), then per key block
//                     P = exp(s - lse), dS = P (dP - D) and dQ += dS K.
//   seg_attn_bwd_dkv  one workgroup per (clip, head, 4 key blocks), a wave per block: loops over the
//                     segments reading that clip, recomputes P and dS, and accumulates dK += dS^T Q,
//                     dV += P'^T dO in registers — every (clip row, head) written by one wave, no
//                     atomics; rows a segment reads as the bias (keep = 0) go to per-wave bias sums.
//
// MFMA: v_mfma_f32_16x16x32_bf16 (A lane (g, li): row li, k 8g..8g+7; B lane: column li, k 8g..;
// D lane: rows 4g..4g+3 of column li).  Score tiles come out with 4 consecutive keys (or queries)
// per lane, which feed the next product's A operand directly when its reduction runs over those
// keys; the B operand is then read transposed from LDS (ds_read_b64_tr_b16) out of rows stored in
// the matching slot order (perm_row).
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>

#include "seg_attention.h"

namespace {

constexpr int HD = 64;       // head dim
constexpr int QT = 32;       // queries per segment (max)
constexpr int KB = 32;       // keys per block
constexpr int kWaves = 4;
constexpr int kThreads = 64 * kWaves;
constexpr int kRS = 144;     // LDS row stride (bytes): 64 bf16 + 16 B, 16-B aligned
constexpr float kNegInf = -INFINITY;

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;

thread_local char g_err[256] = "";

struct Args {
  const uint16_t *q, *pk, *pv, *bk, *bv;
  const int64_t* index;
  const uint8_t *keep, *masked;
  int n, B, K, Lq, H;
  float scale, p;
  const int64_t* seed;
  uint16_t* out;
  float* lse;
  const uint16_t* dout;
  uint16_t *dq, *dpk, *dpv;
  float* dbias;  // (H, P, 2, 64)
  float* D;      // (n, H, 32)
  int* dead;     // (n)
};

__device__ __forceinline__ void wave_lds_fence() { asm volatile("" ::: "memory"); }

__device__ __forceinline__ uint16_t f2bf(float x) {
  const uint32_t u = __float_as_uint(x);
  return (uint16_t)((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
}
__device__ __forceinline__ __bf16 tobf(float x) { return __builtin_bit_cast(__bf16, f2bf(x)); }
__device__ __forceinline__ float bf2f(uint16_t u) { return __uint_as_float((uint32_t)u << 16); }

__device__ __forceinline__ bf16x8 zero8() {
  const __bf16 z = __builtin_bit_cast(__bf16, (uint16_t)0);
  return bf16x8{z, z, z, z, z, z, z, z};
}
__device__ __forceinline__ bf16x8 load8(const uint16_t* p) { return *reinterpret_cast<const bf16x8*>(p); }

// the attention-dropout keep bits (the same 64-bit mix as add_layernorm.hip's branch dropout)
__device__ __forceinline__ uint32_t drop_bits(uint64_t seed, uint64_t e) {
  uint64_t x = seed * 0x9E3779B97F4A7C15ull + e;
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ull;
  x ^= x >> 33;
  return (uint32_t)x;
}
__device__ __forceinline__ float drop_mul(uint64_t seed, uint32_t thresh, float dscale, uint64_t e) {
  return (drop_bits(seed, e) >> 8) >= thresh ? dscale : 0.f;
}

// key / query kk (0..31) of a block -> its LDS row, so that rows 8g .. 8g+7 hold kk = 4g..4g+3 and
// 16+4g..16+4g+3: the k-slot order of an A operand built from two 16-row score tiles
__device__ __forceinline__ int perm_row(int kk) { return 8 * ((kk & 15) >> 2) + 4 * (kk >> 4) + (kk & 3); }

// B operand (k = the tile's 32 LDS rows in order, n = columns cb*16 ..) by two transposed reads
__device__ __forceinline__ bf16x8 tr_b(const unsigned char* tile, int g, int li, int cb) {
  const int qq = li >> 2, pp = li & 3;
  const int col = (cb * 16 + 4 * pp) * 2;
  const bf16x4 x0 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(tile + (8 * g + qq) * kRS + col));
  const bf16x4 x1 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(tile + (8 * g + 4 + qq) * kRS + col));
  return __builtin_shufflevector(x0, x1, 0, 1, 2, 3, 4, 5, 6, 7);
}

__device__ __forceinline__ f32x4 mfma(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

struct BlockMasks {
  uint32_t in, live, keep;  // bit kk: key j0+kk exists / is unmasked / reads the projected row
};

__device__ __forceinline__ BlockMasks block_masks(const Args& a, int s, int j0, int lane) {
  const int j = j0 + (lane & 31);
  const bool lo = lane < 32 && j < a.K;
  const long long e = (long long)s * a.K + j;
  BlockMasks m;
  m.in = (uint32_t)__ballot(lo);
  m.live = (uint32_t)__ballot(lo && (a.masked == nullptr || a.masked[e] == 0));
  m.keep = (uint32_t)__ballot(lo && a.keep[e] != 0);
  return m;
}

// whether segment s has any unmasked key (all threads of the block call it)
__device__ __forceinline__ bool segment_dead(const Args& a, int s) {
  int any = 0;
  if (a.masked == nullptr) {
    any = 1;
  } else {
    for (int j = threadIdx.x; j < a.K; j += kThreads) any |= a.masked[(long long)s * a.K + j] == 0;
  }
  return !__syncthreads_or(any);
}

// 32 rows (keys kk of the block) x 64 head dims of the projected rows (or the bias) into LDS at perm_row
__device__ __forceinline__ void stage_rows(unsigned char* tile, const uint16_t* base, const uint16_t* bias,
                                           const BlockMasks& m, int d, int lane) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = lane + 64 * i, kk = c >> 3, part = c & 7;
    uint4 v = make_uint4(0u, 0u, 0u, 0u);
    if ((m.in >> kk) & 1u) {
      const uint16_t* row = ((m.keep >> kk) & 1u) ? base + (long long)kk * d : bias;
      if (row) v = *reinterpret_cast<const uint4*>(row + part * 8);
    }
    *reinterpret_cast<uint4*>(tile + perm_row(kk) * kRS + part * 16) = v;
  }
}

// A-operand fragments of the block's rows (row kt*16 + li, head dims ks*32 + 8g ..)
__device__ __forceinline__ void row_frags(bf16x8 (&f)[2][2], const uint16_t* base, const uint16_t* bias,
                                          const BlockMasks& m, int d, int g, int li) {
#pragma unroll
  for (int kt = 0; kt < 2; ++kt) {
    const int kk = kt * 16 + li;
    const uint16_t* row = ((m.keep >> kk) & 1u) ? base + (long long)kk * d : bias;
    const bool ok = ((m.in >> kk) & 1u) && row != nullptr;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) f[kt][ks] = ok ? load8(row + ks * 32 + 8 * g) : zero8();
  }
}

__global__ __launch_bounds__(kThreads) void seg_attn_fwd(Args a) {
  __shared__ __attribute__((aligned(16))) unsigned char s_v[kWaves][KB * kRS];
  __shared__ float s_m[kWaves][QT], s_l[kWaves][QT];
  __shared__ float s_o[kWaves][QT][HD + 1];
  const int s = blockIdx.x / a.H, h = blockIdx.x % a.H;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, g = lane >> 4, li = lane & 15;
  const int d = a.H * HD;
  const long long b = a.index[s];
  const bool dead = segment_dead(a, s);
  bf16x8 qf[2][2];  // B operand of S^T = K Q^T: column = query qt*16 + li
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    const int qi = qt * 16 + li;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
      qf[qt][ks] = qi < a.Lq ? load8(a.q + ((long long)s * a.Lq + qi) * d + h * HD + ks * 32 + 8 * g) : zero8();
  }
  float m[2] = {kNegInf, kNegInf}, l[2] = {0.f, 0.f};
  f32x4 o[2][4];
#pragma unroll
  for (int qt = 0; qt < 2; ++qt)
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) o[qt][cb] = f32x4{0.f, 0.f, 0.f, 0.f};
  const uint64_t seed = a.seed ? (uint64_t)a.seed[0] : 0;
  const uint32_t thresh = (uint32_t)fminf(a.p * 16777216.f, 16777216.f);
  const float dscale = 1.f / (1.f - a.p);
  const uint16_t* bk = a.bk ? a.bk + h * HD : nullptr;
  const uint16_t* bv = a.bv ? a.bv + h * HD : nullptr;
  unsigned char* const sv = s_v[wave];
  const int nblk = (a.K + KB - 1) / KB;
  for (int blk = wave; blk < nblk; blk += kWaves) {
    const int j0 = blk * KB;
    const BlockMasks mk = block_masks(a, s, j0, lane);
    if (!dead && mk.live == 0u) continue;  // wave-uniform: no weight on any key of the block
    const long long rbase = (b * a.K + j0) * d + h * HD;
    bf16x8 kf[2][2];
    row_frags(kf, a.pk + rbase, bk, mk, d, g, li);
    stage_rows(sv, a.pv + rbase, bv, mk, d, lane);
    float sc[2][2][4];  // [kt][qt][r]: key kt*16 + 4g + r, query qt*16 + li
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int qt = 0; qt < 2; ++qt) {
        f32x4 t = f32x4{0.f, 0.f, 0.f, 0.f};
        t = mfma(kf[kt][0], qf[qt][0], t);
        t = mfma(kf[kt][1], qf[qt][1], t);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int kk = kt * 16 + 4 * g + r;
          const bool in = (mk.in >> kk) & 1u, live = (mk.live >> kk) & 1u;
          sc[kt][qt][r] = !in ? kNegInf : dead ? 0.f : live ? t[r] * a.scale : kNegInf;
        }
      }
    float alpha[2];
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
      float bm = kNegInf;
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int r = 0; r < 4; ++r) bm = fmaxf(bm, sc[kt][qt][r]);
      bm = fmaxf(bm, __shfl_xor(bm, 16));
      bm = fmaxf(bm, __shfl_xor(bm, 32));
      const float mn = fmaxf(m[qt], bm);
      const float mu = mn == kNegInf ? 0.f : mn;
      alpha[qt] = __expf(m[qt] - mu);
      float ps = 0.f;
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float p = __expf(sc[kt][qt][r] - mu);
          sc[kt][qt][r] = p;
          ps += p;
        }
      ps += __shfl_xor(ps, 16);
      ps += __shfl_xor(ps, 32);
      l[qt] = l[qt] * alpha[qt] + ps;
      m[qt] = mn;
    }
    bf16x8 pa[2];  // A operand of O += P' V: row = query qt*16 + li, k slots = keys 4g.. | 16+4g..
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
      const int qi = qt * 16 + li;
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float p = sc[kt][qt][r];
          if (a.seed) {
            const uint64_t e = ((uint64_t)(s * a.H + h) * a.Lq + qi) * a.K + (j0 + kt * 16 + 4 * g + r);
            p *= drop_mul(seed, thresh, dscale, e);
          }
          pa[qt][kt * 4 + r] = tobf(p);
        }
    }
#pragma unroll
    for (int qt = 0; qt < 2; ++qt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float al = __shfl(alpha[qt], 4 * g + r);  // alpha of query qt*16 + 4g + r (lane li = 4g + r)
#pragma unroll
        for (int cb = 0; cb < 4; ++cb) o[qt][cb][r] *= al;
      }
    wave_lds_fence();
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) {
      const bf16x8 vb = tr_b(sv, g, li, cb);
#pragma unroll
      for (int qt = 0; qt < 2; ++qt) o[qt][cb] = mfma(pa[qt], vb, o[qt][cb]);
    }
    wave_lds_fence();
  }
  if (g == 0) {
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
      s_m[wave][qt * 16 + li] = m[qt];
      s_l[wave][qt * 16 + li] = l[qt];
    }
  }
#pragma unroll
  for (int qt = 0; qt < 2; ++qt)
#pragma unroll
    for (int cb = 0; cb < 4; ++cb)
#pragma unroll
      for (int r = 0; r < 4; ++r) s_o[wave][qt * 16 + 4 * g + r][cb * 16 + li] = o[qt][cb][r];
  __syncthreads();
  const int qi = tid >> 3, c0 = (tid & 7) * 8;
  float M = kNegInf;
#pragma unroll
  for (int w = 0; w < kWaves; ++w) M = fmaxf(M, s_m[w][qi]);
  const float Mu = M == kNegInf ? 0.f : M;
  float f[kWaves], L = 0.f;
#pragma unroll
  for (int w = 0; w < kWaves; ++w) {
    f[w] = __expf(s_m[w][qi] - Mu);
    L += s_l[w][qi] * f[w];
  }
  if ((tid & 7) == 0) a.lse[((long long)s * a.H + h) * QT + qi] = Mu + __logf(L);
  if (qi < a.Lq) {
    const float inv = 1.f / L;
    uint16_t v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      float acc = 0.f;
#pragma unroll
      for (int w = 0; w < kWaves; ++w) acc += s_o[w][qi][c0 + k] * f[w];
      v[k] = f2bf(acc * inv);
    }
    uint4 pk;
    pk.x = v[0] | ((uint32_t)v[1] << 16);
    pk.y = v[2] | ((uint32_t)v[3] << 16);
    pk.z = v[4] | ((uint32_t)v[5] << 16);
    pk.w = v[6] | ((uint32_t)v[7] << 16);
    *reinterpret_cast<uint4*>(a.out + ((long long)s * a.Lq + qi) * d + h * HD + c0) = pk;
  }
}

__global__ __launch_bounds__(kThreads) void seg_attn_bwd_dq(Args a) {
  __shared__ __attribute__((aligned(16))) unsigned char s_k[kWaves][KB * kRS];
  __shared__ float s_dq[kWaves][QT][HD + 1];
  __shared__ float s_D[QT];
  const int s = blockIdx.x / a.H, h = blockIdx.x % a.H;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, g = lane >> 4, li = lane & 15;
  const int d = a.H * HD;
  const long long b = a.index[s];
  const bool dead = segment_dead(a, s);
  if (h == 0 && tid == 0) a.dead[s] = dead ? 1 : 0;
  {  // D = rowsum(dO * O) of the head: 8 threads a query
    const int qi = tid >> 3, c0 = (tid & 7) * 8;
    float acc = 0.f;
    if (qi < a.Lq) {
      const long long off = ((long long)s * a.Lq + qi) * d + h * HD + c0;
      const uint4 x = *reinterpret_cast<const uint4*>(a.dout + off);
      const uint4 y = *reinterpret_cast<const uint4*>(a.out + off);
      const uint32_t xs[4] = {x.x, x.y, x.z, x.w}, ys[4] = {y.x, y.y, y.z, y.w};
#pragma unroll
      for (int k = 0; k < 4; ++k)
        acc += bf2f((uint16_t)xs[k]) * bf2f((uint16_t)ys[k]) + bf2f((uint16_t)(xs[k] >> 16)) * bf2f((uint16_t)(ys[k] >> 16));
    }
    acc += __shfl_xor(acc, 1);
    acc += __shfl_xor(acc, 2);
    acc += __shfl_xor(acc, 4);
    if ((tid & 7) == 0) {
      s_D[qi] = acc;
      a.D[((long long)s * a.H + h) * QT + qi] = acc;
    }
  }
  __syncthreads();
  bf16x8 qf[2][2], df[2][2];  // B operands: column = query qt*16 + li
  float lse[2], Dq[2];
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    const int qi = qt * 16 + li;
    lse[qt] = a.lse[((long long)s * a.H + h) * QT + qi];
    Dq[qt] = s_D[qi];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const long long off = ((long long)s * a.Lq + qi) * d + h * HD + ks * 32 + 8 * g;
      qf[qt][ks] = qi < a.Lq ? load8(a.q + off) : zero8();
      df[qt][ks] = qi < a.Lq ? load8(a.dout + off) : zero8();
    }
  }
  f32x4 dq[2][4];
#pragma unroll
  for (int qt = 0; qt < 2; ++qt)
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) dq[qt][cb] = f32x4{0.f, 0.f, 0.f, 0.f};
  const uint64_t seed = a.seed ? (uint64_t)a.seed[0] : 0;
  const uint32_t thresh = (uint32_t)fminf(a.p * 16777216.f, 16777216.f);
  const float dscale = 1.f / (1.f - a.p);
  const uint16_t* bk = a.bk ? a.bk + h * HD : nullptr;
  const uint16_t* bv = a.bv ? a.bv + h * HD : nullptr;
  unsigned char* const sk = s_k[wave];
  const int nblk = (a.K + KB - 1) / KB;
  // a segment with every key masked has constant scores: no gradient reaches q (nor k)
  for (int blk = wave; !dead && blk < nblk; blk += kWaves) {
    const int j0 = blk * KB;
    const BlockMasks mk = block_masks(a, s, j0, lane);
    if (mk.live == 0u) continue;
    const long long rbase = (b * a.K + j0) * d + h * HD;
    bf16x8 kf[2][2], vf[2][2];
    row_frags(kf, a.pk + rbase, bk, mk, d, g, li);
    row_frags(vf, a.pv + rbase, bv, mk, d, g, li);
    stage_rows(sk, a.pk + rbase, bk, mk, d, lane);
    bf16x8 da[2];  // A operand of dQ += dS K: row = query qt*16 + li, k slots = keys 4g.. | 16+4g..
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int qt = 0; qt < 2; ++qt) {
        f32x4 st = f32x4{0.f, 0.f, 0.f, 0.f}, dp = f32x4{0.f, 0.f, 0.f, 0.f};
        st = mfma(kf[kt][0], qf[qt][0], st);
        st = mfma(kf[kt][1], qf[qt][1], st);
        dp = mfma(vf[kt][0], df[qt][0], dp);
        dp = mfma(vf[kt][1], df[qt][1], dp);
        const int qi = qt * 16 + li;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int kk = kt * 16 + 4 * g + r;
          const bool live = (mk.live >> kk) & 1u;
          const float p = live ? __expf(st[r] * a.scale - lse[qt]) : 0.f;
          float dpv = dp[r];
          if (a.seed) dpv *= drop_mul(seed, thresh, dscale, ((uint64_t)(s * a.H + h) * a.Lq + qi) * a.K + (j0 + kk));
          da[qt][kt * 4 + r] = tobf(p * (dpv - Dq[qt]) * a.scale);
        }
      }
    wave_lds_fence();
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) {
      const bf16x8 kb = tr_b(sk, g, li, cb);
#pragma unroll
      for (int qt = 0; qt < 2; ++qt) dq[qt][cb] = mfma(da[qt], kb, dq[qt][cb]);
    }
    wave_lds_fence();
  }
#pragma unroll
  for (int qt = 0; qt < 2; ++qt)
#pragma unroll
    for (int cb = 0; cb < 4; ++cb)
#pragma unroll
      for (int r = 0; r < 4; ++r) s_dq[wave][qt * 16 + 4 * g + r][cb * 16 + li] = dq[qt][cb][r];
  __syncthreads();
  const int qi = tid >> 3, c0 = (tid & 7) * 8;
  if (qi < a.Lq) {
    uint16_t v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      float acc = 0.f;
#pragma unroll
      for (int w = 0; w < kWaves; ++w) acc += s_dq[w][qi][c0 + k];
      v[k] = f2bf(acc);
    }
    uint4 pk;
    pk.x = v[0] | ((uint32_t)v[1] << 16);
    pk.y = v[2] | ((uint32_t)v[3] << 16);
    pk.z = v[4] | ((uint32_t)v[5] << 16);
    pk.w = v[6] | ((uint32_t)v[7] << 16);
    *reinterpret_cast<uint4*>(a.dq + ((long long)s * a.Lq + qi) * d + h * HD + c0) = pk;
  }
}

__global__ __launch_bounds__(kThreads) void seg_attn_bwd_dkv(Args a, int nkg) {
  __shared__ __attribute__((aligned(16))) unsigned char s_q[QT * kRS];
  __shared__ __attribute__((aligned(16))) unsigned char s_do[QT * kRS];
  __shared__ float s_lse[QT], s_D[QT];
  int bid = blockIdx.x;
  const int kgrp = bid % nkg;
  bid /= nkg;
  const int h = bid % a.H, b = bid / a.H;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, g = lane >> 4, li = lane & 15;
  const int d = a.H * HD;
  const int nblk = (a.K + KB - 1) / KB;
  const int blk = kgrp * kWaves + wave;
  const bool on = blk < nblk;  // wave-uniform
  const int j0 = blk * KB;
  const long long rbase = ((long long)b * a.K + j0) * d + h * HD;
  // B operands of S = Q K^T and dP = dO V^T: column = key kt*16 + li; the projected rows and the bias
  bf16x8 kP[2][2], vP[2][2], kZ[2], vZ[2];
#pragma unroll
  for (int kt = 0; kt < 2; ++kt) {
    const bool ok = on && j0 + kt * 16 + li < a.K;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const long long off = rbase + (long long)(kt * 16 + li) * d + ks * 32 + 8 * g;
      kP[kt][ks] = ok ? load8(a.pk + off) : zero8();
      vP[kt][ks] = ok ? load8(a.pv + off) : zero8();
    }
  }
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) {
    kZ[ks] = a.bk ? load8(a.bk + h * HD + ks * 32 + 8 * g) : zero8();
    vZ[ks] = a.bv ? load8(a.bv + h * HD + ks * 32 + 8 * g) : zero8();
  }
  f32x4 dk[2][4], dv[2][4], zk[4], zv[4];
#pragma unroll
  for (int cb = 0; cb < 4; ++cb) {
    zk[cb] = zv[cb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) dk[kt][cb] = dv[kt][cb] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  const uint64_t seed = a.seed ? (uint64_t)a.seed[0] : 0;
  const uint32_t thresh = (uint32_t)fminf(a.p * 16777216.f, 16777216.f);
  const float dscale = 1.f / (1.f - a.p);
  for (int s = 0; s < a.n; ++s) {
    if (a.index[s] != b) continue;  // block-uniform
    __syncthreads();                // the previous segment's LDS reads are done
    {
      const int qi = tid >> 3, part = tid & 7;
      uint4 xq = make_uint4(0u, 0u, 0u, 0u), xd = xq;
      if (qi < a.Lq) {
        const long long off = ((long long)s * a.Lq + qi) * d + h * HD + part * 8;
        xq = *reinterpret_cast<const uint4*>(a.q + off);
        xd = *reinterpret_cast<const uint4*>(a.dout + off);
      }
      *reinterpret_cast<uint4*>(s_q + perm_row(qi) * kRS + part * 16) = xq;
      *reinterpret_cast<uint4*>(s_do + perm_row(qi) * kRS + part * 16) = xd;
      if (tid < QT) {
        s_lse[tid] = a.lse[((long long)s * a.H + h) * QT + tid];
        s_D[tid] = a.D[((long long)s * a.H + h) * QT + tid];
      }
    }
    const bool dead = a.dead[s] != 0;
    __syncthreads();
    if (!on) continue;
    const BlockMasks mk = block_masks(a, s, j0, lane);
    const uint32_t wts = dead ? mk.in : mk.live;  // keys with a non-zero weight
    if (wts == 0u) continue;
    const bool zrows = (wts & ~mk.keep) != 0u;  // some weighted key reads the bias row
    bf16x8 kf[2][2], vf[2][2];
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {
      const bool kp = (mk.keep >> (kt * 16 + li)) & 1u;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        kf[kt][ks] = kp ? kP[kt][ks] : kZ[ks];
        vf[kt][ks] = kp ? vP[kt][ks] : vZ[ks];
      }
    }
    bf16x8 aa[2], sa[2];  // A operands (row = key kt*16 + li, k slots = queries 4g.. | 16+4g..): P', dS
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
      bf16x8 qa[2], oa[2];
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const int row = perm_row(qt * 16 + li);
        qa[ks] = *reinterpret_cast<const bf16x8*>(s_q + row * kRS + (ks * 32 + 8 * g) * 2);
        oa[ks] = *reinterpret_cast<const bf16x8*>(s_do + row * kRS + (ks * 32 + 8 * g) * 2);
      }
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) {
        f32x4 st = f32x4{0.f, 0.f, 0.f, 0.f}, dp = f32x4{0.f, 0.f, 0.f, 0.f};
        st = mfma(qa[0], kf[kt][0], st);
        st = mfma(qa[1], kf[kt][1], st);
        dp = mfma(oa[0], vf[kt][0], dp);
        dp = mfma(oa[1], vf[kt][1], dp);
        const int kk = kt * 16 + li;
        const bool w = (wts >> kk) & 1u;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int qi = qt * 16 + 4 * g + r;
          const float p = !w ? 0.f : __expf((dead ? 0.f : st[r] * a.scale) - s_lse[qi]);
          const float dm = a.seed ? drop_mul(seed, thresh, dscale, ((uint64_t)(s * a.H + h) * a.Lq + qi) * a.K + (j0 + kk))
                                  : 1.f;
          aa[kt][qt * 4 + r] = tobf(p * dm);
          sa[kt][qt * 4 + r] = tobf(dead ? 0.f : p * (dp[r] * dm - s_D[qi]) * a.scale);
        }
      }
    }
    wave_lds_fence();
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) {
      const bf16x8 ob = tr_b(s_do, g, li, cb), qb = tr_b(s_q, g, li, cb);
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) {
        const bool kp = (mk.keep >> (kt * 16 + li)) & 1u;
        dv[kt][cb] = mfma(kp ? aa[kt] : zero8(), ob, dv[kt][cb]);
        dk[kt][cb] = mfma(kp ? sa[kt] : zero8(), qb, dk[kt][cb]);
        if (zrows) {
          zv[cb] = mfma(kp ? zero8() : aa[kt], ob, zv[cb]);
          zk[cb] = mfma(kp ? zero8() : sa[kt], qb, zk[cb]);
        }
      }
    }
  }
  if (on) {
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int key = j0 + kt * 16 + 4 * g + r;
        if (key >= a.K) continue;
        const long long off = ((long long)b * a.K + key) * d + h * HD + li;
#pragma unroll
        for (int cb = 0; cb < 4; ++cb) {
          a.dpk[off + cb * 16] = f2bf(dk[kt][cb][r]);
          a.dpv[off + cb * 16] = f2bf(dv[kt][cb][r]);
        }
      }
  }
  // bias partial sums of the wave: column sums of zk / zv (rows = keys)
  const long long P = (long long)a.B * nkg * kWaves;
  const long long part = ((long long)b * nkg + kgrp) * kWaves + wave;
#pragma unroll
  for (int cb = 0; cb < 4; ++cb) {
    float sk = zk[cb][0] + zk[cb][1] + zk[cb][2] + zk[cb][3];
    float sv = zv[cb][0] + zv[cb][1] + zv[cb][2] + zv[cb][3];
    sk += __shfl_xor(sk, 16);
    sk += __shfl_xor(sk, 32);
    sv += __shfl_xor(sv, 16);
    sv += __shfl_xor(sv, 32);
    if (g == 0) {
      float* dst = a.dbias + (((long long)h * P + part) * 2) * HD + cb * 16 + li;
      dst[0] = sk;
      dst[HD] = sv;
    }
  }
}

int fail(const char* msg) {
  snprintf(g_err, sizeof(g_err), "%s", msg);
  return 1;
}

bool aligned16(const void* p) { return p == nullptr || (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

int check(const Args& a) {
  if (a.n < 0 || a.B <= 0 || a.K <= 0 || a.H <= 0) return fail("seg_attention: bad sizes");
  if (a.Lq < 1 || a.Lq > QT) return fail("seg_attention: Lq must be in [1, 32]");
  if (!(a.p >= 0.f && a.p < 1.f)) return fail("seg_attention: p_drop must be in [0, 1)");
  if (!a.q || !a.pk || !a.pv || !a.index || !a.keep || !a.lse) return fail("seg_attention: null pointer");
  if (!aligned16(a.q) || !aligned16(a.pk) || !aligned16(a.pv) || !aligned16(a.bk) || !aligned16(a.bv))
    return fail("seg_attention: operands must be 16-byte aligned");
  return 0;
}

}  // namespace

extern "C" {

int mfl_seg_attention_forward(const void* q, const void* pk, const void* pv, const void* bias_k, const void* bias_v,
                              const int64_t* index, const uint8_t* keep, const uint8_t* masked, int64_t n, int64_t B,
                              int64_t K, int64_t Lq, int64_t H, float scale, float p_drop, const int64_t* seed,
                              void* out, float* lse, void* stream) {
  Args a{};
  a.q = static_cast<const uint16_t*>(q);
  a.pk = static_cast<const uint16_t*>(pk);
  a.pv = static_cast<const uint16_t*>(pv);
  a.bk = static_cast<const uint16_t*>(bias_k);
  a.bv = static_cast<const uint16_t*>(bias_v);
  a.index = index;
  a.keep = keep;
  a.masked = masked;
  a.n = (int)n, a.B = (int)B, a.K = (int)K, a.Lq = (int)Lq, a.H = (int)H;
  a.scale = scale, a.p = seed ? p_drop : 0.f, a.seed = seed;
  a.out = static_cast<uint16_t*>(out);
  a.lse = lse;
  if (check(a)) return 1;
  if (!out || !aligned16(out)) return fail("seg_attention: bad output pointer");
  if (n == 0) return 0;
  hipLaunchKernelGGL(seg_attn_fwd, dim3((unsigned)(n * H)), dim3(kThreads), 0, static_cast<hipStream_t>(stream), a);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : fail(hipGetErrorString(e));
}

int64_t mfl_seg_attention_bias_parts(int64_t B, int64_t K) {
  const int64_t nblk = (K + KB - 1) / KB;
  return B * ((nblk + kWaves - 1) / kWaves) * kWaves;
}

int64_t mfl_seg_attention_workspace_bytes(int64_t n, int64_t H) { return n * H * QT * 4 + ((n * 4 + 15) / 16) * 16; }

int mfl_seg_attention_backward(const void* q, const void* pk, const void* pv, const void* bias_k, const void* bias_v,
                               const int64_t* index, const uint8_t* keep, const uint8_t* masked, int64_t n, int64_t B,
                               int64_t K, int64_t Lq, int64_t H, float scale, float p_drop, const int64_t* seed,
                               const void* out, const float* lse, const void* dout, void* dq, void* dpk, void* dpv,
                               float* dbias_part, void* workspace, void* stream) {
  Args a{};
  a.q = static_cast<const uint16_t*>(q);
  a.pk = static_cast<const uint16_t*>(pk);
  a.pv = static_cast<const uint16_t*>(pv);
  a.bk = static_cast<const uint16_t*>(bias_k);
  a.bv = static_cast<const uint16_t*>(bias_v);
  a.index = index;
  a.keep = keep;
  a.masked = masked;
  a.n = (int)n, a.B = (int)B, a.K = (int)K, a.Lq = (int)Lq, a.H = (int)H;
  a.scale = scale, a.p = seed ? p_drop : 0.f, a.seed = seed;
  a.out = static_cast<uint16_t*>(const_cast<void*>(out));
  a.lse = const_cast<float*>(lse);
  a.dout = static_cast<const uint16_t*>(dout);
  a.dq = static_cast<uint16_t*>(dq);
  a.dpk = static_cast<uint16_t*>(dpk);
  a.dpv = static_cast<uint16_t*>(dpv);
  a.dbias = dbias_part;
  a.D = static_cast<float*>(workspace);
  a.dead = reinterpret_cast<int*>(static_cast<char*>(workspace) + n * H * QT * 4);
  if (check(a)) return 1;
  if (!out || !dout || !dq || !dpk || !dpv || !dbias_part || !workspace) return fail("seg_attention: null pointer");
  if (!aligned16(out) || !aligned16(dout) || !aligned16(dq) || !aligned16(workspace))
    return fail("seg_attention: operands must be 16-byte aligned");
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (n > 0) hipLaunchKernelGGL(seg_attn_bwd_dq, dim3((unsigned)(n * H)), dim3(kThreads), 0, st, a);
  const int nblk = (int)((K + KB - 1) / KB), nkg = (nblk + kWaves - 1) / kWaves;
  hipLaunchKernelGGL(seg_attn_bwd_dkv, dim3((unsigned)(B * H * nkg)), dim3(kThreads), 0, st, a, nkg);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : fail(hipGetErrorString(e));
}

const char* mfl_seg_attention_last_error(void) { return g_err; }

}  // extern "C"
