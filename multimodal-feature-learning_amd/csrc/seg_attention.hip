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
constexpr int kMaxBlk = 256;     // key blocks per segment held as LDS bit words: K <= 8192
constexpr int kListChunk = 1024;  // segments scanned per pass of seg_attn_bwd_dkv's clip list
constexpr float kNegInf = -INFINITY;
constexpr float kLog2e = 1.4426950408889634f;

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;

thread_local char g_err[256] = "";

struct Args {
  const uint16_t *q, *pk, *pv, *bk, *bv;
  const int64_t* index;
  const int32_t* order;  // segments in dispatch order (sorted by clip: the clip's rows stay in L2), or null
  const uint8_t *keep, *masked;
  int n, B, K, Lq, H;
  int vbits;  // keep / masked rows readable 16 bytes at a time (K % 16 == 0, 16-byte aligned)
  float scale, p;
  const int64_t* seed;
  uint16_t* out;
  float* lse;
  const uint16_t* dout;
  uint16_t *dq, *dpk, *dpv;
  long long rs_k, rs_v;  // dpk / dpv row strides (elements): d, or a caller's column block of a wider buffer
  float* dbias;  // (H, P, 2, 64)
  float* D;      // (n, H, 32)
  int* dead;     // (n)
  uint16_t* dbits;  // dropout keep bits, (n, H, nblk, 64) words: written by the forward, read by the backward, or null
};

// the word of (segment s, head h, key block blk) in the dropout keep-bit buffer: lane (g, li) of the
// forward's block holds bit kt*8 + qt*4 + r for key kt*16 + 4g + r, query qt*16 + li
__device__ __forceinline__ long long dbits_at(const Args& a, int s, int h, int blk, int nblk) {
  return ((long long)(s * a.H + h) * nblk + blk) * 64;
}

__device__ __forceinline__ void wave_lds_fence() { asm volatile("" ::: "memory"); }

__device__ __forceinline__ uint16_t f2bf(float x) {
  const uint32_t u = __float_as_uint(x);
  return (uint16_t)((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
}
// the MFMA operands' rounding: gfx950's v_cvt_pk_bf16_f32 (round to nearest even, two values an
// instruction) — bitwise f2bf for every finite input, against f2bf's ~5 integer ops a value
__device__ __forceinline__ __bf16 tobf(float x) { return (__bf16)x; }
__device__ __forceinline__ float bf2f(uint16_t u) { return __uint_as_float((uint32_t)u << 16); }

__device__ __forceinline__ bf16x8 zero8() {
  const __bf16 z = __builtin_bit_cast(__bf16, (uint16_t)0);
  return bf16x8{z, z, z, z, z, z, z, z};
}
__device__ __forceinline__ bf16x8 load8(const uint16_t* p) { return *reinterpret_cast<const bf16x8*>(p); }

// the attention-dropout keep bits: a 32-bit mix (murmur3's finaliser) of a key-pair index and the
// seed folded to 32 bits.  One draw covers keys 2i and 2i + 1 of a query row (row = (s * H + h) *
// Lq + q): its low 16 bits decide key 2i, its high 16 bits key 2i + 1, kept iff >= p * 2^16.  The
// finaliser's three 32-bit multiplies run at a quarter of the VALU rate, so a draw per key was ~17 us
// of the DVC step's forward call; a draw per pair halves that.  The index row * ceil(K / 2) + i fits
// 32 bits (n * H * Lq * K < 2^32 is checked on the host)
__device__ __forceinline__ uint32_t drop_bits(uint32_t key, uint32_t e) {
  uint32_t x = e * 0x9E3779B1u + key;
  x ^= x >> 16;
  x *= 0x85EBCA6Bu;
  x ^= x >> 13;
  x *= 0xC2B2AE35u;
  x ^= x >> 16;
  return x;
}
__device__ __forceinline__ uint32_t drop_pair(uint32_t key, uint32_t row, int j, uint32_t k2) {
  return drop_bits(key, row * k2 + ((uint32_t)j >> 1));
}
__device__ __forceinline__ bool pair_keep(uint32_t x, int j, uint32_t thresh) {
  return ((j & 1) ? x >> 16 : x & 0xffffu) >= thresh;
}
__device__ __forceinline__ float drop_mul(uint32_t key, uint32_t thresh, float dscale, uint32_t row, int j,
                                          uint32_t k2) {
  return pair_keep(drop_pair(key, row, j, k2), j, thresh) ? dscale : 0.f;
}
__device__ __forceinline__ uint32_t drop_thresh(float p) { return (uint32_t)fminf(p * 65536.f, 65536.f); }
// bit i of w ? dscale : 0 — the bit sign-extended to an all-ones / zero mask over dscale's bits (two
// VALU ops against the compare-and-select's three; bitwise the same value)
__device__ __forceinline__ float bit_scale(uint32_t w, int i, float dscale) {
  return __uint_as_float((uint32_t)__builtin_amdgcn_sbfe((int)w, i, 1) & __float_as_uint(dscale));
}
__device__ __forceinline__ uint32_t drop_key(const int64_t* seed) {
  if (!seed) return 0u;
  const uint64_t v = (uint64_t)seed[0];
  return (uint32_t)v ^ (uint32_t)(v >> 32);
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

// an LDS word every lane reads at the same (wave-uniform) index, as a scalar: the compiler cannot
// tell it is uniform and branched on conditions derived from it under lane masks
__device__ __forceinline__ uint32_t uword(const uint32_t* w, int i) {
  return (uint32_t)__builtin_amdgcn_readfirstlane((int)w[i]);
}

__device__ __forceinline__ uint32_t in_mask(int j0, int K) {
  return j0 + KB <= K ? 0xffffffffu : (j0 >= K ? 0u : (1u << (K - j0)) - 1u);
}

// bit i of the result: byte i of v is non-zero (nonzero) / zero (!nonzero)
__device__ __forceinline__ uint32_t byte_bits16(uint4 v, bool nonzero) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
  uint32_t r = 0u;
#pragma unroll
  for (int i = 0; i < 16; ++i) r |= (uint32_t)((((w[i >> 2] >> (8 * (i & 3))) & 0xffu) != 0u) == nonzero) << i;
  return r;
}

// the unmasked / kept-row bits of keys j0 .. j0+31 of segment s (masked to the keys that exist)
__device__ __forceinline__ void block_bits(const Args& a, int s, int j0, uint32_t& live, uint32_t& keep) {
  const uint32_t inm = in_mask(j0, a.K);
  const long long e = (long long)s * a.K + j0;
  if (a.vbits) {
    const bool two = j0 + 16 < a.K;
    keep = byte_bits16(*reinterpret_cast<const uint4*>(a.keep + e), true) |
           (two ? byte_bits16(*reinterpret_cast<const uint4*>(a.keep + e + 16), true) << 16 : 0u);
    live = a.masked == nullptr
               ? inm
               : byte_bits16(*reinterpret_cast<const uint4*>(a.masked + e), false) |
                     (two ? byte_bits16(*reinterpret_cast<const uint4*>(a.masked + e + 16), false) << 16 : 0u);
  } else {
    live = keep = 0u;
    for (int kk = 0; kk < KB && j0 + kk < a.K; ++kk) {
      keep |= (uint32_t)(a.keep[e + kk] != 0) << kk;
      live |= (uint32_t)(a.masked == nullptr || a.masked[e + kk] == 0) << kk;
    }
  }
  live &= inm;
  keep &= inm;
}

// the segment's unmasked / kept-row bits per 32-key block into LDS; returns whether every key is
// masked (block-wide: the barrier also publishes the words).  With 16-byte rows (a.vbits) every
// thread turns 16 keys' bytes into bits with one load of each mask — one round trip for K <= 4096
// (the byte-per-lane loop below costs a dependent round trip per 4 blocks: at the DVC step's
// K = 1920 that scan was most of the kernels' time)
__device__ __forceinline__ bool segment_bits(const Args& a, int s, uint32_t* s_live, uint32_t* s_keep, int nblk,
                                             int wave, int lane) {
  int any = 0;
  if (a.vbits) {
    const int nch = a.K >> 4;  // 16-key chunks; chunk c = half (c & 1) of block c / 2
    const int tid = wave * 64 + lane;
    for (int c0 = 0; c0 < nch; c0 += kThreads) {
      const int c = c0 + tid;
      uint32_t lv = 0u, kp = 0u;
      if (c < nch) {
        const long long e = (long long)s * a.K + 16 * c;
        kp = byte_bits16(*reinterpret_cast<const uint4*>(a.keep + e), true);
        lv = a.masked == nullptr ? 0xffffu : byte_bits16(*reinterpret_cast<const uint4*>(a.masked + e), false);
      }
      const uint32_t lv1 = __shfl_xor(lv, 1), kp1 = __shfl_xor(kp, 1);  // (c and c ^ 1: neighbouring lanes)
      if (c < nch && (c & 1) == 0) {
        s_live[c >> 1] = lv | (lv1 << 16);
        s_keep[c >> 1] = kp | (kp1 << 16);
      }
      any |= lv != 0u;
    }
    return !__syncthreads_or(any);
  }
  for (int blk = wave; blk < nblk; blk += kWaves) {
    const int j = blk * KB + (lane & 31);
    const bool lo = lane < 32 && j < a.K;
    const long long e = (long long)s * a.K + j;
    const uint32_t live = (uint32_t)__ballot(lo && (a.masked == nullptr || a.masked[e] == 0));
    const uint32_t keep = (uint32_t)__ballot(lo && a.keep[e] != 0);
    if (lane == 0) {
      s_live[blk] = live;
      s_keep[blk] = keep;
    }
    any |= live != 0u;
  }
  return !__syncthreads_or(any);
}

// fragments of the block's 32 rows (row kt*16 + li, head dims ks*32 + 8g ..): the A operand of a
// product reducing over head dims, and, stored at perm_row, the LDS tile of a transposed B operand
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

__device__ __forceinline__ void store_frags(unsigned char* tile, const bf16x8 (&f)[2][2], int g, int li) {
#pragma unroll
  for (int kt = 0; kt < 2; ++kt)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
      *reinterpret_cast<bf16x8*>(tile + perm_row(kt * 16 + li) * kRS + (ks * 32 + 8 * g) * 2) = f[kt][ks];
}

// the wave's next block at or after `from` (stride kWaves) with a non-zero weight on some key
__device__ __forceinline__ int next_active(const uint32_t* s_live, int from, int nblk, bool dead) {
  int bb = from;
  while (bb < nblk && !dead && uword(s_live, bb) == 0u) bb += kWaves;
  return bb;
}

// the waves' staging tiles (block loop) and their partial O (final combine) share one LDS buffer:
// 36 KB a workgroup, so LDS admits 4 workgroups per CU and the VGPRs 3
constexpr int kStageBytes = kWaves * KB * kRS;
constexpr int kPartBytes = kWaves * QT * (HD + 1) * 4;
constexpr int kRawBytes = kStageBytes > kPartBytes ? kStageBytes : kPartBytes;

__global__ __launch_bounds__(kThreads, 3) void seg_attn_fwd(Args a) {
  __shared__ __attribute__((aligned(16))) unsigned char s_raw[kRawBytes];
  __shared__ float s_m[kWaves][QT], s_l[kWaves][QT];
  float(*const s_o)[QT][HD + 1] = reinterpret_cast<float(*)[QT][HD + 1]>(s_raw);
  __shared__ uint32_t s_live[kMaxBlk], s_keep[kMaxBlk];
  const int s = a.order ? a.order[blockIdx.x / a.H] : (int)(blockIdx.x / a.H), h = blockIdx.x % a.H;
  const int tid = threadIdx.x, wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63, g = lane >> 4, li = lane & 15;  // (wave: scalar)
  const int d = a.H * HD;
  const long long b = a.index[s];
  const int nblk = (a.K + KB - 1) / KB;
  const bool dead = segment_bits(a, s, s_live, s_keep, nblk, wave, lane);
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
  const uint32_t seed = drop_key(a.seed);
  const uint32_t thresh = drop_thresh(a.p), k2 = (uint32_t)(a.K + 1) >> 1;
  const float dscale = 1.f / (1.f - a.p);
  const float sce = dead ? 0.f : a.scale;  // (wave-uniform)
  const uint16_t* bk = a.bk ? a.bk + h * HD : nullptr;
  const uint16_t* bv = a.bv ? a.bv + h * HD : nullptr;
  unsigned char* const sv = s_raw + wave * KB * kRS;
  // software-pipelined over the wave's blocks: the next block's K / V rows load while this one computes
  int blk = next_active(s_live, wave, nblk, dead);
  bf16x8 kf[2][2], vf[2][2];
  if (blk < nblk) {
    const BlockMasks mk{in_mask(blk * KB, a.K), uword(s_live, blk), uword(s_keep, blk)};
    const long long rbase = (b * a.K + blk * KB) * d + h * HD;
    row_frags(kf, a.pk + rbase, bk, mk, d, g, li);
    row_frags(vf, a.pv + rbase, bv, mk, d, g, li);
  }
  while (blk < nblk) {
    const int j0 = blk * KB;
    const BlockMasks mk{in_mask(j0, a.K), uword(s_live, blk), uword(s_keep, blk)};
    wave_lds_fence();
    store_frags(sv, vf, g, li);
    // keys with a score: the unmasked ones, or every existing key of a dead segment, whose scores are
    // all 0 (t * 0: the same softmax as the constant 0 — a signed zero changes no exp or max result)
    const uint32_t ok = dead ? mk.in : (mk.in & mk.live);
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
          sc[kt][qt][r] = ((ok >> kk) & 1u) ? t[r] * sce : kNegInf;
        }
      }
    const int nb = next_active(s_live, blk + kWaves, nblk, dead);
    if (nb < nblk) {
      const BlockMasks mn{in_mask(nb * KB, a.K), uword(s_live, nb), uword(s_keep, nb)};
      const long long rbase = (b * a.K + nb * KB) * d + h * HD;
      row_frags(kf, a.pk + rbase, bk, mn, d, g, li);
      row_frags(vf, a.pv + rbase, bv, mn, d, g, li);
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
    uint32_t kept = 0u;  // the block's keep bits of this lane (dbits_at)
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
      const uint32_t row = (uint32_t)(s * a.H + h) * a.Lq + qt * 16 + li;
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) {
        uint32_t x[2] = {0u, 0u};  // keys j0 + kt*16 + 4g + {0, 1} and {2, 3}: one draw a pair
        if (a.seed) {
#pragma unroll
          for (int rp = 0; rp < 2; ++rp) x[rp] = drop_pair(seed, row, j0 + kt * 16 + 4 * g + 2 * rp, k2);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float p = sc[kt][qt][r];
          if (a.seed) {
            const bool k = pair_keep(x[r >> 1], r, thresh);  // (= drop_mul: the key's parity is r's)
            kept |= (uint32_t)k << (kt * 8 + qt * 4 + r);
            p *= k ? dscale : 0.f;
          }
          pa[qt][kt * 4 + r] = tobf(p);
        }
      }
    }
    if (a.seed && a.dbits) a.dbits[dbits_at(a, s, h, blk, nblk) + lane] = (uint16_t)kept;
    // rescale O only when some query's running max moved (alpha = exp(0) = 1 exactly otherwise, so
    // skipping the multiplies is bitwise the same; after the first blocks the max rarely moves)
    if (__ballot(alpha[0] != 1.f || alpha[1] != 1.f) != 0ull) {
#pragma unroll
      for (int qt = 0; qt < 2; ++qt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float al = __shfl(alpha[qt], 4 * g + r);  // alpha of query qt*16 + 4g + r (lane li = 4g + r)
#pragma unroll
          for (int cb = 0; cb < 4; ++cb) o[qt][cb][r] *= al;
        }
    }
    wave_lds_fence();
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) {
      const bf16x8 vb = tr_b(sv, g, li, cb);
#pragma unroll
      for (int qt = 0; qt < 2; ++qt) o[qt][cb] = mfma(pa[qt], vb, o[qt][cb]);
    }
    blk = nb;
  }
  if (g == 0) {
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
      s_m[wave][qt * 16 + li] = m[qt];
      s_l[wave][qt * 16 + li] = l[qt];
    }
  }
  __syncthreads();  // every wave is done with its staging tile (the buffer becomes the partial O)
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

// kBits: the forward's recorded keep bits are read (a.seed and a.dbits set), else drawn from the seed
template <bool kBits>
__global__ __launch_bounds__(kThreads, 2) void seg_attn_bwd_dq(Args a) {
  __shared__ __attribute__((aligned(16))) unsigned char s_raw[kRawBytes];  // staging tiles, then partial dQ
  float(*const s_dq)[QT][HD + 1] = reinterpret_cast<float(*)[QT][HD + 1]>(s_raw);
  __shared__ float s_D[QT];
  __shared__ uint32_t s_live[kMaxBlk], s_keep[kMaxBlk];
  __shared__ float s_bias[kWaves][2][HD];
  const int s = a.order ? a.order[blockIdx.x / a.H] : (int)(blockIdx.x / a.H), h = blockIdx.x % a.H;
  const int tid = threadIdx.x, wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63, g = lane >> 4, li = lane & 15;  // (wave: scalar)
  const int d = a.H * HD;
  const long long b = a.index[s];
  const int nblk = (a.K + KB - 1) / KB;
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
  const bool dead = segment_bits(a, s, s_live, s_keep, nblk, wave, lane);  // (its barrier publishes s_D)
  if (h == 0 && tid == 0) a.dead[s] = dead ? 1 : 0;
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
  const float sc2 = a.scale * kLog2e, lse2[2] = {lse[0] * kLog2e, lse[1] * kLog2e};
  f32x4 dq[2][4];
#pragma unroll
  for (int qt = 0; qt < 2; ++qt)
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) dq[qt][cb] = f32x4{0.f, 0.f, 0.f, 0.f};
  // per query, over the keys that read the bias row (keep = 0) with a non-zero weight: the sums of
  // dS and of P' — the bias gradients are sum_q cS[q] Q[q] and sum_q cA[q] dO[q]
  float cS[2] = {0.f, 0.f}, cA[2] = {0.f, 0.f};
  const uint32_t seed = drop_key(a.seed);
  const uint32_t thresh = drop_thresh(a.p), k2 = (uint32_t)(a.K + 1) >> 1;
  const float dscale = 1.f / (1.f - a.p);
  const uint16_t* bk = a.bk ? a.bk + h * HD : nullptr;
  const uint16_t* bv = a.bv ? a.bv + h * HD : nullptr;
  unsigned char* const sk = s_raw + wave * KB * kRS;
  if (dead) {  // uniform weights exp(-lse) on every key; only the bias rows' P' sums are needed
    for (int bb = wave; bb < nblk; bb += kWaves) {
      const uint32_t zr = in_mask(bb * KB, a.K) & ~s_keep[bb];
      if (zr == 0u) continue;
      const uint32_t wd = kBits ? a.dbits[dbits_at(a, s, h, bb, nblk) + lane] : 0u;
#pragma unroll
      for (int qt = 0; qt < 2; ++qt) {
        const int qi = qt * 16 + li;
        const float p = __expf(-lse[qt]);
#pragma unroll
        for (int kt = 0; kt < 2; ++kt)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int kk = kt * 16 + 4 * g + r;
            if (!((zr >> kk) & 1u)) continue;
            cA[qt] += kBits     ? p * (((wd >> (kt * 8 + qt * 4 + r)) & 1u) ? dscale : 0.f)
                      : !a.seed ? p
                                : p * drop_mul(seed, thresh, dscale, (uint32_t)(s * a.H + h) * a.Lq + qi,
                                               bb * KB + kk, k2);
          }
      }
    }
  }
  // a segment with every key masked has constant scores: no gradient reaches q (nor k)
  int blk = dead ? nblk : next_active(s_live, wave, nblk, false);
  bf16x8 kf[2][2], vf[2][2];
  constexpr bool bits = kBits;
  uint32_t wb = 0u;  // the block's keep bits (the forward's), loaded with its rows
  if (blk < nblk) {
    const BlockMasks mk{in_mask(blk * KB, a.K), uword(s_live, blk), uword(s_keep, blk)};
    const long long rbase = (b * a.K + blk * KB) * d + h * HD;
    row_frags(kf, a.pk + rbase, bk, mk, d, g, li);
    row_frags(vf, a.pv + rbase, bv, mk, d, g, li);
    if (bits) wb = a.dbits[dbits_at(a, s, h, blk, nblk) + lane];
  }
  while (blk < nblk) {
    const int j0 = blk * KB;
    const BlockMasks mk{in_mask(j0, a.K), uword(s_live, blk), uword(s_keep, blk)};
    wave_lds_fence();
    store_frags(sk, kf, g, li);
    f32x4 st[2][2], dp[2][2];
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int qt = 0; qt < 2; ++qt) {
        st[kt][qt] = dp[kt][qt] = f32x4{0.f, 0.f, 0.f, 0.f};
        st[kt][qt] = mfma(kf[kt][0], qf[qt][0], st[kt][qt]);
        st[kt][qt] = mfma(kf[kt][1], qf[qt][1], st[kt][qt]);
        dp[kt][qt] = mfma(vf[kt][0], df[qt][0], dp[kt][qt]);
        dp[kt][qt] = mfma(vf[kt][1], df[qt][1], dp[kt][qt]);
      }
    const int nb = next_active(s_live, blk + kWaves, nblk, false);
    const uint32_t wc = wb;
    if (nb < nblk) {
      const BlockMasks mn{in_mask(nb * KB, a.K), uword(s_live, nb), uword(s_keep, nb)};
      const long long rbase = (b * a.K + nb * KB) * d + h * HD;
      row_frags(kf, a.pk + rbase, bk, mn, d, g, li);
      row_frags(vf, a.pv + rbase, bv, mn, d, g, li);
      if (bits) wb = a.dbits[dbits_at(a, s, h, nb, nblk) + lane];
    }
    bf16x8 da[2];  // A operand of dQ += dS K: row = query qt*16 + li, k slots = keys 4g.. | 16+4g..
    // (wave-uniform) some key of the block reads the bias row: only then the per-score bias sums, and
    // branch-free (a 0 / 1 factor in an fma: bitwise the conditional add)
    const bool bias_rows = (mk.in & ~mk.keep) != 0u;
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int qt = 0; qt < 2; ++qt) {
        const int qi = qt * 16 + li;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int kk = kt * 16 + 4 * g + r;
          const uint32_t lm = (uint32_t)__builtin_amdgcn_sbfe((int)mk.live, kk, 1);  // (masked exp: see dK / dV)
          // (base-2 operands as in dK / dV: one fma + v_exp_f32)
          const float p =
              __uint_as_float(__float_as_uint(__builtin_amdgcn_exp2f(fmaf(st[kt][qt][r], sc2, -lse2[qt]))) & lm);
          const float dm =
              bits      ? bit_scale(wc, kt * 8 + qt * 4 + r, dscale)
              : !a.seed ? 1.f
                        : drop_mul(seed, thresh, dscale, (uint32_t)(s * a.H + h) * a.Lq + qi, j0 + kk, k2);
          const float ds = p * (dp[kt][qt][r] * dm - Dq[qt]) * a.scale;
          da[qt][kt * 4 + r] = tobf(ds);
          if (bias_rows) {
            const float nk = ((mk.keep >> kk) & 1u) ? 0.f : 1.f;
            cS[qt] = fmaf(nk, ds, cS[qt]);
            cA[qt] = fmaf(nk, p * dm, cA[qt]);
          }
        }
      }
    wave_lds_fence();
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) {
      const bf16x8 kb = tr_b(sk, g, li, cb);
#pragma unroll
      for (int qt = 0; qt < 2; ++qt) dq[qt][cb] = mfma(da[qt], kb, dq[qt][cb]);
    }
    blk = nb;
  }
  __syncthreads();  // every wave is done with its staging tile (the buffer becomes the partial dQ)
#pragma unroll
  for (int qt = 0; qt < 2; ++qt)
#pragma unroll
    for (int cb = 0; cb < 4; ++cb)
#pragma unroll
      for (int r = 0; r < 4; ++r) s_dq[wave][qt * 16 + 4 * g + r][cb * 16 + li] = dq[qt][cb][r];
  {  // the wave's bias partials: sum over its queries of cS Q / cA dO (head dims ks*32 + 8g + j)
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
      cS[qt] += __shfl_xor(cS[qt], 16);
      cS[qt] += __shfl_xor(cS[qt], 32);
      cA[qt] += __shfl_xor(cA[qt], 16);
      cA[qt] += __shfl_xor(cA[qt], 32);
    }
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float vk = 0.f, vv = 0.f;
#pragma unroll
        for (int qt = 0; qt < 2; ++qt) {
          vk += cS[qt] * (float)qf[qt][ks][j];
          vv += cA[qt] * (float)df[qt][ks][j];
        }
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) {
          vk += __shfl_xor(vk, o);
          vv += __shfl_xor(vv, o);
        }
        if (li == 0) {
          s_bias[wave][0][ks * 32 + 8 * g + j] = vk;
          s_bias[wave][1][ks * 32 + 8 * g + j] = vv;
        }
      }
  }
  __syncthreads();
  if (tid < 2 * HD) {  // (H, n, 2, 64) partials: this (segment, head)'s
    const int kv = tid >> 6, c = tid & 63;
    a.dbias[(((long long)h * a.n + s) * 2 + kv) * HD + c] =
        s_bias[0][kv][c] + s_bias[1][kv][c] + s_bias[2][kv][c] + s_bias[3][kv][c];
  }
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

// one segment's operands of seg_attn_bwd_dkv, loaded a segment ahead by each wave: the wave's Q /
// dO rows as fragments (row qt*16 + li, head dims ks*32 + 8g ..), lse / D of query lane & 31, the
// masked / kept bytes of key j0 + (lane & 31), the dead flag
struct SegPrefetch {
  bf16x8 q[2][2], o[2][2];
  float lse, D;
  uint32_t mb, kb;
  uint32_t db;  // the forward's keep-bit word of (s, h, this block), lane's own (dbits_at)
  int dead;
};

__device__ __forceinline__ void load_segment(const Args& a, int s, int h, int d, int j0, int g, int li, int lane,
                                             SegPrefetch& p) {
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    const int qi = qt * 16 + li;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const long long off = ((long long)s * a.Lq + qi) * d + h * HD + ks * 32 + 8 * g;
      p.q[qt][ks] = qi < a.Lq ? load8(a.q + off) : zero8();
      p.o[qt][ks] = qi < a.Lq ? load8(a.dout + off) : zero8();
    }
  }
  p.lse = a.lse[((long long)s * a.H + h) * QT + (lane & 31)];
  p.D = a.D[((long long)s * a.H + h) * QT + (lane & 31)];
  p.dead = a.dead[s];
  p.db = a.dbits ? a.dbits[dbits_at(a, s, h, j0 / KB, (a.K + KB - 1) / KB) + lane] : 0u;
  const int j = j0 + (lane & 31);
  p.mb = 1u;
  p.kb = 0u;
  if (lane < 32 && j < a.K) {
    const long long e = (long long)s * a.K + j;
    p.mb = a.masked ? a.masked[e] : 0u;
    p.kb = a.keep[e];
  }
}

// one workgroup per (clip, head, 32-key block); its 4 waves take the clip's segments round-robin
// (the DVC's composed crops send most segments to a few clips: a wave per block walked all of a heavy
// clip's segments alone) without block barriers — each stages its own copy of a segment's Q / dO
// rows in LDS and prefetches its next segment's while it computes — and add their partial dK / dV
// through LDS at the end
template <bool kBits>
__global__ __launch_bounds__(kThreads, 2) void seg_attn_bwd_dkv(Args a) {
  constexpr int kStage = 2 * QT * kRS;                  // a wave's Q + dO rows
  constexpr int kPart = 2 * 2 * 4 * 64 * 16;            // a wave's dK + dV tiles (f32x4 a lane)
  constexpr int kUnion = (kWaves - 1) * kPart > kWaves * kStage ? (kWaves - 1) * kPart : kWaves * kStage;
  __shared__ __attribute__((aligned(16))) unsigned char s_buf[kUnion];
  // the block's K, V rows: 128-B rows, 16-B chunk c of row r at slot c ^ ((r >> 1) & 7) — the B-operand
  // reads (rows kt*16 + li, chunks ks*4 + g) then meet 16 distinct slots in each ds_read_b128 lane group
  // (the 144-B padded rows of the Q / dO tiles put two lanes of a group on most slots)
  __shared__ __attribute__((aligned(16))) unsigned char s_kv[2 * KB * 128];
  __shared__ __attribute__((aligned(16))) float s_lse[kWaves][QT];
  __shared__ __attribute__((aligned(16))) float s_D[kWaves][QT];
  __shared__ int s_list[kListChunk];
  __shared__ int s_wcnt[kWaves];
  const int nblk = (a.K + KB - 1) / KB;
  int bid = blockIdx.x;
  const int blk = bid % nblk;
  bid /= nblk;
  const int h = bid % a.H, b = bid / a.H;
  const int tid = threadIdx.x, wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63, g = lane >> 4, li = lane & 15;  // (wave: scalar)
  const int d = a.H * HD;
  const bool on = true;
  const int j0 = blk * KB;
  const uint32_t inm = in_mask(j0, a.K);
  const long long rbase = ((long long)b * a.K + j0) * d + h * HD;
  unsigned char* const sq = s_buf + wave * kStage;
  unsigned char* const sd = sq + QT * kRS;
  // the block's projected K and V rows (B operands of S = Q K^T and dP = dO V^T: column = key kt*16
  // + li; keys a segment reads as the bias row get no contribution here — seg_attn_bwd_dq sums
  // those) staged once in LDS for the 4 waves, 16 bytes a thread: per-wave register copies cost 32
  // VGPRs and made the kernel spill at 256
  {
    const int row = tid >> 3, ch = tid & 7;
    const bool ok = on && j0 + row < a.K;
    const long long off = rbase + (long long)row * d + ch * 8;
    const int sw = (ch ^ ((row >> 1) & 7)) << 4;
    *reinterpret_cast<bf16x8*>(s_kv + row * 128 + sw) = ok ? load8(a.pk + off) : zero8();
    *reinterpret_cast<bf16x8*>(s_kv + (KB + row) * 128 + sw) = ok ? load8(a.pv + off) : zero8();
  }
  f32x4 dk[2][4], dv[2][4];
#pragma unroll
  for (int cb = 0; cb < 4; ++cb)
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) dk[kt][cb] = dv[kt][cb] = f32x4{0.f, 0.f, 0.f, 0.f};
  const uint32_t seed = drop_key(a.seed);
  const uint32_t thresh = drop_thresh(a.p), k2 = (uint32_t)(a.K + 1) >> 1;
  const float dscale = 1.f / (1.f - a.p);
  for (int c0 = 0; c0 < a.n; c0 += kListChunk) {
    // the segments of this chunk that read clip b, in order (4 candidates a thread, block prefix sum)
    // (only those giving some kept key of this block a non-zero weight: the others add nothing)
    int flags = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int s = c0 + tid * 4 + i;
      if (s < a.n && a.index[s] == b) {
        uint32_t lv, kp;
        block_bits(a, s, j0, lv, kp);
        if (((a.dead[s] != 0 ? inm : lv) & kp) != 0u) flags |= 1 << i;
      }
    }
    const int cnt = __popc(flags);
    int x = cnt;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int y = __shfl_up(x, o);
      if (lane >= o) x += y;
    }
    __syncthreads();  // the previous chunk's list reads are done
    if (lane == 63) s_wcnt[wave] = x;
    __syncthreads();
    int pos = x - cnt;
    for (int w = 0; w < wave; ++w) pos += s_wcnt[w];
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if ((flags >> i) & 1) s_list[pos++] = c0 + tid * 4 + i;
    const int total = s_wcnt[0] + s_wcnt[1] + s_wcnt[2] + s_wcnt[3];
    __syncthreads();
    SegPrefetch pf;
    if (wave < total) load_segment(a, s_list[wave], h, d, j0, g, li, lane, pf);
    for (int it = wave; it < total; it += kWaves) {
      const int s = s_list[it];
      wave_lds_fence();  // the previous segment's LDS reads are issued before these writes
      store_frags(sq, pf.q, g, li);
      store_frags(sd, pf.o, g, li);
      if (lane < QT) {
        s_lse[wave][lane] = pf.lse * kLog2e;  // (base-2: P = 2^(S sc log2 e - lse log2 e))
        s_D[wave][lane] = pf.D;
      }
      const bool dead = pf.dead != 0;
      const float sc = dead ? 0.f : a.scale;  // (wave-uniform)
      const float sc2 = sc * kLog2e;
      const bool lo = lane < 32;
      const uint32_t live = (uint32_t)__ballot(lo && pf.mb == 0u) & inm;
      const uint32_t keep = (uint32_t)__ballot(lo && pf.kb != 0u) & inm;
      // keep bit of (query qt*16 + 4g + r, key kt*16 + li): bit kt*8 + qt*4 + (li & 3) of the forward
      // lane (li >> 2, 4g + r)'s word, gathered into bit kt*8 + qt*4 + r of one register
      uint32_t dmk = 0u;
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (kBits) dmk |= ((__shfl(pf.db, (li >> 2) * 16 + 4 * g + r) >> (li & 3)) & 0x1111u) << r;
      if (it + kWaves < total) load_segment(a, s_list[it + kWaves], h, d, j0, g, li, lane, pf);  // in flight meanwhile
      const uint32_t wts = (dead ? inm : live) & keep;  // kept keys with a non-zero weight
      if (wts == 0u) continue;
      wave_lds_fence();
      bf16x8 aa[2], sa[2];  // A operands (row = key kt*16 + li, k slots = queries 4g.. | 16+4g..): P', dS
      bf16x8 qa[2][2], oa[2][2];
#pragma unroll
      for (int qt = 0; qt < 2; ++qt)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          const int row = perm_row(qt * 16 + li);
          qa[qt][ks] = *reinterpret_cast<const bf16x8*>(sq + row * kRS + (ks * 32 + 8 * g) * 2);
          oa[qt][ks] = *reinterpret_cast<const bf16x8*>(sd + row * kRS + (ks * 32 + 8 * g) * 2);
        }
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) {
        bf16x8 kb[2], vb[2];
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          const int r = kt * 16 + li, sw = ((ks * 4 + g) ^ ((r >> 1) & 7)) << 4;
          kb[ks] = *reinterpret_cast<const bf16x8*>(s_kv + r * 128 + sw);
          vb[ks] = *reinterpret_cast<const bf16x8*>(s_kv + (KB + r) * 128 + sw);
        }
#pragma unroll
        for (int qt = 0; qt < 2; ++qt) {
          f32x4 st = f32x4{0.f, 0.f, 0.f, 0.f}, dp = f32x4{0.f, 0.f, 0.f, 0.f};
          st = mfma(qa[qt][0], kb[0], st);
          st = mfma(qa[qt][1], kb[1], st);
          dp = mfma(oa[qt][0], vb[0], dp);
          dp = mfma(oa[qt][1], vb[1], dp);
          const int kk = kt * 16 + li;
          // all-ones where key kk has a weight: exp is taken for every score and masked (bitwise the
          // select; as `w ? exp : 0` the compiler branched around each exp under a lane mask)
          const uint32_t wm = (uint32_t)__builtin_amdgcn_sbfe((int)wts, kk, 1);
          // lse / D of queries qt*16 + 4g .. + 3: one 16-B read each
          const float4 l4 = *reinterpret_cast<const float4*>(&s_lse[wave][qt * 16 + 4 * g]);
          const float4 d4 = *reinterpret_cast<const float4*>(&s_D[wave][qt * 16 + 4 * g]);
          const float lr[4] = {l4.x, l4.y, l4.z, l4.w}, dr[4] = {d4.x, d4.y, d4.z, d4.w};
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int qi = qt * 16 + 4 * g + r;
            // (sc = 0 for a dead segment: st * 0 and the dS product's * 0 are the zeros the dead
            // branch gave, bitwise — the finite operands' signed zeros add nothing to dK / dV)
            // (one fma + v_exp_f32 on base-2 operands: __expf's x * log2 e multiply folded into them)
            const float p = __uint_as_float(
                __float_as_uint(__builtin_amdgcn_exp2f(fmaf(st[r], sc2, -lr[r]))) & wm);
            const float dm = kBits     ? bit_scale(dmk, kt * 8 + qt * 4 + r, dscale)
                             : !a.seed ? 1.f
                                       : drop_mul(seed, thresh, dscale, (uint32_t)(s * a.H + h) * a.Lq + qi,
                                                  j0 + kk, k2);
            aa[kt][qt * 4 + r] = tobf(p * dm);
            sa[kt][qt * 4 + r] = tobf(p * (dp[r] * dm - dr[r]) * sc);
          }
        }
      }
#pragma unroll
      for (int cb = 0; cb < 4; ++cb) {
        const bf16x8 ob = tr_b(sd, g, li, cb), qb = tr_b(sq, g, li, cb);
#pragma unroll
        for (int kt = 0; kt < 2; ++kt) {
          dv[kt][cb] = mfma(aa[kt], ob, dv[kt][cb]);
          dk[kt][cb] = mfma(sa[kt], qb, dk[kt][cb]);
        }
      }
    }
  }
  __syncthreads();  // every wave is done with its staging rows (the buffer becomes the partials)
  f32x4* const part = reinterpret_cast<f32x4*>(s_buf);
  if (wave > 0) {
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int cb = 0; cb < 4; ++cb) {
        part[(((wave - 1) * 2 + 0) * 8 + kt * 4 + cb) * 64 + lane] = dk[kt][cb];
        part[(((wave - 1) * 2 + 1) * 8 + kt * 4 + cb) * 64 + lane] = dv[kt][cb];
      }
  }
  __syncthreads();
  if (wave == 0) {
#pragma unroll
    for (int w = 1; w < kWaves; ++w)
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int cb = 0; cb < 4; ++cb) {
          dk[kt][cb] += part[(((w - 1) * 2 + 0) * 8 + kt * 4 + cb) * 64 + lane];
          dv[kt][cb] += part[(((w - 1) * 2 + 1) * 8 + kt * 4 + cb) * 64 + lane];
        }
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int key = j0 + kt * 16 + 4 * g + r;
        if (key >= a.K) continue;
        const long long row = (long long)b * a.K + key, col = h * HD + li;
#pragma unroll
        for (int cb = 0; cb < 4; ++cb) {
          a.dpk[row * a.rs_k + col + cb * 16] = f2bf(dk[kt][cb][r]);
          a.dpv[row * a.rs_v + col + cb * 16] = f2bf(dv[kt][cb][r]);
        }
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
  if (a.K > kMaxBlk * KB) return fail("seg_attention: K must be <= 8192");
  if ((double)a.n * a.H * a.Lq * a.K >= 4294967296.0) return fail("seg_attention: n * H * Lq * K must be < 2^32");
  if (!(a.p >= 0.f && a.p < 1.f)) return fail("seg_attention: p_drop must be in [0, 1)");
  if (!a.q || !a.pk || !a.pv || !a.index || !a.keep || !a.lse) return fail("seg_attention: null pointer");
  if (!aligned16(a.q) || !aligned16(a.pk) || !aligned16(a.pv) || !aligned16(a.bk) || !aligned16(a.bv))
    return fail("seg_attention: operands must be 16-byte aligned");
  return 0;
}

}  // namespace

extern "C" {

int mfl_seg_attention_forward(const void* q, const void* pk, const void* pv, const void* bias_k, const void* bias_v,
                              const int64_t* index, const int32_t* order, const uint8_t* keep, const uint8_t* masked,
                              int64_t n, int64_t B,
                              int64_t K, int64_t Lq, int64_t H, float scale, float p_drop, const int64_t* seed,
                              void* out, float* lse, void* stream) {
  return mfl_seg_attention_forward_ex(q, pk, pv, bias_k, bias_v, index, order, keep, masked, n, B, K, Lq, H, scale,
                                      p_drop, seed, out, lse, nullptr, stream);
}

int64_t mfl_seg_attention_drop_bits_bytes(int64_t n, int64_t K, int64_t H) {
  return n * H * ((K + KB - 1) / KB) * 64 * 2;
}

int mfl_seg_attention_forward_ex(const void* q, const void* pk, const void* pv, const void* bias_k,
                                 const void* bias_v, const int64_t* index, const int32_t* order, const uint8_t* keep,
                                 const uint8_t* masked, int64_t n, int64_t B, int64_t K, int64_t Lq, int64_t H,
                                 float scale, float p_drop, const int64_t* seed, void* out, float* lse,
                                 uint16_t* drop_bits, void* stream) {
  Args a{};
  a.dbits = drop_bits;
  a.q = static_cast<const uint16_t*>(q);
  a.pk = static_cast<const uint16_t*>(pk);
  a.pv = static_cast<const uint16_t*>(pv);
  a.bk = static_cast<const uint16_t*>(bias_k);
  a.bv = static_cast<const uint16_t*>(bias_v);
  a.index = index;
  a.order = order;
  a.keep = keep;
  a.masked = masked;
  a.n = (int)n, a.B = (int)B, a.K = (int)K, a.Lq = (int)Lq, a.H = (int)H;
  a.vbits = K % 16 == 0 && aligned16(keep) && aligned16(masked);
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

int64_t mfl_seg_attention_bias_parts(int64_t n) { return n; }

int64_t mfl_seg_attention_workspace_bytes(int64_t n, int64_t H) { return n * H * QT * 4 + ((n * 4 + 15) / 16) * 16; }

int mfl_seg_attention_backward(const void* q, const void* pk, const void* pv, const void* bias_k, const void* bias_v,
                               const int64_t* index, const int32_t* order, const uint8_t* keep, const uint8_t* masked,
                              int64_t n, int64_t B,
                               int64_t K, int64_t Lq, int64_t H, float scale, float p_drop, const int64_t* seed,
                               const void* out, const float* lse, const void* dout, void* dq, void* dpk, void* dpv,
                               float* dbias_part, void* workspace, void* stream) {
  return mfl_seg_attention_backward_ex2(q, pk, pv, bias_k, bias_v, index, order, keep, masked, n, B, K, Lq, H, scale,
                                        p_drop, seed, out, lse, dout, dq, dpk, dpv, 0, 0, dbias_part, workspace,
                                        nullptr, stream);
}

int mfl_seg_attention_backward_ex(const void* q, const void* pk, const void* pv, const void* bias_k,
                                  const void* bias_v, const int64_t* index, const int32_t* order,
                                  const uint8_t* keep, const uint8_t* masked, int64_t n, int64_t B, int64_t K,
                                  int64_t Lq, int64_t H, float scale, float p_drop, const int64_t* seed,
                                  const void* out, const float* lse, const void* dout, void* dq, void* dpk,
                                  void* dpv, int64_t dpk_row_stride, int64_t dpv_row_stride, float* dbias_part,
                                  void* workspace, void* stream) {
  return mfl_seg_attention_backward_ex2(q, pk, pv, bias_k, bias_v, index, order, keep, masked, n, B, K, Lq, H, scale,
                                        p_drop, seed, out, lse, dout, dq, dpk, dpv, dpk_row_stride, dpv_row_stride,
                                        dbias_part, workspace, nullptr, stream);
}

int mfl_seg_attention_backward_ex2(const void* q, const void* pk, const void* pv, const void* bias_k,
                                   const void* bias_v, const int64_t* index, const int32_t* order,
                                   const uint8_t* keep, const uint8_t* masked, int64_t n, int64_t B, int64_t K,
                                   int64_t Lq, int64_t H, float scale, float p_drop, const int64_t* seed,
                                   const void* out, const float* lse, const void* dout, void* dq, void* dpk,
                                   void* dpv, int64_t dpk_row_stride, int64_t dpv_row_stride, float* dbias_part,
                                   void* workspace, const uint16_t* drop_bits, void* stream) {
  Args a{};
  a.dbits = const_cast<uint16_t*>(drop_bits);
  const long long dmod = H * HD;
  a.rs_k = dpk_row_stride > 0 ? dpk_row_stride : dmod;
  a.rs_v = dpv_row_stride > 0 ? dpv_row_stride : dmod;
  if (a.rs_k < dmod || a.rs_v < dmod) return fail("seg_attention: dK / dV row strides below the model width");
  a.q = static_cast<const uint16_t*>(q);
  a.pk = static_cast<const uint16_t*>(pk);
  a.pv = static_cast<const uint16_t*>(pv);
  a.bk = static_cast<const uint16_t*>(bias_k);
  a.bv = static_cast<const uint16_t*>(bias_v);
  a.index = index;
  a.order = order;
  a.keep = keep;
  a.masked = masked;
  a.n = (int)n, a.B = (int)B, a.K = (int)K, a.Lq = (int)Lq, a.H = (int)H;
  a.vbits = K % 16 == 0 && aligned16(keep) && aligned16(masked);
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
  if (!a.seed) a.dbits = nullptr;
  const int nblk = (int)((K + KB - 1) / KB);
  if (a.dbits) {
    if (n > 0) hipLaunchKernelGGL(seg_attn_bwd_dq<true>, dim3((unsigned)(n * H)), dim3(kThreads), 0, st, a);
    hipLaunchKernelGGL(seg_attn_bwd_dkv<true>, dim3((unsigned)(B * H * nblk)), dim3(kThreads), 0, st, a);
  } else {
    if (n > 0) hipLaunchKernelGGL(seg_attn_bwd_dq<false>, dim3((unsigned)(n * H)), dim3(kThreads), 0, st, a);
    hipLaunchKernelGGL(seg_attn_bwd_dkv<false>, dim3((unsigned)(B * H * nblk)), dim3(kThreads), 0, st, a);
  }
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : fail(hipGetErrorString(e));
}

const char* mfl_seg_attention_last_error(void) { return g_err; }

}  // extern "C"
