// B operand of v_mfma_f32_16x16x32_bf16 built from two ds_read_b64_tr_b16 (as msda_win.hip does)
// with A = identity rows: D[row][col] must equal G[row][col] for row < 16 (sample k = k).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
__device__ short bf(float x) { unsigned u = __float_as_uint(x); return (short)((u + 0x7fffu + ((u >> 16) & 1u)) >> 16); }
__global__ void k(float* out, int* braw) {
  __shared__ __attribute__((aligned(16))) unsigned char g[32 * 144];
  for (int i = threadIdx.x; i < 32 * 64; i += 64) {
    const int r = i / 64, c = i % 64;
    *reinterpret_cast<short*>(g + r * 144 + c * 2) = bf((float)(r * 100 + c));
  }
  __syncthreads();
  const int lane = threadIdx.x, gg = lane >> 4, li = lane & 15;
  bf16x8 a;
  for (int j = 0; j < 8; ++j) a[j] = __builtin_bit_cast(__bf16, bf((8 * gg + j) == li ? 1.f : 0.f));
  const int qq = li >> 2, pp = li & 3;
  const int ra = 8 * gg + qq, rb = 8 * gg + 4 + qq;
  const int cb = 0;
  const int col = (cb * 16 + 4 * pp) * 2;
  const s16x4 x0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(g + ra * 144 + col));
  const s16x4 x1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(g + rb * 144 + col));
  bf16x8 bv;
  for (int j = 0; j < 4; ++j) {
    bv[j] = __builtin_bit_cast(__bf16, x0[j]);
    bv[4 + j] = __builtin_bit_cast(__bf16, x1[j]);
  }
  for (int j = 0; j < 8; ++j) braw[lane * 8 + j] = (int)(__builtin_bit_cast(unsigned short, bv[j]));
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bv, acc, 0, 0, 0);
  for (int j = 0; j < 4; ++j) out[(4 * gg + j) * 16 + li] = acc[j];
}
int main() {
  float* d; int* b;
  (void)hipMalloc(&d, 256 * 4); (void)hipMalloc(&b, 512 * 4);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, b);
  float h[256]; int hb[512];
  (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  (void)hipMemcpy(hb, b, sizeof(hb), hipMemcpyDeviceToHost);
  int bad = 0;
  for (int r = 0; r < 16; ++r) for (int c = 0; c < 16; ++c) if (h[r * 16 + c] != (float)(r * 100 + c)) ++bad;
  printf("mismatches %d\n", bad);
  for (int r = 0; r < 4; ++r) printf("D row %d: %g %g %g %g\n", r, h[r*16], h[r*16+1], h[r*16+2], h[r*16+3]);
  for (int l = 0; l < 2; ++l) {
    printf("lane %d B:", l);
    for (int j = 0; j < 8; ++j) { unsigned u = (unsigned)hb[l*8+j] << 16; float f; memcpy(&f, &u, 4); printf(" %g", f); }
    printf("\n");
  }
  return 0;
}
