// ds_read_b64_tr_b16 semantics probe: LDS tile T[r][c] = r*100 + c (16-bit), 8 rows x 16 cols;
// every lane supplies the address of (row = 4*h + ((lane&15)>>2), cols 4*(lane&3)..+3) of block h
// (h = which read) as tools read it, and prints what it receives.
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
__global__ void k(int* out) {
  __shared__ short t[8 * 16];
  for (int i = threadIdx.x; i < 128; i += 64) t[i] = (short)((i / 16) * 100 + (i % 16));
  __syncthreads();
  const int li = threadIdx.x & 15;
  const int row = li >> 2, chunk = li & 3;
  s16x4 x = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(t + row * 16 + chunk * 4));
  for (int j = 0; j < 4; ++j) out[threadIdx.x * 4 + j] = x[j];
}
int main() {
  int* d; hipMalloc(&d, 64 * 4 * 4);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  int h[256]; hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  for (int l = 0; l < 16; ++l) printf("lane %2d: %d %d %d %d\n", l, h[4*l], h[4*l+1], h[4*l+2], h[4*l+3]);
  return 0;
}
