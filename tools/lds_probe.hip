// LDS read-modify-write throughput probe on gfx950 (design input for msda_gvalue_kernel).
// Each wave issues N row operations; a row op = 64 lanes on 64 consecutive fp32/u32 words
// of one wave-uniform row (bank-conflict free).  Variants:
//   0 ds_add_f32 (float atomicAdd on LDS)   1 ds_add_u32 (int atomicAdd on LDS)
//   2 ds_read_b32 + v_add + ds_write_b32    3 ds_write_b32 only
//   4 ds_add_f32 into per-wave private rows (no cross-wave sharing)
//   5 ds_add_rtn_f32 (returning float atomic)
// Build: hipcc --offload-arch=gfx950 -O3 -o lds_probe tools/lds_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

template <int V>
__global__ __launch_bounds__(256) void probe(float* out, int n_ops, int rows) {
  extern __shared__ float slab[];
  for (int i = threadIdx.x; i < rows * 64; i += blockDim.x) slab[i] = 0.f;
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  unsigned h = 2654435761u * (blockIdx.x * 4 + wave + 1);
  float acc = 0.f;
  for (int i = 0; i < n_ops; ++i) {
    h = h * 1664525u + 1013904223u;
    int row = (h >> 8) % rows;                       // wave-uniform
    if (V == 4) row = (row & ~3) | wave;              // rows private to this wave
    float* p = &slab[row * 64 + lane];
    const float x = 1.0f + lane;
    if (V == 0 || V == 4) atomicAdd(p, x);
    else if (V == 1) atomicAdd(reinterpret_cast<unsigned*>(p), 1u);
    else if (V == 2) *p = *p + x;
    else if (V == 3) *p = x;
    else if (V == 5) acc += atomicAdd(p, x);  // returning form: ds_add_rtn_f32
  }
  __syncthreads();
  for (int i = threadIdx.x; i < rows * 64; i += blockDim.x) acc += slab[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

template <int V>
float run(float* out, int blocks, int n_ops, int rows) {
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  size_t lds = rows * 64 * 4;
  hipLaunchKernelGGL(probe<V>, dim3(blocks), dim3(256), lds, 0, out, n_ops, rows);
  hipEventRecord(a);
  hipLaunchKernelGGL(probe<V>, dim3(blocks), dim3(256), lds, 0, out, n_ops, rows);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms; hipEventElapsedTime(&ms, a, b);
  return ms;
}

int main() {
  const int blocks = 768, n_ops = 2048, rows = 192;
  float* out;
  hipMalloc(&out, blocks * 256 * 4);
  const double ops = (double)blocks * 4 * n_ops;  // wave-instructions
  const char* names[] = {"ds_add_f32", "ds_add_u32", "read+add+write", "write only", "ds_add_f32 private rows", "ds_add_rtn_f32"};
  float t[6];
  t[0] = run<0>(out, blocks, n_ops, rows);
  t[1] = run<1>(out, blocks, n_ops, rows);
  t[2] = run<2>(out, blocks, n_ops, rows);
  t[3] = run<3>(out, blocks, n_ops, rows);
  t[4] = run<4>(out, blocks, n_ops, rows);
  t[5] = run<5>(out, blocks, n_ops, rows);
  for (int v = 0; v < 6; ++v)
    printf("{\"variant\": \"%s\", \"ms\": %.3f, \"ns_per_wave_op_per_CU\": %.2f}\n", names[v], t[v],
           t[v] * 1e6 / (ops / 256.0));
  return 0;
}
