// microbenchmark: issue rate of v_fma_f32 vs v_pk_fma_f32 (and v_pk_mul_f32) on gfx950
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef float f2 __attribute__((ext_vector_type(2)));
constexpr int ITER = 4096;
__global__ __launch_bounds__(256) void scalar_k(float* out, float a, float b) {
  float x[8];
  for (int i = 0; i < 8; ++i) x[i] = threadIdx.x * 0.001f + i;
  for (int it = 0; it < ITER; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = __builtin_fmaf(x[i], a, b);
  }
  float s = 0; for (int i = 0; i < 8; ++i) s += x[i];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}
__global__ __launch_bounds__(256) void packed_k(float* out, float a, float b) {
  f2 x[8];
  for (int i = 0; i < 8; ++i) x[i] = f2{threadIdx.x * 0.001f + i, threadIdx.x * 0.002f - i};
  const f2 av = {a, a * 0.5f}, bv = {b, b * 0.25f};
  for (int it = 0; it < ITER; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = __builtin_elementwise_fma(x[i], av, bv);
  }
  float s = 0; for (int i = 0; i < 8; ++i) s += x[i].x + x[i].y;
  out[blockIdx.x * 256 + threadIdx.x] = s;
}
__global__ __launch_bounds__(256) void packed_bcast_k(float* out, float a, float b) {
  f2 x[8];
  for (int i = 0; i < 8; ++i) x[i] = f2{threadIdx.x * 0.001f + i, threadIdx.x * 0.002f - i};
  for (int it = 0; it < ITER; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = __builtin_elementwise_fma(x[i], (f2)a, (f2)b);
  }
  float s = 0; for (int i = 0; i < 8; ++i) s += x[i].x + x[i].y;
  out[blockIdx.x * 256 + threadIdx.x] = s;
}
__global__ __launch_bounds__(256) void pkmul_k(float* out, float a, float b) {
  f2 x[8];
  for (int i = 0; i < 8; ++i) x[i] = f2{threadIdx.x * 0.001f + i, threadIdx.x * 0.002f - i};
  const f2 av = {a, a * 0.5f};
  for (int it = 0; it < ITER; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = x[i] * av;
  }
  float s = 0; for (int i = 0; i < 8; ++i) s += x[i].x + x[i].y;
  out[blockIdx.x * 256 + threadIdx.x] = s;
}
int main() {
  const int blocks = 256 * 8 * 4;
  float* out; hipMalloc(&out, blocks * 256 * 4);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  const char* names[4] = {"v_fma_f32", "v_pk_fma_f32", "v_pk_fma_f32 (bcast ops)", "v_pk_mul_f32"};
  for (int k = 0; k < 4; ++k) {
    for (int rep = 0; rep < 2; ++rep) {
      hipEventRecord(e0);
      if (k == 0) scalar_k<<<blocks, 256>>>(out, 0.999f, 0.001f);
      if (k == 1) packed_k<<<blocks, 256>>>(out, 0.999f, 0.001f);
      if (k == 2) packed_bcast_k<<<blocks, 256>>>(out, 0.999f, 0.001f);
      if (k == 3) pkmul_k<<<blocks, 256>>>(out, 0.999f, 0.001f);
      hipEventRecord(e1); hipEventSynchronize(e1);
      float ms; hipEventElapsedTime(&ms, e0, e1);
      double instrs = (double)blocks * 4 * ITER * 8;  // wave-instructions
      double lanes_ops = (double)blocks * 256 * ITER * 8 * (k ? 2 : 1);
      if (rep) printf("%-26s %8.3f ms  %.1f G wave-instr/s  %.1f TFLOP/s(fma=2)\n", names[k], ms, instrs / ms / 1e6,
                      lanes_ops * (k == 3 ? 1 : 2) / ms / 1e9);
    }
  }
  return 0;
}
