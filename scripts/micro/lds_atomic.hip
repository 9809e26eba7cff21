// microbenchmark: LDS float-atomic throughput without same-address chains (gfx950,
// 256-lane workgroups, 8 per CU).  Each wave adds into its own 1024-float LDS region; lane l
// of instruction i targets float (l * 17 + i * 5) & 1023 (distinct addresses across lanes and
// consecutive instructions), with 4 / 16 / 64 lanes active.  Also ds_write_b128 + ds_read_b128
// pairs (an LDS transpose of 8 floats per lane).
//   hipcc --offload-arch=gfx950 -O3 lds_atomic.hip -o /tmp/lds_atomic && /tmp/lds_atomic
#include <hip/hip_runtime.h>
#include <stdio.h>
constexpr int ITER = 2048;

template <int KIND>
__global__ __launch_bounds__(256) void k(float* out, float a) {
    __shared__ float lds[4][1024 + 64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int i = lane; i < 1024; i += 64) lds[w][i] = 0.f;
    __syncthreads();
    float x = a * lane;
    if constexpr (KIND <= 2) {
        const bool on = KIND == 0 ? (lane & 15) == 0 : KIND == 1 ? (lane & 3) == 0 : true;
        for (int it = 0; it < ITER; ++it) {
            if (on) {
#pragma unroll
                for (int i = 0; i < 8; ++i) atomicAdd(&lds[w][(lane * 17 + i * 5 + it) & 1023], x);
            }
        }
    } else {
        float4 v0 = make_float4(x, x, x, x), v1 = v0;
        for (int it = 0; it < ITER; ++it) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                *reinterpret_cast<float4*>(&lds[w][lane * 16 + (i & 1) * 4]) = v0;
                *reinterpret_cast<float4*>(&lds[w][lane * 16 + 8 + (i & 1) * 4]) = v1;
                __builtin_amdgcn_s_waitcnt(0xc07f);
                v0 = *reinterpret_cast<const float4*>(&lds[w][((lane ^ 16) * 16 + (i & 1) * 4) & 1023]);
                v1 = *reinterpret_cast<const float4*>(&lds[w][((lane ^ 32) * 16 + 8) & 1023]);
            }
        }
        x = v0.x + v1.y;
    }
    __syncthreads();
    out[blockIdx.x * 256 + threadIdx.x] = lds[w][lane] + x;
}

template <int KIND>
void run(float* out, const char* name, double instr_per_iter) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const int grid = 256 * 8;
    hipLaunchKernelGGL(k<KIND>, dim3(grid), dim3(256), 0, 0, out, 1.0f);
    hipEventRecord(a);
    hipLaunchKernelGGL(k<KIND>, dim3(grid), dim3(256), 0, 0, out, 1.0f);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    const double instrs = (double)grid * 4 * ITER * instr_per_iter;
    printf("%-40s %8.3f ms  %6.2f cycles / wave-instruction / CU\n", name, ms, ms * 1e-3 * 2.4e9 * 256 / instrs);
}

int main() {
    float* out;
    hipMalloc(&out, 256 * 8 * 256 * 4);
    run<0>(out, "ds_add_f32, 4 lanes, distinct", 8);
    run<1>(out, "ds_add_f32, 16 lanes, distinct", 8);
    run<2>(out, "ds_add_f32, 64 lanes, distinct", 8);
    run<3>(out, "ds_write_b128 + ds_read_b128 (x2 each)", 16);
    return 0;
}
