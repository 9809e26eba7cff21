// microbenchmark: ds_read_b128 throughput by address pattern (gfx950, 256-lane workgroups,
// 8 workgroups / CU).  Pattern 0: one address per wave (broadcast); 1: 4 addresses, lane
// groups of 4 (lanes 16m + 4g + e read record g); 2: 4 addresses, records t = 16 k apart
// (bank-conflicting); 3: 16 addresses (lane >> 2); 4: 64 addresses (lane).
//   hipcc --offload-arch=gfx950 -O3 lds_pattern.hip -o /tmp/lds_pattern && /tmp/lds_pattern
#include <hip/hip_runtime.h>
#include <stdio.h>
constexpr int ITER = 4096;

template <int PAT>
__global__ __launch_bounds__(256) void k(float* out, int seed) {
    __shared__ float4 rec[3][512];
    for (int i = threadIdx.x; i < 3 * 512; i += 256) (&rec[0][0])[i] = make_float4(i, i + 1, i + 2, i + 3);
    __syncthreads();
    const int lane = threadIdx.x & 63;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    int base = seed & 127;
    for (int it = 0; it < ITER; ++it) {
        int t;
        if constexpr (PAT == 0) t = base;
        if constexpr (PAT == 1) t = base + 5 * ((lane >> 2) & 3);
        if constexpr (PAT == 2) t = base + 16 * ((lane >> 2) & 3);
        if constexpr (PAT == 3) t = base + (lane >> 2);
        if constexpr (PAT == 4) t = base + lane;
        const float4 a = rec[0][t], b = rec[1][t], c = rec[2][t];
        acc.x += a.x + b.y + c.z;
        acc.y += a.y + b.z + c.w;
        acc.z += a.z + b.w + c.x;
        acc.w += a.w + b.x + c.y;
        base = (base + 7 + (int)acc.w * 0) & 127;
    }
    out[blockIdx.x * 256 + threadIdx.x] = acc.x + acc.y + acc.z + acc.w;
}

template <int PAT>
float run(float* out) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const int grid = 256 * 8;
    hipLaunchKernelGGL(k<PAT>, dim3(grid), dim3(256), 0, 0, out, 3);
    hipEventRecord(a);
    hipLaunchKernelGGL(k<PAT>, dim3(grid), dim3(256), 0, 0, out, 3);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    // 3 ds_read_b128 per iteration per wave
    const double reads = (double)grid * 4 * ITER * 3;
    printf("pattern %d: %.3f ms, %.2f cycles/read/CU at 2.4 GHz\n", PAT, ms, ms * 1e-3 * 2.4e9 * 256 / reads);
    return ms;
}

int main() {
    float* out;
    hipMalloc(&out, 256 * 8 * 256 * 4);
    run<0>(out);
    run<1>(out);
    run<2>(out);
    run<3>(out);
    run<4>(out);
    return 0;
}
