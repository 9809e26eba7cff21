// microbenchmark: does f32 MFMA work hide under VALU work of the same waves? (gfx950)
// 8 waves / SIMD, every wave runs the same mix per iteration:
//   kind 0: 32 v_fmac_f32 (8 chains x 4)                    -> VALU only
//   kind 1: 1 v_mfma_f32_16x16x4_f32 (4 rotating accumulators) -> MFMA only
//   kind 2: 2 MFMA                                           -> MFMA only
//   kind 3: 32 v_fmac + 1 MFMA   kind 4: 32 v_fmac + 2 MFMA  kind 5: 32 v_fmac + 3 MFMA
// (the raster backward with pass 2 on MFMA: ~50 VALU + 2 MFMA per wave step).  If the mixed
// kinds take max(VALU, MFMA) time, the matrix pipe runs under the VALU stream.
//   hipcc --offload-arch=gfx950 -O3 mfma_valu.hip -o /tmp/mfma_valu && /tmp/mfma_valu
#include <hip/hip_runtime.h>
#include <stdio.h>
constexpr int ITER = 2048;
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int NV, int NM>
__global__ __launch_bounds__(256) void k(float* out, float a, float b) {
    float x[8];
    for (int i = 0; i < 8; ++i) x[i] = threadIdx.x * 0.001f + i;
    f32x4 acc[4];
    for (int i = 0; i < 4; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    float ma = x[1], mb = x[2];
    // unrolled by 4 so every accumulator index is static (a dynamic one turns into indexed
    // moves that read the MFMA result -- a dependency -- every iteration)
    for (int it = 0; it < ITER; it += 4) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
#pragma unroll
            for (int m = 0; m < NM; ++m)
                acc[(u * NM + m) & 3] = __builtin_amdgcn_mfma_f32_16x16x4f32(ma, mb, acc[(u * NM + m) & 3], 0, 0, 0);
#pragma unroll
            for (int r = 0; r < NV / 8; ++r) {
#pragma unroll
                for (int i = 0; i < 8; ++i) asm volatile("v_fmac_f32 %0, %1, %2" : "+v"(x[i]) : "v"(a), "v"(b));
            }
        }
    }
    float s = 0;
    for (int i = 0; i < 8; ++i) s += x[i];
    for (int i = 0; i < 4; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int NV, int NM>
float run(float* out, int blocks) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    float best = 1e30f;
    for (int rep = 0; rep < 4; ++rep) {
        hipEventRecord(e0);
        k<NV, NM><<<blocks, 256>>>(out, 0.999f, 0.001f);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        if (rep && ms < best) best = ms;
    }
    return best;
}

int main() {
    const int blocks = 256 * 8 * 4;  // 8 workgroups of 4 waves per CU, 4 rounds
    float* out;
    hipMalloc(&out, (size_t)blocks * 256 * 4);
    struct R { const char* n; float ms; } r[] = {
        {"32 fma", run<32, 0>(out, blocks)},       {"1 mfma", run<0, 1>(out, blocks)},
        {"2 mfma", run<0, 2>(out, blocks)},        {"32 fma + 1 mfma", run<32, 1>(out, blocks)},
        {"32 fma + 2 mfma", run<32, 2>(out, blocks)}, {"32 fma + 3 mfma", run<32, 3>(out, blocks)},
        {"64 fma", run<64, 0>(out, blocks)},       {"64 fma + 2 mfma", run<64, 2>(out, blocks)},
        {"64 fma + 4 mfma", run<64, 4>(out, blocks)},
    };
    for (auto& e : r) printf("%-18s %8.3f ms  (%.2f x the 32-fma time)\n", e.n, e.ms, e.ms / r[0].ms);
    return 0;
}
