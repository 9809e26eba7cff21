// microbenchmark: issue throughput of the instruction kinds in the raster backward step
// (gfx950, 8 waves / SIMD, 8 independent register chains per wave).
//   hipcc --offload-arch=gfx950 -O3 valu_mix.hip -o /tmp/valu_mix && /tmp/valu_mix
#include <hip/hip_runtime.h>
#include <stdio.h>
constexpr int ITER = 2048;

#define BODY8(STMT)                     \
    _Pragma("unroll") for (int i = 0; i < 8; ++i) { STMT; }

template <int KIND>
__global__ __launch_bounds__(256) void k(float* out, float a, float b) {
    float x[8];
    for (int i = 0; i < 8; ++i) x[i] = threadIdx.x * 0.001f + i;
    for (int it = 0; it < ITER; ++it) {
        if constexpr (KIND == 0) BODY8(asm volatile("v_fmac_f32 %0, %1, %2" : "+v"(x[i]) : "v"(a), "v"(b)))
        if constexpr (KIND == 1) BODY8(asm volatile("v_exp_f32 %0, %0" : "+v"(x[i])))
        if constexpr (KIND == 2) BODY8(asm volatile("v_rcp_f32 %0, %0" : "+v"(x[i])))
        if constexpr (KIND == 3)
            BODY8(asm volatile("v_add_f32_dpp %0, %0, %0 row_ror:4 row_mask:0xf bank_mask:0xf bound_ctrl:1"
                               : "+v"(x[i])))
        if constexpr (KIND == 4)
            BODY8(asm volatile("v_add_f32_dpp %0, %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf bound_ctrl:1"
                               : "+v"(x[i])))
        if constexpr (KIND == 5) {
#pragma unroll
            for (int i = 0; i < 8; i += 2) asm volatile("v_permlane32_swap_b32 %0, %1" : "+v"(x[i]), "+v"(x[i + 1]));
        }
        if constexpr (KIND == 6) {
#pragma unroll
            for (int i = 0; i < 8; i += 2) asm volatile("v_permlane16_swap_b32 %0, %1" : "+v"(x[i]), "+v"(x[i + 1]));
        }
        if constexpr (KIND == 7) BODY8(asm volatile("v_mul_f32 %0, %0, %1" : "+v"(x[i]) : "v"(a)))
        if constexpr (KIND == 8) BODY8(asm volatile("v_cmp_le_f32 vcc, %0, %1\n\tv_cndmask_b32 %0, 0, %0, vcc"
                                                    : "+v"(x[i]) : "v"(a) : "vcc"))
        if constexpr (KIND == 9) {  // readlane + salu use
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                int s;
                asm volatile("v_readlane_b32 %0, %1, 5" : "=s"(s) : "v"(x[i]));
                asm volatile("s_add_u32 %0, %0, 1" : "+s"(s));
                asm volatile("v_add_u32 %0, %1, %0" : "+v"(x[i]) : "s"(s));
            }
        }
        if constexpr (KIND == 11) {  // ds_swizzle xor 16 (LDS pipe)
#pragma unroll
            for (int i = 0; i < 8; ++i) x[i] = __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(x[i]), 0x401f));
        }
        if constexpr (KIND == 12) {  // ds_bpermute xor 32 (LDS pipe)
            const int addr = ((threadIdx.x & 63) ^ 32) * 4;
#pragma unroll
            for (int i = 0; i < 8; ++i) x[i] = __int_as_float(__builtin_amdgcn_ds_bpermute(addr, __float_as_int(x[i])));
        }
        if constexpr (KIND == 13) {  // 1 ds_bpermute + 4 v_fma per chain
            const int addr = ((threadIdx.x & 63) ^ 32) * 4;
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                float y = __int_as_float(__builtin_amdgcn_ds_bpermute(addr, __float_as_int(x[i])));
                asm volatile("v_fmac_f32 %0, %1, %2\n\tv_fmac_f32 %0, %1, %2\n\tv_fmac_f32 %0, %1, %2\n\tv_fmac_f32 %0, %1, %2"
                             : "+v"(y) : "v"(a), "v"(b));
                x[i] = y;
            }
        }
        if constexpr (KIND == 14) {  // 1 v_permlane32_swap per 2 chains + 4 v_fma per chain (same mix on VALU)
#pragma unroll
            for (int i = 0; i < 8; i += 2) {
                asm volatile("v_permlane32_swap_b32 %0, %1" : "+v"(x[i]), "+v"(x[i + 1]));
                asm volatile("v_fmac_f32 %0, %1, %2\n\tv_fmac_f32 %0, %1, %2\n\tv_fmac_f32 %0, %1, %2\n\tv_fmac_f32 %0, %1, %2"
                             : "+v"(x[i]) : "v"(a), "v"(b));
                asm volatile("v_fmac_f32 %0, %1, %2\n\tv_fmac_f32 %0, %1, %2\n\tv_fmac_f32 %0, %1, %2\n\tv_fmac_f32 %0, %1, %2"
                             : "+v"(x[i + 1]) : "v"(a), "v"(b));
            }
        }
        if constexpr (KIND == 15) {  // 4 v_fma per chain only (baseline for 13/14)
#pragma unroll
            for (int i = 0; i < 8; ++i)
                asm volatile("v_fmac_f32 %0, %1, %2\n\tv_fmac_f32 %0, %1, %2\n\tv_fmac_f32 %0, %1, %2\n\tv_fmac_f32 %0, %1, %2"
                             : "+v"(x[i]) : "v"(a), "v"(b));
        }
        if constexpr (KIND >= 16 && KIND <= 18) {  // ds_add_f32 from 4 / 16 / 64 lanes, distinct addresses
            __shared__ float lds[4][256];
            const int lane = threadIdx.x & 63;
            const bool on = KIND == 16 ? (lane & 15) == 0 : KIND == 17 ? (lane & 3) == 0 : true;
            float* dst = &lds[threadIdx.x >> 6][lane * 3 % 256];
            if (on) {
#pragma unroll
                for (int i = 0; i < 8; ++i) atomicAdd(dst + i * 0, x[i]);
            }
        }
        if constexpr (KIND == 10) {  // v_pk_fma_f32
#pragma unroll
            for (int i = 0; i < 8; i += 2) {
                asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(*(double*)&x[i]) : "v"(*(double*)&x[0]), "v"(*(double*)&x[2]));
            }
        }
    }
    float s = 0;
    for (int i = 0; i < 8; ++i) s += x[i];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int KIND>
float run(float* out, int blocks) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    float best = 1e30f;
    for (int rep = 0; rep < 3; ++rep) {
        hipEventRecord(e0);
        k<KIND><<<blocks, 256>>>(out, 0.999f, 0.001f);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        if (rep && ms < best) best = ms;
    }
    return best;
}

int main() {
    const int blocks = 256 * 8 * 4;  // 8 WG of 4 waves per CU, 4 rounds
    float* out;
    hipMalloc(&out, (size_t)blocks * 256 * 4);
    const char* names[] = {"v_fmac_f32", "v_exp_f32", "v_rcp_f32", "v_add_f32_dpp row_ror", "v_add_f32_dpp quad_perm",
                           "v_permlane32_swap", "v_permlane16_swap", "v_mul_f32", "v_cmp+v_cndmask (2 instr)",
                           "v_readlane+s_add+v_add (2 VALU)", "v_pk_fma_f32", "ds_swizzle_b32 xor16",
                           "ds_bpermute_b32 xor32", "bpermute + 4 fma (per chain)", "permlane32 (1/2) + 4 fma",
                           "4 fma", "ds_add_f32 4 lanes", "ds_add_f32 16 lanes", "ds_add_f32 64 lanes"};
    float ms[19];
    ms[0] = run<0>(out, blocks);
    ms[1] = run<1>(out, blocks);
    ms[2] = run<2>(out, blocks);
    ms[3] = run<3>(out, blocks);
    ms[4] = run<4>(out, blocks);
    ms[5] = run<5>(out, blocks);
    ms[6] = run<6>(out, blocks);
    ms[7] = run<7>(out, blocks);
    ms[8] = run<8>(out, blocks);
    ms[9] = run<9>(out, blocks);
    ms[10] = run<10>(out, blocks);
    ms[11] = run<11>(out, blocks);
    ms[12] = run<12>(out, blocks);
    ms[13] = run<13>(out, blocks);
    ms[14] = run<14>(out, blocks);
    ms[15] = run<15>(out, blocks);
    ms[16] = run<16>(out, blocks);
    ms[17] = run<17>(out, blocks);
    ms[18] = run<18>(out, blocks);
    const double waves = (double)blocks * 4;
    for (int i = 0; i < 19; ++i) {
        const double n_instr = waves * ITER * ((i == 5 || i == 6 || i == 10) ? 4 : 8);
        printf("%-34s %8.3f ms  %7.1f G wave-instr/s  (%.2f x fma time per instr)\n", names[i], ms[i],
               n_instr / ms[i] / 1e6, (ms[i] / n_instr) / (ms[0] / (waves * ITER * 8)));
    }
    return 0;
}
