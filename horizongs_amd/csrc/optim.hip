// K17: the optimizer step of the reference train loop (train.py:274-277,
// gaussians.optimizer.step() of torch.optim.Adam(l, lr=0.0, eps=1e-15) built at
// scene/lod_model.py:320), for every parameter group in ONE launch.
//
// torch's Adam (foreach and single-tensor forms, amsgrad/weight_decay/maximize off):
//   m  = lerp(m, g, 1 - beta1)            = m + (1 - beta1) (g - m)
//   v  = v * beta2 + (1 - beta2) g g
//   p  = p - step_size * m / (sqrt(v) / bc2_sqrt + eps)
// with step_size = lr / (1 - beta1^t) and bc2_sqrt = sqrt(1 - beta2^t) computed on the
// host in double per parameter (torch keeps `step` per parameter state).
//
// CDNA4 mapping: HBM-bound (28 B per element: p, g, m, v read; p, m, v written).
// Every tensor of the step is described in the kernel arguments; a workgroup takes a
// 2048-element chunk of one tensor (scalar lookup over the chunk prefix), each lane
// two independent float4 rows (all loads issued before the first use), streamed with
// non-temporal loads / stores (every byte is touched once per step).  Tensors whose
// four pointers are not 16-B aligned, and ragged tails, take a scalar path.
#include "common.h"

namespace hgsr {

constexpr int kAdamMaxT = 16;            // tensors per launch (more: several launches)
constexpr int kAdamChunk = 2048;         // elements per workgroup (1024 / 4096 / 8192: slower)
constexpr int kAdamVec = kAdamChunk / 4 / 256;  // float4 rows per lane
typedef float f4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ float4 ld_nt(const float* p, int64_t i) {
    const f4v v = __builtin_nontemporal_load(reinterpret_cast<const f4v*>(p) + i);
    return make_float4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void st_nt(float* p, int64_t i, float4 v) {
    __builtin_nontemporal_store(f4v{v.x, v.y, v.z, v.w}, reinterpret_cast<f4v*>(p) + i);
}

struct AdamArgs {
    float* p[kAdamMaxT];
    const float* g[kAdamMaxT];
    float* m[kAdamMaxT];
    float* v[kAdamMaxT];
    int64_t n[kAdamMaxT];
    float step_size[kAdamMaxT];
    float bc2_sqrt[kAdamMaxT];
    int vec[kAdamMaxT];
    int chunk0[kAdamMaxT + 1];  // first workgroup of each tensor
    int nt;
    float w1;     // 1 - beta1 (the lerp weight)
    float beta2;
    float w2;     // 1 - beta2
    float eps;
};

__device__ __forceinline__ void adam_elem(float& p, float g, float& m, float& v, float w1, float beta2, float w2,
                                          float eps, float step_size, float bc2_sqrt) {
    // Contraction is spelled out: left to the compiler, the float4 and the scalar path
    // fused different products, so a tensor's result depended on its alignment (a shard
    // segment at an odd offset of a flat bucket stepped differently from the whole tensor).
#pragma clang fp contract(off)
    m = __builtin_fmaf(w1, g - m, m);
    v = __builtin_fmaf(v, beta2, (w2 * g) * g);
    const float denom = sqrtf(v) / bc2_sqrt + eps;
    p = __builtin_fmaf(-step_size, m / denom, p);
}

__global__ __launch_bounds__(256) void adam_kernel(const AdamArgs a) {
    const int b = blockIdx.x;
    int t = 0;
#pragma unroll
    for (int k = 1; k < kAdamMaxT; ++k)
        if (k < a.nt && b >= a.chunk0[k]) t = k;
    const int64_t base = (int64_t)(b - a.chunk0[t]) * kAdamChunk;
    const int64_t n = a.n[t];
    float* __restrict__ P = a.p[t];
    const float* __restrict__ G = a.g[t];
    float* __restrict__ M = a.m[t];
    float* __restrict__ V = a.v[t];
    const float ss = a.step_size[t], bc = a.bc2_sqrt[t];
    if (a.vec[t] && base + kAdamChunk <= n) {
        float4 p[kAdamVec], g[kAdamVec], m[kAdamVec], v[kAdamVec];
#pragma unroll
        for (int r = 0; r < kAdamVec; ++r) {
            const int64_t i = base / 4 + r * 256 + threadIdx.x;
            p[r] = ld_nt(P, i);
            g[r] = ld_nt(G, i);
            m[r] = ld_nt(M, i);
            v[r] = ld_nt(V, i);
        }
#pragma unroll
        for (int r = 0; r < kAdamVec; ++r) {
            adam_elem(p[r].x, g[r].x, m[r].x, v[r].x, a.w1, a.beta2, a.w2, a.eps, ss, bc);
            adam_elem(p[r].y, g[r].y, m[r].y, v[r].y, a.w1, a.beta2, a.w2, a.eps, ss, bc);
            adam_elem(p[r].z, g[r].z, m[r].z, v[r].z, a.w1, a.beta2, a.w2, a.eps, ss, bc);
            adam_elem(p[r].w, g[r].w, m[r].w, v[r].w, a.w1, a.beta2, a.w2, a.eps, ss, bc);
            const int64_t i = base / 4 + r * 256 + threadIdx.x;
            st_nt(P, i, p[r]);
            st_nt(M, i, m[r]);
            st_nt(V, i, v[r]);
        }
        return;
    }
    for (int64_t i = base + threadIdx.x; i < min(base + (int64_t)kAdamChunk, n); i += 256) {
        float p = P[i], m = M[i], v = V[i];
        adam_elem(p, G[i], m, v, a.w1, a.beta2, a.w2, a.eps, ss, bc);
        P[i] = p;
        M[i] = m;
        V[i] = v;
    }
}

}  // namespace hgsr

using namespace hgsr;

extern "C" int hgsr_adam_step(int n_tensors, const hgsr_adam_tensor* tensors, double beta1, double beta2,
                              double eps, hgsr_stream_t stream) {
    HGSR_REQUIRE(n_tensors >= 0 && (n_tensors == 0 || tensors), "adam: bad tensor list");
    HGSR_REQUIRE(beta1 >= 0.0 && beta1 < 1.0 && beta2 >= 0.0 && beta2 < 1.0, "adam: betas must lie in [0, 1)");
    hipStream_t s = as_stream(stream);
    AdamArgs a{};
    a.w1 = (float)(1.0 - beta1);
    a.beta2 = (float)beta2;
    a.w2 = (float)(1.0 - beta2);
    a.eps = (float)eps;
    auto flush = [&](void) -> int {
        if (a.nt == 0) return HGSR_OK;
        const int nwg = a.chunk0[a.nt];
        if (nwg > 0) {
            KernelTimer kt("adam", s);
            hipLaunchKernelGGL(adam_kernel, dim3(nwg), dim3(256), 0, s, a);
        }
        a.nt = 0;
        a.chunk0[0] = 0;
        return check_launch("adam");
    };
    for (int i = 0; i < n_tensors; ++i) {
        const hgsr_adam_tensor& t = tensors[i];
        HGSR_REQUIRE(t.numel >= 0, "adam: tensor %d has negative numel", i);
        if (t.numel == 0 || !t.grad) continue;  // torch skips parameters without a gradient
        HGSR_REQUIRE(t.param && t.exp_avg && t.exp_avg_sq, "adam: null pointer in tensor %d", i);
        HGSR_REQUIRE(t.step >= 1, "adam: step must be >= 1 (got %lld)", (long long)t.step);
        const int64_t chunks = (t.numel + kAdamChunk - 1) / kAdamChunk;
        HGSR_REQUIRE(chunks < (1ll << 30), "adam: tensor %d too large", i);
        if (a.nt == kAdamMaxT || (int64_t)a.chunk0[a.nt] + chunks >= (1ll << 31))
            if (int st = flush()) return st;
        const int k = a.nt;
        a.p[k] = t.param;
        a.g[k] = t.grad;
        a.m[k] = t.exp_avg;
        a.v[k] = t.exp_avg_sq;
        a.n[k] = t.numel;
        // torch: bias_correction1 = 1 - beta1 ** step; step_size = lr / bias_correction1;
        //        bias_correction2_sqrt = (1 - beta2 ** step) ** 0.5   (Python floats)
        a.step_size[k] = (float)(t.lr / (1.0 - pow(beta1, (double)t.step)));
        a.bc2_sqrt[k] = (float)sqrt(1.0 - pow(beta2, (double)t.step));
        const uintptr_t al = (uintptr_t)t.param | (uintptr_t)t.grad | (uintptr_t)t.exp_avg | (uintptr_t)t.exp_avg_sq;
        a.vec[k] = (al & 15) == 0;
        a.chunk0[k + 1] = a.chunk0[k] + (int)chunks;
        a.nt = k + 1;
    }
    return flush();
}
