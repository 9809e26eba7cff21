// The 3DGS parametrisation's activations of a training step, fused: scales = exp(log_scales)
// [N,3] and opacities = sigmoid(logits) [N] in ONE elementwise pass, and their vjps
// (v_log_scales = v_scales * scales, v_logits = v_opac * o * (1 - o)) in another -- the
// reference's get_scaling / get_opacity activations (scene/basic_model.py scaling_activation
// = exp, opacity_activation = sigmoid) without four separate torch launches per step.
// HBM-bound: 16 B read + 16 B written per Gaussian forward, 32 B read + 16 B written backward.
#include <initializer_list>

#include "common.h"

namespace hgsr {

// Both kernels treat the [N,3] scale arrays as 3N independent floats and run two flat
// ranges in one grid: float4 items [0, S4) over the scales (3N / 4 of them), then float4
// items over the N opacities; a scalar tail covers counts that are not multiples of 4.
// (Vector loads / stores need 16-B aligned bases; the host falls back to V = 1 otherwise.)
template <int V>
struct Vec;
template <>
struct Vec<4> {
    using T = float4;
    __device__ static float get(const T& v, int k) { return k == 0 ? v.x : k == 1 ? v.y : k == 2 ? v.z : v.w; }
    __device__ static void set(T& v, int k, float x) {
        if (k == 0) v.x = x; else if (k == 1) v.y = x; else if (k == 2) v.z = x; else v.w = x;
    }
};
template <>
struct Vec<1> {
    using T = float;
    __device__ static float get(const T& v, int) { return v; }
    __device__ static void set(T& v, int, float x) { v = x; }
};

__device__ __forceinline__ float sigmoidf_(float x) { return 1.0f / (1.0f + expf(-x)); }

template <int V>
__global__ __launch_bounds__(256) void activate_fwd_kernel(int64_t ns, int64_t no, const float* __restrict__ log_scales,
                                                           const float* __restrict__ logits,
                                                           float* __restrict__ scales, float* __restrict__ opac) {
    using T = typename Vec<V>::T;
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t s_items = ns / V, o_items = no / V;
    if (i < s_items) {
        T x = reinterpret_cast<const T*>(log_scales)[i];
#pragma unroll
        for (int k = 0; k < V; ++k) Vec<V>::set(x, k, expf(Vec<V>::get(x, k)));
        reinterpret_cast<T*>(scales)[i] = x;
    } else if (i < s_items + o_items) {
        const int64_t j = i - s_items;
        T x = reinterpret_cast<const T*>(logits)[j];
#pragma unroll
        for (int k = 0; k < V; ++k) Vec<V>::set(x, k, sigmoidf_(Vec<V>::get(x, k)));
        reinterpret_cast<T*>(opac)[j] = x;
    } else if (V > 1) {  // tails
        const int64_t r = i - s_items - o_items;
        const int64_t st = ns - s_items * V, ot = no - o_items * V;
        if (r < st) scales[s_items * V + r] = expf(log_scales[s_items * V + r]);
        else if (r < st + ot) opac[o_items * V + r - st] = sigmoidf_(logits[o_items * V + r - st]);
    }
}

template <int V>
__global__ __launch_bounds__(256) void activate_bwd_kernel(int64_t ns, int64_t no, const float* __restrict__ scales,
                                                           const float* __restrict__ opac,
                                                           const float* __restrict__ v_scales,
                                                           const float* __restrict__ v_opac,
                                                           float* __restrict__ v_log_scales,
                                                           float* __restrict__ v_logits) {
    using T = typename Vec<V>::T;
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t s_items = ns / V, o_items = no / V;
    auto sc = [&](T& g, const T& a, const T& b) {
#pragma unroll
        for (int k = 0; k < V; ++k) Vec<V>::set(g, k, Vec<V>::get(a, k) * Vec<V>::get(b, k));
    };
    auto op = [&](T& g, const T& a, const T& o) {
#pragma unroll
        for (int k = 0; k < V; ++k) {
            const float ok = Vec<V>::get(o, k);
            Vec<V>::set(g, k, Vec<V>::get(a, k) * (ok * (1.0f - ok)));
        }
    };
    if (i < s_items) {
        if (!v_log_scales) return;
        T g;
        if (v_scales) sc(g, reinterpret_cast<const T*>(v_scales)[i], reinterpret_cast<const T*>(scales)[i]);
        else g = T{};
        reinterpret_cast<T*>(v_log_scales)[i] = g;
    } else if (i < s_items + o_items) {
        if (!v_logits) return;
        const int64_t j = i - s_items;
        T g;
        if (v_opac) op(g, reinterpret_cast<const T*>(v_opac)[j], reinterpret_cast<const T*>(opac)[j]);
        else g = T{};
        reinterpret_cast<T*>(v_logits)[j] = g;
    } else if (V > 1) {  // tails
        const int64_t r = i - s_items - o_items;
        const int64_t st = ns - s_items * V, ot = no - o_items * V;
        if (r < st) {
            const int64_t e = s_items * V + r;
            if (v_log_scales) v_log_scales[e] = v_scales ? v_scales[e] * scales[e] : 0.f;
        } else if (r < st + ot) {
            const int64_t e = o_items * V + r - st;
            if (v_logits) v_logits[e] = v_opac ? v_opac[e] * (opac[e] * (1.0f - opac[e])) : 0.f;
        }
    }
}

static bool aligned16(std::initializer_list<const void*> ps) {
    for (const void* p : ps)
        if (p && (reinterpret_cast<uintptr_t>(p) & 15)) return false;
    return true;
}

}  // namespace hgsr

using namespace hgsr;

extern "C" int hgsr_activate_fwd(int64_t N, const float* log_scales, const float* logits, float* scales,
                                 float* opacities, hgsr_stream_t stream) {
    HGSR_REQUIRE(N >= 0, "bad dims");
    if (N == 0) return HGSR_OK;
    HGSR_REQUIRE(log_scales && logits && scales && opacities, "null pointer");
    const int64_t ns = 3 * N;
    if (aligned16({log_scales, logits, scales, opacities})) {
        const int64_t items = ns / 4 + N / 4 + (ns % 4) + (N % 4);
        hipLaunchKernelGGL(activate_fwd_kernel<4>, dim3((unsigned)((items + 255) / 256)), dim3(256), 0,
                           as_stream(stream), ns, N, log_scales, logits, scales, opacities);
    } else {
        hipLaunchKernelGGL(activate_fwd_kernel<1>, dim3((unsigned)((ns + N + 255) / 256)), dim3(256), 0,
                           as_stream(stream), ns, N, log_scales, logits, scales, opacities);
    }
    return check_launch("activate_fwd");
}

extern "C" int hgsr_activate_bwd(int64_t N, const float* scales, const float* opacities, const float* v_scales,
                                 const float* v_opacities, float* v_log_scales, float* v_logits,
                                 hgsr_stream_t stream) {
    HGSR_REQUIRE(N >= 0, "bad dims");
    if (N == 0) return HGSR_OK;
    HGSR_REQUIRE(scales && opacities, "null pointer");
    const int64_t ns = 3 * N;
    if (aligned16({scales, opacities, v_scales, v_opacities, v_log_scales, v_logits})) {
        const int64_t items = ns / 4 + N / 4 + (ns % 4) + (N % 4);
        hipLaunchKernelGGL(activate_bwd_kernel<4>, dim3((unsigned)((items + 255) / 256)), dim3(256), 0,
                           as_stream(stream), ns, N, scales, opacities, v_scales, v_opacities, v_log_scales, v_logits);
    } else {
        hipLaunchKernelGGL(activate_bwd_kernel<1>, dim3((unsigned)((ns + N + 255) / 256)), dim3(256), 0,
                           as_stream(stream), ns, N, scales, opacities, v_scales, v_opacities, v_log_scales,
                           v_logits);
    }
    return check_launch("activate_bwd");
}
