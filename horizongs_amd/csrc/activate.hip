// The 3DGS parametrisation's activations of a training step, fused: scales = exp(log_scales)
// [N,3] and opacities = sigmoid(logits) [N] in ONE elementwise pass, and their vjps
// (v_log_scales = v_scales * scales, v_logits = v_opac * o * (1 - o)) in another -- the
// reference's get_scaling / get_opacity activations (scene/basic_model.py scaling_activation
// = exp, opacity_activation = sigmoid) without four separate torch launches per step.
// HBM-bound: 16 B read + 16 B written per Gaussian each way.
#include "common.h"

namespace hgsr {

__global__ __launch_bounds__(256) void activate_fwd_kernel(int64_t N, const float* __restrict__ log_scales,
                                                           const float* __restrict__ logits,
                                                           float* __restrict__ scales, float* __restrict__ opac) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= N) return;
#pragma unroll
    for (int k = 0; k < 3; ++k) scales[i * 3 + k] = expf(log_scales[i * 3 + k]);
    opac[i] = 1.0f / (1.0f + expf(-logits[i]));
}

__global__ __launch_bounds__(256) void activate_bwd_kernel(int64_t N, const float* __restrict__ scales,
                                                           const float* __restrict__ opac,
                                                           const float* __restrict__ v_scales,
                                                           const float* __restrict__ v_opac,
                                                           float* __restrict__ v_log_scales,
                                                           float* __restrict__ v_logits) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= N) return;
    if (v_log_scales) {
#pragma unroll
        for (int k = 0; k < 3; ++k)
            v_log_scales[i * 3 + k] = v_scales ? v_scales[i * 3 + k] * scales[i * 3 + k] : 0.f;
    }
    if (v_logits) {
        const float o = opac[i];
        v_logits[i] = v_opac ? v_opac[i] * (o * (1.0f - o)) : 0.f;
    }
}

}  // namespace hgsr

using namespace hgsr;

extern "C" int hgsr_activate_fwd(int64_t N, const float* log_scales, const float* logits, float* scales,
                                 float* opacities, hgsr_stream_t stream) {
    HGSR_REQUIRE(N >= 0, "bad dims");
    if (N == 0) return HGSR_OK;
    HGSR_REQUIRE(log_scales && logits && scales && opacities, "null pointer");
    hipLaunchKernelGGL(activate_fwd_kernel, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, as_stream(stream), N,
                       log_scales, logits, scales, opacities);
    return check_launch("activate_fwd");
}

extern "C" int hgsr_activate_bwd(int64_t N, const float* scales, const float* opacities, const float* v_scales,
                                 const float* v_opacities, float* v_log_scales, float* v_logits,
                                 hgsr_stream_t stream) {
    HGSR_REQUIRE(N >= 0, "bad dims");
    if (N == 0) return HGSR_OK;
    HGSR_REQUIRE(scales && opacities, "null pointer");
    hipLaunchKernelGGL(activate_bwd_kernel, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, as_stream(stream), N,
                       scales, opacities, v_scales, v_opacities, v_log_scales, v_logits);
    return check_launch("activate_bwd");
}
