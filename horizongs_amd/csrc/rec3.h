// 3DGS raster record shared by the projection (fused pack) and the raster kernels.
#pragma once
#include "common.h"

namespace hgsr {

// 48-B raster record of one (camera, Gaussian).  The conic is stored pre-scaled,
// {a', b', c'} = log2(e) * {a/2, b, c/2}, so that
//   sigma' = dx (a' dx + b' dy) + c' dy^2 = log2(e) * sigma,  vis = exp2(-sigma')
// costs three products and two FMAs and feeds v_exp_f32 directly (same value as
// gsplat's exp(-sigma) up to the last ulps; forward and backward share sigma2()).
constexpr float kLog2e = 1.4426950408889634f;
struct Rec3 {
    float4 g0;  // x, y, a', b'
    float4 g1;  // c', opacity, footprint half-extent x, half-extent y
    float4 col; // colour (D <= 4, zero padded)
};

// Exact screen-space half-extents of the region where alpha = o*exp(-sigma) can
// reach 1/255: 0.5 d^T Conic d <= L, L = ln(255 o); the ellipse's bounding box
// is |dx| <= sqrt(2L * Cov_xx), |dy| <= sqrt(2L * Cov_yy) with Cov = Conic^-1.
// Padded by 1 % + 0.01 px (the kernels use the hardware exp).  Purely a skip
// test: a Gaussian outside a wave's quadrant by this box has alpha < 1/255 at
// every pixel of it, so skipping it changes no result.
__device__ __forceinline__ float2 footprint(float a, float b, float c, float opac) {
    const float L = __logf(255.0f * opac);
    const float det = a * c - b * b;
    if (!(L > 0.f) || !(det > 0.f)) return make_float2(-1e30f, -1e30f);
    const float k = 2.0f * L / det;
    return make_float2(sqrtf(k * c) * 1.01f + 0.01f, sqrtf(k * a) * 1.01f + 0.01f);
}

// the record of one (camera, Gaussian) from its projection and channels
__device__ __forceinline__ Rec3 make_rec3(float2 m, float a, float b, float c, float o, const float (&col)[4]) {
    const float2 ext = footprint(a, b, c, o);
    Rec3 r;
    r.g0 = make_float4(m.x, m.y, (0.5f * kLog2e) * a, kLog2e * b);
    r.g1 = make_float4((0.5f * kLog2e) * c, o, ext.x, ext.y);
    r.col = make_float4(col[0], col[1], col[2], col[3]);
    return r;
}

}  // namespace hgsr
