// 3DGS raster record shared by the projection (fused pack) and the raster kernels.
#pragma once
#include "common.h"

namespace hgsr {

// 64-B raster record of one (camera, Gaussian).  The conic is stored pre-scaled,
// {a', b', c'} = log2(e) * {a/2, b, c/2}, so that
//   sigma' = dx (a' dx + b' dy) + c' dy^2 = log2(e) * sigma,  vis = exp2(-sigma')
// costs three products and two FMAs and feeds v_exp_f32 directly (same value as
// gsplat's exp(-sigma) up to the last ulps; forward and backward share sigma2()).
constexpr float kLog2e = 1.4426950408889634f;
// The fourth quad carries the pair's gradient-slot base {seg - y0 w - x0, w} (isect.hip
// launch_grad_slots writes it at the start of a backward; the forward never reads it), so the
// backward's slot lookup hits the 64-B sector its record DMA fetches instead of a separate
// gather (a 48-B record plus an 8-B slot array read ~2x the record bytes: 984 vs ~490 MB
// corrected FETCH per c2 launch, profiles/r06_pmc_traffic.json).  At 64 B a record is one
// aligned sector; at 48 B one in two straddles two.
struct Rec3 {
    float4 g0;  // x, y, a', b'
    float4 g1;  // c', opacity, footprint half-extent x, half-extent y
    float4 col; // colour (D <= 4, zero padded)
    int4 sl;    // gradient-slot base, slot width, 0, 0
};
static_assert(sizeof(Rec3) == 64, "Rec3 is one 64-B sector");

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
    r.sl = make_int4(0, 0, 0, 0);
    return r;
}

}  // namespace hgsr
