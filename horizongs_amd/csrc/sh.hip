// K3: spherical-harmonics colour (degree <= 3), forward and backward.
// Basis polynomials and constants: reference utils/sh_utils.py:26-112 (pinned by
// tests/golden/sh_eval.npz).  Coefficient layout [n, K, 3] (gsplat).
// One lane per Gaussian; HBM-bound (reads K*12 + 12 B, writes 12 B).
#include "common.h"

namespace hgsr {

__constant__ float kC0 = 0.28209479177387814f;
__constant__ float kC1 = 0.4886025119029199f;
__constant__ float kC2[5] = {1.0925484305920792f, -1.0925484305920792f, 0.31539156525252005f,
                             -1.0925484305920792f, 0.5462742152960396f};
__constant__ float kC3[7] = {-0.5900435899266435f, 2.890611442640554f, -0.4570457994644658f,
                             0.3731763325901154f, -0.4570457994644658f, 1.445305721320277f,
                             -0.5900435899266435f};

template <int DEG>
__device__ __forceinline__ void sh_basis(float x, float y, float z, float* b) {
    b[0] = kC0;
    if (DEG < 1) return;
    b[1] = -kC1 * y;
    b[2] = kC1 * z;
    b[3] = -kC1 * x;
    if (DEG < 2) return;
    const float xx = x * x, yy = y * y, zz = z * z, xy = x * y, yz = y * z, xz = x * z;
    b[4] = kC2[0] * xy;
    b[5] = kC2[1] * yz;
    b[6] = kC2[2] * (2.0f * zz - xx - yy);
    b[7] = kC2[3] * xz;
    b[8] = kC2[4] * (xx - yy);
    if (DEG < 3) return;
    b[9] = kC3[0] * y * (3.0f * xx - yy);
    b[10] = kC3[1] * xy * z;
    b[11] = kC3[2] * y * (4.0f * zz - xx - yy);
    b[12] = kC3[3] * z * (2.0f * zz - 3.0f * xx - 3.0f * yy);
    b[13] = kC3[4] * x * (4.0f * zz - xx - yy);
    b[14] = kC3[5] * z * (xx - yy);
    b[15] = kC3[6] * x * (xx - 3.0f * yy);
}

template <int DEG>
__device__ __forceinline__ void sh_basis_grad(float x, float y, float z, float* bx, float* by, float* bz) {
    constexpr int NB = (DEG + 1) * (DEG + 1);
#pragma unroll
    for (int k = 0; k < NB; ++k) { bx[k] = 0.f; by[k] = 0.f; bz[k] = 0.f; }
    if (DEG < 1) return;
    by[1] = -kC1; bz[2] = kC1; bx[3] = -kC1;
    if (DEG < 2) return;
    bx[4] = kC2[0] * y; by[4] = kC2[0] * x;
    by[5] = kC2[1] * z; bz[5] = kC2[1] * y;
    bx[6] = kC2[2] * (-2.0f * x); by[6] = kC2[2] * (-2.0f * y); bz[6] = kC2[2] * (4.0f * z);
    bx[7] = kC2[3] * z; bz[7] = kC2[3] * x;
    bx[8] = kC2[4] * (2.0f * x); by[8] = kC2[4] * (-2.0f * y);
    if (DEG < 3) return;
    const float xx = x * x, yy = y * y, zz = z * z;
    bx[9] = kC3[0] * y * 6.0f * x; by[9] = kC3[0] * (3.0f * xx - 3.0f * yy);
    bx[10] = kC3[1] * y * z; by[10] = kC3[1] * x * z; bz[10] = kC3[1] * x * y;
    bx[11] = kC3[2] * y * (-2.0f * x); by[11] = kC3[2] * (4.0f * zz - xx - 3.0f * yy); bz[11] = kC3[2] * y * 8.0f * z;
    bx[12] = kC3[3] * z * (-6.0f * x); by[12] = kC3[3] * z * (-6.0f * y); bz[12] = kC3[3] * (6.0f * zz - 3.0f * xx - 3.0f * yy);
    bx[13] = kC3[4] * (4.0f * zz - 3.0f * xx - yy); by[13] = kC3[4] * x * (-2.0f * y); bz[13] = kC3[4] * x * 8.0f * z;
    bx[14] = kC3[5] * z * 2.0f * x; by[14] = kC3[5] * z * (-2.0f * y); bz[14] = kC3[5] * (xx - yy);
    bx[15] = kC3[6] * (3.0f * xx - 3.0f * yy); by[15] = kC3[6] * x * (-6.0f * y);
}

template <int DEG>
__global__ __launch_bounds__(256) void sh_fwd_kernel(int K, int64_t n, const float* __restrict__ dirs,
                                                     const float* __restrict__ coeffs,
                                                     const uint8_t* __restrict__ masks,
                                                     float* __restrict__ colors) {
    constexpr int NB = (DEG + 1) * (DEG + 1);
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float r0 = 0.f, r1 = 0.f, r2 = 0.f;
    if (!masks || masks[i]) {
        const float x = dirs[i * 3], y = dirs[i * 3 + 1], z = dirs[i * 3 + 2];
        const float inv = 1.0f / sqrtf(x * x + y * y + z * z);
        float b[NB];
        sh_basis<DEG>(x * inv, y * inv, z * inv, b);
        const float* c = coeffs + i * K * 3;
#pragma unroll
        for (int k = 0; k < NB; ++k) {
            r0 += b[k] * c[k * 3 + 0];
            r1 += b[k] * c[k * 3 + 1];
            r2 += b[k] * c[k * 3 + 2];
        }
    }
    colors[i * 3 + 0] = r0;
    colors[i * 3 + 1] = r1;
    colors[i * 3 + 2] = r2;
}

template <int DEG>
__global__ __launch_bounds__(256) void sh_bwd_kernel(int K, int64_t n, const float* __restrict__ dirs,
                                                     const float* __restrict__ coeffs,
                                                     const uint8_t* __restrict__ masks,
                                                     const float* __restrict__ v_colors,
                                                     float* __restrict__ v_coeffs,
                                                     float* __restrict__ v_dirs) {
    constexpr int NB = (DEG + 1) * (DEG + 1);
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float* vc = v_coeffs + i * K * 3;
    const bool on = !masks || masks[i];
    if (!on) {
        for (int k = 0; k < K * 3; ++k) vc[k] = 0.f;
        return;
    }
    const float x = dirs[i * 3], y = dirs[i * 3 + 1], z = dirs[i * 3 + 2];
    const float inv = 1.0f / sqrtf(x * x + y * y + z * z);
    const float ux = x * inv, uy = y * inv, uz = z * inv;
    float b[NB];
    sh_basis<DEG>(ux, uy, uz, b);
    const float g0 = v_colors[i * 3], g1 = v_colors[i * 3 + 1], g2 = v_colors[i * 3 + 2];
#pragma unroll
    for (int k = 0; k < NB; ++k) {
        vc[k * 3 + 0] = b[k] * g0;
        vc[k * 3 + 1] = b[k] * g1;
        vc[k * 3 + 2] = b[k] * g2;
    }
    for (int k = NB * 3; k < K * 3; ++k) vc[k] = 0.f;
    if (DEG < 1 || !v_dirs) return;
    float bx[NB], by[NB], bz[NB];
    sh_basis_grad<DEG>(ux, uy, uz, bx, by, bz);
    const float* c = coeffs + i * K * 3;
    float gu0 = 0.f, gu1 = 0.f, gu2 = 0.f;
#pragma unroll
    for (int k = 0; k < NB; ++k) {
        const float vb = c[k * 3] * g0 + c[k * 3 + 1] * g1 + c[k * 3 + 2] * g2;
        gu0 += vb * bx[k];
        gu1 += vb * by[k];
        gu2 += vb * bz[k];
    }
    const float dot = gu0 * ux + gu1 * uy + gu2 * uz;
    v_dirs[i * 3 + 0] += (gu0 - dot * ux) * inv;
    v_dirs[i * 3 + 1] += (gu1 - dot * uy) * inv;
    v_dirs[i * 3 + 2] += (gu2 - dot * uz) * inv;
}

}  // namespace hgsr

using namespace hgsr;

extern "C" int hgsr_sh_fwd(int degree, int K, int64_t n, const float* dirs, const float* coeffs,
                           const uint8_t* masks, float* colors, hgsr_stream_t stream) {
    HGSR_REQUIRE(degree >= 0 && degree <= 3, "sh degree %d unsupported (0..3)", degree);
    HGSR_REQUIRE(K >= (degree + 1) * (degree + 1), "K=%d too small for degree %d", K, degree);
    if (n == 0) return HGSR_OK;
    HGSR_REQUIRE(dirs && coeffs && colors, "null pointer");
    dim3 grid((unsigned)((n + 255) / 256));
    hipStream_t s = as_stream(stream);
    KernelTimer kt("sh_fwd", s);
    switch (degree) {
        case 0: hipLaunchKernelGGL(sh_fwd_kernel<0>, grid, dim3(256), 0, s, K, n, dirs, coeffs, masks, colors); break;
        case 1: hipLaunchKernelGGL(sh_fwd_kernel<1>, grid, dim3(256), 0, s, K, n, dirs, coeffs, masks, colors); break;
        case 2: hipLaunchKernelGGL(sh_fwd_kernel<2>, grid, dim3(256), 0, s, K, n, dirs, coeffs, masks, colors); break;
        default: hipLaunchKernelGGL(sh_fwd_kernel<3>, grid, dim3(256), 0, s, K, n, dirs, coeffs, masks, colors); break;
    }
    return check_launch("sh_fwd");
}

extern "C" int hgsr_sh_bwd(int degree, int K, int64_t n, const float* dirs, const float* coeffs,
                           const uint8_t* masks, const float* v_colors, float* v_coeffs, float* v_dirs,
                           hgsr_stream_t stream) {
    HGSR_REQUIRE(degree >= 0 && degree <= 3, "sh degree %d unsupported (0..3)", degree);
    HGSR_REQUIRE(K >= (degree + 1) * (degree + 1), "K=%d too small for degree %d", K, degree);
    if (n == 0) return HGSR_OK;
    HGSR_REQUIRE(dirs && coeffs && v_colors && v_coeffs, "null pointer");
    dim3 grid((unsigned)((n + 255) / 256));
    hipStream_t s = as_stream(stream);
    KernelTimer kt("sh_bwd", s);
    switch (degree) {
        case 0: hipLaunchKernelGGL(sh_bwd_kernel<0>, grid, dim3(256), 0, s, K, n, dirs, coeffs, masks, v_colors, v_coeffs, v_dirs); break;
        case 1: hipLaunchKernelGGL(sh_bwd_kernel<1>, grid, dim3(256), 0, s, K, n, dirs, coeffs, masks, v_colors, v_coeffs, v_dirs); break;
        case 2: hipLaunchKernelGGL(sh_bwd_kernel<2>, grid, dim3(256), 0, s, K, n, dirs, coeffs, masks, v_colors, v_coeffs, v_dirs); break;
        default: hipLaunchKernelGGL(sh_bwd_kernel<3>, grid, dim3(256), 0, s, K, n, dirs, coeffs, masks, v_colors, v_coeffs, v_dirs); break;
    }
    return check_launch("sh_bwd");
}
