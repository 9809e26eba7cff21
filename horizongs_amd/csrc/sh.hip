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

// rasterization()'s SH colours in one pass each way (gsplat rendering: dirs = means - campos,
// colors = spherical_harmonics(dirs, coeffs, masks = radii > 0), clamp_min(colors + 0.5, 0)):
// no dirs tensor, no elementwise offset / clamp kernels and no clamp mask in the backward,
// whose v_means (= v_dirs) is written directly.  Lane per Gaussian, cameras in a loop
// (deterministic sums over cameras for shared coefficients).  A workgroup's 256 coefficient
// rows (K x 3 floats each, contiguous in HBM) come in -- and the backward's gradient rows go
// out -- as contiguous float4 runs through LDS: lane-strided 108-B rows made every load and
// store instruction touch 64 cache lines.
constexpr int kShMaxK = 16;  // (degree 3 + 1)^2: at most 48 KB of dynamic LDS per workgroup

template <int DEG>
__device__ __forceinline__ bool sh_rgb_eval(int K, const float* __restrict__ m, const float* __restrict__ cp,
                                            const float* c, bool on, float (&u)[3], float& inv,
                                            float (&b)[(DEG + 1) * (DEG + 1)], float (&r)[3]) {
    constexpr int NB = (DEG + 1) * (DEG + 1);
    r[0] = r[1] = r[2] = 0.f;
    if (!on) return false;
    const float x = m[0] - cp[0], y = m[1] - cp[1], z = m[2] - cp[2];
    inv = 1.0f / sqrtf(x * x + y * y + z * z);
    u[0] = x * inv, u[1] = y * inv, u[2] = z * inv;
    sh_basis<DEG>(u[0], u[1], u[2], b);
#pragma unroll
    for (int k = 0; k < NB; ++k) {
        r[0] += b[k] * c[k * 3 + 0];
        r[1] += b[k] * c[k * 3 + 1];
        r[2] += b[k] * c[k * 3 + 2];
    }
    return true;
}

// camera c's centre: campos[c] given, else -R^T t of the world-to-camera view matrix
// viewmats[c] (row-major 4x4): the renderer's camera centres without a batched GEMM + negation in
// torch per view
__device__ __forceinline__ void cam_center(const float* __restrict__ campos, const float* __restrict__ viewmats,
                                           int c, float (&cp)[3]) {
    if (viewmats) {
        const float* v = viewmats + c * 16;
#pragma unroll
        for (int j = 0; j < 3; ++j) cp[j] = -(v[j] * v[3] + v[4 + j] * v[7] + v[8 + j] * v[11]);
    } else {
#pragma unroll
        for (int j = 0; j < 3; ++j) cp[j] = campos[c * 3 + j];
    }
}

template <int DEG>
__global__ __launch_bounds__(256) void sh_rgb_fwd_kernel(int C, int N, int K, const float* __restrict__ means,
                                                         const float* __restrict__ campos,
                                                         const float* __restrict__ viewmats,
                                                         const float* __restrict__ coeffs, int shared,
                                                         const int32_t* __restrict__ radii,
                                                         float* __restrict__ colors) {
    // (the forward only reads its rows: staging them through LDS measured slower, 83 -> 90 us at c4)
    constexpr int NB = (DEG + 1) * (DEG + 1);
    const int g = blockIdx.x * 256 + threadIdx.x;
    if (g >= N) return;
    for (int c = 0; c < C; ++c) {
        const int64_t i = (int64_t)c * N + g;
        float u[3], inv, b[NB], r[3], cp[3];
        cam_center(campos, viewmats, c, cp);
        sh_rgb_eval<DEG>(K, means + (int64_t)g * 3, cp, coeffs + (shared ? g : i) * K * 3,
                         radii[i] > 0, u, inv, b, r);
#pragma unroll
        for (int q = 0; q < 3; ++q) colors[i * 3 + q] = fmaxf(r[q] + 0.5f, 0.0f);
    }
}

template <int DEG>
__global__ __launch_bounds__(256) void sh_rgb_bwd_kernel(int C, int N, int K, const float* __restrict__ means,
                                                         const float* __restrict__ campos,
                                                         const float* __restrict__ viewmats,
                                                         const float* __restrict__ coeffs, int shared,
                                                         const int32_t* __restrict__ radii,
                                                         const float* __restrict__ v_colors,
                                                         float* __restrict__ v_coeffs, float* __restrict__ v_means) {
    constexpr int NB = (DEG + 1) * (DEG + 1);
    extern __shared__ __attribute__((aligned(16))) float s_cf[];  // [256][K x 3], sized at launch
    const int g0 = blockIdx.x * 256, nloc = min(256, N - g0), t = threadIdx.x, g = g0 + t;
    const int row = K * 3;
    float* const my = s_cf + t * row;  // this lane's row: coefficients in, their gradient out
    float vm[3] = {0.f, 0.f, 0.f};
    float vsum[NB * 3];  // shared coefficients: summed over cameras
#pragma unroll
    for (int k = 0; k < NB * 3; ++k) vsum[k] = 0.f;
    for (int c = 0; c < C; ++c) {
        const int64_t base = shared ? (int64_t)g0 : (int64_t)c * N + g0;
        if (c == 0 || !shared) {
            if (c > 0) __syncthreads();  // the previous camera's gradient rows have left
            stage_floats(coeffs + base * row, nloc * row, s_cf);
            __syncthreads();
        }
        if (t < nloc) {
            const int64_t i = (int64_t)c * N + g;
            float u[3], inv, b[NB], r[3], cp[3];
            cam_center(campos, viewmats, c, cp);
            const bool on = sh_rgb_eval<DEG>(K, means + (int64_t)g * 3, cp, my, radii[i] > 0, u, inv, b, r);
            // clamp_min backward: the gradient passes where colour + 0.5 >= 0
            float gq[3];
#pragma unroll
            for (int q = 0; q < 3; ++q) gq[q] = (on && r[q] + 0.5f >= 0.0f) ? v_colors[i * 3 + q] : 0.f;
            if (DEG >= 1 && on && v_means) {
                float bx[NB], by[NB], bz[NB];
                sh_basis_grad<DEG>(u[0], u[1], u[2], bx, by, bz);
                float gu0 = 0.f, gu1 = 0.f, gu2 = 0.f;
#pragma unroll
                for (int k = 0; k < NB; ++k) {
                    const float vb = my[k * 3] * gq[0] + my[k * 3 + 1] * gq[1] + my[k * 3 + 2] * gq[2];
                    gu0 += vb * bx[k];
                    gu1 += vb * by[k];
                    gu2 += vb * bz[k];
                }
                const float dot = gu0 * u[0] + gu1 * u[1] + gu2 * u[2];
                vm[0] += (gu0 - dot * u[0]) * inv;
                vm[1] += (gu1 - dot * u[1]) * inv;
                vm[2] += (gu2 - dot * u[2]) * inv;
            }
            if (shared) {
#pragma unroll
                for (int k = 0; k < NB; ++k)
#pragma unroll
                    for (int q = 0; q < 3; ++q) vsum[k * 3 + q] += b[k] * gq[q];
            } else {  // the row's coefficients are no longer needed: its gradient replaces them
#pragma unroll
                for (int k = 0; k < NB; ++k)
#pragma unroll
                    for (int q = 0; q < 3; ++q) my[k * 3 + q] = on ? b[k] * gq[q] : 0.f;
                for (int k = NB * 3; k < row; ++k) my[k] = 0.f;
            }
        }
        if (!shared) {
            __syncthreads();
            unstage_floats(s_cf, nloc * row, v_coeffs + base * row);
        }
    }
    if (shared) {
        if (t < nloc) {
#pragma unroll
            for (int k = 0; k < NB * 3; ++k) my[k] = vsum[k];
            for (int k = NB * 3; k < row; ++k) my[k] = 0.f;
        }
        __syncthreads();
        unstage_floats(s_cf, nloc * row, v_coeffs + (int64_t)g0 * row);
    }
    if (v_means && t < nloc)
#pragma unroll
        for (int q = 0; q < 3; ++q) v_means[(int64_t)g * 3 + q] = vm[q];
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

extern "C" int hgsr_sh_rgb_fwd(int degree, int C, int N, int K, const float* means, const float* campos,
                               const float* viewmats, const float* coeffs, int shared, const int32_t* radii,
                               float* colors, hgsr_stream_t stream) {
    HGSR_REQUIRE(degree >= 0 && degree <= 3, "sh degree %d unsupported (0..3)", degree);
    HGSR_REQUIRE(K >= (degree + 1) * (degree + 1), "K=%d too small for degree %d", K, degree);
    HGSR_REQUIRE(C >= 1 && N >= 0, "bad dims C=%d N=%d", C, N);
    // the backward stages K coefficient rows in LDS: refuse here, not one step later in it
    HGSR_REQUIRE(K <= kShMaxK, "sh_rgb: K=%d coefficients per Gaussian (at most %d)", K, kShMaxK);
    if (N == 0) return HGSR_OK;
    HGSR_REQUIRE(means && (campos || viewmats) && coeffs && radii && colors, "null pointer");
    dim3 grid((unsigned)((N + 255) / 256));
    hipStream_t s = as_stream(stream);
    KernelTimer kt("sh_fwd", s);
#define SH_RGB_F(D) hipLaunchKernelGGL(sh_rgb_fwd_kernel<D>, grid, dim3(256), 0, s, C, N, K, means, campos, \
                                       viewmats, coeffs, shared, radii, colors)
    switch (degree) {
        case 0: SH_RGB_F(0); break;
        case 1: SH_RGB_F(1); break;
        case 2: SH_RGB_F(2); break;
        default: SH_RGB_F(3); break;
    }
#undef SH_RGB_F
    return check_launch("sh_rgb_fwd");
}

extern "C" int hgsr_sh_rgb_bwd(int degree, int C, int N, int K, const float* means, const float* campos,
                               const float* viewmats, const float* coeffs, int shared, const int32_t* radii,
                               const float* v_colors, float* v_coeffs, float* v_means, hgsr_stream_t stream) {
    HGSR_REQUIRE(degree >= 0 && degree <= 3, "sh degree %d unsupported (0..3)", degree);
    HGSR_REQUIRE(K >= (degree + 1) * (degree + 1), "K=%d too small for degree %d", K, degree);
    HGSR_REQUIRE(C >= 1 && N >= 0, "bad dims C=%d N=%d", C, N);
    HGSR_REQUIRE(K <= kShMaxK, "sh_rgb: K=%d coefficients per Gaussian (at most %d)", K, kShMaxK);
    if (N == 0) return HGSR_OK;
    HGSR_REQUIRE(means && (campos || viewmats) && coeffs && radii && v_colors && v_coeffs, "null pointer");
    dim3 grid((unsigned)((N + 255) / 256));
    hipStream_t s = as_stream(stream);
    KernelTimer kt("sh_bwd", s);
    const size_t lds = (size_t)256 * K * 3 * sizeof(float);
#define SH_RGB_B(D) hipLaunchKernelGGL(sh_rgb_bwd_kernel<D>, grid, dim3(256), lds, s, C, N, K, means, campos,   \
                                       viewmats, coeffs, shared, radii, v_colors, v_coeffs, v_means)
    switch (degree) {
        case 0: SH_RGB_B(0); break;
        case 1: SH_RGB_B(1); break;
        case 2: SH_RGB_B(2); break;
        default: SH_RGB_B(3); break;
    }
#undef SH_RGB_B
    return check_launch("sh_rgb_bwd");
}
