// K13: normals from the rendered depth map (2DGS branch), forward and backward.
//
// Reference semantics: the FantasticOven2 gsplat fork's depth_to_normal, reached from
// rasterization_2dgs (gaussian_renderer/render.py:62-76) and consumed by the normal
// consistency term of train.py:180-188.  Per camera, with c2w = [R | o]:
//   dir(y, x) = R ((x - cx + 0.5) / fx, (y - cy + 0.5) / fy, 1)   (normalised if !z_depth)
//   P(y, x)   = o + depth(y, x) dir(y, x)
//   a = P(y+1, x) - P(y-1, x),  b = P(y, x+1) - P(y, x-1),  n = normalize(a x b)
// on interior pixels, 0 on the one-pixel border.  The torch version costs ~25 launches
// (two of them 130-us hipBLASLt GEMMs of shape 3 x 3 x HW) per direction per view.
//
// CDNA4 mapping: one lane per pixel, 16 x 16 pixel tiles per workgroup so the 4- (forward)
// or 12-neighbour (backward) depth reads hit L1/L2; the origin cancels in a and b and is
// never added (fewer roundings than o + d dir followed by the difference).  The backward
// gathers instead of scattering: d depth(p) = dir(p) . (A(p - y) - A(p + y) + B(p - x) -
// B(p + x)) with A = b x g_raw, B = g_raw x a the cross-product vjps of the neighbours,
// points and vjps staged once per 16 x 16 tile in LDS.
#include "common.h"

namespace hgsr {

struct NrmCam {
    float r[9];   // c2w rotation, row-major
    float fx, fy, cx, cy;
};

struct NrmDims {
    int C, H, W;
    int z_depth;
    int from_viewmat;  // the camera matrices are world -> camera viewmats: R_c2w = R^T
    const float* depth;  // [C,H,W] with strides
    int64_t ds[3];
};

__device__ __forceinline__ NrmCam nrm_cam(const float* __restrict__ c2w, const float* __restrict__ Ks, int c,
                                          int from_viewmat) {
    NrmCam k;
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) k.r[i * 3 + j] = from_viewmat ? c2w[c * 16 + j * 4 + i] : c2w[c * 16 + i * 4 + j];
    k.fx = Ks[c * 9 + 0];
    k.fy = Ks[c * 9 + 4];
    k.cx = Ks[c * 9 + 2];
    k.cy = Ks[c * 9 + 5];
    return k;
}

__device__ __forceinline__ float3 nrm_dir(const NrmCam& k, int y, int x, int z_depth) {
    const float u = ((float)x - k.cx + 0.5f) / k.fx, v = ((float)y - k.cy + 0.5f) / k.fy;
    float3 d = make_float3(k.r[0] * u + k.r[1] * v + k.r[2], k.r[3] * u + k.r[4] * v + k.r[5],
                           k.r[6] * u + k.r[7] * v + k.r[8]);
    if (!z_depth) {
        const float inv = 1.0f / fmaxf(sqrtf(d.x * d.x + d.y * d.y + d.z * d.z), 1e-12f);
        d = make_float3(d.x * inv, d.y * inv, d.z * inv);
    }
    return d;
}

// P(y, x) - o
__device__ __forceinline__ float3 nrm_point(const NrmDims& g, const NrmCam& k, int c, int y, int x) {
    const float dep = g.depth[c * g.ds[0] + y * g.ds[1] + x * g.ds[2]];
    const float3 d = nrm_dir(k, y, x, g.z_depth);
    return make_float3(dep * d.x, dep * d.y, dep * d.z);
}

__device__ __forceinline__ float3 sub3(float3 a, float3 b) { return make_float3(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ float3 cross3(float3 a, float3 b) {
    return make_float3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}

__device__ __forceinline__ bool interior(const NrmDims& g, int y, int x) {
    return y >= 1 && y <= g.H - 2 && x >= 1 && x <= g.W - 2;
}

// pixel id of this lane: 16 x 16 tiles, tile-major grid over (camera, tile row, tile column)
__device__ __forceinline__ bool nrm_pixel(const NrmDims& g, int& c, int& y, int& x) {
    const int tw = (g.W + 15) / 16, th = (g.H + 15) / 16;
    const int b = blockIdx.x;
    c = b / (tw * th);
    const int t = b - c * tw * th;
    y = (t / tw) * 16 + (threadIdx.x >> 4);
    x = (t % tw) * 16 + (threadIdx.x & 15);
    return y < g.H && x < g.W;
}

__global__ __launch_bounds__(256) void depth_normal_fwd_kernel(NrmDims g, const float* __restrict__ c2w,
                                                               const float* __restrict__ Ks,
                                                               float* __restrict__ normals) {
    int c, y, x;
    if (!nrm_pixel(g, c, y, x)) return;
    float3 n = make_float3(0.f, 0.f, 0.f);
    if (interior(g, y, x)) {
        const NrmCam k = nrm_cam(c2w, Ks, c, g.from_viewmat);
        const float3 a = sub3(nrm_point(g, k, c, y + 1, x), nrm_point(g, k, c, y - 1, x));
        const float3 b = sub3(nrm_point(g, k, c, y, x + 1), nrm_point(g, k, c, y, x - 1));
        n = cross3(a, b);
        const float inv = 1.0f / fmaxf(sqrtf(n.x * n.x + n.y * n.y + n.z * n.z), 1e-12f);
        n = make_float3(n.x * inv, n.y * inv, n.z * inv);
    }
    float* o = normals + (((int64_t)c * g.H + y) * g.W + x) * 3;
    o[0] = n.x;
    o[1] = n.y;
    o[2] = n.z;
}

// LDS-tiled backward: the 20 x 20 points of the tile (+2 halo) are unprojected once, the
// cross-product vjps of the 18 x 18 (+1 halo) normals once, then every pixel gathers its
// four neighbours' terms (each point / vjp evaluated once instead of 4x / 4x recomputed).
constexpr int kNT = 16, kNP = kNT + 4, kNV = kNT + 2;
__global__ __launch_bounds__(256) void depth_normal_bwd_kernel(NrmDims g, const float* __restrict__ c2w,
                                                               const float* __restrict__ Ks,
                                                               const float* __restrict__ g_normals,
                                                               float* __restrict__ g_depth) {
    __shared__ float s_p[3][kNP * kNP];
    __shared__ float s_a[3][kNV * kNV], s_b[3][kNV * kNV];
    const int tw = (g.W + kNT - 1) / kNT, th = (g.H + kNT - 1) / kNT;
    const int c = blockIdx.x / (tw * th);
    const int t = blockIdx.x - c * tw * th;
    const int ty0 = (t / tw) * kNT, tx0 = (t % tw) * kNT;
    const NrmCam k = nrm_cam(c2w, Ks, c, g.from_viewmat);
    for (int e = threadIdx.x; e < kNP * kNP; e += 256) {
        const int y = ty0 - 2 + e / kNP, x = tx0 - 2 + e % kNP;
        float3 p = make_float3(0.f, 0.f, 0.f);
        if (y >= 0 && y < g.H && x >= 0 && x < g.W) p = nrm_point(g, k, c, y, x);
        s_p[0][e] = p.x;
        s_p[1][e] = p.y;
        s_p[2][e] = p.z;
    }
    __syncthreads();
    auto P = [&](int ly, int lx) {  // local point coordinates relative to (ty0 - 2, tx0 - 2)
        const int e = ly * kNP + lx;
        return make_float3(s_p[0][e], s_p[1][e], s_p[2][e]);
    };
    for (int e = threadIdx.x; e < kNV * kNV; e += 256) {
        const int vy = e / kNV, vx = e % kNV;          // vjp pixel (ty0 - 1 + vy, tx0 - 1 + vx)
        const int y = ty0 - 1 + vy, x = tx0 - 1 + vx;
        float3 A = make_float3(0.f, 0.f, 0.f), B = A;
        if (interior(g, y, x)) {
            const int ly = vy + 1, lx = vx + 1;
            const float3 a = sub3(P(ly + 1, lx), P(ly - 1, lx));
            const float3 b = sub3(P(ly, lx + 1), P(ly, lx - 1));
            const float3 n = cross3(a, b);
            const float nr = sqrtf(n.x * n.x + n.y * n.y + n.z * n.z);
            const float* gp = g_normals + (((int64_t)c * g.H + y) * g.W + x) * 3;
            const float3 gv = make_float3(gp[0], gp[1], gp[2]);
            float3 gr;
            if (nr > 1e-12f) {
                // d/dn (n / |n|) = (I - u u^T) / |n|
                const float inv = 1.0f / nr;
                const float3 u = make_float3(n.x * inv, n.y * inv, n.z * inv);
                const float ug = u.x * gv.x + u.y * gv.y + u.z * gv.z;
                gr = make_float3((gv.x - u.x * ug) * inv, (gv.y - u.y * ug) * inv, (gv.z - u.z * ug) * inv);
            } else {
                gr = make_float3(gv.x * 1e12f, gv.y * 1e12f, gv.z * 1e12f);  // n / eps
            }
            A = cross3(b, gr);
            B = cross3(gr, a);
        }
        s_a[0][e] = A.x; s_a[1][e] = A.y; s_a[2][e] = A.z;
        s_b[0][e] = B.x; s_b[1][e] = B.y; s_b[2][e] = B.z;
    }
    __syncthreads();
    const int ly = threadIdx.x >> 4, lx = threadIdx.x & 15;
    const int y = ty0 + ly, x = tx0 + lx;
    if (y >= g.H || x >= g.W) return;
    // this pixel is the +y end of a at (y-1, x), the -y end at (y+1, x), the +x end of b at
    // (y, x-1) and the -x end at (y, x+1); vjp array index of pixel (y', x') = (y'-ty0+1, x'-tx0+1)
    const int vc = (ly + 1) * kNV + (lx + 1);
    float G[3];
#pragma unroll
    for (int q = 0; q < 3; ++q) G[q] = s_a[q][vc - kNV] - s_a[q][vc + kNV] + s_b[q][vc - 1] - s_b[q][vc + 1];
    const float3 d = nrm_dir(k, y, x, g.z_depth);
    g_depth[((int64_t)c * g.H + y) * g.W + x] = d.x * G[0] + d.y * G[1] + d.z * G[2];
}

}  // namespace hgsr

using namespace hgsr;

static int nrm_check(int C, int H, int W, const float* depth, const float* c2w, const float* Ks) {
    HGSR_REQUIRE(C >= 1 && H >= 1 && W >= 1, "depth_normal: bad dims");
    HGSR_REQUIRE(depth && c2w && Ks, "depth_normal: null pointer");
    HGSR_REQUIRE((int64_t)C * ((H + 15) / 16) * ((W + 15) / 16) < (1ll << 31), "depth_normal: image too large");
    return HGSR_OK;
}

extern "C" int hgsr_depth_normal_fwd(int C, int H, int W, const float* depth, const int64_t* depth_strides,
                                     const float* camtoworlds, const float* Ks, int z_depth, int from_viewmat,
                                     float* normals, hgsr_stream_t stream) {
    if (int st = nrm_check(C, H, W, depth, camtoworlds, Ks)) return st;
    HGSR_REQUIRE(depth_strides && normals, "depth_normal: null pointer");
    const NrmDims g{C, H, W, z_depth, from_viewmat, depth, {depth_strides[0], depth_strides[1], depth_strides[2]}};
    const unsigned grid = (unsigned)(C * ((H + 15) / 16) * ((W + 15) / 16));
    KernelTimer kt("depth_normal_fwd", as_stream(stream));
    hipLaunchKernelGGL(depth_normal_fwd_kernel, dim3(grid), dim3(256), 0, as_stream(stream), g, camtoworlds, Ks,
                       normals);
    return check_launch("depth_normal_fwd");
}

extern "C" int hgsr_depth_normal_bwd(int C, int H, int W, const float* depth, const int64_t* depth_strides,
                                     const float* camtoworlds, const float* Ks, int z_depth, int from_viewmat,
                                     const float* v_normals, float* v_depth, hgsr_stream_t stream) {
    if (int st = nrm_check(C, H, W, depth, camtoworlds, Ks)) return st;
    HGSR_REQUIRE(depth_strides && v_normals && v_depth, "depth_normal: null pointer");
    const NrmDims g{C, H, W, z_depth, from_viewmat, depth, {depth_strides[0], depth_strides[1], depth_strides[2]}};
    const unsigned grid = (unsigned)(C * ((H + 15) / 16) * ((W + 15) / 16));
    KernelTimer kt("depth_normal_bwd", as_stream(stream));
    hipLaunchKernelGGL(depth_normal_bwd_kernel, dim3(grid), dim3(256), 0, as_stream(stream), g, camtoworlds, Ks,
                       v_normals, v_depth);
    return check_launch("depth_normal_bwd");
}

namespace hgsr {
// out[c, m] = R_c v (transpose = 0) or R_c^T v (transpose = 1) for vectors in[c, m] (3 floats)
__global__ __launch_bounds__(256) void rotate3_kernel(int C, int64_t M, const float* __restrict__ R, int cam_stride,
                                                      int row_stride, int transpose, const float* __restrict__ in,
                                                      float* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= (int64_t)C * M) return;
    const int c = (int)(i / M);
    float r[9];
#pragma unroll
    for (int k = 0; k < 9; ++k)
        r[k] = transpose ? R[c * cam_stride + (k % 3) * row_stride + k / 3] : R[c * cam_stride + (k / 3) * row_stride + k % 3];
    const float x = in[i * 3], y = in[i * 3 + 1], z = in[i * 3 + 2];
    out[i * 3] = r[0] * x + r[1] * y + r[2] * z;
    out[i * 3 + 1] = r[3] * x + r[4] * y + r[5] * z;
    out[i * 3 + 2] = r[6] * x + r[7] * y + r[8] * z;
}
}  // namespace hgsr

extern "C" int hgsr_rotate3(int C, int64_t M, const float* R, int cam_stride, int row_stride, int transpose,
                            const float* in, float* out, hgsr_stream_t stream) {
    HGSR_REQUIRE(C >= 1 && M >= 0 && cam_stride >= 0 && row_stride >= 3, "rotate3: bad dims");
    if (M == 0) return HGSR_OK;
    HGSR_REQUIRE(R && in && out, "rotate3: null pointer");
    const int64_t n = (int64_t)C * M;
    hipLaunchKernelGGL(rotate3_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, as_stream(stream), C, M, R,
                       cam_stride, row_stride, transpose, in, out);
    return check_launch("rotate3");
}
