// K1/K2/K10: Gaussian projection, 3DGS (EWA) and 2DGS (surfel ray transform),
// forward and backward.  One lane per (camera, Gaussian); HBM-bound.
//
// Compiled with -ffp-contract=off: radii, means2d and depths feed the integer
// tile/intersection keys, which must be bit-identical to the CPU restatement
// (oracle/hgsr_oracle.c), so every expression keeps the oracle's operation
// order and rounding (correctly rounded divide/sqrt, no FMA contraction).
//
// Semantics: gsplat fully_fused_projection / fully_fused_projection_2dgs as
// called at reference gaussian_renderer/render.py:149-186 and inside
// gsplat.rasterization[_2dgs] (render.py:40-76).
#include "common.h"

namespace hgsr {

struct Mat3 {
    float m[3][3];
};

__device__ __forceinline__ Mat3 mm3(const Mat3& a, const Mat3& b) {
    Mat3 o;
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) o.m[i][j] = a.m[i][0] * b.m[0][j] + a.m[i][1] * b.m[1][j] + a.m[i][2] * b.m[2][j];
    return o;
}
// a * b^T
__device__ __forceinline__ Mat3 mm3_bt(const Mat3& a, const Mat3& b) {
    Mat3 o;
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) o.m[i][j] = a.m[i][0] * b.m[j][0] + a.m[i][1] * b.m[j][1] + a.m[i][2] * b.m[j][2];
    return o;
}
// a^T * b
__device__ __forceinline__ Mat3 mm3_at(const Mat3& a, const Mat3& b) {
    Mat3 o;
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) o.m[i][j] = a.m[0][i] * b.m[0][j] + a.m[1][i] * b.m[1][j] + a.m[2][i] * b.m[2][j];
    return o;
}

struct View {
    Mat3 R;
    float t[3];
    float fx, fy, cx, cy;
};

__device__ __forceinline__ View load_view(const float* __restrict__ vm, const float* __restrict__ K) {
    View v;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
#pragma unroll
        for (int j = 0; j < 3; ++j) v.R.m[i][j] = vm[i * 4 + j];
        v.t[i] = vm[i * 4 + 3];
    }
    v.fx = K[0];
    v.cx = K[2];
    v.fy = K[4];
    v.cy = K[5];
    return v;
}

__device__ __forceinline__ void to_camera(const View& v, const float* m, float mc[3]) {
#pragma unroll
    for (int i = 0; i < 3; ++i) mc[i] = v.R.m[i][0] * m[0] + v.R.m[i][1] * m[1] + v.R.m[i][2] * m[2] + v.t[i];
}

__device__ __forceinline__ Mat3 quat_to_rotmat(float4 q) {
    float w = q.x, x = q.y, y = q.z, z = q.w;
    float n2 = x * x + y * y + z * z + w * w;
    float inv = 1.0f / sqrtf(n2);
    x = x * inv; y = y * inv; z = z * inv; w = w * inv;
    float x2 = x * x, y2 = y * y, z2 = z * z;
    float xy = x * y, xz = x * z, yz = y * z;
    float wx = w * x, wy = w * y, wz = w * z;
    Mat3 R;
    R.m[0][0] = 1.0f - 2.0f * (y2 + z2);
    R.m[0][1] = 2.0f * (xy - wz);
    R.m[0][2] = 2.0f * (xz + wy);
    R.m[1][0] = 2.0f * (xy + wz);
    R.m[1][1] = 1.0f - 2.0f * (x2 + z2);
    R.m[1][2] = 2.0f * (yz - wx);
    R.m[2][0] = 2.0f * (xz - wy);
    R.m[2][1] = 2.0f * (yz + wx);
    R.m[2][2] = 1.0f - 2.0f * (x2 + y2);
    return R;
}

__device__ __forceinline__ float4 quat_to_rotmat_vjp(float4 q, const Mat3& vR) {
    float w = q.x, x = q.y, y = q.z, z = q.w;
    float n2 = x * x + y * y + z * z + w * w;
    float inv = 1.0f / sqrtf(n2);
    x = x * inv; y = y * inv; z = z * inv; w = w * inv;
    const float(*v)[3] = vR.m;
    float gw = 2.0f * (x * (v[2][1] - v[1][2]) + y * (v[0][2] - v[2][0]) + z * (v[1][0] - v[0][1]));
    float gx = 2.0f * (-2.0f * x * (v[1][1] + v[2][2]) + y * (v[1][0] + v[0][1]) + z * (v[2][0] + v[0][2]) + w * (v[2][1] - v[1][2]));
    float gy = 2.0f * (x * (v[1][0] + v[0][1]) - 2.0f * y * (v[0][0] + v[2][2]) + z * (v[2][1] + v[1][2]) + w * (v[0][2] - v[2][0]));
    float gz = 2.0f * (x * (v[2][0] + v[0][2]) + y * (v[2][1] + v[1][2]) - 2.0f * z * (v[0][0] + v[1][1]) + w * (v[1][0] - v[0][1]));
    float dot = gw * w + gx * x + gy * y + gz * z;
    return make_float4((gw - dot * w) * inv, (gx - dot * x) * inv, (gy - dot * y) * inv, (gz - dot * z) * inv);
}

struct Lims {
    float xp, xn, yp, yn;
};

__device__ __forceinline__ Lims make_lims(const View& v, int W, int H) {
    Lims l;
    float tan_fovx = 0.5f * (float)W / v.fx;
    float tan_fovy = 0.5f * (float)H / v.fy;
    l.xp = ((float)W - v.cx) / v.fx + 0.3f * tan_fovx;
    l.xn = v.cx / v.fx + 0.3f * tan_fovx;
    l.yp = ((float)H - v.cy) / v.fy + 0.3f * tan_fovy;
    l.yn = v.cy / v.fy + 0.3f * tan_fovy;
    return l;
}

__device__ __forceinline__ float3 ld3(const float* p) { return make_float3(p[0], p[1], p[2]); }

__device__ __forceinline__ Mat3 covar_from_qs(float4 q, float3 s, Mat3& Rq) {
    Rq = quat_to_rotmat(q);
    Mat3 M;
    const float sv[3] = {s.x, s.y, s.z};
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) M.m[i][j] = Rq.m[i][j] * sv[j];
    return mm3_bt(M, M);
}

// ---------------------------------------------------------------- 3DGS fwd
struct Proj3 {
    int32_t rad;
    float2 m2;
    float dep, ca, cb, cc;
};

// gsplat fully_fused_projection (pinhole, non-packed) of one Gaussian; shared by the
// projection and the anchor prefilter so both decide radius > 0 with the same bits
__device__ __forceinline__ Proj3 project3d_one(const View& v, const Lims& L, const float m[3], float4 q, float3 s,
                                               int W, int H, float eps2d, float near_plane, float far_plane,
                                               float radius_clip) {
    Proj3 r{0, make_float2(0.f, 0.f), 0.f, 0.f, 0.f, 0.f};
    float mc[3];
    to_camera(v, m, mc);
    if (!(mc[2] < near_plane || mc[2] > far_plane)) {
        Mat3 Rq;
        const Mat3 cov = covar_from_qs(q, s, Rq);
        const Mat3 covc = mm3_bt(mm3(v.R, cov), v.R);
        const float x = mc[0], y = mc[1], z = mc[2];
        const float rz = 1.0f / z;
        const float rz2 = rz * rz;
        const float tx = z * fminf(L.xp, fmaxf(-L.xn, x * rz));
        const float ty = z * fminf(L.yp, fmaxf(-L.yn, y * rz));
        const float J[2][3] = {{v.fx * rz, 0.f, -v.fx * tx * rz2}, {0.f, v.fy * rz, -v.fy * ty * rz2}};
        float JS[2][3];
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 3; ++j) JS[i][j] = J[i][0] * covc.m[0][j] + J[i][1] * covc.m[1][j] + J[i][2] * covc.m[2][j];
        float c2[2][2];
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) c2[i][j] = JS[i][0] * J[j][0] + JS[i][1] * J[j][1] + JS[i][2] * J[j][2];
        const float mx = v.fx * x * rz + v.cx;
        const float my = v.fy * y * rz + v.cy;
        c2[0][0] = c2[0][0] + eps2d;
        c2[1][1] = c2[1][1] + eps2d;
        const float det = c2[0][0] * c2[1][1] - c2[0][1] * c2[1][0];
        if (det > 0.f) {
            const float idet = 1.0f / det;
            const float b = 0.5f * (c2[0][0] + c2[1][1]);
            const float v1 = b + sqrtf(fmaxf(0.01f, b * b - det));
            const float radius = ceilf(3.0f * sqrtf(v1));
            if (radius > radius_clip && !(mx + radius <= 0.f || mx - radius >= (float)W ||
                                          my + radius <= 0.f || my - radius >= (float)H)) {
                r.rad = (int32_t)radius;
                r.m2 = make_float2(mx, my);
                r.dep = z;
                r.ca = c2[1][1] * idet;
                r.cb = -c2[0][1] * idet;
                r.cc = c2[0][0] * idet;
            }
        }
    }
    return r;
}

__global__ __launch_bounds__(256) void project3d_fwd_kernel(
    int N, const float* __restrict__ means, const float4* __restrict__ quats,
    const float* __restrict__ scales, const float* __restrict__ viewmats,
    const float* __restrict__ Ks, int W, int H, float eps2d, float near_plane, float far_plane,
    float radius_clip, int32_t* __restrict__ radii, float2* __restrict__ means2d,
    float* __restrict__ depths, float* __restrict__ conics) {
    const int g = blockIdx.x * blockDim.x + threadIdx.x;
    const int c = blockIdx.y;
    if (g >= N) return;
    const int64_t o = (int64_t)c * N + g;
    const View v = load_view(viewmats + c * 16, Ks + c * 9);
    const Lims L = make_lims(v, W, H);
    const float m[3] = {means[(int64_t)g * 3], means[(int64_t)g * 3 + 1], means[(int64_t)g * 3 + 2]};
    const Proj3 r = project3d_one(v, L, m, quats[g], ld3(scales + (int64_t)g * 3), W, H, eps2d, near_plane,
                                  far_plane, radius_clip);
    radii[o] = r.rad;
    means2d[o] = r.m2;
    depths[o] = r.dep;
    conics[o * 3 + 0] = r.ca;
    conics[o * 3 + 1] = r.cb;
    conics[o * 3 + 2] = r.cc;
}

// Anchor prefilter (reference gaussian_renderer/render.py:120-197 prefilter_voxel after
// set_anchor_mask, scene/lod_model.py:286-290): visible[a] = LoD level test (when `level`
// is given; the test of hgsr_lod_mask) AND radius > 0 of the anchor projected with its
// first three scales (gsplat projection, camera 0).  One byte per anchor; no projection
// outputs are written (the reference keeps only radii > 0).
__global__ __launch_bounds__(256) void anchor_prefilter_kernel(
    int A, const float* __restrict__ anchor, const float4* __restrict__ quats, const float* __restrict__ scales,
    int scale_stride, const float* __restrict__ viewmat, const float* __restrict__ K, int W, int H, float eps2d,
    float near_plane, float far_plane, const int32_t* __restrict__ level, const float* __restrict__ extra_level,
    const float* __restrict__ cam, float res_scale, float standard_dist, float log2_fork, int max_level,
    uint8_t* __restrict__ visible) {
    const int a = blockIdx.x * 256 + threadIdx.x;
    if (a >= A) return;
    const float m[3] = {anchor[(int64_t)a * 3], anchor[(int64_t)a * 3 + 1], anchor[(int64_t)a * 3 + 2]};
    bool vis = true;
    if (level) {
        const float dx = m[0] - cam[0], dy = m[1] - cam[1], dz = m[2] - cam[2];
        const float dist = sqrtf(dx * dx + dy * dy + dz * dz) * res_scale;
        const float pred = log2f(standard_dist / dist) / log2_fork + extra_level[a];
        const float fl = floorf(pred);
        const int il = fl <= 0.f ? 0 : (fl >= (float)max_level ? max_level : (int)fl);
        vis = level[a] <= il;
    }
    if (vis) {
        const View v = load_view(viewmat, K);
        const Lims L = make_lims(v, W, H);
        const Proj3 r = project3d_one(v, L, m, quats[a], ld3(scales + (int64_t)a * scale_stride), W, H, eps2d,
                                      near_plane, far_plane, 0.0f);
        vis = r.rad > 0;
    }
    visible[a] = vis ? 1 : 0;
}

// ---------------------------------------------------------------- 3DGS bwd
// One lane per Gaussian, looping over cameras: deterministic accumulation.
// 3 waves per SIMD (<= 168 VGPRs, a few spills): 0.079 -> 0.071 ms at 2M Gaussians; 4 spills heavily.
// Branch-free camera loop with every load of a camera consumed at one point: 0.071 -> 0.059-0.066 ms
// (the same for project3d_fwd / project2d_bwd measured no change)
__global__ __launch_bounds__(256, 3) void project3d_bwd_kernel(
    int C, int N, const float* __restrict__ means, const float4* __restrict__ quats,
    const float* __restrict__ scales, const float* __restrict__ viewmats,
    const float* __restrict__ Ks, int W, int H, const int32_t* __restrict__ radii,
    const float* __restrict__ conics, const float2* __restrict__ v_means2d,
    const float* __restrict__ v_depths, const float* __restrict__ v_conics,
    float* __restrict__ v_means, float4* __restrict__ v_quats, float* __restrict__ v_scales,
    const float* __restrict__ v_scales_in, const float* __restrict__ v_means_in) {
    const int g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= N) return;
    const float m[3] = {means[(int64_t)g * 3], means[(int64_t)g * 3 + 1], means[(int64_t)g * 3 + 2]};
    const float4 q = quats[g];
    const float3 s3 = ld3(scales + (int64_t)g * 3);
    const float s[3] = {s3.x, s3.y, s3.z};
    float vm_acc[3] = {0.f, 0.f, 0.f};
    float vs_acc[3] = {0.f, 0.f, 0.f};
    float4 vq_acc = make_float4(0.f, 0.f, 0.f, 0.f);
    // branch-free camera loop: every load of a camera is issued together and consumed at
    // one point (one memory round trip per camera -- camera 0's together with the
    // Gaussian's own -- instead of a radius load, a branch and then the rest in three
    // waits); a culled pair's contributions are computed from whatever it holds and
    // selected away
    int32_t rad;
    float3 cn, vcn;
    float2 vm2;
    float vdep;
    auto load_cam = [&](int64_t o) {
        rad = radii[o];
        cn = ld3(conics + o * 3);
        vcn = ld3(v_conics + o * 3);
        vm2 = v_means2d[o];
        vdep = v_depths[o];
    };
#define HGSR_CAM_READY asm volatile("" ::"v"(rad), "v"(cn.x), "v"(cn.y), "v"(cn.z), "v"(vcn.x), "v"(vcn.y), \
                                    "v"(vcn.z), "v"(vm2.x), "v"(vm2.y), "v"(vdep))
    load_cam(g);
    // the other consumer's scale gradient travels with the first round trip (loaded after the
    // camera loop it costs one more exposed memory latency per lane at 3 waves / SIMD)
    const float3 vsi = v_scales_in ? ld3(v_scales_in + (int64_t)g * 3) : make_float3(0.f, 0.f, 0.f);
    const float3 vmi = v_means_in ? ld3(v_means_in + (int64_t)g * 3) : make_float3(0.f, 0.f, 0.f);
    HGSR_CAM_READY;
    asm volatile("" ::"v"(m[0]), "v"(m[1]), "v"(m[2]), "v"(q.x), "v"(q.y), "v"(q.z), "v"(q.w), "v"(s3.x),
                 "v"(s3.y), "v"(s3.z), "v"(vsi.x), "v"(vsi.y), "v"(vsi.z), "v"(vmi.x), "v"(vmi.y), "v"(vmi.z));
    Mat3 Rq;
    const Mat3 cov = covar_from_qs(q, s3, Rq);
    for (int c = 0; c < C; ++c) {
        if (c > 0) {
            load_cam((int64_t)c * N + g);
            HGSR_CAM_READY;
        }
#undef HGSR_CAM_READY
        const bool live = rad > 0;
        const View v = load_view(viewmats + c * 16, Ks + c * 9);
        const Lims L = make_lims(v, W, H);
        const float Ci[2][2] = {{cn.x, cn.y}, {cn.y, cn.z}};
        const float vCi[2][2] = {{vcn.x, 0.5f * vcn.y}, {0.5f * vcn.y, vcn.z}};
        float T1[2][2], vc2[2][2];
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) T1[i][j] = Ci[i][0] * vCi[0][j] + Ci[i][1] * vCi[1][j];
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) vc2[i][j] = -(T1[i][0] * Ci[0][j] + T1[i][1] * Ci[1][j]);
        float mc[3];
        to_camera(v, m, mc);
        const Mat3 covc = mm3_bt(mm3(v.R, cov), v.R);
        const float x = mc[0], y = mc[1], z = mc[2];
        const float rz = 1.0f / z, rz2 = rz * rz, rz3 = rz2 * rz;
        const float ux = x * rz, uy = y * rz;
        const float tx = z * fminf(L.xp, fmaxf(-L.xn, ux));
        const float ty = z * fminf(L.yp, fmaxf(-L.yn, uy));
        const float J[2][3] = {{v.fx * rz, 0.f, -v.fx * tx * rz2}, {0.f, v.fy * rz, -v.fy * ty * rz2}};
        Mat3 vcovc;
#pragma unroll
        for (int i = 0; i < 3; ++i)
#pragma unroll
            for (int j = 0; j < 3; ++j) {
                float acc = 0.f;
#pragma unroll
                for (int a = 0; a < 2; ++a)
#pragma unroll
                    for (int b2 = 0; b2 < 2; ++b2) acc += J[a][i] * vc2[a][b2] * J[b2][j];
                vcovc.m[i][j] = acc;
            }
        float vJ[2][3];
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
            for (int j = 0; j < 3; ++j) {
                float acc = 0.f;
#pragma unroll
                for (int b2 = 0; b2 < 2; ++b2)
#pragma unroll
                    for (int k = 0; k < 3; ++k) acc += (vc2[a][b2] + vc2[b2][a]) * J[b2][k] * covc.m[k][j];
                vJ[a][j] = acc;
            }
        float vmc[3];
        vmc[0] = v.fx * rz * vm2.x;
        vmc[1] = v.fy * rz * vm2.y;
        vmc[2] = -(v.fx * x * vm2.x + v.fy * y * vm2.y) * rz2;
        vmc[2] += -v.fx * rz2 * vJ[0][0] - v.fy * rz2 * vJ[1][1];
        if (ux <= L.xp && ux >= -L.xn) {
            vmc[0] += -v.fx * rz2 * vJ[0][2];
            vmc[2] += 2.0f * v.fx * tx * rz3 * vJ[0][2];
        } else {
            vmc[2] += v.fx * tx * rz3 * vJ[0][2];
        }
        if (uy <= L.yp && uy >= -L.yn) {
            vmc[1] += -v.fy * rz2 * vJ[1][2];
            vmc[2] += 2.0f * v.fy * ty * rz3 * vJ[1][2];
        } else {
            vmc[2] += v.fy * ty * rz3 * vJ[1][2];
        }
        vmc[2] += vdep;
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            const float d = v.R.m[0][j] * vmc[0] + v.R.m[1][j] * vmc[1] + v.R.m[2][j] * vmc[2];
            vm_acc[j] += live ? d : 0.f;
        }
        const Mat3 vcov = mm3(mm3_at(v.R, vcovc), v.R);
        Mat3 Mm, vsym;
#pragma unroll
        for (int i = 0; i < 3; ++i)
#pragma unroll
            for (int j = 0; j < 3; ++j) {
                Mm.m[i][j] = Rq.m[i][j] * s[j];
                vsym.m[i][j] = vcov.m[i][j] + vcov.m[j][i];
            }
        const Mat3 vM = mm3(vsym, Mm);
        Mat3 vRq;
#pragma unroll
        for (int i = 0; i < 3; ++i)
#pragma unroll
            for (int j = 0; j < 3; ++j) vRq.m[i][j] = vM.m[i][j] * s[j];
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            const float d = Rq.m[0][j] * vM.m[0][j] + Rq.m[1][j] * vM.m[1][j] + Rq.m[2][j] * vM.m[2][j];
            vs_acc[j] += live ? d : 0.f;
        }
        const float4 vq = quat_to_rotmat_vjp(q, vRq);
        vq_acc.x += live ? vq.x : 0.f;
        vq_acc.y += live ? vq.y : 0.f;
        vq_acc.z += live ? vq.z : 0.f;
        vq_acc.w += live ? vq.w : 0.f;
    }
    // overwrite semantics: a Gaussian culled in every camera gets zeros; v_scales_in / v_means_in
    // (another consumer's gradient of the scales / means) are added here instead of by a
    // separate sum -- one fp32 add of two terms, the same value autograd's sum gives
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        v_means[(int64_t)g * 3 + j] = v_means_in ? vm_acc[j] + (j == 0 ? vmi.x : (j == 1 ? vmi.y : vmi.z)) : vm_acc[j];
        v_scales[(int64_t)g * 3 + j] = v_scales_in ? vs_acc[j] + (j == 0 ? vsi.x : (j == 1 ? vsi.y : vsi.z)) : vs_acc[j];
    }
    v_quats[g] = vq_acc;
}

// ---------------------------------------------------------------- 2DGS fwd
struct Surfel {
    Mat3 RRq, Rq;
    float RS[3][3];
    float mc[3];
};

__device__ __forceinline__ Surfel surfel_frame(const View& v, const float* m, float4 q, float3 s) {
    Surfel f;
    to_camera(v, m, f.mc);
    f.Rq = quat_to_rotmat(q);
    f.RRq = mm3(v.R, f.Rq);
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        f.RS[i][0] = f.RRq.m[i][0] * s.x;
        f.RS[i][1] = f.RRq.m[i][1] * s.y;
        f.RS[i][2] = f.RRq.m[i][2];
    }
    return f;
}

__global__ __launch_bounds__(256) void project2d_fwd_kernel(
    int N, const float* __restrict__ means, const float4* __restrict__ quats,
    const float* __restrict__ scales, const float* __restrict__ viewmats,
    const float* __restrict__ Ks, int W, int H, float near_plane, float far_plane,
    float radius_clip, int32_t* __restrict__ radii, float2* __restrict__ means2d,
    float* __restrict__ depths, float* __restrict__ ray_transforms, float* __restrict__ normals) {
    // the 12-B rows (means, scales) come in and the 36-B ray transforms / 12-B normals go out
    // as contiguous runs through LDS
    __shared__ __attribute__((aligned(16))) float s_io[256 * 12];
    const int g0 = blockIdx.x * blockDim.x, t = threadIdx.x, g = g0 + t;
    const int c = blockIdx.y;
    const int nloc = min(256, N - g0);
    const bool live = t < nloc;
    const int64_t o = (int64_t)c * N + g, o0 = (int64_t)c * N + g0;
    stage_floats(means + (int64_t)g0 * 3, nloc * 3, s_io);
    stage_floats(scales + (int64_t)g0 * 3, nloc * 3, s_io + 768);
    __syncthreads();
    const float m[3] = {s_io[t * 3], s_io[t * 3 + 1], s_io[t * 3 + 2]};
    const float3 s3 = make_float3(s_io[768 + t * 3], s_io[768 + t * 3 + 1], s_io[768 + t * 3 + 2]);
    __syncthreads();  // s_io now collects the outputs
    const View v = load_view(viewmats + c * 16, Ks + c * 9);
    const Surfel f = surfel_frame(v, m, live ? quats[g] : make_float4(1.f, 0.f, 0.f, 0.f), s3);
    float M[3][3] = {{0.f, 0.f, 0.f}, {0.f, 0.f, 0.f}, {0.f, 0.f, 0.f}};
    float nrm[3] = {0.f, 0.f, 0.f};
    int32_t rad = 0;
    float2 m2 = make_float2(0.f, 0.f);
    float dep = 0.f;
    if (live && !(f.mc[2] < near_plane || f.mc[2] > far_plane)) {
        float WH[3][3];
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            WH[i][0] = f.RS[i][0];
            WH[i][1] = f.RS[i][1];
            WH[i][2] = f.mc[i];
        }
        float Mt[3][3];
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            Mt[0][j] = v.fx * WH[0][j] + v.cx * WH[2][j];
            Mt[1][j] = v.fy * WH[1][j] + v.cy * WH[2][j];
            Mt[2][j] = WH[2][j];
        }
        const float dist = Mt[2][0] * Mt[2][0] + Mt[2][1] * Mt[2][1] - Mt[2][2] * Mt[2][2];
        if (dist != 0.f) {
            const float f0 = 1.0f / dist, f2 = -(1.0f / dist);
            const float mx = f0 * Mt[0][0] * Mt[2][0] + f0 * Mt[0][1] * Mt[2][1] + f2 * Mt[0][2] * Mt[2][2];
            const float my = f0 * Mt[1][0] * Mt[2][0] + f0 * Mt[1][1] * Mt[2][1] + f2 * Mt[1][2] * Mt[2][2];
            const float tpx = f0 * Mt[0][0] * Mt[0][0] + f0 * Mt[0][1] * Mt[0][1] + f2 * Mt[0][2] * Mt[0][2];
            const float tpy = f0 * Mt[1][0] * Mt[1][0] + f0 * Mt[1][1] * Mt[1][1] + f2 * Mt[1][2] * Mt[1][2];
            const float hx = mx * mx - tpx, hy = my * my - tpy;
            const float radius = ceilf(3.33f * sqrtf(fmaxf(1e-4f, fmaxf(hx, hy))));
            if (radius > radius_clip && !(mx + radius <= 0.f || mx - radius >= (float)W ||
                                          my + radius <= 0.f || my - radius >= (float)H)) {
                const float n0 = f.RS[0][2], n1 = f.RS[1][2], n2 = f.RS[2][2];
                const float d = -n0 * f.mc[0] + -n1 * f.mc[1] + -n2 * f.mc[2];
                const float sgn = d > 0.f ? 1.0f : -1.0f;
                rad = (int32_t)radius;
                m2 = make_float2(mx, my);
                dep = f.mc[2];
#pragma unroll
                for (int i = 0; i < 3; ++i)
#pragma unroll
                    for (int j = 0; j < 3; ++j) M[i][j] = Mt[i][j];
                nrm[0] = n0 * sgn;
                nrm[1] = n1 * sgn;
                nrm[2] = n2 * sgn;
            }
        }
    }
    if (live) {
        radii[o] = rad;
        means2d[o] = m2;
        depths[o] = dep;
    }
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) s_io[t * 9 + i * 3 + j] = M[i][j];
#pragma unroll
    for (int i = 0; i < 3; ++i) s_io[256 * 9 + t * 3 + i] = nrm[i];
    __syncthreads();
    for (int e = t; e < nloc * 9; e += 256) ray_transforms[o0 * 9 + e] = s_io[e];
    for (int e = t; e < nloc * 3; e += 256) normals[o0 * 3 + e] = s_io[256 * 9 + e];
}

// ---------------------------------------------------------------- 2DGS bwd
__global__ __launch_bounds__(256) void project2d_bwd_kernel(
    int C, int N, const float* __restrict__ means, const float4* __restrict__ quats,
    const float* __restrict__ scales, const float* __restrict__ viewmats,
    const float* __restrict__ Ks, const int32_t* __restrict__ radii,
    const float* __restrict__ ray_transforms, const float2* __restrict__ v_means2d,
    const float* __restrict__ v_depths, const float* __restrict__ v_ray_transforms,
    const float* __restrict__ v_normals, float* __restrict__ v_means, float4* __restrict__ v_quats,
    float* __restrict__ v_scales, const float* __restrict__ v_scales_in) {
    const int g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= N) return;
    const float m[3] = {means[(int64_t)g * 3], means[(int64_t)g * 3 + 1], means[(int64_t)g * 3 + 2]};
    const float4 q = quats[g];
    const float3 s = ld3(scales + (int64_t)g * 3);
    const float3 vsi = v_scales_in ? ld3(v_scales_in + (int64_t)g * 3) : make_float3(0.f, 0.f, 0.f);  // (issued early)
    float vm_acc[3] = {0.f, 0.f, 0.f};
    float vs0 = 0.f, vs1 = 0.f;
    float4 vq_acc = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int c = 0; c < C; ++c) {
        const int64_t o = (int64_t)c * N + g;
        if (radii[o] <= 0) continue;
        const View v = load_view(viewmats + c * 16, Ks + c * 9);
        const Surfel f = surfel_frame(v, m, q, s);
        const float* M = ray_transforms + o * 9;
        float vM[3][3];
#pragma unroll
        for (int i = 0; i < 3; ++i)
#pragma unroll
            for (int j = 0; j < 3; ++j) vM[i][j] = v_ray_transforms[o * 9 + i * 3 + j];
        const float2 vm2 = v_means2d[o];
        const float dist = M[6] * M[6] + M[7] * M[7] - M[8] * M[8];
        const float id = 1.0f / dist;
        const float e[3] = {1.f, 1.f, -1.f};
        const float mx = (M[0] * M[6] + M[1] * M[7] - M[2] * M[8]) * id;
        const float my = (M[3] * M[6] + M[4] * M[7] - M[5] * M[8]) * id;
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            vM[0][j] += vm2.x * e[j] * M[6 + j] * id;
            vM[1][j] += vm2.y * e[j] * M[6 + j] * id;
            vM[2][j] += (vm2.x * e[j] * M[j] + vm2.y * e[j] * M[3 + j]) * id -
                        (vm2.x * mx + vm2.y * my) * 2.0f * e[j] * M[6 + j] * id;
        }
        float vWH[3][3];
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            vWH[0][j] = v.fx * vM[0][j];
            vWH[1][j] = v.fy * vM[1][j];
            vWH[2][j] = v.cx * vM[0][j] + v.cy * vM[1][j] + vM[2][j];
        }
        const float vmc[3] = {vWH[0][2], vWH[1][2], vWH[2][2] + v_depths[o]};
        const float n0 = f.RS[0][2], n1 = f.RS[1][2], n2 = f.RS[2][2];
        const float d = -n0 * f.mc[0] + -n1 * f.mc[1] + -n2 * f.mc[2];
        const float sgn = d > 0.f ? 1.0f : -1.0f;
        Mat3 vRRq;
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            vRRq.m[i][0] = vWH[i][0] * s.x;
            vRRq.m[i][1] = vWH[i][1] * s.y;
            vRRq.m[i][2] = sgn * v_normals[o * 3 + i];
            vs0 += vWH[i][0] * f.RRq.m[i][0];
            vs1 += vWH[i][1] * f.RRq.m[i][1];
        }
        const Mat3 vRq = mm3_at(v.R, vRRq);
        const float4 vq = quat_to_rotmat_vjp(q, vRq);
        vq_acc.x += vq.x; vq_acc.y += vq.y; vq_acc.z += vq.z; vq_acc.w += vq.w;
#pragma unroll
        for (int j = 0; j < 3; ++j) vm_acc[j] += v.R.m[0][j] * vmc[0] + v.R.m[1][j] * vmc[1] + v.R.m[2][j] * vmc[2];
    }
    // overwrite semantics: a Gaussian culled in every camera gets zeros
#pragma unroll
    for (int j = 0; j < 3; ++j) v_means[(int64_t)g * 3 + j] = vm_acc[j];
    if (v_scales_in) {
        v_scales[(int64_t)g * 3 + 0] = vs0 + vsi.x;
        v_scales[(int64_t)g * 3 + 1] = vs1 + vsi.y;
        v_scales[(int64_t)g * 3 + 2] = 0.f + vsi.z;
    } else {
        v_scales[(int64_t)g * 3 + 0] = vs0;
        v_scales[(int64_t)g * 3 + 1] = vs1;
        v_scales[(int64_t)g * 3 + 2] = 0.f;
    }
    v_quats[g] = vq_acc;
}

}  // namespace hgsr

using namespace hgsr;

static int check_common(int C, int N, const void* means, const void* quats, const void* scales,
                        const void* viewmats, const void* Ks, int W, int H) {
    HGSR_REQUIRE(C >= 1 && N >= 0 && W > 0 && H > 0, "bad dims C=%d N=%d W=%d H=%d", C, N, W, H);
    HGSR_REQUIRE(C <= 65535, "too many cameras (%d)", C);
    HGSR_REQUIRE(N == 0 || (means && quats && scales && viewmats && Ks), "null input pointer");
    return HGSR_OK;
}

extern "C" int hgsr_project3d_fwd(int C, int N, const float* means, const float* quats,
                                  const float* scales, const float* viewmats, const float* Ks,
                                  int width, int height, float eps2d, float near_plane,
                                  float far_plane, float radius_clip, int32_t* radii,
                                  float* means2d, float* depths, float* conics,
                                  hgsr_stream_t stream) {
    int st = check_common(C, N, means, quats, scales, viewmats, Ks, width, height);
    if (st) return st;
    HGSR_REQUIRE(N == 0 || (radii && means2d && depths && conics), "null output pointer");
    if (N == 0) return HGSR_OK;
    dim3 grid((N + 255) / 256, C);
    KernelTimer kt("project3d_fwd", as_stream(stream));
    hipLaunchKernelGGL(project3d_fwd_kernel, grid, dim3(256), 0, as_stream(stream), N, means,
                       reinterpret_cast<const float4*>(quats), scales, viewmats, Ks, width, height,
                       eps2d, near_plane, far_plane, radius_clip, radii,
                       reinterpret_cast<float2*>(means2d), depths, conics);
    return check_launch("project3d_fwd");
}

extern "C" int hgsr_project3d_bwd(int C, int N, const float* means, const float* quats,
                                  const float* scales, const float* viewmats, const float* Ks,
                                  int width, int height, float eps2d, const int32_t* radii,
                                  const float* conics, const float* v_means2d,
                                  const float* v_depths, const float* v_conics, float* v_means,
                                  float* v_quats, float* v_scales, const float* v_scales_in,
                                  const float* v_means_in, hgsr_stream_t stream) {
    (void)eps2d;
    int st = check_common(C, N, means, quats, scales, viewmats, Ks, width, height);
    if (st) return st;
    HGSR_REQUIRE(N == 0 || (radii && conics && v_means2d && v_depths && v_conics && v_means && v_quats && v_scales),
                 "null pointer");
    if (N == 0) return HGSR_OK;
    KernelTimer kt("project3d_bwd", as_stream(stream));
    hipLaunchKernelGGL(project3d_bwd_kernel, dim3((N + 255) / 256), dim3(256), 0, as_stream(stream), C, N,
                       means, reinterpret_cast<const float4*>(quats), scales, viewmats, Ks, width,
                       height, radii, conics, reinterpret_cast<const float2*>(v_means2d), v_depths,
                       v_conics, v_means, reinterpret_cast<float4*>(v_quats), v_scales, v_scales_in, v_means_in);
    return check_launch("project3d_bwd");
}

extern "C" int hgsr_project2d_fwd(int C, int N, const float* means, const float* quats,
                                  const float* scales, const float* viewmats, const float* Ks,
                                  int width, int height, float near_plane, float far_plane,
                                  float radius_clip, int32_t* radii, float* means2d, float* depths,
                                  float* ray_transforms, float* normals, hgsr_stream_t stream) {
    int st = check_common(C, N, means, quats, scales, viewmats, Ks, width, height);
    if (st) return st;
    HGSR_REQUIRE(N == 0 || (radii && means2d && depths && ray_transforms && normals), "null output pointer");
    if (N == 0) return HGSR_OK;
    dim3 grid((N + 255) / 256, C);
    KernelTimer kt("project2d_fwd", as_stream(stream));
    hipLaunchKernelGGL(project2d_fwd_kernel, grid, dim3(256), 0, as_stream(stream), N, means,
                       reinterpret_cast<const float4*>(quats), scales, viewmats, Ks, width, height,
                       near_plane, far_plane, radius_clip, radii, reinterpret_cast<float2*>(means2d),
                       depths, ray_transforms, normals);
    return check_launch("project2d_fwd");
}

extern "C" int hgsr_project2d_bwd(int C, int N, const float* means, const float* quats,
                                  const float* scales, const float* viewmats, const float* Ks,
                                  int width, int height, const int32_t* radii,
                                  const float* ray_transforms, const float* v_means2d,
                                  const float* v_depths, const float* v_ray_transforms,
                                  const float* v_normals, float* v_means, float* v_quats,
                                  float* v_scales, const float* v_scales_in, hgsr_stream_t stream) {
    int st = check_common(C, N, means, quats, scales, viewmats, Ks, width, height);
    if (st) return st;
    HGSR_REQUIRE(N == 0 || (radii && ray_transforms && v_means2d && v_depths && v_ray_transforms && v_normals &&
                            v_means && v_quats && v_scales),
                 "null pointer");
    if (N == 0) return HGSR_OK;
    KernelTimer kt("project2d_bwd", as_stream(stream));
    hipLaunchKernelGGL(project2d_bwd_kernel, dim3((N + 255) / 256), dim3(256), 0, as_stream(stream), C, N,
                       means, reinterpret_cast<const float4*>(quats), scales, viewmats, Ks, radii,
                       ray_transforms, reinterpret_cast<const float2*>(v_means2d), v_depths,
                       v_ray_transforms, v_normals, v_means, reinterpret_cast<float4*>(v_quats), v_scales,
                       v_scales_in);
    return check_launch("project2d_bwd");
}

extern "C" int hgsr_anchor_prefilter(int A, const float* anchor, const float* quats, const float* scales,
                                     int scale_stride, const float* viewmat, const float* K, int width, int height,
                                     float eps2d, float near_plane, float far_plane, const int32_t* level,
                                     const float* extra_level, const float* cam_center, float res_scale,
                                     float standard_dist, float log2_fork, int max_level, uint8_t* visible,
                                     hgsr_stream_t stream) {
    HGSR_REQUIRE(A >= 0 && width > 0 && height > 0 && scale_stride >= 3, "bad dims");
    if (A == 0) return HGSR_OK;
    HGSR_REQUIRE(anchor && quats && scales && viewmat && K && visible, "null pointer");
    HGSR_REQUIRE(!level || (extra_level && cam_center && max_level >= 0), "LoD inputs incomplete");
    KernelTimer kt("anchor_prefilter", as_stream(stream));
    hipLaunchKernelGGL(anchor_prefilter_kernel, dim3((A + 255) / 256), dim3(256), 0, as_stream(stream), A, anchor,
                       reinterpret_cast<const float4*>(quats), scales, scale_stride, viewmat, K, width, height, eps2d,
                       near_plane, far_plane, level, extra_level, cam_center, res_scale, standard_dist, log2_fork,
                       max_level, visible);
    return check_launch("anchor_prefilter");
}
