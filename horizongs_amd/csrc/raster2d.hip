// K11/K12: 2DGS surfel tile rasterization, forward and backward (gsplat
// rasterize_to_pixels_2dgs semantics, reached from reference
// gaussian_renderer/render.py:62-76).  Same CDNA4 structure as raster3d.hip:
// a 256-lane workgroup per 16x16 tile (four 8x8 wave quadrants), LDS-staged
// surfel batches, workgroup early-out vote, wave-ballot skips and one packed
// atomic record per (surfel, tile) in the backward.
//
// Per pair: h_u = px*w - u, h_v = py*w - v (rows u,v,w of the ray transform),
// x = h_u x h_v, s = x.xy / x.z, G = min(|s|^2, 2|mean2d - p|^2), alpha =
// min(0.999, o*exp(-G/2)).  The last colour channel is the depth (RGB+ED).
#include "common.h"

namespace hgsr {

constexpr int kFwd2Batch = 128;
constexpr int kBwd2Batch = 32;
constexpr int kRec2 = 32;  // xy(2) rt(9) opac(1) normal(3) densify(2) color(D<=4) absxy(2)

struct Tile2 {
    int cam, tile, i, j;
    bool inside;
    float px, py;
    int32_t start, end;
    int64_t pix;
};

__device__ __forceinline__ Tile2 tile2_ctx(int C, int W, int H, int tw, int th,
                                           const int32_t* __restrict__ offsets, int64_t n_isects) {
    Tile2 t;
    const int n_tiles = tw * th;
    const int bid = xcd_remap(blockIdx.x, gridDim.x);
    t.cam = bid / n_tiles;
    t.tile = bid - t.cam * n_tiles;
    const int ty = t.tile / tw, tx = t.tile - ty * tw;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    t.i = ty * kTile + (wave >> 1) * 8 + (lane >> 3);
    t.j = tx * kTile + (wave & 1) * 8 + (lane & 7);
    t.inside = t.i < H && t.j < W;
    t.px = (float)t.j + 0.5f;
    t.py = (float)t.i + 0.5f;
    const int64_t bin = (int64_t)t.cam * n_tiles + t.tile;
    t.start = offsets[bin];
    t.end = (bin == (int64_t)C * n_tiles - 1) ? (int32_t)n_isects : offsets[bin + 1];
    t.pix = ((int64_t)t.cam * H + t.i) * W + t.j;
    return t;
}

struct SurfelRec {
    float u[3], v[3], w[3];
    float mx, my, opac;
};

__device__ __forceinline__ void stage_surfel(float* s, int64_t g, const float2* __restrict__ means2d,
                                             const float* __restrict__ rt, const float* __restrict__ opac) {
    const float* M = rt + g * 9;
#pragma unroll
    for (int k = 0; k < 9; ++k) s[k] = M[k];
    const float2 m = means2d[g];
    s[9] = m.x;
    s[10] = m.y;
    s[11] = opac[g];
}

template <int D>
__global__ __launch_bounds__(256) void raster2d_fwd_kernel(
    int C, int W, int H, int tw, int th, const float2* __restrict__ means2d, const float* __restrict__ rt,
    const float* __restrict__ colors, const float* __restrict__ opacities, const float* __restrict__ normals,
    const float* __restrict__ backgrounds, const int32_t* __restrict__ offsets, int64_t n_isects,
    const int32_t* __restrict__ flatten_ids, float* __restrict__ render_colors, float* __restrict__ render_alphas,
    float* __restrict__ render_normals, float* __restrict__ render_distort, float* __restrict__ render_median,
    int32_t* __restrict__ last_ids, int32_t* __restrict__ median_ids) {
    constexpr int S = 12 + D + 3;  // floats staged per surfel
    __shared__ float s_rec[kFwd2Batch * S];
    const Tile2 tc = tile2_ctx(C, W, H, tw, th, offsets, n_isects);
    const int tid = threadIdx.x;
    float T = 1.0f, distort = 0.f, acc_vd = 0.f, median = 0.f;
    float acc[D], nacc[3] = {0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < D; ++k) acc[k] = 0.f;
    int32_t cur = 0, med_idx = 0;
    bool done = !tc.inside;
    const int nb = (tc.end - tc.start + kFwd2Batch - 1) / kFwd2Batch;
    for (int b = 0; b < nb; ++b) {
        if (__syncthreads_count(done) == 256) break;
        const int32_t bs = tc.start + b * kFwd2Batch;
        if (tid < kFwd2Batch && bs + tid < tc.end) {
            const int32_t g = flatten_ids[bs + tid];
            float* s = s_rec + tid * S;
            stage_surfel(s, g, means2d, rt, opacities);
#pragma unroll
            for (int k = 0; k < D; ++k) s[12 + k] = colors[(int64_t)g * D + k];
#pragma unroll
            for (int k = 0; k < 3; ++k) s[12 + D + k] = normals[(int64_t)g * 3 + k];
        }
        __syncthreads();
        const int cnt = min(kFwd2Batch, tc.end - bs);
        for (int t = 0; t < cnt && !done; ++t) {
            const float* s = s_rec + t * S;
            const float hu0 = tc.px * s[6] - s[0], hu1 = tc.px * s[7] - s[1], hu2 = tc.px * s[8] - s[2];
            const float hv0 = tc.py * s[6] - s[3], hv1 = tc.py * s[7] - s[4], hv2 = tc.py * s[8] - s[5];
            const float cx = hu1 * hv2 - hu2 * hv1;
            const float cy = hu2 * hv0 - hu0 * hv2;
            const float cz = hu0 * hv1 - hu1 * hv0;
            if (cz == 0.f) continue;
            const float sx = cx / cz, sy = cy / cz;
            const float g3 = sx * sx + sy * sy;
            const float dx = s[9] - tc.px, dy = s[10] - tc.py;
            const float g2 = 2.0f * (dx * dx + dy * dy);
            const float sigma = 0.5f * fminf(g3, g2);
            const float alpha = fminf(0.999f, s[11] * __expf(-sigma));
            if (sigma < 0.f || alpha < 1.0f / 255.0f) continue;
            const float nT = T * (1.0f - alpha);
            if (nT <= 1e-4f) {
                done = true;
                break;
            }
            const float vis = alpha * T;
#pragma unroll
            for (int k = 0; k < D; ++k) acc[k] += s[12 + k] * vis;
#pragma unroll
            for (int k = 0; k < 3; ++k) nacc[k] += s[12 + D + k] * vis;
            const float depth = s[12 + D - 1];
            distort += 2.0f * (vis * depth * (1.0f - T) - vis * acc_vd);
            acc_vd += vis * depth;
            if (T > 0.5f) {
                median = depth;
                med_idx = bs + t;
            }
            cur = bs + t;
            T = nT;
        }
    }
    if (tc.inside) {
        render_alphas[tc.pix] = 1.0f - T;
#pragma unroll
        for (int k = 0; k < D; ++k)
            render_colors[tc.pix * D + k] = backgrounds ? acc[k] + T * backgrounds[tc.cam * D + k] : acc[k];
#pragma unroll
        for (int k = 0; k < 3; ++k) render_normals[tc.pix * 3 + k] = nacc[k];
        render_distort[tc.pix] = distort;
        render_median[tc.pix] = median;
        last_ids[tc.pix] = cur;
        median_ids[tc.pix] = med_idx;
    }
}

__device__ __forceinline__ int32_t wave_max2(int32_t v) {
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) v = max(v, __shfl_xor(v, d));
    return v;
}

template <int D, bool ABS>
__global__ __launch_bounds__(256) void raster2d_bwd_kernel(
    int C, int W, int H, int tw, int th, const float2* __restrict__ means2d, const float* __restrict__ rt,
    const float* __restrict__ colors, const float* __restrict__ opacities, const float* __restrict__ normals,
    const float* __restrict__ backgrounds, const int32_t* __restrict__ offsets, int64_t n_isects,
    const int32_t* __restrict__ flatten_ids, const float* __restrict__ render_alphas,
    const int32_t* __restrict__ last_ids, const float* __restrict__ v_render_colors,
    const float* __restrict__ v_render_alphas, const float* __restrict__ v_render_normals,
    float* __restrict__ acc_rows) {
    constexpr int S = 12 + D + 3;
    constexpr int KV = 17 + D + (ABS ? 2 : 0);
    // record layout: 0-1 xy, 2-10 rt, 11 opac, 12-14 normal, 15-16 densify, 17.. color, then abs
    __shared__ float s_rec[kBwd2Batch * S];
    __shared__ int32_t s_id[kBwd2Batch];
    __shared__ float s_part[kBwd2Batch * 4 * KV];
    __shared__ int32_t s_last[4];
    const Tile2 tc = tile2_ctx(C, W, H, tw, th, offsets, n_isects);
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const float T_final = tc.inside ? 1.0f - render_alphas[tc.pix] : 1.0f;
    float T = T_final;
    float buf[D], vo[D], nbuf[3] = {0.f, 0.f, 0.f}, vn[3];
    float bg_dot = 0.f;
#pragma unroll
    for (int k = 0; k < D; ++k) {
        buf[k] = 0.f;
        vo[k] = tc.inside ? v_render_colors[tc.pix * D + k] : 0.f;
        if (backgrounds) bg_dot += backgrounds[tc.cam * D + k] * vo[k];
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) vn[k] = tc.inside ? v_render_normals[tc.pix * 3 + k] : 0.f;
    const float va = tc.inside ? v_render_alphas[tc.pix] : 0.f;
    const int32_t bin_final = tc.inside ? last_ids[tc.pix] : 0;
    const int32_t wave_final = wave_max2(tc.inside ? bin_final : -1);
    if (lane == 0) s_last[wave] = wave_final;
    __syncthreads();
    const int32_t blk_final = max(max(s_last[0], s_last[1]), max(s_last[2], s_last[3]));
    const int32_t end = min(tc.end, blk_final + 1);
    const int nb = end > tc.start ? (end - tc.start + kBwd2Batch - 1) / kBwd2Batch : 0;
    for (int b = 0; b < nb; ++b) {
        const int32_t batch_end = end - 1 - b * kBwd2Batch;
        const int bsz = min(kBwd2Batch, batch_end + 1 - tc.start);
        __syncthreads();
        if (tid < bsz) {
            const int32_t g = flatten_ids[batch_end - tid];
            s_id[tid] = g;
            float* s = s_rec + tid * S;
            stage_surfel(s, g, means2d, rt, opacities);
#pragma unroll
            for (int k = 0; k < D; ++k) s[12 + k] = colors[(int64_t)g * D + k];
#pragma unroll
            for (int k = 0; k < 3; ++k) s[12 + D + k] = normals[(int64_t)g * 3 + k];
        }
        for (int e = tid; e < kBwd2Batch * 4 * KV; e += 256) s_part[e] = 0.f;
        __syncthreads();
        const int t0 = max(0, batch_end - wave_final);
        for (int t = t0; t < bsz; ++t) {
            const float* s = s_rec + t * S;
            bool valid = tc.inside && (batch_end - t <= bin_final);
            const float hu0 = tc.px * s[6] - s[0], hu1 = tc.px * s[7] - s[1], hu2 = tc.px * s[8] - s[2];
            const float hv0 = tc.py * s[6] - s[3], hv1 = tc.py * s[7] - s[4], hv2 = tc.py * s[8] - s[5];
            const float cx = hu1 * hv2 - hu2 * hv1;
            const float cy = hu2 * hv0 - hu0 * hv2;
            const float cz = hu0 * hv1 - hu1 * hv0;
            valid = valid && cz != 0.f;
            const float iz = 1.0f / cz;
            const float sx = cx * iz, sy = cy * iz;
            const float g3 = sx * sx + sy * sy;
            const float dx = s[9] - tc.px, dy = s[10] - tc.py;
            const float g2 = 2.0f * (dx * dx + dy * dy);
            const float sigma = 0.5f * fminf(g3, g2);
            const float vis = __expf(-sigma);
            const float alpha = fminf(0.999f, s[11] * vis);
            valid = valid && !(sigma < 0.f || alpha < 1.0f / 255.0f);
            if (!__any(valid)) continue;
            float gv[KV];
#pragma unroll
            for (int k = 0; k < KV; ++k) gv[k] = 0.f;
            if (valid) {
                const float ra = __builtin_amdgcn_rcpf(1.0f - alpha);
                T = T * ra;
                const float fac = alpha * T;
                float v_alpha = 0.f;
#pragma unroll
                for (int k = 0; k < D; ++k) {
                    const float ck = s[12 + k];
                    gv[17 + k] = fac * vo[k];
                    v_alpha += (ck * T - buf[k] * ra) * vo[k];
                    buf[k] += ck * fac;
                }
#pragma unroll
                for (int k = 0; k < 3; ++k) {
                    const float nk = s[12 + D + k];
                    gv[12 + k] = fac * vn[k];
                    v_alpha += (nk * T - nbuf[k] * ra) * vn[k];
                    nbuf[k] += nk * fac;
                }
                v_alpha += T_final * ra * va;
                v_alpha += -T_final * ra * bg_dot;
                if (s[11] * vis <= 0.999f) {
                    const float v_sigma = -s[11] * vis * v_alpha;
                    float vu[3] = {0.f, 0.f, 0.f}, vv[3] = {0.f, 0.f, 0.f}, vw[3] = {0.f, 0.f, 0.f};
                    float vx = 0.f, vy = 0.f;
                    if (g3 <= g2) {
                        const float vs0 = v_sigma * sx, vs1 = v_sigma * sy;
                        const float vc0 = vs0 * iz, vc1 = vs1 * iz, vc2 = -(vs0 * sx + vs1 * sy) * iz;
                        // v_hu = hv x vc ; v_hv = vc x hu
                        const float vhu0 = hv1 * vc2 - hv2 * vc1, vhu1 = hv2 * vc0 - hv0 * vc2, vhu2 = hv0 * vc1 - hv1 * vc0;
                        const float vhv0 = vc1 * hu2 - vc2 * hu1, vhv1 = vc2 * hu0 - vc0 * hu2, vhv2 = vc0 * hu1 - vc1 * hu0;
                        vu[0] = -vhu0; vu[1] = -vhu1; vu[2] = -vhu2;
                        vv[0] = -vhv0; vv[1] = -vhv1; vv[2] = -vhv2;
                        vw[0] = tc.px * vhu0 + tc.py * vhv0;
                        vw[1] = tc.px * vhu1 + tc.py * vhv1;
                        vw[2] = tc.px * vhu2 + tc.py * vhv2;
                    } else {
                        vx = 2.0f * v_sigma * dx;
                        vy = 2.0f * v_sigma * dy;
                    }
                    gv[0] = vx;
                    gv[1] = vy;
#pragma unroll
                    for (int k = 0; k < 3; ++k) {
                        gv[2 + k] = vu[k];
                        gv[5 + k] = vv[k];
                        gv[8 + k] = vw[k];
                    }
                    gv[11] = vis * v_alpha;
                    gv[15] = vu[0] * s[6] + vu[1] * s[7] + vu[2] * s[8] + vx;
                    gv[16] = vv[0] * s[6] + vv[1] * s[7] + vv[2] * s[8] + vy;
                    if (ABS) {
                        gv[17 + D] = fabsf(vx);
                        gv[18 + D] = fabsf(vy);
                    }
                }
            }
            float* dst = s_part + (t * 4 + wave) * KV;
#pragma unroll
            for (int k = 0; k < KV; ++k) {
                const float sm = wave_sum_to_lane63(gv[k]);
                if (lane == 63) dst[k] = sm;
            }
        }
        __syncthreads();
        for (int e = tid; e < bsz * KV; e += 256) {
            const int t = e / KV, k = e - t * KV;
            const float* p = s_part + t * 4 * KV + k;
            const float sm = p[0] + p[KV] + p[2 * KV] + p[3 * KV];
            if (sm != 0.f) atomicAdd(acc_rows + (int64_t)s_id[t] * kRec2 + k, sm);
        }
    }
}

template <int D, bool ABS>
__global__ __launch_bounds__(256) void split2_kernel(int64_t n, const float* __restrict__ rows,
                                                     float2* __restrict__ v_means2d, float* __restrict__ v_rt,
                                                     float* __restrict__ v_colors, float* __restrict__ v_opacities,
                                                     float* __restrict__ v_normals, float2* __restrict__ v_densify,
                                                     float2* __restrict__ v_abs) {
    const int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (g >= n) return;
    const float* r = rows + g * kRec2;
    float2 m = v_means2d[g];
    m.x += r[0]; m.y += r[1];
    v_means2d[g] = m;
#pragma unroll
    for (int k = 0; k < 9; ++k) v_rt[g * 9 + k] += r[2 + k];
    v_opacities[g] += r[11];
#pragma unroll
    for (int k = 0; k < 3; ++k) v_normals[g * 3 + k] += r[12 + k];
    if (v_densify) {
        float2 d = v_densify[g];
        d.x += r[15]; d.y += r[16];
        v_densify[g] = d;
    }
#pragma unroll
    for (int k = 0; k < D; ++k) v_colors[g * D + k] += r[17 + k];
    if (ABS) {
        float2 a = v_abs[g];
        a.x += r[17 + D]; a.y += r[18 + D];
        v_abs[g] = a;
    }
}

}  // namespace hgsr

using namespace hgsr;

static int check_raster2(int C, int N, int D, int W, int H, int tile_size, int tw, int th) {
    HGSR_REQUIRE(C >= 1 && N >= 0 && W > 0 && H > 0, "bad dims");
    HGSR_REQUIRE(D >= 1 && D <= 4, "channels per call must be 1..4 (got %d)", D);
    HGSR_REQUIRE(tile_size == kTile, "tile_size must be %d (got %d)", kTile, tile_size);
    HGSR_REQUIRE(tw == (W + kTile - 1) / kTile && th == (H + kTile - 1) / kTile, "tile grid mismatch");
    return HGSR_OK;
}

extern "C" int hgsr_raster2d_fwd(int C, int N, int D, const float* means2d, const float* ray_transforms,
                                 const float* colors, const float* opacities, const float* normals,
                                 const float* backgrounds, int width, int height, int tile_size, int tile_w,
                                 int tile_h, const int32_t* isect_offsets, int64_t n_isects,
                                 const int32_t* flatten_ids, float* render_colors, float* render_alphas,
                                 float* render_normals, float* render_distort, float* render_median,
                                 int32_t* last_ids, int32_t* median_ids, hgsr_stream_t stream) {
    if (int st = check_raster2(C, N, D, width, height, tile_size, tile_w, tile_h)) return st;
    HGSR_REQUIRE(isect_offsets && render_colors && render_alphas && render_normals && render_distort &&
                     render_median && last_ids && median_ids,
                 "null pointer");
    HGSR_REQUIRE(n_isects == 0 || (means2d && ray_transforms && colors && opacities && normals && flatten_ids),
                 "null pointer");
    const dim3 grid(C * tile_w * tile_h);
    hipStream_t s = as_stream(stream);
    const float2* m2 = reinterpret_cast<const float2*>(means2d);
    KernelTimer kt("raster2d_fwd", s);
#define LAUNCH_F2(DD)                                                                                           \
    hipLaunchKernelGGL(raster2d_fwd_kernel<DD>, grid, dim3(256), 0, s, C, width, height, tile_w, tile_h, m2,     \
                       ray_transforms, colors, opacities, normals, backgrounds, isect_offsets, n_isects,         \
                       flatten_ids, render_colors, render_alphas, render_normals, render_distort, render_median, \
                       last_ids, median_ids)
    switch (D) {
        case 1: LAUNCH_F2(1); break;
        case 2: LAUNCH_F2(2); break;
        case 3: LAUNCH_F2(3); break;
        default: LAUNCH_F2(4); break;
    }
#undef LAUNCH_F2
    return check_launch("raster2d_fwd");
}

extern "C" size_t hgsr_raster2d_bwd_ws_bytes(int C, int N, int D) {
    (void)D;
    return (size_t)C * N * kRec2 * sizeof(float);
}

extern "C" int hgsr_raster2d_bwd(int C, int N, int D, const float* means2d, const float* ray_transforms,
                                 const float* colors, const float* opacities, const float* normals,
                                 const float* backgrounds, int width, int height, int tile_size, int tile_w,
                                 int tile_h, const int32_t* isect_offsets, int64_t n_isects,
                                 const int32_t* flatten_ids, const float* render_alphas, const int32_t* last_ids,
                                 const float* v_render_colors, const float* v_render_alphas,
                                 const float* v_render_normals, float* v_means2d, float* v_ray_transforms,
                                 float* v_colors, float* v_opacities, float* v_normals, float* v_densify,
                                 void* ws, size_t ws_bytes, hgsr_stream_t stream) {
    if (int st = check_raster2(C, N, D, width, height, tile_size, tile_w, tile_h)) return st;
    HGSR_REQUIRE(ws_bytes >= hgsr_raster2d_bwd_ws_bytes(C, N, D), "raster2d_bwd workspace too small");
    if (n_isects == 0 || N == 0) return HGSR_OK;
    HGSR_REQUIRE(means2d && ray_transforms && colors && opacities && normals && isect_offsets && flatten_ids &&
                     render_alphas && last_ids && v_render_colors && v_render_alphas && v_render_normals &&
                     v_means2d && v_ray_transforms && v_colors && v_opacities && v_normals && ws,
                 "null pointer");
    hipStream_t s = as_stream(stream);
    float* rows = (float*)ws;
    if (int st = memset_async(rows, hgsr_raster2d_bwd_ws_bytes(C, N, D), s, "raster2d_bwd")) return st;
    const dim3 grid(C * tile_w * tile_h);
    const float2* m2 = reinterpret_cast<const float2*>(means2d);
#define LAUNCH_B2(DD)                                                                                            \
    {                                                                                                            \
        KernelTimer kt("raster2d_bwd", s);                                                                       \
        hipLaunchKernelGGL((raster2d_bwd_kernel<DD, false>), grid, dim3(256), 0, s, C, width, height, tile_w, tile_h, \
                       m2, ray_transforms, colors, opacities, normals, backgrounds, isect_offsets, n_isects,       \
                       flatten_ids, render_alphas, last_ids, v_render_colors, v_render_alphas, v_render_normals,  \
                       rows);                                                                                    \
    }                                                                                                            \
    hipLaunchKernelGGL((split2_kernel<DD, false>), dim3((unsigned)(((int64_t)C * N + 255) / 256)), dim3(256), 0, \
                       s, (int64_t)C * N, rows, reinterpret_cast<float2*>(v_means2d), v_ray_transforms, v_colors, \
                       v_opacities, v_normals, reinterpret_cast<float2*>(v_densify), nullptr)
    switch (D) {
        case 1: LAUNCH_B2(1); break;
        case 2: LAUNCH_B2(2); break;
        case 3: LAUNCH_B2(3); break;
        default: LAUNCH_B2(4); break;
    }
#undef LAUNCH_B2
    return check_launch("raster2d_bwd");
}
