// K8/K9: 3DGS tile rasterization, forward and backward (gsplat
// rasterize_to_pixels semantics, as reached from reference
// gaussian_renderer/render.py:40-54).
//
// CDNA4 mapping: one 256-lane workgroup per 16x16 tile = four wave64s, each
// wave owning an 8x8 quadrant (compact footprint -> more wave-uniform skips in
// the backward).  Gaussian records of the tile's depth-sorted list are staged in
// LDS in batches and read back as broadcasts; the forward early-outs per tile
// with a workgroup vote.  The backward replays back-to-front from each pixel's
// last contributor, skips Gaussians no lane of the wave sees (wave ballot),
// reduces each Gaussian's gradient across the wave with DPP row ops, combines
// the four waves through LDS and issues ONE packed record of atomics per
// (Gaussian, tile) into a 64-byte-aligned accumulator row (one memory request).
// Work is bounded by the latest last_id in the tile (block-level skip of the
// never-reached tail).
#include "common.h"

namespace hgsr {

constexpr int kFwdBatch = 256;
constexpr int kBwdBatch = 64;
constexpr int kRec3 = 16;  // floats per accumulator row: xy(2) conic(3) opac(1) color(D<=4) absxy(2)

struct TileCtx {
    int cam, tile, i, j;
    bool inside;
    float px, py;
    int32_t start, end;
    int64_t pix;
};

__device__ __forceinline__ TileCtx tile_ctx(int C, int W, int H, int tw, int th,
                                            const int32_t* __restrict__ offsets, int64_t n_isects) {
    TileCtx t;
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

template <int D>
__global__ __launch_bounds__(256) void raster3d_fwd_kernel(
    int C, int W, int H, int tw, int th, const float2* __restrict__ means2d,
    const float* __restrict__ conics, const float* __restrict__ colors,
    const float* __restrict__ opacities, const float* __restrict__ backgrounds,
    const int32_t* __restrict__ offsets, int64_t n_isects, const int32_t* __restrict__ flatten_ids,
    float* __restrict__ render_colors, float* __restrict__ render_alphas, int32_t* __restrict__ last_ids) {
    __shared__ float2 s_xy[kFwdBatch];
    __shared__ float4 s_co[kFwdBatch];  // conic a, b, c, opacity
    __shared__ float s_col[kFwdBatch * D];
    const TileCtx tc = tile_ctx(C, W, H, tw, th, offsets, n_isects);
    const int tid = threadIdx.x;
    float T = 1.0f;
    float acc[D];
#pragma unroll
    for (int k = 0; k < D; ++k) acc[k] = 0.f;
    int32_t cur = 0;
    bool done = !tc.inside;
    const int nb = (tc.end - tc.start + kFwdBatch - 1) / kFwdBatch;
    for (int b = 0; b < nb; ++b) {
        if (__syncthreads_count(done) == 256) break;
        const int32_t bs = tc.start + b * kFwdBatch;
        const int32_t idx = bs + tid;
        if (idx < tc.end) {
            const int32_t g = flatten_ids[idx];
            s_xy[tid] = means2d[g];
            s_co[tid] = make_float4(conics[(int64_t)g * 3], conics[(int64_t)g * 3 + 1], conics[(int64_t)g * 3 + 2],
                                    opacities[g]);
#pragma unroll
            for (int k = 0; k < D; ++k) s_col[tid * D + k] = colors[(int64_t)g * D + k];
        }
        __syncthreads();
        const int cnt = min(kFwdBatch, tc.end - bs);
        for (int t = 0; t < cnt && !done; ++t) {
            const float2 xy = s_xy[t];
            const float4 co = s_co[t];
            const float dx = xy.x - tc.px, dy = xy.y - tc.py;
            const float sigma = 0.5f * (co.x * dx * dx + co.z * dy * dy) + co.y * dx * dy;
            const float alpha = fminf(0.999f, co.w * __expf(-sigma));
            if (sigma < 0.f || alpha < 1.0f / 255.0f) continue;
            const float nT = T * (1.0f - alpha);
            if (nT <= 1e-4f) {
                done = true;
                break;
            }
            const float vis = alpha * T;
#pragma unroll
            for (int k = 0; k < D; ++k) acc[k] += s_col[t * D + k] * vis;
            cur = bs + t;
            T = nT;
        }
    }
    if (tc.inside) {
        render_alphas[tc.pix] = 1.0f - T;
#pragma unroll
        for (int k = 0; k < D; ++k)
            render_colors[tc.pix * D + k] = backgrounds ? acc[k] + T * backgrounds[tc.cam * D + k] : acc[k];
        last_ids[tc.pix] = cur;
    }
}

__device__ __forceinline__ int32_t wave_max_i32(int32_t v) {
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) v = max(v, __shfl_xor(v, d));
    return v;
}

template <int D, bool ABS>
__global__ __launch_bounds__(256) void raster3d_bwd_kernel(
    int C, int W, int H, int tw, int th, const float2* __restrict__ means2d,
    const float* __restrict__ conics, const float* __restrict__ colors,
    const float* __restrict__ opacities, const float* __restrict__ backgrounds,
    const int32_t* __restrict__ offsets, int64_t n_isects, const int32_t* __restrict__ flatten_ids,
    const float* __restrict__ render_alphas, const int32_t* __restrict__ last_ids,
    const float* __restrict__ v_render_colors, const float* __restrict__ v_render_alphas,
    float* __restrict__ acc_rows) {
    constexpr int KV = 6 + D + (ABS ? 2 : 0);
    __shared__ float2 s_xy[kBwdBatch];
    __shared__ float4 s_co[kBwdBatch];
    __shared__ float s_col[kBwdBatch * D];
    __shared__ int32_t s_id[kBwdBatch];
    __shared__ float s_part[kBwdBatch * 4 * KV];
    __shared__ int32_t s_last[4];
    const TileCtx tc = tile_ctx(C, W, H, tw, th, offsets, n_isects);
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const float T_final = tc.inside ? 1.0f - render_alphas[tc.pix] : 1.0f;
    float T = T_final;
    float buf[D], vo[D];
    float bg_dot = 0.f;
#pragma unroll
    for (int k = 0; k < D; ++k) {
        buf[k] = 0.f;
        vo[k] = tc.inside ? v_render_colors[tc.pix * D + k] : 0.f;
        if (backgrounds) bg_dot += backgrounds[tc.cam * D + k] * vo[k];
    }
    const float va = tc.inside ? v_render_alphas[tc.pix] : 0.f;
    const int32_t bin_final = tc.inside ? last_ids[tc.pix] : 0;
    const int32_t wave_final = wave_max_i32(tc.inside ? bin_final : -1);
    if (lane == 0) s_last[wave] = wave_final;
    __syncthreads();
    const int32_t blk_final = max(max(s_last[0], s_last[1]), max(s_last[2], s_last[3]));
    // Gaussians after the block's last contributor are never reached
    const int32_t end = min(tc.end, blk_final + 1);
    const int nb = end > tc.start ? (end - tc.start + kBwdBatch - 1) / kBwdBatch : 0;
    for (int b = 0; b < nb; ++b) {
        const int32_t batch_end = end - 1 - b * kBwdBatch;
        const int bsz = min(kBwdBatch, batch_end + 1 - tc.start);
        __syncthreads();
        if (tid < bsz) {
            const int32_t g = flatten_ids[batch_end - tid];
            s_id[tid] = g;
            s_xy[tid] = means2d[g];
            s_co[tid] = make_float4(conics[(int64_t)g * 3], conics[(int64_t)g * 3 + 1], conics[(int64_t)g * 3 + 2],
                                    opacities[g]);
#pragma unroll
            for (int k = 0; k < D; ++k) s_col[tid * D + k] = colors[(int64_t)g * D + k];
        }
        for (int e = tid; e < kBwdBatch * 4 * KV; e += 256) s_part[e] = 0.f;
        __syncthreads();
        const int t0 = max(0, batch_end - wave_final);
        for (int t = t0; t < bsz; ++t) {
            bool valid = tc.inside && (batch_end - t <= bin_final);
            const float2 xy = s_xy[t];
            const float4 co = s_co[t];
            const float dx = xy.x - tc.px, dy = xy.y - tc.py;
            const float sigma = 0.5f * (co.x * dx * dx + co.z * dy * dy) + co.y * dx * dy;
            const float vis = __expf(-sigma);
            const float alpha = fminf(0.999f, co.w * vis);
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
                    const float ck = s_col[t * D + k];
                    gv[6 + k] = fac * vo[k];
                    v_alpha += (ck * T - buf[k] * ra) * vo[k];
                    buf[k] += ck * fac;
                }
                v_alpha += T_final * ra * va;
                v_alpha += -T_final * ra * bg_dot;
                if (co.w * vis <= 0.999f) {
                    const float v_sigma = -co.w * vis * v_alpha;
                    gv[0] = v_sigma * (co.x * dx + co.y * dy);
                    gv[1] = v_sigma * (co.y * dx + co.z * dy);
                    gv[2] = 0.5f * v_sigma * dx * dx;
                    gv[3] = v_sigma * dx * dy;
                    gv[4] = 0.5f * v_sigma * dy * dy;
                    gv[5] = vis * v_alpha;
                    if (ABS) {
                        gv[6 + D] = fabsf(gv[0]);
                        gv[7 + D] = fabsf(gv[1]);
                    }
                }
            }
            float* dst = s_part + (t * 4 + wave) * KV;
#pragma unroll
            for (int k = 0; k < KV; ++k) {
                const float s = wave_sum_to_lane63(gv[k]);
                if (lane == 63) dst[k] = s;
            }
        }
        __syncthreads();
        for (int e = tid; e < bsz * KV; e += 256) {
            const int t = e / KV, k = e - t * KV;
            const float* p = s_part + t * 4 * KV + k;
            const float s = p[0] + p[KV] + p[2 * KV] + p[3 * KV];
            if (s != 0.f) atomicAdd(acc_rows + (int64_t)s_id[t] * kRec3 + k, s);
        }
    }
}

// scatter accumulator rows into gsplat's separate gradient tensors (+=)
template <int D, bool ABS>
__global__ __launch_bounds__(256) void split3_kernel(int64_t n, const float* __restrict__ rows,
                                                     float2* __restrict__ v_means2d, float* __restrict__ v_conics,
                                                     float* __restrict__ v_colors, float* __restrict__ v_opacities,
                                                     float2* __restrict__ v_abs) {
    const int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (g >= n) return;
    const float4* r4 = reinterpret_cast<const float4*>(rows + g * kRec3);
    float r[kRec3];
#pragma unroll
    for (int q = 0; q < kRec3 / 4; ++q) {
        const float4 v = r4[q];
        r[q * 4] = v.x; r[q * 4 + 1] = v.y; r[q * 4 + 2] = v.z; r[q * 4 + 3] = v.w;
    }
    float2 m = v_means2d[g];
    m.x += r[0]; m.y += r[1];
    v_means2d[g] = m;
    v_conics[g * 3] += r[2];
    v_conics[g * 3 + 1] += r[3];
    v_conics[g * 3 + 2] += r[4];
    v_opacities[g] += r[5];
#pragma unroll
    for (int k = 0; k < D; ++k) v_colors[g * D + k] += r[6 + k];
    if (ABS) {
        float2 a = v_abs[g];
        a.x += r[6 + D]; a.y += r[7 + D];
        v_abs[g] = a;
    }
}

}  // namespace hgsr

using namespace hgsr;

static int check_raster(int C, int N, int D, int W, int H, int tile_size, int tw, int th) {
    HGSR_REQUIRE(C >= 1 && N >= 0 && W > 0 && H > 0, "bad dims");
    HGSR_REQUIRE(D >= 1 && D <= 4, "channels per call must be 1..4 (got %d); chunk wider colours", D);
    HGSR_REQUIRE(tile_size == kTile, "tile_size must be %d (got %d)", kTile, tile_size);
    HGSR_REQUIRE(tw == (W + kTile - 1) / kTile && th == (H + kTile - 1) / kTile, "tile grid mismatch");
    HGSR_REQUIRE((int64_t)C * tw * th < (1ll << 31), "too many tiles");
    return HGSR_OK;
}

extern "C" int hgsr_raster3d_fwd(int C, int N, int D, const float* means2d, const float* conics,
                                 const float* colors, const float* opacities, const float* backgrounds,
                                 int width, int height, int tile_size, int tile_w, int tile_h,
                                 const int32_t* isect_offsets, int64_t n_isects, const int32_t* flatten_ids,
                                 float* render_colors, float* render_alphas, int32_t* last_ids,
                                 hgsr_stream_t stream) {
    if (int st = check_raster(C, N, D, width, height, tile_size, tile_w, tile_h)) return st;
    HGSR_REQUIRE(isect_offsets && render_colors && render_alphas && last_ids, "null pointer");
    HGSR_REQUIRE(n_isects == 0 || (means2d && conics && colors && opacities && flatten_ids), "null pointer");
    const dim3 grid(C * tile_w * tile_h);
    hipStream_t s = as_stream(stream);
    const float2* m2 = reinterpret_cast<const float2*>(means2d);
    KernelTimer kt("raster3d_fwd", s);
#define LAUNCH_F(DD)                                                                                      \
    hipLaunchKernelGGL(raster3d_fwd_kernel<DD>, grid, dim3(256), 0, s, C, width, height, tile_w, tile_h, m2, \
                       conics, colors, opacities, backgrounds, isect_offsets, n_isects, flatten_ids,        \
                       render_colors, render_alphas, last_ids)
    switch (D) {
        case 1: LAUNCH_F(1); break;
        case 2: LAUNCH_F(2); break;
        case 3: LAUNCH_F(3); break;
        default: LAUNCH_F(4); break;
    }
#undef LAUNCH_F
    return check_launch("raster3d_fwd");
}

extern "C" size_t hgsr_raster3d_bwd_ws_bytes(int C, int N, int D) {
    (void)D;
    return (size_t)C * N * kRec3 * sizeof(float);
}

extern "C" int hgsr_raster3d_bwd(int C, int N, int D, const float* means2d, const float* conics,
                                 const float* colors, const float* opacities, const float* backgrounds,
                                 int width, int height, int tile_size, int tile_w, int tile_h,
                                 const int32_t* isect_offsets, int64_t n_isects, const int32_t* flatten_ids,
                                 const float* render_alphas, const int32_t* last_ids,
                                 const float* v_render_colors, const float* v_render_alphas, float* v_means2d,
                                 float* v_conics, float* v_colors, float* v_opacities, float* v_means2d_abs,
                                 void* ws, size_t ws_bytes, hgsr_stream_t stream) {
    if (int st = check_raster(C, N, D, width, height, tile_size, tile_w, tile_h)) return st;
    HGSR_REQUIRE(ws_bytes >= hgsr_raster3d_bwd_ws_bytes(C, N, D), "raster3d_bwd workspace too small");
    if (n_isects == 0 || N == 0) return HGSR_OK;
    HGSR_REQUIRE(means2d && conics && colors && opacities && isect_offsets && flatten_ids && render_alphas &&
                     last_ids && v_render_colors && v_render_alphas && v_means2d && v_conics && v_colors &&
                     v_opacities && ws,
                 "null pointer");
    hipStream_t s = as_stream(stream);
    float* rows = (float*)ws;
    if (int st = memset_async(rows, hgsr_raster3d_bwd_ws_bytes(C, N, D), s, "raster3d_bwd")) return st;
    const dim3 grid(C * tile_w * tile_h);
    const float2* m2 = reinterpret_cast<const float2*>(means2d);
    const bool abs = v_means2d_abs != nullptr;
#define LAUNCH_B(DD, AA)                                                                                     \
    {                                                                                                        \
        KernelTimer kt("raster3d_bwd", s);                                                                   \
        hipLaunchKernelGGL((raster3d_bwd_kernel<DD, AA>), grid, dim3(256), 0, s, C, width, height, tile_w, tile_h, \
                       m2, conics, colors, opacities, backgrounds, isect_offsets, n_isects, flatten_ids,       \
                       render_alphas, last_ids, v_render_colors, v_render_alphas, rows);                       \
    }                                                                                                        \
    hipLaunchKernelGGL((split3_kernel<DD, AA>), dim3((unsigned)(((int64_t)C * N + 255) / 256)), dim3(256), 0, s, \
                       (int64_t)C * N, rows, reinterpret_cast<float2*>(v_means2d), v_conics, v_colors,         \
                       v_opacities, reinterpret_cast<float2*>(v_means2d_abs))
    switch (D * 2 + (abs ? 1 : 0)) {
        case 2: LAUNCH_B(1, false); break;
        case 3: LAUNCH_B(1, true); break;
        case 4: LAUNCH_B(2, false); break;
        case 5: LAUNCH_B(2, true); break;
        case 6: LAUNCH_B(3, false); break;
        case 7: LAUNCH_B(3, true); break;
        case 8: LAUNCH_B(4, false); break;
        default: LAUNCH_B(4, true); break;
    }
#undef LAUNCH_B
    return check_launch("raster3d_bwd");
}
