// K11/K12: 2DGS surfel tile rasterization, forward and backward (gsplat
// rasterize_to_pixels_2dgs semantics, reached from reference
// gaussian_renderer/render.py:62-76).  Same CDNA4 structure as raster3d.hip:
// a 256-lane workgroup per 16x16 tile (four 8x8 wave quadrants), LDS-staged
// surfel batches, workgroup early-out vote, wave-ballot skips and, in the
// backward, each wave's partial of a (tile, surfel) pair stored as one 80-B row of
// the pair's gradient slot (plain stores; split2 sums a surfel's slots in a fixed
// order: bit-reproducible).
//
// Per pair: h_u = px*w - u, h_v = py*w - v (rows u,v,w of the ray transform),
// x = h_u x h_v, s = x.xy / x.z, G = min(|s|^2, 2|mean2d - p|^2), alpha =
// min(0.999, o*exp(-G/2)).  The last colour channel is the depth (RGB+ED).
#include "common.h"

namespace hgsr {

#ifndef HGSR_FWD2_BATCH
#define HGSR_FWD2_BATCH 64
#endif
// records per forward batch (a multiple of 64): 64 -> 64 VGPRs, 12.6 KB of LDS, 8 waves / SIMD;
// raster2d_fwd 0.682 -> 0.633 ms at c3 against 128 (25 KB, 6 waves)
constexpr int kFwd2Batch = HGSR_FWD2_BATCH;
constexpr int kBwd2Batch = 64;
// floats per gradient-slot row (80 B, 16-B aligned): accumulator value idx at idx -- v_xy 0-1,
// (p - m)x v_c 2-4, (p - m)y v_c 5-7, v_c 8-10, opacity 11, normal 12-14, colour 15 + k (19 used
// at D = 4; a row is written only where koff says, the reader takes the first 15 + D)
constexpr int kRow2 = 20;

struct Tile2 {
    int cam, tile, i, j;
    bool inside;
    float px, py;
    int32_t start, end;
    int64_t pix;
};

// info (nullable): a deferred count's device-resident {n_isects, largest bin, overflow}, as
// in raster3d.hip tile_ctx
__device__ __forceinline__ Tile2 tile2_ctx(int C, int W, int H, int tw, int th,
                                           const int32_t* __restrict__ offsets, int64_t n_isects,
                                           const int64_t* __restrict__ info, const int32_t* __restrict__ order) {
    Tile2 t;
    const int n_tiles = tw * th;
    const int bid = raster_bin(order);
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
    const int64_t n = info ? info[0] : n_isects;
    t.end = (bin == (int64_t)C * n_tiles - 1) ? (int32_t)n : offsets[bin + 1];
    if (info && info[2]) t.end = t.start;
    t.pix = ((int64_t)t.cam * H + t.i) * W + t.j;
    return t;
}

// Raster record of one (camera, surfel).  With rows u, v, w of the ray
// transform, h_u x h_v = (p_x w - u) x (p_y w - v) = p_x A + p_y B + C for
// A = v x w, B = w x u, C = u x v.  Relative to the projected mean m this is
// (p_x - m_x) A + (p_y - m_y) B + C' with C' = C + m_x A + m_y B (the hit at m), so
// the kernels store A, B, C' (from f64) and evaluate the hit with six FMAs on
// small offsets, keeping cancellation out of both passes.
// 128 B: the seventh quad carries the pair's gradient-slot base (as Rec3::sl: written by a
// training forward's pack, read by the backward from the sectors its record DMA fetched); a
// 96-B record touched two 64-B sectors too, so the forward reads no more.
struct Rec2 {
    float4 r0;  // A.x A.y A.z B.x
    float4 r1;  // B.y B.z C'.x C'.y
    float4 r2;  // C'.z mean_x mean_y opacity
    float4 col; // colour (D <= 4, zero padded; the last channel is the depth in RGB+ED)
    float4 r4;  // normal xyz, low-pass disk radius
    float4 box; // centre xy and half-extents of the surfel ellipse's screen bounding box
    int4 sl;    // gradient-slot base, slot width, 0, 0
    float4 pad;
};
static_assert(sizeof(Rec2) == 128, "Rec2 is two 64-B sectors");

// Skip-test geometry.  alpha >= 1/255 needs sigma = min(|s|^2, 2|m-p|^2)/2 <= L =
// ln(255 o), i.e. either the ray-plane hit s lies in the UV disk of radius
// sqrt(2L) or p lies within sqrt(L) of the projected centre.  The disk projects to
// the conic with dual Q* = M diag(R^2, R^2, -1) M^T (M = [u; v; w]); while Q*_22 < 0
// it is an ellipse whose bounding box is centre Q*_i2/Q*_22, half-extent
// sqrt(c_i^2 - Q*_ii/Q*_22).  Near-degenerate views (plane through the camera)
// get an unbounded box.  Evaluated in f64 and padded (1 % + 0.01 px) because the
// kernels use the hardware exp/rcp; it only ever skips pairs with alpha < 1/255.
__device__ __forceinline__ void surfel_footprint(const float* u, const float* v, const float* w, float opac,
                                                 float4& box, float& disk) {
    const float L = __logf(255.0f * opac);
    if (!(L > 0.f)) {
        box = make_float4(0.f, 0.f, -1e30f, -1e30f);
        disk = -1e30f;
        return;
    }
    disk = sqrtf(L) * 1.01f + 0.01f;
    const double R2 = 2.0 * (double)L;
    const double f[3] = {R2, R2, -1.0};
    double q00 = 0, q02 = 0, q11 = 0, q12 = 0, q22 = 0;
    for (int k = 0; k < 3; ++k) {
        q00 += (double)u[k] * u[k] * f[k];
        q02 += (double)u[k] * w[k] * f[k];
        q11 += (double)v[k] * v[k] * f[k];
        q12 += (double)v[k] * w[k] * f[k];
        q22 += (double)w[k] * w[k] * f[k];
    }
    const double w2 = (double)w[2] * w[2];
    if (!(q22 < -1e-3 * w2)) {
        box = make_float4(0.f, 0.f, 1e30f, 1e30f);
        return;
    }
    const double cx = q02 / q22, cy = q12 / q22;
    const double ex2 = cx * cx - q00 / q22, ey2 = cy * cy - q11 / q22;
    const double ex = sqrt(fmax(ex2, 0.0)), ey = sqrt(fmax(ey2, 0.0));
    box = make_float4((float)cx, (float)cy, (float)(ex * 1.01 + 0.01 + 1e-6 * fabs(cx)),
                      (float)(ey * 1.01 + 0.01 + 1e-6 * fabs(cy)));
}

__device__ __forceinline__ void cross3d(const double* a, const double* b, double* c) {
    c[0] = a[1] * b[2] - a[2] * b[1];
    c[1] = a[2] * b[0] - a[0] * b[2];
    c[2] = a[0] * b[1] - a[1] * b[0];
}

// A = v x w, B = w x u, C' = (m_x w - u) x (m_y w - v), in f64, rounded once
__device__ __forceinline__ void cross_abc(const float* M, float mx, float my, float* abc) {
    const double u[3] = {M[0], M[1], M[2]}, v[3] = {M[3], M[4], M[5]}, w[3] = {M[6], M[7], M[8]};
    double A[3], B[3], C[3], hu[3], hv[3];
    for (int k = 0; k < 3; ++k) {
        hu[k] = (double)mx * w[k] - u[k];
        hv[k] = (double)my * w[k] - v[k];
    }
    cross3d(v, w, A);
    cross3d(w, u, B);
    cross3d(hu, hv, C);
    for (int k = 0; k < 3; ++k) {
        abc[k] = (float)A[k];
        abc[3 + k] = (float)B[k];
        abc[6 + k] = (float)C[k];
    }
}

// One workgroup packs 256 consecutive (camera, surfel) records.  The ray transforms (36 B
// each) and normals (12 B) come in as contiguous float4 runs through LDS and the 128-B
// records leave the same way: lane-strided AoS loads / stores made every instruction touch
// ~36 cache lines.  SLOTS: the gradient slots with the records, as pack3_kernel.
template <int D, bool SLOTS>
__global__ __launch_bounds__(256) void pack2_kernel(int64_t n, int N, const float2* __restrict__ means2d,
                                                    const float* __restrict__ rt, ChanSrc cs,
                                                    const float* __restrict__ normals, Rec2* __restrict__ rec,
                                                    RectFromRadii rr, const int32_t* __restrict__ bpre,
                                                    int32_t* __restrict__ seg) {
    constexpr int kOP = 33;  // record pitch in LDS (32 floats + 1: conflict-free lane stride)
    __shared__ __attribute__((aligned(16))) float s_buf[256 * kOP];
    const int64_t i0 = (int64_t)blockIdx.x * 256;
    const int nloc = (int)min((int64_t)256, n - i0);
    const int t = threadIdx.x;
    const int64_t i = i0 + t;
    stage_floats(rt + i0 * 9, nloc * 9, s_buf);
    stage_floats(normals + i0 * 3, nloc * 3, s_buf + 256 * 9);
    int area = 0, inc = 0, x0 = 0, y0 = 0, w = 0;
    __shared__ int s_ws[4];
    if (SLOTS) {
        static_assert(kSlotRow == 256, "one prefix row per workgroup");
        if (t < nloc) area = rr(i, x0, y0, w);
        inc = area;
        const int lane = t & 63;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const int o = __shfl_up(inc, d);
            if (lane >= d) inc += o;
        }
        if (lane == 63) s_ws[t >> 6] = inc;
    }
    __syncthreads();
    int sl_x = 0, sl_w = 0;
    if (SLOTS && t < nloc) {
        int e = bpre[blockIdx.x] + inc - area;
#pragma unroll
        for (int v = 0; v < 4; ++v) e += v < (t >> 6) ? s_ws[v] : 0;
        seg[i] = e;
        sl_x = e - y0 * w - x0;
        sl_w = w;
    }
    float M[9], nr[3];
#pragma unroll
    for (int k = 0; k < 9; ++k) M[k] = s_buf[t * 9 + k];
#pragma unroll
    for (int k = 0; k < 3; ++k) nr[k] = s_buf[256 * 9 + t * 3 + k];
    __syncthreads();  // s_buf now holds the records
    if (t < nloc) {
        const int64_t c = i / N, g = i - c * N;
        const float2 m = means2d[i];
        const float o = cs.opac[c * cs.op_cstride + g];
        float4 box;
        float disk;
        surfel_footprint(M, M + 3, M + 6, o, box, disk);
        float abc[9];
        cross_abc(M, m.x, m.y, abc);
        float col[4] = {0.f, 0.f, 0.f, 0.f};
        const float* src = cs.colors + c * cs.col_cstride + g * cs.dc;
#pragma unroll
        for (int k = 0; k < D; ++k) col[k] = k < cs.dc ? src[k] : cs.depths[i];
        const float r[32] = {abc[0], abc[1], abc[2], abc[3], abc[4], abc[5], abc[6], abc[7],
                             abc[8], m.x,    m.y,    o,      col[0], col[1], col[2], col[3],
                             nr[0],  nr[1],  nr[2],  disk,   box.x,  box.y,  box.z,  box.w,
                             __int_as_float(sl_x), __int_as_float(sl_w), 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int k = 0; k < 32; ++k) s_buf[t * kOP + k] = r[k];
    }
    __syncthreads();
    float4* dst = reinterpret_cast<float4*>(rec + i0);
    for (int q = t; q < nloc * 8; q += 256) {
        const int e = q >> 3, f = q & 7;
        const float* p = s_buf + e * kOP + 4 * f;
        dst[q] = make_float4(p[0], p[1], p[2], p[3]);
    }
}

// Does the surfel reach the 8x8 quadrant centred at (qx, qy)?  Both passes use this test, so
// they skip the same records.  The record's boxes give a cheap conservative answer; the
// exact refinement follows.
// With q = p - m (pixel centre relative to the projected mean) the hit is
// c = q_x A + q_y B + C' and the UV-disk branch is valid iff |c_xy|^2 <= 2L c_z^2, i.e.
// f(q) = a q_x^2 + b q_x q_y + c q_y^2 + d q_x + e q_y + f0 <= 0.  When the quadratic part
// is positive definite that set is an ellipse and f is convex, so its minimum over the
// quadrant's pixel-centre rectangle is at the unconstrained minimiser (if inside) or on an
// edge (a 1-D parabola minimised in closed form).  Otherwise (the plane nearly through the
// camera) the f64 bounding box of the record decides, as before.  The low-pass branch
// (|q|^2 <= L) is tested against the nearest point of the rectangle.  Conservative: L is
// inflated by 2 % + 0.02, far above the rounding of the per-pixel evaluation and of the
// hardware exp / rcp, so a skipped record has alpha < 1/255 at every pixel of the quadrant.
__device__ __forceinline__ bool reaches2_exact(const float4 r0, const float4 r1, const float4 r2, const float4 r4,
                                               const float4 box, float qx, float qy) {
    const bool in_box = fabsf(box.x - qx) <= box.z + 3.5f && fabsf(box.y - qy) <= box.w + 3.5f;
    const bool in_dbox = fabsf(r2.y - qx) <= r4.w + 3.5f && fabsf(r2.z - qy) <= r4.w + 3.5f;
    const float X0 = qx - 3.5f - r2.y, X1 = qx + 3.5f - r2.y, Y0 = qy - 3.5f - r2.z, Y1 = qy + 3.5f - r2.z;
    const float Lp = 1.02f * __logf(255.0f * r2.w) + 0.02f;
    const float nx = fminf(fmaxf(0.f, X0), X1), ny = fminf(fmaxf(0.f, Y0), Y1);
    const bool in_disk = in_dbox & (nx * nx + ny * ny <= Lp);
    const float L2 = 2.0f * Lp;
    const float Ax = r0.x, Ay = r0.y, Az = r0.z, Bx = r0.w, By = r1.x, Bz = r1.y, Cx = r1.z, Cy = r1.w, Cz = r2.x;
    const float a = Ax * Ax + Ay * Ay - L2 * Az * Az;
    const float b = 2.0f * (Ax * Bx + Ay * By - L2 * Az * Bz);
    const float c = Bx * Bx + By * By - L2 * Bz * Bz;
    const float d = 2.0f * (Ax * Cx + Ay * Cy - L2 * Az * Cz);
    const float e = 2.0f * (Bx * Cx + By * Cy - L2 * Bz * Cz);
    const float f0 = Cx * Cx + Cy * Cy - L2 * Cz * Cz;
    const float det = 4.0f * a * c - b * b;
    const bool pd = (a > 0.f) & (c > 0.f) & (det > 1e-3f * 4.0f * a * c);
    const float i2a = 0.5f * __builtin_amdgcn_rcpf(a), i2c = 0.5f * __builtin_amdgcn_rcpf(c);
    auto F = [&](float x, float y) { return fmaf(fmaf(a, x, fmaf(b, y, d)), x, fmaf(fmaf(c, y, e), y, f0)); };
    const float yA = fminf(fmaxf(-(b * X0 + e) * i2c, Y0), Y1), yB = fminf(fmaxf(-(b * X1 + e) * i2c, Y0), Y1);
    const float xA = fminf(fmaxf(-(b * Y0 + d) * i2a, X0), X1), xB = fminf(fmaxf(-(b * Y1 + d) * i2a, X0), X1);
    const float m = fminf(fminf(F(X0, yA), F(X1, yB)), fminf(F(xA, Y0), F(xB, Y1)));
    const float idet = __builtin_amdgcn_rcpf(det);
    const float sx = (b * e - 2.0f * c * d) * idet, sy = (b * d - 2.0f * a * e) * idet;
    const bool centre_in = (sx >= X0) & (sx <= X1) & (sy >= Y0) & (sy <= Y1);
    const bool in_ell = pd ? (centre_in | (m <= 0.f)) : true;
    return (in_box & in_ell) | in_disk;
}

__device__ __forceinline__ int lanes_below2(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
}

// per-pair surfel geometry shared by forward and backward
struct Hit2 {
    float iz, sx, sy, g3, dx, dy, g2, sigma;
    bool ok;  // the ray is not parallel to the surfel plane
};

__device__ __forceinline__ Hit2 hit2(const float4 r0, const float4 r1, const float4 r2, float px, float py) {
    Hit2 h;
    h.dx = r2.y - px;
    h.dy = r2.z - py;
    // c = (p - m)_x A + (p - m)_y B + C'
    const float cx = fmaf(-h.dx, r0.x, fmaf(-h.dy, r0.w, r1.z));
    const float cy = fmaf(-h.dx, r0.y, fmaf(-h.dy, r1.x, r1.w));
    const float cz = fmaf(-h.dx, r0.z, fmaf(-h.dy, r1.y, r2.x));
    h.ok = cz != 0.f;
    h.iz = h.ok ? __builtin_amdgcn_rcpf(cz) : 0.f;
    h.sx = cx * h.iz;
    h.sy = cy * h.iz;
    h.g3 = h.sx * h.sx + h.sy * h.sy;
    h.g2 = 2.0f * (h.dx * h.dx + h.dy * h.dy);
    // log2(e) * sigma, sigma = min(g3, g2) / 2: feeds v_exp_f32 directly (vis = exp2(-sigma'))
    h.sigma = (0.5f * 1.4426950408889634f) * fminf(h.g3, h.g2);
    return h;
}

template <int D>
__global__ __launch_bounds__(256) void raster2d_fwd_kernel(
    int C, int W, int H, int tw, int th, const Rec2* __restrict__ rec, const float* __restrict__ backgrounds,
    int bg_ch, int ed_ch, const int32_t* __restrict__ offsets, int64_t n_isects,
    const int32_t* __restrict__ flatten_ids, float* __restrict__ render_colors, float* __restrict__ render_alphas,
    float* __restrict__ render_normals,
    float* __restrict__ render_distort, float* __restrict__ render_median, int32_t* __restrict__ last_ids,
    int32_t* __restrict__ median_ids, uint64_t* __restrict__ qmask, int64_t qstride, float4* __restrict__ zero_rows,
    int64_t zero_n4, const int64_t* __restrict__ isect_info, const float* __restrict__ normal_rot,
    const int32_t* __restrict__ order,
    int32_t* __restrict__ tile_end) {
    constexpr int NB = kFwd2Batch;
    // one LDS object: every component of record t sits at a compile-time offset from one address;
    // double-buffered and filled by LDS-DMA one batch ahead (no staging VGPRs: 96 -> 72 VGPRs)
    __shared__ struct {
        float4 r0[2][NB], r1[2][NB], r2[2][NB], col[2][NB], r4[2][NB], box[2][NB];
    } sr;
    __shared__ uint8_t s_list[4][NB];
    __shared__ int s_vote[2][4];
    const Tile2 tc = tile2_ctx(C, W, H, tw, th, offsets, n_isects, isect_info, order);
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const float qx = (float)(tc.j - (lane & 7)) + 4.0f;
    const float qy = (float)(tc.i - (lane >> 3)) + 4.0f;
    // a stopped lane (exclusive stop at T <= 1e-4) carries T negated: no separate flag
    float T = tc.inside ? 1.0f : -1.0f, distort = 0.f, acc_vd = 0.f, median = 0.f;
    float acc[4] = {0.f, 0.f, 0.f, 0.f}, nacc[3] = {0.f, 0.f, 0.f};
    int32_t cur = 0, med_idx = 0;
    const int nb = (tc.end - tc.start + NB - 1) / NB;
    const int32_t last = tc.end - 1;
    const bool loader = tid < NB;  // waves 0, 1: one record each (clamped ids)
    // global_load_lds_dwordx4: per-lane source, LDS destination = wave base + 16 B x lane
    auto dma_batch = [&](int buf, int32_t id) {
        const float4* r = reinterpret_cast<const float4*>(rec + id);
        const int w0 = tid & ~63;
        float4* const dst[6] = {&sr.r0[buf][w0], &sr.r1[buf][w0], &sr.r2[buf][w0],
                                &sr.col[buf][w0], &sr.r4[buf][w0], &sr.box[buf][w0]};
#pragma unroll
        for (int q = 0; q < 6; ++q) lds_dma16(r + q, dst[q]);
    };
    int32_t nid = 0;
    if (nb > 0 && loader) {
        dma_batch(0, flatten_ids[min(tc.start + tid, last)]);
        nid = flatten_ids[min(tc.start + NB + tid, last)];
    }
    uint8_t* my_list = s_list[wave];
    for (int b = 0; b < nb; ++b) {
        const int cur_b = b & 1;
        const bool wave_done = __all(T < 0.f);
        if (lane == 0) s_vote[b & 1][wave] = wave_done;
        // this wave's DMA of batch b has landed; the barrier publishes it (and the vote) to
        // the workgroup, and every wave is past batch b-1, whose buffer the next DMA refills
        __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt(0)
        lds_barrier();
        if (s_vote[b & 1][0] & s_vote[b & 1][1] & s_vote[b & 1][2] & s_vote[b & 1][3]) break;
        const int32_t bs = tc.start + b * NB;
        const int cnt = min(NB, tc.end - bs);
        if (b + 1 < nb && loader) {
            dma_batch(cur_b ^ 1, nid);
            nid = flatten_ids[min(bs + 2 * NB + tid, last)];
        }
        if (wave_done) continue;
        const float4 *s_r0 = sr.r0[cur_b], *s_r1 = sr.r1[cur_b], *s_r2 = sr.r2[cur_b], *s_col = sr.col[cur_b],
                     *s_r4 = sr.r4[cur_b], *s_box = sr.box[cur_b];
        int n_mine = 0;
        // quadrant mask words of this batch (read by the backward), one per 64 records
        uint64_t* const qw = qmask ? qmask + wave * qstride +
                                         qmask_word0(tc.start, (int64_t)tc.cam * (tw * th) + tc.tile) +
                                         (int64_t)b * (NB / 64)
                                   : nullptr;
#pragma unroll
        for (int k = 0; k < NB / 64; ++k) {
            const int t = k * 64 + lane;
            const bool rel = t < cnt && reaches2_exact(s_r0[t], s_r1[t], s_r2[t], s_r4[t], s_box[t], qx, qy);
            const uint64_t m = __ballot(rel);
            if (rel) my_list[n_mine + lanes_below2(m)] = (uint8_t)t;
            n_mine += __popcll(m);
            if (qw && lane == k && k * 64 < cnt) qw[k] = m;  // only words holding records of this tile
        }
        if (n_mine == 0) continue;
        static_assert(NB == 64 || NB == 128, "list registers hold 64 or 128 entries");
        const int lst0 = my_list[lane];
        // the second half exists only for 128-record batches (s_list rows are NB long)
        const int lst1 = NB > 64 ? my_list[(NB > 64 ? 64 : 0) + lane] : 0;
        auto step = [&](const int t) {
            const float4 r0 = s_r0[t], r1 = s_r1[t], r2 = s_r2[t], c = s_col[t], r4 = s_r4[t];
            const Hit2 h = hit2(r0, r1, r2, tc.px, tc.py);
            const float alpha = fminf(0.999f, r2.w * __builtin_amdgcn_exp2f(-h.sigma));
            const bool valid = h.ok & (h.sigma >= 0.f) & (alpha >= 1.0f / 255.0f);
            const float nT = T * (1.0f - alpha);
            const bool ok = valid & (nT > 1e-4f);  // a stopped lane's nT is negative
            const float vis = ok ? alpha * T : 0.f;
            const float ck[4] = {c.x, c.y, c.z, c.w};
#pragma unroll
            for (int k = 0; k < D; ++k) acc[k] += ck[k] * vis;
            nacc[0] += r4.x * vis;
            nacc[1] += r4.y * vis;
            nacc[2] += r4.z * vis;
            const float depth = ck[D - 1];
            distort += 2.0f * (vis * depth * (1.0f - T) - vis * acc_vd);
            acc_vd += vis * depth;
            const bool med = ok & (T > 0.5f);
            median = med ? depth : median;
            med_idx = med ? bs + t : med_idx;
            cur = ok ? bs + t : cur;
            T = ok ? nT : (valid ? -fabsf(T) : T);
        };
        const int n0 = min(n_mine, 64);
        int i = 0;
        for (; i < n0; ++i) {
            step(__builtin_amdgcn_readlane(lst0, i));
            if (__all(T < 0.f)) break;
        }
        if (NB > 64 && i == n0)
            for (; i < n_mine; ++i) {
                step(__builtin_amdgcn_readlane(lst1, i - 64));
                if (__all(T < 0.f)) break;
            }
    }
    if (tc.inside) {
        T = fabsf(T);
        const float alpha = 1.0f - T;
        render_alphas[tc.pix] = alpha;
#pragma unroll
        for (int k = 0; k < D; ++k) {
            float v = (backgrounds && k < bg_ch) ? acc[k] + T * backgrounds[tc.cam * bg_ch + k] : acc[k];
            if (k == ed_ch) v = v / fmaxf(alpha, 1e-10f);  // expected depth (rasterization ED)
            render_colors[tc.pix * D + k] = v;
        }
        if (normal_rot) {
            // world frame (rasterization_2dgs): R^T n, R = the camera's viewmat rotation
            const float* R = normal_rot + tc.cam * 16;
            float nw[3];
#pragma unroll
            for (int k = 0; k < 3; ++k) nw[k] = R[k] * nacc[0] + R[4 + k] * nacc[1] + R[8 + k] * nacc[2];
#pragma unroll
            for (int k = 0; k < 3; ++k) nacc[k] = nw[k];
        }
#pragma unroll
        for (int k = 0; k < 3; ++k) render_normals[tc.pix * 3 + k] = nacc[k];
        render_distort[tc.pix] = distort;
        render_median[tc.pix] = median;
        last_ids[tc.pix] = cur;
        median_ids[tc.pix] = med_idx;
    }
    if (tile_end) {  // the tile's latest contributor + 1 (the backward's tile order), as raster3d_fwd
        __shared__ int32_t s_end[4];
        int32_t m = tc.inside ? cur : -1;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) m = max(m, __shfl_xor(m, d));
        if (lane == 0) s_end[wave] = m;
        __syncthreads();
        if (tid == 0)
            tile_end[(int64_t)tc.cam * (tw * th) + tc.tile] = max(max(s_end[0], s_end[1]), max(s_end[2], s_end[3])) + 1;
    }
    // the backward's accumulator rows, cleared here (after the last load) instead of by a
    // memset on the step's critical path
    zero_share(zero_rows, zero_n4);
}

__device__ __forceinline__ int32_t wave_max2(int32_t v) {
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) v = max(v, __shfl_xor(v, d));
    return v;
}

// ---------------------------------------------------------------- backward, transposed inputs
// The 2DGS backward without a per-step 19-value wave reduction (round 2's kernel spent 15
// permlane swaps, 15 adds and 20 DPP adds a step on it).  As in the 3DGS backward, pass 1 composites
// the steps per lane (pixel) and queues the ones some pixel composites, two numbers per pixel:
// F = fac = alpha T with the sigma branch in its sign bit (set: the low-pass disk, clear: the
// ray-plane hit) and V = dL/dsigma.  They are transposed through LDS so that lane 16 s + r holds
// step s's values for the 4 pixels of one column (rows y0, y0 + 2, y0 + 4, y0 + 6); pass 2
// re-evaluates the hit of that step's surfel at those 4 pixels (the same float operations as
// pass 1: identical values), forms the 19 accumulator terms (v_xy, (p - m) x v_c, v_c, the
// opacity sum, fac x normal / colour upstream) summed over its 4 pixels, and a 16-lane
// transpose-reduce (4 DPP levels, the value set halved at each) leaves 2 of the 19 sums per lane,
// stored as one float2 per lane into the wave's row of the (tile, surfel) pair's gradient slot.
#ifndef HGSR_BWD2TP_WAVES
#define HGSR_BWD2TP_WAVES 5
#endif
#ifndef HGSR_BWD2TP_U1  // unroll of the pass-1 step loop (1: rolled)
#define HGSR_BWD2TP_U1 1
#endif
#ifndef HGSR_BWD2TP_U2  // unroll of the pass-2 pixel loop
#define HGSR_BWD2TP_U2 1
#endif
// one transpose-reduce level over a 16-lane row: N values -> N / 2, lanes with `bit` set keep the
// upper half; the partner (DPP control CTRL, an involution with the opposite bit) sends the rest
template <int CTRL, int N>
__device__ __forceinline__ void tr_level(const float (&v)[N], float (&w)[N / 2], bool bit) {
#pragma unroll
    for (int i = 0; i < N / 2; ++i) {
        const float keep = bit ? v[i + N / 2] : v[i];
        const float give = bit ? v[i] : v[i + N / 2];
        w[i] = keep + dpp<CTRL>(give);
    }
}

template <int D>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(HGSR_BWD2TP_WAVES, 8))) void
raster2d_bwd_tp_kernel(int C, int W, int H, int tw, int th, const Rec2* __restrict__ rec,
                       const float* __restrict__ backgrounds, int bg_ch, int ed_ch,
                       const float* __restrict__ render_colors, const int32_t* __restrict__ offsets,
                       int64_t n_isects, const int32_t* __restrict__ flatten_ids,
                       const float* __restrict__ render_alphas, const int32_t* __restrict__ last_ids,
                       const float* __restrict__ v_render_colors, const float* __restrict__ v_render_alphas,
                       const float* __restrict__ v_render_normals, float* __restrict__ rows,
                       uint8_t* __restrict__ flags, int64_t n_slots,
                       unsigned long long* __restrict__ pair_counter, const uint64_t* __restrict__ qmask,
                       int64_t qstride, const float* __restrict__ normal_rot,
                       const float* __restrict__ v_depth_extra, const int32_t* __restrict__ order) {
    constexpr int KV = 15 + D;
    constexpr int NB = kBwd2Batch;
    __shared__ struct {
        float4 r0[2][NB], r1[2][NB], r2[2][NB], col[2][NB], r4[2][NB], box[2][NB];
    } sr;
    __shared__ int32_t s_e[2][NB];  // the batch's records' gradient slots (-1: none)
    __shared__ __attribute__((aligned(16))) uint8_t s_list[4][NB];
    __shared__ int32_t s_last[4];
    __shared__ __attribute__((aligned(16))) float s_tp[4][4 * 16 * 4 * 2];
    __shared__ __attribute__((aligned(16))) float s_pv[4][64 * 8];  // per pixel: vo[4], vn[3], 0
    const Tile2 tc = tile2_ctx(C, W, H, tw, th, offsets, n_isects, nullptr, order);
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const float qx = (float)(tc.j - (lane & 7)) + 4.0f;
    const float qy = (float)(tc.i - (lane >> 3)) + 4.0f;
    const int tile_y = tc.tile / tw, tile_x = tc.tile - tile_y * tw;
    // per-pixel upstream terms of pixel (i, j), as raster2d_bwd_kernel: colour (ED divided, the
    // depth channel plus the depth->normal gradient), normal (back to the camera frame), the
    // alpha / background term; returns T_final
    auto pixel_terms = [&](int i, int j, float (&vo)[4], float (&vn)[3], float& va_term) {
        const bool in = i < H && j < W;
        const int64_t pix = ((int64_t)tc.cam * H + i) * W + j;
        const float Tf = in ? 1.0f - render_alphas[pix] : 1.0f;
#pragma unroll
        for (int k = 0; k < 4; ++k) vo[k] = (in && k < D) ? v_render_colors[pix * D + k] : 0.f;
#pragma unroll
        for (int k = 0; k < 3; ++k) vn[k] = in ? v_render_normals[pix * 3 + k] : 0.f;
        if (normal_rot) {
            const float* R = normal_rot + tc.cam * 16;
            float vc[3];
#pragma unroll
            for (int q = 0; q < 3; ++q) vc[q] = R[4 * q] * vn[0] + R[4 * q + 1] * vn[1] + R[4 * q + 2] * vn[2];
#pragma unroll
            for (int q = 0; q < 3; ++q) vn[q] = vc[q];
        }
        if (v_depth_extra && in) vo[D - 1] += v_depth_extra[pix];
        float va = in ? v_render_alphas[pix] : 0.f;
        if (ed_ch >= 0 && in) {
            const float alpha = 1.0f - Tf, ac = fmaxf(alpha, 1e-10f);
            float v_ed = 0.f;
#pragma unroll
            for (int k = 0; k < D; ++k)
                if (k == ed_ch) {
                    v_ed = vo[k];
                    vo[k] = v_ed / ac;
                }
            if (alpha >= 1e-10f) va -= v_ed * render_colors[pix * D + ed_ch] / ac;
        }
        float bg_dot = 0.f;
#pragma unroll
        for (int k = 0; k < D; ++k)
            if (backgrounds && k < bg_ch) bg_dot += backgrounds[tc.cam * bg_ch + k] * vo[k];
        va_term = Tf * (va - bg_dot);
        return Tf;
    };
    float vo[4], vn[3], va_term;
    const float T_final = pixel_terms(tc.i, tc.j, vo, vn, va_term);
    float T = T_final, Bsum = 0.f;
    // pass-2 role: step lane >> 4, column cx, rows y0 + 2 m of the quadrant; the pixels'
    // upstream colour / normal terms come from the wave's LDS table (pixel = lane of pass 1)
    const int r16 = lane & 15, cx = r16 & 7, y0 = r16 >> 3;
    const int qi0 = tc.i - (lane >> 3), qj0 = tc.j - (lane & 7);
    const float p2x = (float)(qj0 + cx) + 0.5f, p2y0 = (float)(qi0 + y0) + 0.5f;
    float* const pv = s_pv[wave];
    // pixel p = lane: colour terms at float 128 (p >> 4) + 4 (p & 15), normal terms 64 further; pass 2
    // reads 16 distinct pixels p = r + 16 m per 16-B read, conflict-free on CDNA4's banks
    *reinterpret_cast<float4*>(pv + 128 * (lane >> 4) + 4 * (lane & 15)) = make_float4(vo[0], vo[1], vo[2], vo[3]);
    *reinterpret_cast<float4*>(pv + 128 * (lane >> 4) + 64 + 4 * (lane & 15)) = make_float4(vn[0], vn[1], vn[2], 0.f);
    // this lane's two output sums after the transpose-reduce: index b3 10 + b2 5 + b1 3 + b0 2 + q
    int koff[2];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        const int b3 = (r16 >> 3) & 1, b2 = (r16 >> 2) & 1, b1 = (r16 >> 1) & 1, b0 = r16 & 1;
        const int l = b0 * 2 + q, k = b1 * 3 + l, idx = b3 * 10 + b2 * 5 + k;
        koff[q] = (l < 3 && k < 5 && idx < KV) ? idx : -1;
    }
    const int32_t bin_final = tc.inside ? last_ids[tc.pix] : -1;
    const int32_t wave_final = wave_max2(bin_final);
    if (lane == 0) s_last[wave] = wave_final;
    lds_barrier();
    const int32_t blk_final = max(max(s_last[0], s_last[1]), max(s_last[2], s_last[3]));
    const int32_t end = min(tc.end, blk_final + 1);
    const int nb = end > tc.start ? (end - tc.start + NB - 1) / NB : 0;
    if (pair_counter && threadIdx.x == 0 && end > tc.start)
        atomicAdd(pair_slot(pair_counter, 0), (unsigned long long)(end - tc.start) * kTilePixels);
    float4* const stage_arr[6] = {&sr.r0[0][0], &sr.r1[0][0], &sr.r2[0][0], &sr.col[0][0], &sr.r4[0][0], &sr.box[0][0]};
    int32_t cid = 0, nid = 0;
    int2 csl = make_int2(-1, 0);  // slot base of cid (raster3d_bwd_kernel)
    const bool loader = tid < NB;
    auto dma_batch = [&](int buf, int32_t id) {
        const float4* r = reinterpret_cast<const float4*>(rec + id);
#pragma unroll
        for (int q = 0; q < 6; ++q) lds_dma16(r + q, stage_arr[q] + buf * NB);
    };
    if (nb > 0 && loader) {
        cid = flatten_ids[max(end - 1 - tid, tc.start)];
        dma_batch(0, cid);
        csl = *reinterpret_cast<const int2*>(&rec[cid].sl);
        nid = flatten_ids[max(end - 1 - NB - tid, tc.start)];
    }
    uint8_t* my_list = s_list[wave];
    uint32_t stepped = 0;
    uint64_t qw[2] = {0, 0};
    auto qfetch = [&](int bb) {
        const int64_t lo = (end - 1 - (int64_t)bb * NB - tc.start) - (NB - 1);
        const int64_t bin = (int64_t)tc.cam * (tw * th) + tc.tile;
        const int idx = __builtin_amdgcn_readfirstlane(
            (int)(__builtin_amdgcn_readfirstlane(wave) * qstride + qmask_word0(tc.start, bin) + (lo >> 6)));
        const uint64_t* qp = qmask + idx;
        qw[0] = qp[0];
        qw[1] = qp[1];
    };
    if (qmask && nb > 0) qfetch(0);
    const int gsl = lane >> 4;  // pass-2 queue entry of this lane
    for (int b = 0; b < nb; ++b) {
        const int cur = b & 1, prv = cur ^ 1;
        const int32_t batch_end = end - 1 - b * NB;
        const int bsz = min(NB, batch_end + 1 - tc.start);
        __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt(0): batch b's DMA has landed
        if (tid < bsz) {
            const int64_t e = (int64_t)csl.x + (int64_t)tile_y * csl.y + tile_x;
            s_e[cur][tid] = (e >= 0 && e < n_slots) ? (int32_t)e : -1;
        }
        if (b + 1 < nb && loader) {
            cid = nid;
            dma_batch(prv, cid);
            csl = *reinterpret_cast<const int2*>(&rec[cid].sl);
            nid = flatten_ids[max(batch_end - 2 * NB - tid, tc.start)];
        }
        lds_barrier();
        const int t0 = max(0, batch_end - wave_final);
        uint64_t m;
        bool rel;
        if (qmask) {
            const int64_t R = batch_end - tc.start, lo = R - (NB - 1);
            const uint64_t w0 = qw[0], w1 = qw[1];
            if (b + 1 < nb) qfetch(b + 1);
            const int sh = (int)(lo & 63);
            const uint64_t win = sh ? (w0 >> sh) | (w1 << (64 - sh)) : w0;
            const uint64_t below_z = bsz >= 64 ? ~0ull : ((1ull << bsz) - 1);
            const uint64_t below_a = t0 >= 64 ? ~0ull : ((1ull << t0) - 1);
            const uint64_t mk = __builtin_bitreverse64(win) & below_z & ~below_a;
            m = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)mk) |
                ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(mk >> 32)) << 32);
            rel = (m >> lane) & 1;
        } else {
            rel = lane < bsz && lane >= t0 &&
                  reaches2_exact(sr.r0[cur][lane], sr.r1[cur][lane], sr.r2[cur][lane], sr.r4[cur][lane],
                                 sr.box[cur][lane], qx, qy);
            m = __ballot(rel);
        }
        if (rel) my_list[lanes_below2(m)] = (uint8_t)lane;
        const int n_mine = __popcll(m);
        stepped += (uint32_t)n_mine;
        if (n_mine > 0) {
            const uint32_t lstp = reinterpret_cast<const uint32_t*>(my_list)[lane < NB / 4 ? lane : 0];
            float* const tp = s_tp[wave];
            // pass 2 over the 4 queued steps (packed record indices, NB = empty entry): step `gsl`'s
            // surfel at this lane's 4 pixels, the 16-lane transpose-reduce, the sums stored
            auto pass2 = [&](const uint32_t qpk) {
                const int t = (int)__builtin_amdgcn_ubfe(qpk, 8 * gsl, 8);
                const int tt = t < NB ? t : 0;
                const int se = s_e[cur][tt];
                const float4 r0 = sr.r0[cur][tt], r1 = sr.r1[cur][tt], r2 = sr.r2[cur][tt];
                float g[20];
#pragma unroll
                for (int k = 0; k < 20; ++k) g[k] = 0.f;
#pragma unroll HGSR_BWD2TP_U2
                for (int mq = 0; mq < 4; ++mq) {
                    const float2 fv = *reinterpret_cast<const float2*>(tp + 128 * mq + 32 * gsl + 2 * r16);
                    // pixel (y0 + 2 mq) * 8 + cx = r16 + 16 mq
                    const float4 po = *reinterpret_cast<const float4*>(pv + 128 * mq + 4 * r16);
                    const float4 pn = *reinterpret_cast<const float4*>(pv + 128 * mq + 64 + 4 * r16);
                    const float pvo[4] = {po.x, po.y, po.z, po.w}, pvn[3] = {pn.x, pn.y, pn.z};
                    const Hit2 h = hit2(r0, r1, r2, p2x, p2y0 + (float)(2 * mq));
                    const float fac = fabsf(fv.x);
                    const bool ell = !__builtin_signbit(fv.x);
                    const float v_sigma = fv.y;
                    const float ve = ell ? v_sigma : 0.f, vp = ell ? 0.f : v_sigma;
                    const float vs0 = ve * h.sx, vs1 = ve * h.sy;
                    const float vc0 = vs0 * h.iz, vc1 = vs1 * h.iz, vc2 = -(vs0 * h.sx + vs1 * h.sy) * h.iz;
                    g[0] += 2.0f * vp * h.dx;
                    g[1] += 2.0f * vp * h.dy;
                    g[2] -= h.dx * vc0; g[3] -= h.dx * vc1; g[4] -= h.dx * vc2;
                    g[5] -= h.dy * vc0; g[6] -= h.dy * vc1; g[7] -= h.dy * vc2;
                    g[8] += vc0; g[9] += vc1; g[10] += vc2;
                    g[11] += v_sigma;  // -> the opacity sum below
#pragma unroll
                    for (int k = 0; k < 3; ++k) g[12 + k] += fac * pvn[k];
#pragma unroll
                    for (int k = 0; k < D; ++k) g[15 + k] += fac * pvo[k];
                }
                // opacity: sum vis va2 = -sum v_sigma / opacity
                g[11] = r2.w != 0.f ? -g[11] / r2.w : 0.f;
                // 16-lane transpose-reduce: 20 -> 10 -> 5 -> 3 -> 2 values per lane
                float w1[10], w2[5], w3[3], w4[2];
                tr_level<0x128, 20>(g, w1, (r16 >> 3) & 1);  // row_ror:8, partner r ^ 8
                tr_level<0x141, 10>(w1, w2, (r16 >> 2) & 1);  // row_half_mirror, partner 7 - r
                {
                    const float w2p[6] = {w2[0], w2[1], w2[2], w2[3], w2[4], 0.f};
                    tr_level<0x4E, 6>(w2p, w3, (r16 >> 1) & 1);  // quad_perm [2,3,0,1]
                }
                {
                    const float w3p[4] = {w3[0], w3[1], w3[2], 0.f};
                    tr_level<0xB1, 4>(w3p, w4, r16 & 1);  // quad_perm [1,0,3,2]
                }
#pragma unroll
                for (int q = 0; q < 2; ++q) asm volatile("" : "+v"(w4[q]));
                if (t < NB && se >= 0) {  // this wave's row of the (tile, surfel) pair's slot
                    const int64_t rw = (int64_t)se * kSlotWaves + wave;
                    float* const row = rows + rw * kRow2;
#pragma unroll
                    for (int q = 0; q < 2; ++q)
                        if (koff[q] >= 0) row[koff[q]] = w4[q];
                    if (r16 == 0) flags[rw] = 1;
                }
            };
            // pass 1, one step at a time; a step with a valid pixel is queued -- its (F, V) go to
            // queue slot qn of the wave's transpose buffer (float 128 m + 32 qn + 2 r for lane L =
            // pixel r + 16 m: conflict-free 8-B writes, and 8-B reads by lane 16 s + r at 128 m + 32 s
            // + 2 r conflict-free too; the [qn][r][m] layout read 4-way) --
            // and a full queue runs pass 2 (a step nobody composites contributes nothing: skipped)
            int qn = 0;
            uint32_t qpk = 0;
            for (int i = 0; i < n_mine; ++i) {
                const uint32_t word = (uint32_t)__builtin_amdgcn_readlane((int)lstp, i >> 2);
                const int t = (int)((word >> (8 * (i & 3))) & 0xffu);
                const float4 r0 = sr.r0[cur][t], r1 = sr.r1[cur][t], r2 = sr.r2[cur][t], c = sr.col[cur][t],
                             r4 = sr.r4[cur][t];
                const Hit2 h = hit2(r0, r1, r2, tc.px, tc.py);
                const float vis = __builtin_amdgcn_exp2f(-h.sigma);
                const float araw = r2.w * vis;
                const float alpha = fminf(0.999f, araw);
                const bool valid = (batch_end - t <= bin_final) & h.ok & (h.sigma >= 0.f) & (alpha >= 1.0f / 255.0f);
                if (!__any(valid)) continue;
                const float al = valid ? alpha : 0.f;
                const float ra = __builtin_amdgcn_rcpf(1.0f - al);
                const float Tn = T * ra;
                const float fac = al * Tn;
                const float ck[4] = {c.x, c.y, c.z, c.w};
                float cv = r4.x * vn[0] + r4.y * vn[1] + r4.z * vn[2];
#pragma unroll
                for (int k = 0; k < D; ++k) cv += ck[k] * vo[k];
                const float v_alpha = Tn * cv + ra * (va_term - Bsum);
                Bsum += fac * cv;
                const float va2 = (valid & (araw <= 0.999f)) ? v_alpha : 0.f;
                T = Tn;
                // sigma = min(g3, g2) / 2: the sign bit of F carries the branch (set: low-pass)
                const float Fq = (h.g3 <= h.g2) ? fac : -fac;
                *reinterpret_cast<float2*>(tp + 128 * (lane >> 4) + 32 * qn + 2 * r16) = make_float2(Fq, -araw * va2);
                qpk |= (uint32_t)t << (8 * qn);
                if (++qn == 4) {
                    pass2(qpk);
                    qn = 0;
                    qpk = 0;
                }
            }
            if (qn > 0) {  // the partial queue: empty slots composite nothing
                for (int q = qn; q < 4; ++q) {
                    *reinterpret_cast<float2*>(tp + 128 * (lane >> 4) + 32 * q + 2 * r16) = make_float2(0.f, 0.f);
                    qpk |= (uint32_t)NB << (8 * q);
                }
                pass2(qpk);
            }
        }
        lds_barrier();
    }
    if (pair_counter && lane == 0 && stepped)
        atomicAdd(pair_slot(pair_counter, 1), (unsigned long long)stepped * 64ull);
}

// Per surfel: fold the accumulated sums into gsplat's gradient tensors (overwrite), in f64.
// gA = sum p_x v_c = gA' + m_x gC (gA' = sum (p-m)_x v_c), gB likewise, gC = sum v_c; with
// d(a x b).g = da.(b x g) + db.(g x a):
//   v_u = gB x w + v x gC,  v_v = w x gA + gC x u,  v_w = gA x v + u x gB;
// the densification proxy (d loss / d screen translation) is v_xy - (A.gC, B.gC).
template <int D>
__global__ __launch_bounds__(256) void split2_kernel(int C, int N, const float* __restrict__ rows,
                                                    const uint8_t* __restrict__ flags, const int32_t* __restrict__ seg,
                                                     const int32_t* __restrict__ pbase, const float* __restrict__ partial,
                                                    const float* __restrict__ rt, const float2* __restrict__ means2d,
                                                    float2* __restrict__ v_means2d, float* __restrict__ v_rt,
                                                    ChanDst cd, float* __restrict__ v_normals,
                                                    float2* __restrict__ v_densify) {
    constexpr int KV = 15 + D;
    constexpr int kScr = reduce_slots_floats<KV>();
    __shared__ __attribute__((aligned(16))) float s_scr[4][kScr];  // per wave (each wave owns 64 surfels)
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t g0 = ((int64_t)blockIdx.x * 4 + wave) * 64, g = g0 + lane;
    if (g0 >= N) return;  // wave-uniform; the waves never synchronise with each other
    const int nloc = (int)min((int64_t)64, (int64_t)N - g0);
    const bool live = lane < nloc;
    float col_sum[4] = {0.f, 0.f, 0.f, 0.f}, op_sum = 0.f;
    for (int c = 0; c < C; ++c) {
        const int64_t i = (int64_t)c * N + g;
        float r[KV];
        reduce_slots<KV, (KV + 3) / 4, kRow2, kSlotWaves, 2>(rows, flags, seg, pbase, partial, (int64_t)c * N + g0, nloc, s_scr[wave], r);
        if (!live) continue;
        double u[3], v[3], w[3], gA[3], gB[3], gC[3];
        const float2 mm = means2d[i];
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            u[k] = rt[i * 9 + k];
            v[k] = rt[i * 9 + 3 + k];
            w[k] = rt[i * 9 + 6 + k];
            gC[k] = r[8 + k];
            gA[k] = (double)r[2 + k] + (double)mm.x * gC[k];
            gB[k] = (double)r[5 + k] + (double)mm.y * gC[k];
        }
        double t0[3], t1[3];
        cross3d(gB, w, t0);
        cross3d(v, gC, t1);
#pragma unroll
        for (int k = 0; k < 3; ++k) v_rt[i * 9 + k] = (float)(t0[k] + t1[k]);
        cross3d(w, gA, t0);
        cross3d(gC, u, t1);
#pragma unroll
        for (int k = 0; k < 3; ++k) v_rt[i * 9 + 3 + k] = (float)(t0[k] + t1[k]);
        cross3d(gA, v, t0);
        cross3d(u, gB, t1);
#pragma unroll
        for (int k = 0; k < 3; ++k) v_rt[i * 9 + 6 + k] = (float)(t0[k] + t1[k]);
        v_means2d[i] = make_float2(r[0], r[1]);
#pragma unroll
        for (int k = 0; k < 3; ++k) v_normals[i * 3 + k] = r[12 + k];
        if (v_densify) {
            double A[3], B[3];
            cross3d(v, w, A);
            cross3d(w, u, B);
            v_densify[i] = make_float2((float)((double)r[0] - (A[0] * gC[0] + A[1] * gC[1] + A[2] * gC[2])),
                                       (float)((double)r[1] - (B[0] * gC[0] + B[1] * gC[1] + B[2] * gC[2])));
        }
        if (cd.op_shared) op_sum += r[11];
        else cd.opac[i] = r[11];
#pragma unroll
        for (int k = 0; k < D; ++k) {
            if (k < cd.dc) {
                if (cd.col_shared) col_sum[k] += r[15 + k];
                else cd.colors[i * cd.dc + k] = r[15 + k];
            } else if (cd.depths) {
                cd.depths[i] = r[15 + k];
            }
        }
    }
    if (!live) return;
    if (cd.op_shared) cd.opac[g] = op_sum;
    if (cd.col_shared)
#pragma unroll
        for (int k = 0; k < D; ++k)
            if (k < cd.dc) cd.colors[g * cd.dc + k] = col_sum[k];
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

static size_t rec2_bytes(int C, int N) { return ((size_t)C * N * sizeof(Rec2) + 255) & ~(size_t)255; }

// slots (nullable): as pack3's (the rectangles and launch_slot_prefix's buffer)
static int pack2(int C, int N, int D, const float* means2d, const float* rt, const ChanSrc& cs,
                 const float* normals, Rec2* rec, hipStream_t s, const RectFromRadii* rr = nullptr,
                 void* slots = nullptr) {
    const int64_t n = (int64_t)C * N;
    if (n == 0) return HGSR_OK;
    const dim3 grid((unsigned)((n + 255) / 256));
    const float2* m2 = reinterpret_cast<const float2*>(means2d);
    int32_t* const seg = (int32_t*)slots;
    const int32_t* const bpre = slots ? (const int32_t*)((char*)slots + (((size_t)(n + 1) * 4 + 255) & ~(size_t)255))
                                      : nullptr;
    const RectFromRadii none{nullptr, nullptr, 0, 0, 0};
#define LAUNCH_P2(DD)                                                                                           \
    if (slots)                                                                                                  \
        hipLaunchKernelGGL((pack2_kernel<DD, true>), grid, dim3(256), 0, s, n, N, m2, rt, cs, normals, rec, *rr, \
                           bpre, seg);                                                                          \
    else                                                                                                        \
        hipLaunchKernelGGL((pack2_kernel<DD, false>), grid, dim3(256), 0, s, n, N, m2, rt, cs, normals, rec,    \
                           none, (const int32_t*)nullptr, (int32_t*)nullptr)
    switch (D) {
        case 1: LAUNCH_P2(1); break;
        case 2: LAUNCH_P2(2); break;
        case 3: LAUNCH_P2(3); break;
        default: LAUNCH_P2(4); break;
    }
#undef LAUNCH_P2
    return check_launch("raster2d_pack");
}

// the records, then the slot prefix a training forward fills (hgsr_raster2d_pack_fused with radii)
extern "C" size_t hgsr_raster2d_fwd_ws_bytes(int C, int N, int D) {
    (void)D;
    return rec2_bytes(C, N) + slot_prefix_bytes((int64_t)C * N);
}

static int raster2d_fwd_launch(int C, int D, const Rec2* rec, const float* backgrounds, int bg_ch, int ed_ch,
                               int width, int height, int tile_w, int tile_h, const int32_t* isect_offsets,
                               int64_t n_isects, const int32_t* flatten_ids, float* render_colors,
                               float* render_alphas, float* render_normals, float* render_distort,
                               float* render_median, int32_t* last_ids, int32_t* median_ids, hipStream_t s,
                               void* qbuf = nullptr, size_t qbytes = 0, float* zero_rows = nullptr,
                               size_t zero_bytes = 0, const int64_t* isect_info = nullptr,
                               const float* normal_rot = nullptr);

static int raster2d_fwd_impl(int C, int N, int D, const float* means2d, const float* rt, const ChanSrc& cs,
                             const float* normals, const float* backgrounds, int bg_ch, int ed_ch, int width,
                             int height, int tile_size, int tile_w, int tile_h, const int32_t* isect_offsets,
                             int64_t n_isects, const int32_t* flatten_ids, float* render_colors,
                             float* render_alphas, float* render_normals, float* render_distort,
                             float* render_median, int32_t* last_ids, int32_t* median_ids, void* ws,
                             size_t ws_bytes, hgsr_stream_t stream) {
    if (int st = check_raster2(C, N, D, width, height, tile_size, tile_w, tile_h)) return st;
    HGSR_REQUIRE(ws_bytes >= hgsr_raster2d_fwd_ws_bytes(C, N, D), "raster2d_fwd workspace too small");
    HGSR_REQUIRE(isect_offsets && render_colors && render_alphas && render_normals && render_distort &&
                     render_median && last_ids && median_ids,
                 "null pointer");
    HGSR_REQUIRE(n_isects == 0 || (means2d && rt && (cs.colors || cs.dc == 0) && cs.opac && normals &&
                                   flatten_ids && ws),
                 "null pointer");
    hipStream_t s = as_stream(stream);
    Rec2* rec = (Rec2*)ws;
    if (n_isects > 0)
        if (int st = pack2(C, N, D, means2d, rt, cs, normals, rec, s)) return st;
    return raster2d_fwd_launch(C, D, rec, backgrounds, bg_ch, ed_ch, width, height, tile_w, tile_h, isect_offsets,
                               n_isects, flatten_ids, render_colors, render_alphas, render_normals, render_distort,
                               render_median, last_ids, median_ids, s);
}

static int raster2d_fwd_launch(int C, int D, const Rec2* rec, const float* backgrounds, int bg_ch, int ed_ch,
                               int width, int height, int tile_w, int tile_h, const int32_t* isect_offsets,
                               int64_t n_isects, const int32_t* flatten_ids, float* render_colors,
                               float* render_alphas, float* render_normals, float* render_distort,
                               float* render_median, int32_t* last_ids, int32_t* median_ids, hipStream_t s,
                               void* qbuf, size_t qbytes, float* zero_rows, size_t zero_bytes,
                               const int64_t* isect_info, const float* normal_rot) {
    const int64_t n_bins = (int64_t)C * tile_w * tile_h;
    const dim3 grid((unsigned)n_bins);
    float4* const z4 = reinterpret_cast<float4*>(zero_rows);
    const int64_t zn4 = (int64_t)(zero_bytes / sizeof(float4));
    uint64_t* const qmask = qmask_words(qbuf, n_bins);
    const int64_t qstride = qbuf ? qmask_stride_of(qbytes, n_bins) : 0;
    int32_t* order = (qbuf && HGSR_TILE_ORDER && n_isects > 0) ? tile_order_of(qbuf) : nullptr;
    if (order)
        if (int st = launch_tile_order(n_bins, isect_offsets, n_isects, isect_info, order, s)) return st;
    KernelTimer kt("raster2d_fwd", s);
#define LAUNCH_F2(DD)                                                                                            \
    hipLaunchKernelGGL(raster2d_fwd_kernel<DD>, grid, dim3(256), 0, s, C, width, height, tile_w, tile_h, rec,     \
                       backgrounds, bg_ch, ed_ch, isect_offsets, n_isects, flatten_ids, render_colors,           \
                       render_alphas, render_normals, render_distort, render_median, last_ids, median_ids, qmask,   \
                       qstride, z4, zn4, isect_info, normal_rot, order,                                        \
                       (HGSR_BWD_ORDER && order) ? tile_end_of(qbuf, n_bins) : nullptr)
    switch (D) {
        case 1: LAUNCH_F2(1); break;
        case 2: LAUNCH_F2(2); break;
        case 3: LAUNCH_F2(3); break;
        default: LAUNCH_F2(4); break;
    }
#undef LAUNCH_F2
    return check_launch("raster2d_fwd");
}

extern "C" int hgsr_raster2d_fwd(int C, int N, int D, const float* means2d, const float* ray_transforms,
                                 const float* colors, const float* opacities, const float* normals,
                                 const float* backgrounds, int width, int height, int tile_size, int tile_w,
                                 int tile_h, const int32_t* isect_offsets, int64_t n_isects,
                                 const int32_t* flatten_ids, float* render_colors, float* render_alphas,
                                 float* render_normals, float* render_distort, float* render_median,
                                 int32_t* last_ids, int32_t* median_ids, void* ws, size_t ws_bytes,
                                 hgsr_stream_t stream) {
    const ChanSrc cs{colors, (int64_t)N * D, D, nullptr, opacities, (int64_t)N};
    return raster2d_fwd_impl(C, N, D, means2d, ray_transforms, cs, normals, backgrounds, D, -1, width, height,
                             tile_size, tile_w, tile_h, isect_offsets, n_isects, flatten_ids, render_colors,
                             render_alphas, render_normals, render_distort, render_median, last_ids, median_ids, ws,
                             ws_bytes, stream);
}

extern "C" int hgsr_raster2d_fwd_fused(int C, int N, int Dc, const float* means2d, const float* ray_transforms,
                                       const float* colors, int colors_shared, const float* depths,
                                       int expected_depth, const float* opacities, int opacities_shared,
                                       const float* normals, const float* backgrounds, int width, int height,
                                       int tile_size, int tile_w, int tile_h, const int32_t* isect_offsets,
                                       int64_t n_isects, const int32_t* flatten_ids, float* render_colors,
                                       float* render_alphas, float* render_normals, float* render_distort,
                                       float* render_median, int32_t* last_ids, int32_t* median_ids, void* ws,
                                       size_t ws_bytes, hgsr_stream_t stream) {
    HGSR_REQUIRE(Dc >= 0 && Dc <= 4 && (Dc > 0 || depths), "fused raster: 0..4 colour channels (got %d)", Dc);
    HGSR_REQUIRE(!(expected_depth && !depths), "expected_depth needs depths");
    const int D = Dc + (depths ? 1 : 0);
    const ChanSrc cs{colors, colors_shared ? 0 : (int64_t)N * Dc, Dc, depths, opacities,
                     opacities_shared ? 0 : (int64_t)N};
    return raster2d_fwd_impl(C, N, D, means2d, ray_transforms, cs, normals, backgrounds, Dc,
                             expected_depth ? Dc : -1, width, height, tile_size, tile_w, tile_h, isect_offsets,
                             n_isects, flatten_ids, render_colors, render_alphas, render_normals, render_distort,
                             render_median, last_ids, median_ids, ws, ws_bytes, stream);
}

extern "C" int hgsr_raster2d_pack_fused(int C, int N, int Dc, const float* means2d, const float* ray_transforms,
                                        const float* colors, int colors_shared, const float* depths,
                                        const float* opacities, int opacities_shared, const float* normals,
                                        const int32_t* radii, const int32_t* tiles_per_gauss, int tile_size,
                                        int tile_w, int tile_h, void* ws, size_t ws_bytes, hgsr_stream_t stream) {
    HGSR_REQUIRE(C >= 1 && N >= 0, "bad dims");
    HGSR_REQUIRE(Dc >= 0 && Dc <= 4 && (Dc > 0 || depths), "fused raster: 0..4 colour channels (got %d)", Dc);
    const int D = Dc + (depths ? 1 : 0);
    HGSR_REQUIRE(D <= 4, "channels per call must be 1..4 (got %d)", D);
    HGSR_REQUIRE(ws_bytes >= hgsr_raster2d_fwd_ws_bytes(C, N, D), "raster2d_pack workspace too small");
    HGSR_REQUIRE(N == 0 || (means2d && ray_transforms && (colors || Dc == 0) && opacities && normals && ws),
                 "null pointer");
    const ChanSrc cs{colors, colors_shared ? 0 : (int64_t)N * Dc, Dc, depths, opacities,
                     opacities_shared ? 0 : (int64_t)N};
    hipStream_t s = as_stream(stream);
    if (!radii || N == 0) return pack2(C, N, D, means2d, ray_transforms, cs, normals, (Rec2*)ws, s);
    // a backward follows: the records carry their gradient slots (pack3's scheme)
    HGSR_REQUIRE(tile_size > 0 && tile_w > 0 && tile_h > 0, "bad tile grid");
    const RectFromRadii rr{reinterpret_cast<const float2*>(means2d), radii, tile_size, tile_w, tile_h};
    void* const slots = (char*)ws + rec2_bytes(C, N);
    if (int st = launch_slot_prefix((int64_t)C * N, rr, slots, s, tiles_per_gauss)) return st;
    return pack2(C, N, D, means2d, ray_transforms, cs, normals, (Rec2*)ws, s, &rr, slots);
}

extern "C" int hgsr_raster2d_fwd_packed(int C, int N, int Dc, int with_depth, int expected_depth,
                                        const float* backgrounds, int width, int height, int tile_size, int tile_w,
                                        int tile_h, const int32_t* isect_offsets, int64_t n_isects,
                                        const int32_t* flatten_ids, float* render_colors, float* render_alphas,
                                        float* render_normals, float* render_distort, float* render_median,
                                        int32_t* last_ids, int32_t* median_ids, const void* records,
                                        size_t records_bytes, void* qmask, size_t qmask_bytes, void* bwd_ws,
                                        size_t bwd_ws_bytes, const int64_t* isect_info, const float* normal_rot,
                                        hgsr_stream_t stream) {
    HGSR_REQUIRE(Dc >= 0 && Dc <= 4 && (Dc > 0 || with_depth), "fused raster: 0..4 colour channels (got %d)", Dc);
    HGSR_REQUIRE(!(expected_depth && !with_depth), "expected_depth needs depths");
    const int D = Dc + (with_depth ? 1 : 0);
    if (int st = check_raster2(C, N, D, width, height, tile_size, tile_w, tile_h)) return st;
    HGSR_REQUIRE(records_bytes >= hgsr_raster2d_fwd_ws_bytes(C, N, D), "raster2d_fwd_packed: records too small");
    HGSR_REQUIRE(isect_offsets && render_colors && render_alphas && render_normals && render_distort &&
                     render_median && last_ids && median_ids,
                 "null pointer");
    HGSR_REQUIRE(n_isects == 0 || (flatten_ids && records), "null pointer");
    HGSR_REQUIRE(!qmask || qmask_bytes >= hgsr_raster3d_qmask_bytes(C, tile_w, tile_h, n_isects),
                 "raster2d_fwd_packed: quadrant-mask buffer too small");
    // bwd_ws (nullable): the backward's workspace, whose gradient-slot flags this launch clears
    const size_t flags_b = slot_flag_bytes(n_isects, kSlotWaves);
    HGSR_REQUIRE(!bwd_ws || (bwd_ws_bytes >= flags_b && (reinterpret_cast<uintptr_t>(bwd_ws) & 15) == 0),
                 "raster2d_fwd_packed: bwd_ws too small or not 16-B aligned");
    return raster2d_fwd_launch(C, D, (const Rec2*)records, backgrounds, Dc, expected_depth ? Dc : -1, width, height,
                               tile_w, tile_h, isect_offsets, n_isects, flatten_ids, render_colors, render_alphas,
                               render_normals, render_distort, render_median, last_ids, median_ids,
                               as_stream(stream), qmask, qmask_bytes, (float*)bwd_ws, bwd_ws ? flags_b : 0, isect_info,
                               normal_rot);
}

// backward workspace: [slot flags (cleared by a forward given it)][slot rows][slot index (seg,
// slot) + its scan scratch][the packed records unless the forward's are reused]
static size_t rows2_bytes(int64_t n_isects) {
    return ((size_t)n_isects * kSlotWaves * kRow2 * sizeof(float) + 255) & ~(size_t)255;
}

extern "C" size_t hgsr_raster2d_bwd_ws_bytes(int C, int N, int D, int64_t n_isects, int reuse_fwd) {
    (void)D;
    return slot_flag_bytes(n_isects, kSlotWaves) + rows2_bytes(n_isects) + grad_slot_bytes((int64_t)C * N, true, n_isects) +
           (reuse_fwd ? 0 : rec2_bytes(C, N));
}

static int raster2d_bwd_impl(int C, int N, int D, const float* means2d, const float* rt, const ChanSrc& cs,
                             const float* normals, const float* backgrounds, int bg_ch, int ed_ch,
                             const float* render_colors, int width, int height, int tile_size, int tile_w,
                             int tile_h, const int32_t* isect_offsets, int64_t n_isects, const int32_t* flatten_ids,
                             const float* render_alphas, const int32_t* last_ids, const float* v_render_colors,
                             const float* v_render_alphas, const float* v_render_normals, float* v_means2d,
                             float* v_rt, const ChanDst& cd, float* v_normals, float* v_densify,
                             const void* fwd_ws, void* ws, size_t ws_bytes, hgsr_stream_t stream, const void* qbuf = nullptr,
                             size_t qmask_bytes = 0, bool flags_zeroed = false, const float* normal_rot = nullptr,
                             const float* v_depth_extra = nullptr, const int32_t* radii = nullptr,
                             bool fwd_slots = false) {
    if (int st = check_raster2(C, N, D, width, height, tile_size, tile_w, tile_h)) return st;
    HGSR_REQUIRE(ws_bytes >= hgsr_raster2d_bwd_ws_bytes(C, N, D, n_isects, fwd_ws != nullptr),
                 "raster2d_bwd workspace too small");
    HGSR_REQUIRE(ed_ch < 0 || render_colors, "expected-depth backward needs render_colors");
    if (N == 0) return HGSR_OK;
    HGSR_REQUIRE(v_means2d && v_rt && (cd.colors || cd.dc == 0) && cd.opac && v_normals, "null pointer");
    hipStream_t s = as_stream(stream);
    const int64_t n = (int64_t)C * N;
    if (n_isects == 0) {  // nothing composited: every gradient is zero
        if (int st = memset_async(v_means2d, n * 2 * sizeof(float), s, "raster2d_bwd")) return st;
        if (int st = memset_async(v_rt, n * 9 * sizeof(float), s, "raster2d_bwd")) return st;
        if (cd.dc)
            if (int st = memset_async(cd.colors, (cd.col_shared ? N : n) * cd.dc * sizeof(float), s, "raster2d_bwd"))
                return st;
        if (cd.depths)
            if (int st = memset_async(cd.depths, n * sizeof(float), s, "raster2d_bwd")) return st;
        if (int st = memset_async(cd.opac, (cd.op_shared ? N : n) * sizeof(float), s, "raster2d_bwd")) return st;
        if (int st = memset_async(v_normals, n * 3 * sizeof(float), s, "raster2d_bwd")) return st;
        if (v_densify)
            if (int st = memset_async(v_densify, n * 2 * sizeof(float), s, "raster2d_bwd")) return st;
        return HGSR_OK;
    }
    HGSR_REQUIRE(means2d && rt && normals && isect_offsets && flatten_ids && render_alphas && last_ids &&
                     v_render_colors && v_render_alphas && v_render_normals && ws,
                 "null pointer");
    uint8_t* const flags = (uint8_t*)ws;
    float* const rows = (float*)((char*)ws + slot_flag_bytes(n_isects, kSlotWaves));
    char* const sbuf = (char*)rows + rows2_bytes(n_isects);
    const float2* m2 = reinterpret_cast<const float2*>(means2d);
    if (!flags_zeroed)  // else hgsr_raster2d_fwd_packed cleared them (bwd_ws)
        if (int st = memset_async(flags, slot_flag_bytes(n_isects, kSlotWaves), s, "raster2d_bwd")) return st;
    // the forward's records when the caller kept them, else pack again; the gradient slots as in
    // raster3d_bwd_impl (in the records from a training forward's pack, else made here)
    Rec2* rec = (Rec2*)const_cast<void*>(fwd_ws);
    if (!rec) {
        rec = (Rec2*)(sbuf + grad_slot_bytes(n, true, n_isects));
        if (int st = pack2(C, N, D, means2d, rt, cs, normals, rec, s)) return st;
    }
    GradSlots gs;
    if (fwd_ws && fwd_slots) {
        void* const slots = (char*)const_cast<void*>(fwd_ws) + rec2_bytes(C, N);
        if (int st = launch_grad_pieces(n, (const int32_t*)slots, n_isects, sbuf, s, gs, slot_prefix_npieces(slots, n),
                                        flags_zeroed))
            return st;
    } else if (int st = launch_grad_slots(C, N, means2d, radii, tile_size, tile_w, tile_h, isect_offsets, flatten_ids,
                                          n_isects, sbuf, s, gs, reinterpret_cast<int2*>(&rec->sl),
                                          sizeof(Rec2) / sizeof(int2))) {
        return st;
    }
    const int64_t n_bins = (int64_t)C * tile_w * tile_h;
    const dim3 grid((unsigned)n_bins);
    unsigned long long* const pairs = timing_pair_counter("raster2d_bwd");
    const uint64_t* const qmask = qmask_words(qbuf, n_bins);
    const int64_t qstride = qbuf ? qmask_stride_of(qmask_bytes, n_bins) : 0;
    // the forward writes the order only for a non-empty view
    const int32_t* const order = (qbuf && HGSR_TILE_ORDER && n_isects > 0) ? tile_order_of(qbuf) : nullptr;
    if (HGSR_BWD_ORDER && order) {  // tiles by the ranges the backward walks (raster3d_bwd_impl)
        void* const qb = const_cast<void*>(qbuf);
        if (int st = launch_tile_order(n_bins, isect_offsets, n_isects, nullptr, tile_order_of(qb), s,
                                       tile_end_of(qb, n_bins)))
            return st;
    }
#define LAUNCH_B2(DD)                                                                                             \
    {                                                                                                             \
        KernelTimer kt("raster2d_bwd", s);                                                                        \
        hipLaunchKernelGGL((raster2d_bwd_tp_kernel<DD>), grid, dim3(256), 0, s, C, width, height, tile_w, tile_h,  \
                           rec, backgrounds, bg_ch, ed_ch, render_colors, isect_offsets, n_isects, flatten_ids,    \
                           render_alphas, last_ids, v_render_colors, v_render_alphas, v_render_normals, rows,      \
                           flags, n_isects, pairs, qmask, qstride, normal_rot, v_depth_extra, order);              \
    }                                                                                                             \
    hipLaunchKernelGGL((reduce_pieces_kernel<15 + DD, (15 + DD + 3) / 4, kRow2, kSlotWaves>), dim3(piece_grid(gs)), \
                       dim3(256), 0, s, rows, flags, gs.seg, gs.pbase, gs.pieces, gs.npieces, gs.partial);          \
    hipLaunchKernelGGL((split2_kernel<DD>), dim3((unsigned)(((int64_t)N + 255) / 256)), dim3(256), 0, s, C, N,    \
                       rows, flags, gs.seg, gs.pbase, gs.partial, rt, m2,                                          \
                       reinterpret_cast<float2*>(v_means2d), v_rt, cd, v_normals, reinterpret_cast<float2*>(v_densify))
    switch (D) {
        case 1: LAUNCH_B2(1); break;
        case 2: LAUNCH_B2(2); break;
        case 3: LAUNCH_B2(3); break;
        default: LAUNCH_B2(4); break;
    }
#undef LAUNCH_B2
    return check_launch("raster2d_bwd");
}

extern "C" int hgsr_raster2d_bwd(int C, int N, int D, const float* means2d, const float* ray_transforms,
                                 const float* colors, const float* opacities, const float* normals,
                                 const float* backgrounds, int width, int height, int tile_size, int tile_w,
                                 int tile_h, const int32_t* isect_offsets, int64_t n_isects,
                                 const int32_t* flatten_ids, const float* render_alphas, const int32_t* last_ids,
                                 const float* v_render_colors, const float* v_render_alphas,
                                 const float* v_render_normals, float* v_means2d, float* v_ray_transforms,
                                 float* v_colors, float* v_opacities, float* v_normals, float* v_densify,
                                 const void* fwd_ws, void* ws, size_t ws_bytes, hgsr_stream_t stream) {
    const ChanSrc cs{colors, (int64_t)N * D, D, nullptr, opacities, (int64_t)N};
    const ChanDst cd{v_colors, false, D, nullptr, v_opacities, false};
    return raster2d_bwd_impl(C, N, D, means2d, ray_transforms, cs, normals, backgrounds, D, -1, nullptr, width,
                             height, tile_size, tile_w, tile_h, isect_offsets, n_isects, flatten_ids, render_alphas,
                             last_ids, v_render_colors, v_render_alphas, v_render_normals, v_means2d,
                             v_ray_transforms, cd, v_normals, v_densify, fwd_ws, ws, ws_bytes, stream);
}

extern "C" int hgsr_raster2d_bwd_fused(int C, int N, int Dc, const float* means2d, const float* ray_transforms,
                                       const float* colors, int colors_shared, const float* depths,
                                       int expected_depth, const float* opacities, int opacities_shared,
                                       const float* normals, const float* backgrounds, int width, int height,
                                       int tile_size, int tile_w, int tile_h, const int32_t* isect_offsets,
                                       int64_t n_isects, const int32_t* flatten_ids, const float* render_colors,
                                       const float* render_alphas, const int32_t* last_ids,
                                       const float* v_render_colors, const float* v_render_alphas,
                                       const float* v_render_normals, float* v_means2d, float* v_ray_transforms,
                                       float* v_colors, float* v_depths, float* v_opacities, float* v_normals,
                                       float* v_densify, const void* fwd_ws, void* ws, size_t ws_bytes,
                                       const void* qmask, size_t qmask_bytes, int ws_zeroed,
                                       const float* normal_rot, const float* v_depth_extra, const int32_t* radii,
                                       int fwd_slots, hgsr_stream_t stream) {
    HGSR_REQUIRE(Dc >= 0 && Dc <= 4 && (Dc > 0 || depths), "fused raster: 0..4 colour channels (got %d)", Dc);
    HGSR_REQUIRE(!(expected_depth && !depths), "expected_depth needs depths");
    HGSR_REQUIRE(!depths || v_depths, "null pointer");
    HGSR_REQUIRE(!v_depth_extra || depths, "v_depth_extra needs the depth channel");
    HGSR_REQUIRE(!qmask || qmask_bytes >= hgsr_raster3d_qmask_bytes(C, tile_w, tile_h, n_isects),
                 "raster2d_bwd_fused: quadrant-mask buffer too small");
    const int D = Dc + (depths ? 1 : 0);
    const ChanSrc cs{colors, colors_shared ? 0 : (int64_t)N * Dc, Dc, depths, opacities,
                     opacities_shared ? 0 : (int64_t)N};
    const ChanDst cd{v_colors, colors_shared != 0, Dc, depths ? v_depths : nullptr, v_opacities,
                     opacities_shared != 0};
    return raster2d_bwd_impl(C, N, D, means2d, ray_transforms, cs, normals, backgrounds, Dc,
                             expected_depth ? Dc : -1, render_colors, width, height, tile_size, tile_w, tile_h,
                             isect_offsets, n_isects, flatten_ids, render_alphas, last_ids, v_render_colors,
                             v_render_alphas, v_render_normals, v_means2d, v_ray_transforms, cd, v_normals,
                             v_densify, fwd_ws, ws, ws_bytes, stream, qmask, qmask_bytes,
                             ws_zeroed != 0, normal_rot, v_depth_extra, radii, fwd_slots != 0);
}
