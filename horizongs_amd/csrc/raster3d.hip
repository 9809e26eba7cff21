// K8/K9: 3DGS tile rasterization, forward and backward (gsplat
// rasterize_to_pixels semantics, as reached from reference
// gaussian_renderer/render.py:40-54).
//
// CDNA4 mapping
//  * one 256-lane workgroup per 16x16 tile = four wave64s, each owning an 8x8
//    quadrant (compact footprint -> more wave-uniform skips in the backward);
//  * the Gaussians' raster attributes are first packed into 48-B records
//    {x, y, a, b | c, opacity | colour[4]} (one coalesced pass over N), so a batch
//    load is 3 x 16-B loads per Gaussian instead of 5 scattered gathers;
//  * batches of the tile's depth-sorted list are register-prefetched one batch
//    ahead (global latency hidden under the current batch) and staged in LDS,
//    read back as wave-wide broadcasts;
//  * inner loops are branch-free (predicated per lane) with a wave-uniform
//    early exit, so the scalar unit is not saturated by exec-mask bookkeeping;
//  * backward: replay back-to-front bounded by the tile's latest contributor,
//    wave-ballot skip of Gaussians no lane sees, all gradient components
//    reduced across the wave together (step-major DPP, no hazard stalls), and
//    each wave's sums stored as one 64-B row in the (tile, Gaussian) pair's own
//    gradient slot (one plain store per 4 steps, no atomics); split3 sums each
//    Gaussian's slots in a fixed order, so the gradients are bit-reproducible.
#include "rec3.h"

namespace hgsr {

constexpr int kFwdBatch = 256;
constexpr int kBwdBatch = 128;
// floats per gradient-slot row (64 B, one full sector per store): sigma moments Sx Sy Sxx Sxy Syy
// at 0-4, S0 = sum v_sigma at 5, colour channel k at 6 + k, |v_xy| at 10-11 (absgrad), 12-15 zero
constexpr int kRow3 = 16;

struct TileCtx {
    int cam, tile, i, j;
    bool inside;
    float px, py;
    int32_t start, end;
    int64_t pix;
};

// info (nullable): the device-resident {n_isects, largest bin, overflow} of a deferred
// intersection count (hgsr_isect_emit_sorted with isect_info): the last bin ends at info[0],
// and an overflowed emission (capacity exceeded; the host re-runs it) leaves every tile empty
__device__ __forceinline__ TileCtx tile_ctx(int C, int W, int H, int tw, int th,
                                            const int32_t* __restrict__ offsets, int64_t n_isects,
                                            const int64_t* __restrict__ info, const int32_t* __restrict__ order) {
    TileCtx t;
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

// sigma' of a record at offset (dx, dy), factored as dx (a' dx + b' dy) + (c' dy) dy
__device__ __forceinline__ float sigma2(const float4 g0, const float4 g1, float dx, float dy) {
    const float h = __builtin_fmaf(g0.w, dy, g0.z * dx);
    return __builtin_fmaf(g1.x * dy, dy, dx * h);
}

// One workgroup packs 256 consecutive (camera, Gaussian) records; the conics (12 B each)
// come in and the 64-B records leave as contiguous float4 runs through LDS (lane-strided
// AoS loads / stores touch ~12-48 cache lines per instruction): 37.6 -> 29.3 us at c2 (48-B
// records).  SLOTS (a forward a backward follows): the workgroup's 256 entries are one row of
// the slot-area prefix (launch_slot_prefix summed and scanned the rows), so a block scan of the
// rectangles' areas gives seg and each record's gradient-slot base here, written with the record
// instead of scattered into the records by the backward (8 B into each 64-B record: 60 us at c2);
// else the slot quad is zero.
template <int D, bool SLOTS>
__global__ __launch_bounds__(256) void pack3_kernel(int64_t n, int N, const float2* __restrict__ means2d,
                                                    const float* __restrict__ conics, ChanSrc cs,
                                                    Rec3* __restrict__ rec, RectFromRadii rr,
                                                    const int32_t* __restrict__ bpre, int32_t* __restrict__ seg) {
    constexpr int kOP = 17;  // record pitch in LDS (16 floats + 1: conflict-free lane stride)
    __shared__ __attribute__((aligned(16))) float s_buf[256 * kOP];
    const int64_t i0 = (int64_t)blockIdx.x * 256;
    const int nloc = (int)min((int64_t)256, n - i0);
    const int t = threadIdx.x;
    const int64_t i = i0 + t;
    stage_floats(conics + i0 * 3, nloc * 3, s_buf);
    int4 sl = make_int4(0, 0, 0, 0);
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
    const float a = s_buf[t * 3], b = s_buf[t * 3 + 1], cc = s_buf[t * 3 + 2];
    if (SLOTS && t < nloc) {
        int e = bpre[blockIdx.x] + inc - area;
#pragma unroll
        for (int v = 0; v < 4; ++v) e += v < (t >> 6) ? s_ws[v] : 0;
        seg[i] = e;
        sl = make_int4(e - y0 * w - x0, w, 0, 0);
    }
    __syncthreads();  // s_buf now holds the records
    if (t < nloc) {
        const int64_t c = i / N, g = i - c * N;
        const float2 m = means2d[i];
        const float o = cs.opac[c * cs.op_cstride + g];
        float col[4] = {0.f, 0.f, 0.f, 0.f};
        const float* src = cs.colors + c * cs.col_cstride + g * cs.dc;
#pragma unroll
        for (int k = 0; k < D; ++k) col[k] = k < cs.dc ? src[k] : cs.depths[i];
        Rec3 r = make_rec3(m, a, b, cc, o, col);
        r.sl = sl;
        const float v[16] = {r.g0.x, r.g0.y, r.g0.z, r.g0.w, r.g1.x, r.g1.y, r.g1.z, r.g1.w,
                             r.col.x, r.col.y, r.col.z, r.col.w, __int_as_float(r.sl.x), __int_as_float(r.sl.y),
                             __int_as_float(r.sl.z), __int_as_float(r.sl.w)};
#pragma unroll
        for (int k = 0; k < 16; ++k) s_buf[t * kOP + k] = v[k];
    }
    __syncthreads();
    float4* dst = reinterpret_cast<float4*>(rec + i0);
    for (int q = t; q < nloc * 4; q += 256) {
        const int e = q >> 2, f = q & 3;
        const float* p = s_buf + e * kOP + 4 * f;
        dst[q] = make_float4(p[0], p[1], p[2], p[3]);
    }
}

// does the footprint box of (g0, g1) reach the 8x8 quadrant centred at (qx, qy)?
__device__ __forceinline__ bool reaches(const float4 g0, const float4 g1, float qx, float qy) {
    return fabsf(g0.x - qx) <= g1.z + 3.5f && fabsf(g0.y - qy) <= g1.w + 3.5f;
}

// Exact refinement of reaches(): the minimum of sigma' = a'dx^2 + b'dx dy + c'dy^2 over
// the quadrant's pixel-centre rectangle (dx = x - px, px in qx +- 3.5) against the alpha
// >= 1/255 level sigma' <= log2(255 o).  A convex quadratic attains its minimum over a
// rectangle at the origin (if inside) or on an edge, where it is a 1-D parabola minimised
// in closed form.  Conservative: a relative + absolute slack covers the rounding of the
// per-pixel evaluation and of v_exp_f32, so a skipped record has alpha < 1/255 at every
// pixel of the quadrant (forward and backward skip the same records).
__device__ __forceinline__ bool ellipse_reaches(const float4 g0, const float4 g1, float qx, float qy) {
    const float cx = g0.x - qx, cy = g0.y - qy;
    const float x0 = cx - 3.5f, x1 = cx + 3.5f, y0 = cy - 3.5f, y1 = cy + 3.5f;
    const float a = g0.z, b = g0.w, c = g1.x;
    const float lim = __builtin_amdgcn_logf(255.0f * g1.y);  // log2
    const float ia = -0.5f * __builtin_amdgcn_rcpf(a), ic = -0.5f * __builtin_amdgcn_rcpf(c);
    auto q = [&](float dx, float dy) { return a * dx * dx + b * dx * dy + c * dy * dy; };
    const float dya = fminf(fmaxf(b * x0 * ic, y0), y1), dyb = fminf(fmaxf(b * x1 * ic, y0), y1);
    const float dxa = fminf(fmaxf(b * y0 * ia, x0), x1), dxb = fminf(fmaxf(b * y1 * ia, x0), x1);
    float m = fminf(fminf(q(x0, dya), q(x1, dyb)), fminf(q(dxa, y0), q(dxb, y1)));
    const bool inside = x0 <= 0.f && x1 >= 0.f && y0 <= 0.f && y1 >= 0.f;
    m = inside ? 0.f : m;
    return m <= lim + 1e-3f * fabsf(lim) + 1e-3f;
}

__device__ __forceinline__ int lanes_below(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
}

// one front-to-back compositing step, branch-free (predicated per lane).  A lane
// that has stopped (gsplat: the Gaussian that would push T to <= 1e-4 ends the pixel,
// exclusively) carries T negated, so "done" costs no separate flag: its next T is
// negative, never kept, and |T| is the final transmittance.
template <int D>
__device__ __forceinline__ void fwd_step(const float4 g0, const float4 g1, const float4 c, uint32_t idx, float px,
                                         float py, float& T, float (&acc)[4], uint32_t& cur) {
    const float dx = g0.x - px, dy = g0.y - py;
    const float sigma = sigma2(g0, g1, dx, dy);
    const float alpha = fminf(0.999f, g1.y * __builtin_amdgcn_exp2f(-sigma));
    const float nT = T * (1.0f - alpha);
    const bool valid = (sigma >= 0.f) & (alpha >= 1.0f / 255.0f);
    const bool ok = valid & (nT > 1e-4f);  // T < 0 (stopped) gives nT < 0
    const float vis = ok ? alpha * T : 0.f;
    acc[0] += c.x * vis;
    if (D > 1) acc[1] += c.y * vis;
    if (D > 2) acc[2] += c.z * vis;
    if (D > 3) acc[3] += c.w * vis;
    T = ok ? nT : (valid ? -fabsf(T) : T);
    cur = ok ? idx : cur;
}

template <int D>
__global__ __launch_bounds__(256) void raster3d_fwd_kernel(
    int C, int W, int H, int tw, int th, const Rec3* __restrict__ rec, const float* __restrict__ backgrounds,
    int bg_ch, int ed_ch, const int32_t* __restrict__ offsets, int64_t n_isects,
    const int32_t* __restrict__ flatten_ids, float* __restrict__ render_colors, float* __restrict__ render_alphas,
    int32_t* __restrict__ last_ids, uint64_t* __restrict__ qmask, int64_t qstride, float4* __restrict__ zero_rows,
    int64_t zero_n4, const int64_t* __restrict__ isect_info, const int32_t* __restrict__ order,
    int32_t* __restrict__ tile_end) {
    // slot kFwdBatch is a zero-opacity dummy used to pad the per-wave lists
    __shared__ float4 s_g0[kFwdBatch + 1];
    __shared__ float4 s_g1[kFwdBatch + 1];
    __shared__ float4 s_col[kFwdBatch + 1];
    // per-wave compacted lists hold LDS byte offsets (16 x slot) of the records: the
    // list read yields the record addresses directly and the last-contributor update
    // keeps the offset, rebased once per batch
    __shared__ uint32_t s_list[4][kFwdBatch + 4];
    __shared__ int s_vote[2][4];
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const TileCtx tc = tile_ctx(C, W, H, tw, th, offsets, n_isects, isect_info, order);
    const float qx = (float)(tc.j - (lane & 7)) + 4.0f;   // centre of this wave's quadrant
    const float qy = (float)(tc.i - (lane >> 3)) + 4.0f;
    if (tid == 0) {
        s_g0[kFwdBatch] = make_float4(0.f, 0.f, 0.f, 0.f);
        s_g1[kFwdBatch] = make_float4(0.f, 0.f, -1e30f, -1e30f);
        s_col[kFwdBatch] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
    float T = tc.inside ? 1.0f : -1.0f;  // negative = stopped
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    int32_t cur = 0;
    const int nb = (tc.end - tc.start + kFwdBatch - 1) / kFwdBatch;
    // two-deep software pipeline of the batch loads: ids two batches ahead,
    // records one batch ahead; indices are clamped so every load is unconditional
    // (no phi copies forcing an early vmcnt wait)
    const int32_t last = tc.end - 1;
    float4 n0 = make_float4(0.f, 0.f, 0.f, 0.f), n1 = n0, n2 = n0;
    int32_t nid = 0;
    if (nb > 0) {
        const int32_t id0 = flatten_ids[min(tc.start + tid, last)];
        const float4* r = reinterpret_cast<const float4*>(rec + id0);
        n0 = r[0]; n1 = r[1]; n2 = r[2];
        nid = flatten_ids[min(tc.start + kFwdBatch + tid, last)];
    }
    uint32_t* my_list = s_list[wave];
    const char* lds_g0 = reinterpret_cast<const char*>(s_g0);
    const char* lds_g1 = reinterpret_cast<const char*>(s_g1);
    const char* lds_col = reinterpret_cast<const char*>(s_col);
    for (int b = 0; b < nb; ++b) {
        // workgroup early-out vote (double-buffered slots; LDS-only barriers so the
        // prefetch loads stay in flight)
        const bool wave_done = __all(T < 0.f);
        if (lane == 0) s_vote[b & 1][wave] = wave_done;
        lds_barrier();
        if (s_vote[b & 1][0] & s_vote[b & 1][1] & s_vote[b & 1][2] & s_vote[b & 1][3]) break;
        const int32_t bs = tc.start + b * kFwdBatch;
        const int cnt = min(kFwdBatch, tc.end - bs);
        if (tid < cnt) {
            s_g0[tid] = n0;
            s_g1[tid] = n1;
            s_col[tid] = n2;
        }
        lds_barrier();
        // prefetch: records of batch b+1 (ids already here), ids of batch b+2
        {
            const float4* r = reinterpret_cast<const float4*>(rec + nid);
            n0 = r[0]; n1 = r[1]; n2 = r[2];
            nid = flatten_ids[min(bs + 2 * kFwdBatch + tid, last)];
        }
        if (wave_done) continue;
        // order-preserving compaction of the batch to the Gaussians that can reach
        // this wave's quadrant (each lane tests 4 of them)
        int n_mine = 0;
        // quadrant mask words of this batch (read by the backward), one per 64 records
        uint64_t* const qw = qmask ? qmask + wave * qstride + qmask_word0(tc.start, (int64_t)tc.cam * (tw * th) + tc.tile) +
                                         (int64_t)b * (kFwdBatch / 64)
                                   : nullptr;
#pragma unroll
        for (int k = 0; k < kFwdBatch / 64; ++k) {
            const int t = k * 64 + lane;
            const bool rel = t < cnt && reaches(s_g0[t], s_g1[t], qx, qy) && ellipse_reaches(s_g0[t], s_g1[t], qx, qy);
            const uint64_t m = __ballot(rel);
            if (rel) my_list[n_mine + lanes_below(m)] = (uint32_t)t * 16u;
            n_mine += __popcll(m);
            if (qw && lane == k && k * 64 < cnt) qw[k] = m;  // only words holding records of this tile
        }
        if (lane < 4) my_list[n_mine + lane] = (uint32_t)kFwdBatch * 16u;  // pad to a multiple of 4
        uint32_t cur_off = 0xffffffffu;  // byte offset of this batch's latest contributor, if any
        for (int i = 0; i < n_mine; i += 4) {
            const uint4 o = *reinterpret_cast<const uint4*>(my_list + i);
            auto ld = [](const char* base, uint32_t off) { return *reinterpret_cast<const float4*>(base + off); };
            const float4 a0 = ld(lds_g0, o.x), a1 = ld(lds_g0, o.y), a2 = ld(lds_g0, o.z), a3 = ld(lds_g0, o.w);
            const float4 b0 = ld(lds_g1, o.x), b1 = ld(lds_g1, o.y), b2 = ld(lds_g1, o.z), b3 = ld(lds_g1, o.w);
            const float4 c0 = ld(lds_col, o.x), c1 = ld(lds_col, o.y), c2 = ld(lds_col, o.z), c3 = ld(lds_col, o.w);
            fwd_step<D>(a0, b0, c0, o.x, tc.px, tc.py, T, acc, cur_off);
            fwd_step<D>(a1, b1, c1, o.y, tc.px, tc.py, T, acc, cur_off);
            fwd_step<D>(a2, b2, c2, o.z, tc.px, tc.py, T, acc, cur_off);
            fwd_step<D>(a3, b3, c3, o.w, tc.px, tc.py, T, acc, cur_off);
            if (__all(T < 0.f)) break;
        }
        if (cur_off != 0xffffffffu) cur = bs + (int32_t)(cur_off >> 4);
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
        last_ids[tc.pix] = cur;
    }
    if (tile_end) {
        // the tile's latest contributor + 1 (the backward's trimmed range, for its tile order)
        int32_t m = tc.inside ? cur : -1;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) m = max(m, __shfl_xor(m, d));
        __shared__ int32_t s_end[4];
        if (lane == 0) s_end[wave] = m;
        __syncthreads();
        if (tid == 0)
            tile_end[(int64_t)tc.cam * (tw * th) + tc.tile] = max(max(s_end[0], s_end[1]), max(s_end[2], s_end[3])) + 1;
    }
    // the backward's accumulator rows, cleared here (after the last load: no wait covers
    // these stores) instead of by a memset on the step's critical path
    zero_share(zero_rows, zero_n4);
}

__device__ __forceinline__ int32_t wave_max_i32(int32_t v) {
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) v = max(v, __shfl_xor(v, d));
    return v;
}

// Backward "input transpose".  Per step a wave composites one Gaussian over its 8x8
// quadrant (pass 1) and keeps only two numbers per pixel: fac = alpha T (the colour
// weight) and v_sigma.  Every 4 steps the 4 x 2 registers are transposed across the
// wave through LDS (four 8-B writes, two 16-B reads per lane; measured 623-635 -> 585 us
// at c2 against eight v_permlane32/16_swap, which cost ~3 VALU slots each) so that lane
// L = 16 s + r holds step s's
// values for the 4 pixels r + 16 m (m = 0..3) -- one pixel column, rows y0, y0+2, y0+4,
// y0+6 -- and accumulates the 10 gradient values of that Gaussian over them in
// registers (pass 2).  With dx constant down a column the sigma moments factor:
//   Sx = dx S0, Sxx = dx^2 S0, Sxy = dx Sy,  S0 = sum v_sigma, Sy = sum v_sigma dy,
//   Syy = sum v_sigma dy^2,
// and the opacity gradient sum vis va = -S0 / opacity is formed once per Gaussian in
// split3.  A 16-lane DPP tree finishes the sums (colours pre-permuted per lane class so
// that the first two levels transpose instead of add).  Two transposed inputs replace
// the ten reduced outputs of a per-step wave reduction.

// 7 waves / SIMD: the LDS transpose buffer (8 KB per workgroup) allows 7 workgroups per CU;
// 72 VGPRs (two spilled values outside the step loop)
#ifndef HGSR_BWD_WAVES_N
#define HGSR_BWD_WAVES_N 7
#endif
#if HGSR_BWD_WAVES_N > 0
#define HGSR_BWD_WAVES __attribute__((amdgpu_waves_per_eu(HGSR_BWD_WAVES_N, 8)))
#else
#define HGSR_BWD_WAVES
#endif
struct Pass2Lane {
    float pxc, py0c;         // pixel-centre x of this lane's column, y of its first row
    float vo[4][4];          // [m][slot]: upstream colour gradient of pixel m, lane-permuted channels
};

#if HGSR_PROBE_WAIT
// raster3d_bwd's wait sites (scripts/micro/wait_probe.py): 0 setup, 1 batch-top vmcnt wait, 2 DMA /
// slot issue, 3 first barrier, 4 compaction, 5 steps + pass 2, 6 second barrier, 7 tail; [8] waves
__device__ unsigned long long g_wait_bwd3[16];
extern "C" int hgsr_probe_wait_read(unsigned long long* host, int reset) {
    if (hipMemcpyFromSymbol(host, HIP_SYMBOL(g_wait_bwd3), sizeof(g_wait_bwd3)) != hipSuccess) return 1;
    if (reset) {
        static const unsigned long long zero[16] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_wait_bwd3), zero, sizeof(zero)) != hipSuccess) return 1;
    }
    return 0;
}
#endif

template <int D, bool ABS>
__global__ __launch_bounds__(256) HGSR_BWD_WAVES void raster3d_bwd_kernel(
    int C, int W, int H, int tw, int th, const Rec3* __restrict__ rec, const float* __restrict__ backgrounds,
    int bg_ch, int ed_ch, const float* __restrict__ render_colors, const int32_t* __restrict__ offsets,
    int64_t n_isects, const int32_t* __restrict__ flatten_ids, const float* __restrict__ render_alphas,
    const int32_t* __restrict__ last_ids, const float* __restrict__ v_render_colors,
    const float* __restrict__ v_render_alphas, float* __restrict__ rows, uint8_t* __restrict__ flags,
    int64_t n_slots, unsigned long long* __restrict__ pair_counter,
    const uint64_t* __restrict__ qmask, int64_t qstride, const int32_t* __restrict__ order,
    const int32_t* __restrict__ tile_end) {
    constexpr int NB = kBwdBatch;
    HGSR_WP_DECL(g_wait_bwd3);
    // double-buffered staging: batch b+1 is loaded while batch b is composited (two
    // barriers per batch); slot NB is a zero-opacity dummy
    // one LDS object, so every component of record t sits at a compile-time offset from one
    // address; filled by LDS-DMA (no staging VGPRs)
    __shared__ struct {
        float4 g0[2][NB + 1], g1[2][NB + 1], col[2][NB + 1];
    } sr;
    __shared__ int32_t s_e[2][NB];  // the batch's records' gradient slots (-1: none)
    __shared__ __attribute__((aligned(16))) uint8_t s_list[4][NB];  // read back as 32-bit words
    __shared__ int32_t s_last[4];
    // pass-1 -> pass-2 transpose through LDS: [step s][column lane r][pixel m][F, V]
    __shared__ __attribute__((aligned(16))) float s_tp[4][4 * 16 * 4 * 2];
    const TileCtx tc = tile_ctx(C, W, H, tw, th, offsets, n_isects, nullptr, order);
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const float qx = (float)(tc.j - (lane & 7)) + 4.0f;
    const float qy = (float)(tc.i - (lane >> 3)) + 4.0f;
    const int tile_y = tc.tile / tw, tile_x = tc.tile - tile_y * tw;
    // per-pixel upstream terms of pixel (i, j); the ED channel is divided by max(alpha, 1e-10)
    auto pixel_terms = [&](int i, int j, float (&v)[4], float& vterm) {
        const bool in = i < H && j < W;
        const int64_t pix = ((int64_t)tc.cam * H + i) * W + j;
        const float Tf = in ? 1.0f - render_alphas[pix] : 1.0f;
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] = (in && k < D) ? v_render_colors[pix * D + k] : 0.f;
        float va = in ? v_render_alphas[pix] : 0.f;
        if (ed_ch >= 0 && in) {
            // ED = raw / max(alpha, 1e-10): d/d raw = 1/ac, d/d alpha = -ED/ac (alpha >= 1e-10)
            const float alpha = 1.0f - Tf, ac = fmaxf(alpha, 1e-10f);
            float v_ed = 0.f;
#pragma unroll
            for (int k = 0; k < D; ++k)
                if (k == ed_ch) {
                    v_ed = v[k];
                    v[k] = v_ed / ac;
                }
            if (alpha >= 1e-10f) va -= v_ed * render_colors[pix * D + ed_ch] / ac;
        }
        float bg_dot = 0.f;
#pragma unroll
        for (int k = 0; k < D; ++k)
            if (backgrounds && k < bg_ch) bg_dot += backgrounds[tc.cam * bg_ch + k] * v[k];
        vterm = Tf * (va - bg_dot);  // multiplied by ra per Gaussian
        return Tf;
    };
    float vo[4], va_term;
    const float T_final = pixel_terms(tc.i, tc.j, vo, va_term);
    float T = T_final;
    // B = sum_k buf_k * vo_k, the upstream-weighted colour composited behind the
    // current Gaussian: v_alpha only ever needs this dot product, never buf_k itself
    float B = 0.f;
    // pass-2 role of this lane: column cx = r & 7, rows y0 + 2m of the quadrant
    const int r16 = lane & 15, cx = r16 & 7, y0 = r16 >> 3;
    const int qi0 = tc.i - (lane >> 3), qj0 = tc.j - (lane & 7);  // quadrant origin
    Pass2Lane p2;
    p2.pxc = (float)(qj0 + cx) + 0.5f;
    p2.py0c = (float)(qi0 + y0) + 0.5f;
    {
        // colour slots permuted by lane class (bit 3, bit 2 of r) so the first two DPP
        // levels of the 16-lane tree transpose (see the reduction below):
        // class (b3,b2) = (0,0): 0 1 2 3, (1,0): 1 0 3 2, (0,1): 2 3 0 1, (1,1): 3 2 1 0
        const int perm = ((r16 >> 3) & 1) | (((r16 >> 2) & 1) << 1);
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            float v[4], vt;
            pixel_terms(qi0 + y0 + 2 * m, qj0 + cx, v, vt);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int k = q ^ perm;
                p2.vo[m][q] = k == 0 ? v[0] : k == 1 ? v[1] : k == 2 ? v[2] : v[3];
            }
        }
    }
    const int32_t bin_final = tc.inside ? last_ids[tc.pix] : -1;
    if (tid < 6) {
        const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
        sr.g0[tid >> 1][NB] = z;  // both buffers' dummy records: opacity 0, never composited
        sr.g1[tid >> 1][NB] = z;
        sr.col[tid >> 1][NB] = z;  // (published by the first batch's barrier)
    }
    // the tile's latest contributor: the forward's tile_end when it kept one (a load issued with
    // the tile's offsets, so the first ids and DMA do not wait for the pixels' last ids and a
    // workgroup barrier), else the maximum of the pixels' last ids
    int32_t blk_final;
    if (tile_end) {
        blk_final = __builtin_amdgcn_readfirstlane(tile_end[(int64_t)tc.cam * (tw * th) + tc.tile]) - 1;
    } else {
        const int32_t wf = wave_max_i32(bin_final);
        if (lane == 0) s_last[wave] = wf;
        lds_barrier();
        blk_final = max(max(s_last[0], s_last[1]), max(s_last[2], s_last[3]));
    }
    // Gaussians after the block's last contributor are never reached
    const int32_t end = min(tc.end, blk_final + 1);
    const int nb = end > tc.start ? (end - tc.start + NB - 1) / NB : 0;
    if (pair_counter && threadIdx.x == 0 && end > tc.start)  // measurement only (bench roofline)
        atomicAdd(pair_slot(pair_counter, 0), (unsigned long long)(end - tc.start) * kTilePixels);
    // records are staged with LDS-DMA (global_load_lds_dwordx4: per-lane source, LDS
    // destination wave base + 16 B x lane) one batch ahead; ids two batches ahead in a
    // register; lanes < NB (waves 0, 1) load one Gaussian each, clamped indices; with each record
    // its slot base {seg - y0 w - x0, w} (Rec3::sl, the same 64-B sector as the DMA: an L2 hit),
    // so the record's gradient slot is base + y w + x
    int32_t cid = 0, nid = 0;
    int2 csl = make_int2(-1, 0);
    const bool loader = tid < NB;
    auto dma_batch = [&](int buf, int32_t id) {
        const float4* r = reinterpret_cast<const float4*>(rec + id);
        const int w0 = tid & ~63;
        lds_dma16(r, &sr.g0[buf][w0]);
        lds_dma16(r + 1, &sr.g1[buf][w0]);
        lds_dma16(r + 2, &sr.col[buf][w0]);
    };
    if (nb > 0 && loader) {
        cid = flatten_ids[max(end - 1 - tid, tc.start)];
        dma_batch(0, cid);
        csl = *reinterpret_cast<const int2*>(&rec[cid].sl);
        nid = flatten_ids[max(end - 1 - NB - tid, tc.start)];
    }
    uint8_t* my_list = s_list[wave];
    uint32_t stepped = 0;  // compacted list entries this wave stepped (bench roofline only)
    const int gsl = lane >> 4;  // pass-2 Gaussian (list entry of the 4-step group) of this lane
    // pass-2 output lane roles: after the 16-lane tree every lane of a row holds the six
    // sigma sums (and |v_xy|) and each quad one colour channel; lane r16 = 4 q + 3 adds its
    // quad's channel, lanes 0-2 / 4-6 the sums 0-2 / 3-5, lanes 8 / 9 the |v_xy| pair (ABS)
    const int qlo = r16 & 3;
    const bool qb2 = (r16 >> 2) & 1, qsel1 = qlo == 1, qsel2 = qlo == 2, qcol = qlo == 3;
    const int koff = qlo == 3 ? 6 + ((r16 >> 3) | ((r16 >> 1) & 2))
                   : r16 < 8  ? qlo + (qb2 ? 3 : 0)
                   : (ABS && r16 == 8) ? 10
                   : (ABS && r16 == 9) ? 11 : -1;
    // the row position lane r16 stores: koff, the unused lanes 8-10 (without ABS 8, 9) and 12-14
    // on 10-15, so the 16 lanes of a Gaussian write one whole 64-B row
    const int spos = (int)((0x9FED7CBA85436210ull >> (4 * r16)) & 15);
    // quadrant-mask words of batch bb: wave-uniform index, so they are scalar loads
    uint64_t qw[3] = {0, 0, 0};
    auto qfetch = [&](int bb) {
        const int64_t lo = (end - 1 - (int64_t)bb * NB - tc.start) - (NB - 1);
        const int64_t bin = (int64_t)tc.cam * (tw * th) + tc.tile;
        const int idx = __builtin_amdgcn_readfirstlane(
            (int)(__builtin_amdgcn_readfirstlane(wave) * qstride + qmask_word0(tc.start, bin) + (lo >> 6)));
        const uint64_t* qp = qmask + idx;
        qw[0] = qp[0];
        qw[1] = qp[1];
        qw[2] = qp[2];
    };
    if (qmask && nb > 0) qfetch(0);
    // this quadrant's latest contributor (after the first batch's loads are out)
    const int32_t wave_final = wave_max_i32(bin_final);
    HGSR_WP_MARK(0);
    for (int b = 0; b < nb; ++b) {
        const int cur = b & 1, prv = cur ^ 1;
        const int32_t batch_end = end - 1 - b * NB;
        const int bsz = min(NB, batch_end + 1 - tc.start);
        // batch b's DMA (issued one iteration ago, before batch b-1's gradient atomics) lands
        // before the barrier below publishes it; then DMA batch b+1 into the other buffer
        // (its previous records were last read before the previous barrier)
        __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt(0)
        HGSR_WP_MARK(1);
        if (tid < bsz) {
            const int64_t e = (int64_t)csl.x + (int64_t)tile_y * csl.y + tile_x;
            s_e[cur][tid] = (e >= 0 && e < n_slots) ? (int32_t)e : -1;  // (inconsistent lists: no store)
        }
        if (b + 1 < nb && loader) {
            cid = nid;
            dma_batch(prv, cid);
            csl = *reinterpret_cast<const int2*>(&rec[cid].sl);
            nid = flatten_ids[max(batch_end - 2 * NB - tid, tc.start)];
        }
        HGSR_WP_MARK(2);
        lds_barrier();
        HGSR_WP_MARK(3);
        // phase 2: composite batch b, first the per-wave list of its records that reach this
        // quadrant and are not behind every pixel's last contributor (order-preserving)
        const int t0 = max(0, batch_end - wave_final);
        int n_mine = 0;
        if (qmask) {
            // the forward's culling bits: record t <-> tile-relative bit R - t, R = batch_end -
            // start; the 128-bit window [R - 127, R] (3 words, prefetched one batch ahead) is
            // realigned and bit-reversed
            const int64_t R = batch_end - tc.start, lo = R - (NB - 1);
            const uint64_t w0 = qw[0], w1 = qw[1], w2 = qw[2];
            if (b + 1 < nb) qfetch(b + 1);  // scalar loads, done long before the next batch
            const int sh = (int)(lo & 63);
            const uint64_t wlo = sh ? (w0 >> sh) | (w1 << (64 - sh)) : w0;
            const uint64_t whi = sh ? (w1 >> sh) | (w2 << (64 - sh)) : w1;
            uint64_t mk[2] = {__builtin_bitreverse64(whi), __builtin_bitreverse64(wlo)};
#pragma unroll
            for (int k = 0; k < 2; ++k) {  // keep t in [t0, bsz)
                const int a = min(max(t0 - 64 * k, 0), 64), z = min(max(bsz - 64 * k, 0), 64);
                const uint64_t below_z = z >= 64 ? ~0ull : ((1ull << z) - 1);
                const uint64_t below_a = a >= 64 ? ~0ull : ((1ull << a) - 1);
                mk[k] &= below_z & ~below_a;
                // (uint32_t casts: readfirstlane returns int, which would sign-extend)
                const uint64_t m = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)mk[k]) |
                                   ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(mk[k] >> 32)) << 32);
                if ((m >> lane) & 1) my_list[n_mine + lanes_below(m)] = (uint8_t)(k * 64 + lane);
                n_mine += __popcll(m);
            }
        } else {
            // order-preserving compaction to the Gaussians that reach this quadrant and
            // are not behind every pixel's last contributor
#pragma unroll
            for (int k = 0; k < NB / 64; ++k) {
                const int t = k * 64 + lane;
                const bool rel = t < bsz && t >= t0 && reaches(sr.g0[cur][t], sr.g1[cur][t], qx, qy) &&
                                 ellipse_reaches(sr.g0[cur][t], sr.g1[cur][t], qx, qy);
                const uint64_t m = __ballot(rel);
                if (rel) my_list[n_mine + lanes_below(m)] = (uint8_t)t;
                n_mine += __popcll(m);
            }
        }
        // padded with the dummy to a multiple of 4
        if (lane < 4 && n_mine + lane < NB) my_list[n_mine + lane] = (uint8_t)NB;
        stepped += (uint32_t)n_mine;
        HGSR_WP_MARK(4);
        if (n_mine > 0) {
            // the list comes back into registers once per batch; the loop reads
            // entries with readlane so no LDS index read sits on the critical path
            // (four 8-bit entries per lane: lanes 0-31 hold the whole list)
            const uint32_t lstp = reinterpret_cast<const uint32_t*>(my_list)[lane & 31];
            // pass 1: composite record t for this lane's pixel (branch-free: a padding entry
            // is the zero-opacity dummy and composites nothing); returns fac and v_sigma
            auto step = [&](const int t, float& F, float& V) {
                const float4 g0 = sr.g0[cur][t], g1 = sr.g1[cur][t], c = sr.col[cur][t];
                const float dx = g0.x - tc.px, dy = g0.y - tc.py;
                const float sigma = sigma2(g0, g1, dx, dy);
                const float vis = __builtin_amdgcn_exp2f(-sigma);
                const float araw = g1.y * vis;
                const float alpha = fminf(0.999f, araw);
                const bool valid = (batch_end - t <= bin_final) & (sigma >= 0.f) & (alpha >= 1.0f / 255.0f);
                const float ck[4] = {c.x, c.y, c.z, c.w};
                // an invalid lane composites alpha = 0: T, fac and B come out unchanged
                const float al = valid ? alpha : 0.f;
                const float ra = __builtin_amdgcn_rcpf(1.0f - al);
                const float Tn = T * ra;
                const float fac = al * Tn;
                float cv = ck[0] * vo[0];
#pragma unroll
                for (int k = 1; k < D; ++k) cv += ck[k] * vo[k];
                const float v_alpha = Tn * cv + ra * (va_term - B);
                B += fac * cv;
                // alpha clamped at 0.999 (or not composited): no gradient through it
                const float va2 = (valid & (araw <= 0.999f)) ? v_alpha : 0.f;
                T = Tn;
                F = fac;
                V = -araw * va2;  // dL/dsigma (unscaled sigma)
            };
            // pass 2 over 4 composited steps (records ts[0..3], values F/V in pass-1 layout)
            auto pass2 = [&](const uint32_t packed, float (&F)[4], float (&V)[4]) {
                // this lane's Gaussian (step `gsl`), extracted from the group's packed list
                // entries: its position and id reads are independent and go out before the
                // transpose
                const int t = (int)__builtin_amdgcn_ubfe(packed, 8 * gsl, 8);
                float4 g0;
                if (ABS) {
                    g0 = sr.g0[cur][t];
                } else {
                    const float2 xy = *reinterpret_cast<const float2*>(&sr.g0[cur][t]);
                    g0 = make_float4(xy.x, xy.y, 0.f, 0.f);
                }
                const float g1x = ABS ? sr.g1[cur][t].x : 0.f;
                const int se = s_e[cur][t < NB ? t : 0];
                {
                    // lane L = pixel r + 16 m writes (F[s], V[s]) at float 128 s + 64 (m >> 1) + 4 r +
                    // 2 (m & 1); lane 16 s + r reads its step's column as two 16-B chunks, pixels
                    // 0-1 at 128 s + 4 r and 2-3 at + 64 (a wave's LDS operations complete in order).
                    // On CDNA4's banking the reads are conflict-free and the writes 2-way (the
                    // [s][r][m] layout read 2-way and wrote 4-way: 72M of raster3d_bwd's 161M LDS
                    // cycles at c2 were conflict cycles, profiles/r05_pmc_lds.txt)
                    float* tp = s_tp[wave];
                    const int rr = lane & 15, mm = lane >> 4;
#pragma unroll
                    for (int q = 0; q < 4; ++q)
                        *reinterpret_cast<float2*>(tp + 128 * q + 64 * (mm >> 1) + 4 * rr + 2 * (mm & 1)) =
                            make_float2(F[q], V[q]);
                    const float4 lo = *reinterpret_cast<const float4*>(tp + 128 * gsl + 4 * rr);
                    const float4 hi = *reinterpret_cast<const float4*>(tp + 128 * gsl + 64 + 4 * rr);
                    F[0] = lo.x; V[0] = lo.y; F[1] = lo.z; V[1] = lo.w;
                    F[2] = hi.x; V[2] = hi.y; F[3] = hi.z; V[3] = hi.w;
                }
                // now F[m], V[m]: step `gsl`, pixel (column cx, row y0 + 2m)
                const float dx = g0.x - p2.pxc, dy0 = g0.y - p2.py0c;
                float S0, Sy, Syy, P[4], A0 = 0.f, A1 = 0.f;
                float ax = 0.f, ay = 0.f, bx = 0.f, c2 = 0.f;
                if (ABS) {
                    ax = 2.f * g0.z * dx;
                    bx = g0.w * dx;
                    ay = g0.w;
                    c2 = 2.f * g1x;
                }
                // the sums start from the first pixel's terms (an add to +0 is not foldable)
#pragma unroll
                for (int m = 0; m < 4; ++m) {
                    const float dy = dy0 - (float)(2 * m);
                    const float vdy = V[m] * dy;
                    S0 = m ? S0 + V[m] : V[m];
                    Sy = m ? Sy + vdy : vdy;
                    Syy = m ? __builtin_fmaf(vdy, dy, Syy) : vdy * dy;
#pragma unroll
                    for (int q = 0; q < 4; ++q) P[q] = m ? __builtin_fmaf(F[m], p2.vo[m][q], P[q]) : F[m] * p2.vo[m][q];
                    if (ABS) {  // |per-pixel v_means2d| up to ln 2: |v_sigma (2a'dx + b'dy)|, |v_sigma (b'dx + 2c'dy)|
                        A0 += fabsf(V[m] * __builtin_fmaf(ay, dy, ax));
                        A1 += fabsf(V[m] * __builtin_fmaf(c2, dy, bx));
                    }
                }
                // level 1 (xor 8: the two lanes of a column): plain sums before the dx
                // products; colours transposed (slot q of class b3 = 1 holds slot q^1's channel)
                // row_ror:8 = 0x128, row_half_mirror = 0x141, quad_perm [1,0,3,2] = 0xB1, [2,3,0,1] = 0x4E
                S0 += dpp<0x128>(S0);
                Sy += dpp<0x128>(Sy);
                Syy += dpp<0x128>(Syy);
                if (ABS) {
                    A0 += dpp<0x128>(A0);
                    A1 += dpp<0x128>(A1);
                }
                const float C01 = P[0] + dpp<0x128>(P[1]), C23 = P[2] + dpp<0x128>(P[3]);
                float g[7];
                g[0] = dx * S0;       // Sx
                g[1] = Sy;            // Sy
                g[2] = dx * dx * S0;  // Sxx
                g[3] = dx * Sy;       // Sxy
                g[4] = Syy;           // Syy
                g[5] = S0;            // sum v_sigma (split3: opacity gradient = -S0 / opacity)
                // opaque products: the next level's DPP add must not be contracted into an FMA
                // (that recomputes the product and needs a separate DPP move)
                asm volatile("" : "+v"(g[0]));
                asm volatile("" : "+v"(g[2]));
                asm volatile("" : "+v"(g[3]));
                // level 2 (half mirror, partner r ^ 7): colours transposed again
                g[6] = C01 + dpp<0x141>(C23);
#pragma unroll
                for (int k = 0; k < 6; ++k) g[k] += dpp<0x141>(g[k]);
                if (ABS) {
                    A0 += dpp<0x141>(A0);
                    A1 += dpp<0x141>(A1);
                }
#pragma unroll
                for (int k = 0; k < 7; ++k) g[k] += dpp<0xB1>(g[k]);
                if (ABS) {
                    A0 += dpp<0xB1>(A0);
                    A1 += dpp<0xB1>(A1);
                }
#pragma unroll
                for (int k = 0; k < 7; ++k) g[k] += dpp<0x4E>(g[k]);
                if (ABS) {
                    A0 += dpp<0x4E>(A0);
                    A1 += dpp<0x4E>(A1);
                }
#pragma unroll
                for (int k = 0; k < 7; ++k) asm volatile("" : "+v"(g[k]));
                {
                    // the wave's partial of this (tile, Gaussian) pair goes to its own row of the
                    // pair's gradient slot: one plain 64-B store per Gaussian, no atomics
                    constexpr float kLn2 = 0.6931471805599453f;
                    const float a = qb2 ? g[3] : g[0], b = qb2 ? g[4] : g[1], c = qb2 ? g[5] : g[2];
                    float v = qsel1 ? b : a;
                    v = qsel2 ? c : v;
                    v = qcol ? g[6] : v;
                    if (ABS) v = r16 == 8 ? kLn2 * A0 : r16 == 9 ? kLn2 * A1 : v;
                    if (t < NB && se >= 0) {
                        const int64_t rw = (int64_t)se * kSlotWaves + wave;
                        rows[rw * kRow3 + spos] = koff >= 0 ? v : 0.f;
                        if (r16 == 0) flags[rw] = 1;
                    }
                }
            };
            for (int i = 0; i < n_mine; i += 4) {
                // the group's four list entries in one scalar register
                const uint32_t packed = (uint32_t)__builtin_amdgcn_readlane((int)lstp, i >> 2);
                float F[4], V[4];
#pragma unroll
                for (int q = 0; q < 4; ++q) step((int)((packed >> (8 * q)) & 0xffu), F[q], V[q]);
                pass2(packed, F, V);
            }
        }
        HGSR_WP_MARK(5);
        lds_barrier();
        HGSR_WP_MARK(6);
    }
    if (pair_counter && lane == 0 && stepped)  // measurement only: lane-pairs stepped
        atomicAdd(pair_slot(pair_counter, 1), (unsigned long long)stepped * 64ull);
    HGSR_WP_MARK(7);
    HGSR_WP_FLUSH();
}

// Gradient slots -> gsplat's separate gradient tensors (overwrite): each (camera, Gaussian)'s
// slot rows summed in a fixed order (reduce_slots), cameras in order per Gaussian.  The sums are
// sigma moments (Sx, Sy, Sxx, Sxy, Syy) = sum_p v_sigma (dx, dy, dx^2, dx dy, dy^2):
// v_means2d = Q (Sx, Sy) with Q the conic, v_conic = (Sxx / 2, Sxy, Syy / 2); value 5 is
// S0 = sum_p v_sigma, and v_opacity = sum_p vis v_alpha = -S0 / opacity.
template <int D, bool ABS>
__global__ __launch_bounds__(256) void split3_kernel(int C, int N, const float* __restrict__ rows,
                                                     const uint8_t* __restrict__ flags, const int32_t* __restrict__ seg,
                                                     const int32_t* __restrict__ pbase, const float* __restrict__ partial,
                                                     const float* __restrict__ opac, int64_t op_cstride,
                                                     const float* __restrict__ conics,
                                                     float2* __restrict__ v_means2d, float* __restrict__ v_conics,
                                                     ChanDst cd, float2* __restrict__ v_abs) {
    constexpr int kScr = reduce_slots_floats<12>();
    __shared__ __attribute__((aligned(16))) float s_scr[4][kScr];  // per wave (each wave owns 64 Gaussians)
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t g0 = ((int64_t)blockIdx.x * 4 + wave) * 64, g = g0 + lane;
    if (g0 >= N) return;  // wave-uniform; the waves never synchronise with each other
    const int nloc = (int)min((int64_t)64, (int64_t)N - g0);
    const bool live = lane < nloc;
    float col_sum[4] = {0.f, 0.f, 0.f, 0.f}, op_sum = 0.f;
    for (int c = 0; c < C; ++c) {
        const int64_t i = (int64_t)c * N + g;
        float r[12];
        reduce_slots<12, 3, kRow3, kSlotWaves, 2>(rows, flags, seg, pbase, partial, (int64_t)c * N + g0, nloc, s_scr[wave], r);
        if (!live) continue;
        const float qa = conics[i * 3], qb = conics[i * 3 + 1], qc = conics[i * 3 + 2];
        v_means2d[i] = make_float2(qa * r[0] + qb * r[1], qb * r[0] + qc * r[1]);
        v_conics[i * 3] = 0.5f * r[2];
        v_conics[i * 3 + 1] = r[3];
        v_conics[i * 3 + 2] = 0.5f * r[4];
        // S0 != 0 only if the Gaussian composited somewhere, i.e. opacity >= 1/255
        // (the records' opacity, read from its coalesced source instead of a 48-B record each)
        const float v_op = r[5] != 0.f ? -r[5] / opac[c * op_cstride + g] : 0.f;
        if (cd.op_shared) op_sum += v_op;
        else cd.opac[i] = v_op;
#pragma unroll
        for (int k = 0; k < D; ++k) {
            if (k < cd.dc) {
                if (cd.col_shared) col_sum[k] += r[6 + k];
                else cd.colors[i * cd.dc + k] = r[6 + k];
            } else if (cd.depths) {
                cd.depths[i] = r[6 + k];
            }
        }
        if (ABS) v_abs[i] = make_float2(r[10], r[11]);
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

static int check_raster(int C, int N, int D, int W, int H, int tile_size, int tw, int th) {
    HGSR_REQUIRE(C >= 1 && N >= 0 && W > 0 && H > 0, "bad dims");
    HGSR_REQUIRE(D >= 1 && D <= 4, "channels per call must be 1..4 (got %d); chunk wider colours", D);
    HGSR_REQUIRE(tile_size == kTile, "tile_size must be %d (got %d)", kTile, tile_size);
    HGSR_REQUIRE(tw == (W + kTile - 1) / kTile && th == (H + kTile - 1) / kTile, "tile grid mismatch");
    HGSR_REQUIRE((int64_t)C * tw * th < (1ll << 31), "too many tiles");
    return HGSR_OK;
}

static size_t rec_bytes(int C, int N) { return ((size_t)C * N * sizeof(Rec3) + 255) & ~(size_t)255; }

// slots (nullable): the rectangles, and the buffer launch_slot_prefix filled (seg, then the row
// prefix), for records that carry their gradient slots
static int pack3(int C, int N, int D, const float* means2d, const float* conics, const ChanSrc& cs, Rec3* rec,
                 hipStream_t s, const RectFromRadii* rr = nullptr, void* slots = nullptr) {
    const int64_t n = (int64_t)C * N;
    if (n == 0) return HGSR_OK;
    const dim3 grid((unsigned)((n + 255) / 256));
    const float2* m2 = reinterpret_cast<const float2*>(means2d);
    int32_t* const seg = (int32_t*)slots;
    const int32_t* const bpre = slots ? (const int32_t*)((char*)slots + (((size_t)(n + 1) * 4 + 255) & ~(size_t)255))
                                      : nullptr;
    const RectFromRadii none{nullptr, nullptr, 0, 0, 0};
#define LAUNCH_P(DD)                                                                                            \
    if (slots)                                                                                                  \
        hipLaunchKernelGGL((pack3_kernel<DD, true>), grid, dim3(256), 0, s, n, N, m2, conics, cs, rec, *rr, bpre, \
                           seg);                                                                                \
    else                                                                                                        \
        hipLaunchKernelGGL((pack3_kernel<DD, false>), grid, dim3(256), 0, s, n, N, m2, conics, cs, rec, none,    \
                           (const int32_t*)nullptr, (int32_t*)nullptr)
    switch (D) {
        case 1: LAUNCH_P(1); break;
        case 2: LAUNCH_P(2); break;
        case 3: LAUNCH_P(3); break;
        default: LAUNCH_P(4); break;
    }
#undef LAUNCH_P
    return check_launch("raster3d_pack");
}

// the tiles' dispatch order, then the 4 quadrant-mask arrays (common.h qmask_words)
extern "C" size_t hgsr_raster3d_qmask_bytes(int C, int tile_w, int tile_h, int64_t n_isects) {
    const int64_t n_bins = (int64_t)C * tile_w * tile_h;
    return tile_order_bytes(n_bins) + (size_t)(4 * qmask_stride(n_isects, n_bins)) * sizeof(uint64_t);
}

// the records, then the slot prefix a training forward fills (hgsr_raster3d_pack_fused with radii)
extern "C" size_t hgsr_raster3d_fwd_ws_bytes(int C, int N, int D) {
    (void)D;
    return rec_bytes(C, N) + slot_prefix_bytes((int64_t)C * N);
}

static int raster3d_fwd_launch(int C, int D, const Rec3* rec, const float* backgrounds, int bg_ch, int ed_ch,
                               int width, int height, int tile_w, int tile_h, const int32_t* isect_offsets,
                               int64_t n_isects, const int32_t* flatten_ids, float* render_colors,
                               float* render_alphas, int32_t* last_ids, hipStream_t s, void* qbuf = nullptr,
                               size_t qbytes = 0, float* zero_rows = nullptr, size_t zero_bytes = 0,
                               const int64_t* isect_info = nullptr);

static int raster3d_fwd_impl(int C, int N, int D, const float* means2d, const float* conics, const ChanSrc& cs,
                             const float* backgrounds, int bg_ch, int ed_ch, int width, int height, int tile_size,
                             int tile_w, int tile_h, const int32_t* isect_offsets, int64_t n_isects,
                             const int32_t* flatten_ids, float* render_colors, float* render_alphas,
                             int32_t* last_ids, void* ws, size_t ws_bytes, hgsr_stream_t stream) {
    if (int st = check_raster(C, N, D, width, height, tile_size, tile_w, tile_h)) return st;
    HGSR_REQUIRE(ws_bytes >= hgsr_raster3d_fwd_ws_bytes(C, N, D), "raster3d_fwd workspace too small");
    HGSR_REQUIRE(isect_offsets && render_colors && render_alphas && last_ids, "null pointer");
    HGSR_REQUIRE(n_isects == 0 || (means2d && conics && (cs.colors || cs.dc == 0) && cs.opac && flatten_ids && ws),
                 "null pointer");
    hipStream_t s = as_stream(stream);
    Rec3* rec = (Rec3*)ws;
    if (n_isects > 0)
        if (int st = pack3(C, N, D, means2d, conics, cs, rec, s)) return st;
    return raster3d_fwd_launch(C, D, rec, backgrounds, bg_ch, ed_ch, width, height, tile_w, tile_h, isect_offsets,
                               n_isects, flatten_ids, render_colors, render_alphas, last_ids, s);
}

static int raster3d_fwd_launch(int C, int D, const Rec3* rec, const float* backgrounds, int bg_ch, int ed_ch,
                               int width, int height, int tile_w, int tile_h, const int32_t* isect_offsets,
                               int64_t n_isects, const int32_t* flatten_ids, float* render_colors,
                               float* render_alphas, int32_t* last_ids, hipStream_t s, void* qbuf,
                               size_t qbytes, float* zero_rows, size_t zero_bytes, const int64_t* isect_info) {
    const int64_t n_bins = (int64_t)C * tile_w * tile_h;
    const dim3 grid((unsigned)n_bins);
    float4* const z4 = reinterpret_cast<float4*>(zero_rows);
    const int64_t zn4 = (int64_t)(zero_bytes / sizeof(float4));
    uint64_t* const qmask = qmask_words(qbuf, n_bins);
    const int64_t qstride = qbuf ? qmask_stride_of(qbytes, n_bins) : 0;
    // heaviest-first tile order, kept in the mask buffer for the backward
    int32_t* const order = (qbuf && HGSR_TILE_ORDER) ? tile_order_of(qbuf) : nullptr;
    if (order && n_isects > 0)
        if (int st = launch_tile_order(n_bins, isect_offsets, n_isects, isect_info, order, s)) return st;
    KernelTimer kt("raster3d_fwd", s);
#define LAUNCH_F(DD)                                                                                           \
    hipLaunchKernelGGL(raster3d_fwd_kernel<DD>, grid, dim3(256), 0, s, C, width, height, tile_w, tile_h, rec,    \
                       backgrounds, bg_ch, ed_ch, isect_offsets, n_isects, flatten_ids, render_colors,          \
                       render_alphas, last_ids, qmask, qstride, z4, zn4, isect_info, n_isects > 0 ? order : nullptr, \
                       (HGSR_BWD_ORDER && order && n_isects > 0) ? tile_end_of(qbuf, n_bins) : nullptr)
    switch (D) {
        case 1: LAUNCH_F(1); break;
        case 2: LAUNCH_F(2); break;
        case 3: LAUNCH_F(3); break;
        default: LAUNCH_F(4); break;
    }
#undef LAUNCH_F
    return check_launch("raster3d_fwd");
}

extern "C" int hgsr_raster3d_fwd(int C, int N, int D, const float* means2d, const float* conics,
                                 const float* colors, const float* opacities, const float* backgrounds,
                                 int width, int height, int tile_size, int tile_w, int tile_h,
                                 const int32_t* isect_offsets, int64_t n_isects, const int32_t* flatten_ids,
                                 float* render_colors, float* render_alphas, int32_t* last_ids, void* ws,
                                 size_t ws_bytes, hgsr_stream_t stream) {
    const ChanSrc cs{colors, (int64_t)N * D, D, nullptr, opacities, (int64_t)N};
    return raster3d_fwd_impl(C, N, D, means2d, conics, cs, backgrounds, D, -1, width, height, tile_size, tile_w,
                             tile_h, isect_offsets, n_isects, flatten_ids, render_colors, render_alphas, last_ids,
                             ws, ws_bytes, stream);
}

extern "C" int hgsr_raster3d_fwd_fused(int C, int N, int Dc, const float* means2d, const float* conics,
                                       const float* colors, int colors_shared, const float* depths,
                                       int expected_depth, const float* opacities, int opacities_shared,
                                       const float* backgrounds, int width, int height, int tile_size,
                                       int tile_w, int tile_h, const int32_t* isect_offsets, int64_t n_isects,
                                       const int32_t* flatten_ids, float* render_colors, float* render_alphas,
                                       int32_t* last_ids, void* ws, size_t ws_bytes, hgsr_stream_t stream) {
    HGSR_REQUIRE(Dc >= 0 && Dc <= 4 && (Dc > 0 || depths), "fused raster: 0..4 colour channels (got %d)", Dc);
    HGSR_REQUIRE(!(expected_depth && !depths), "expected_depth needs depths");
    const int D = Dc + (depths ? 1 : 0);
    const ChanSrc cs{colors, colors_shared ? 0 : (int64_t)N * Dc, Dc, depths, opacities,
                     opacities_shared ? 0 : (int64_t)N};
    return raster3d_fwd_impl(C, N, D, means2d, conics, cs, backgrounds, Dc, expected_depth ? Dc : -1, width,
                             height, tile_size, tile_w, tile_h, isect_offsets, n_isects, flatten_ids,
                             render_colors, render_alphas, last_ids, ws, ws_bytes, stream);
}

extern "C" int hgsr_raster3d_pack_fused(int C, int N, int Dc, const float* means2d, const float* conics,
                                        const float* colors, int colors_shared, const float* depths,
                                        const float* opacities, int opacities_shared, const int32_t* radii,
                                        const int32_t* tiles_per_gauss, int tile_size, int tile_w, int tile_h,
                                        void* ws, size_t ws_bytes, hgsr_stream_t stream) {
    HGSR_REQUIRE(C >= 1 && N >= 0, "bad dims");
    HGSR_REQUIRE(Dc >= 0 && Dc <= 4 && (Dc > 0 || depths), "fused raster: 0..4 colour channels (got %d)", Dc);
    const int D = Dc + (depths ? 1 : 0);
    HGSR_REQUIRE(D <= 4, "channels per call must be 1..4 (got %d)", D);
    HGSR_REQUIRE(ws_bytes >= hgsr_raster3d_fwd_ws_bytes(C, N, D), "raster3d_pack workspace too small");
    HGSR_REQUIRE(N == 0 || (means2d && conics && (colors || Dc == 0) && opacities && ws), "null pointer");
    const ChanSrc cs{colors, colors_shared ? 0 : (int64_t)N * Dc, Dc, depths, opacities,
                     opacities_shared ? 0 : (int64_t)N};
    hipStream_t s = as_stream(stream);
    if (!radii || N == 0) return pack3(C, N, D, means2d, conics, cs, (Rec3*)ws, s);
    // a backward follows: the records carry their gradient slots (isect_tiles' rectangles)
    HGSR_REQUIRE(tile_size > 0 && tile_w > 0 && tile_h > 0, "bad tile grid");
    const RectFromRadii rr{reinterpret_cast<const float2*>(means2d), radii, tile_size, tile_w, tile_h};
    void* const slots = (char*)ws + rec_bytes(C, N);
    if (int st = launch_slot_prefix((int64_t)C * N, rr, slots, s, tiles_per_gauss)) return st;
    return pack3(C, N, D, means2d, conics, cs, (Rec3*)ws, s, &rr, slots);
}

extern "C" int hgsr_raster3d_fwd_packed(int C, int N, int Dc, int with_depth, int expected_depth,
                                        const float* backgrounds, int width, int height, int tile_size,
                                        int tile_w, int tile_h, const int32_t* isect_offsets, int64_t n_isects,
                                        const int32_t* flatten_ids, float* render_colors, float* render_alphas,
                                        int32_t* last_ids, const void* records, size_t records_bytes,
                                        void* qmask, size_t qmask_bytes, void* bwd_ws, size_t bwd_ws_bytes,
                                        const int64_t* isect_info, hgsr_stream_t stream) {
    HGSR_REQUIRE(Dc >= 0 && Dc <= 4 && (Dc > 0 || with_depth), "fused raster: 0..4 colour channels (got %d)", Dc);
    HGSR_REQUIRE(!(expected_depth && !with_depth), "expected_depth needs depths");
    const int D = Dc + (with_depth ? 1 : 0);
    if (int st = check_raster(C, N, D, width, height, tile_size, tile_w, tile_h)) return st;
    HGSR_REQUIRE(records_bytes >= hgsr_raster3d_fwd_ws_bytes(C, N, D), "raster3d_fwd_packed: records too small");
    HGSR_REQUIRE(isect_offsets && render_colors && render_alphas && last_ids, "null pointer");
    HGSR_REQUIRE(n_isects == 0 || (flatten_ids && records), "null pointer");
    HGSR_REQUIRE(!qmask || qmask_bytes >= hgsr_raster3d_qmask_bytes(C, tile_w, tile_h, n_isects),
                 "raster3d_fwd_packed: quadrant-mask buffer too small");
    // bwd_ws (nullable): the backward's workspace, whose gradient-slot flags this launch clears
    const size_t flags_b = slot_flag_bytes(n_isects, kSlotWaves);
    HGSR_REQUIRE(!bwd_ws || (bwd_ws_bytes >= flags_b && (reinterpret_cast<uintptr_t>(bwd_ws) & 15) == 0),
                 "raster3d_fwd_packed: bwd_ws too small or not 16-B aligned");
    // the quadrant-mask stride follows the buffer (sized for the capacity of a deferred count;
    // the backward, given the same buffer, derives the same stride)
    return raster3d_fwd_launch(C, D, (const Rec3*)records, backgrounds, Dc, expected_depth ? Dc : -1, width, height,
                               tile_w, tile_h, isect_offsets, n_isects, flatten_ids, render_colors, render_alphas,
                               last_ids, as_stream(stream), qmask, qmask_bytes, (float*)bwd_ws, bwd_ws ? flags_b : 0,
                               isect_info);
}

// backward workspace: [slot flags (cleared by a forward given it)][slot rows][slot index (seg,
// slot) + its scan scratch][the packed records unless the forward's are reused]
static size_t rows3_bytes(int64_t n_isects) {
    return ((size_t)n_isects * kSlotWaves * kRow3 * sizeof(float) + 255) & ~(size_t)255;
}

extern "C" size_t hgsr_raster3d_bwd_ws_bytes(int C, int N, int D, int64_t n_isects, int reuse_fwd) {
    (void)D;
    return slot_flag_bytes(n_isects, kSlotWaves) + rows3_bytes(n_isects) + grad_slot_bytes((int64_t)C * N, true, n_isects) +
           (reuse_fwd ? 0 : rec_bytes(C, N));
}

static int raster3d_bwd_impl(int C, int N, int D, const float* means2d, const float* conics, const ChanSrc& cs,
                             const float* backgrounds, int bg_ch, int ed_ch, const float* render_colors,
                             int width, int height, int tile_size, int tile_w, int tile_h,
                             const int32_t* isect_offsets, int64_t n_isects, const int32_t* flatten_ids,
                             const float* render_alphas, const int32_t* last_ids, const float* v_render_colors,
                             const float* v_render_alphas, float* v_means2d, float* v_conics, const ChanDst& cd,
                             float* v_means2d_abs, const void* fwd_ws, void* ws, size_t ws_bytes,
                             hgsr_stream_t stream, const void* qbuf = nullptr, size_t qmask_bytes = 0,
                             bool flags_zeroed = false, const int32_t* radii = nullptr, bool fwd_slots = false) {
    if (int st = check_raster(C, N, D, width, height, tile_size, tile_w, tile_h)) return st;
    HGSR_REQUIRE(ws_bytes >= hgsr_raster3d_bwd_ws_bytes(C, N, D, n_isects, fwd_ws != nullptr),
                 "raster3d_bwd workspace too small");
    HGSR_REQUIRE(ed_ch < 0 || render_colors, "expected-depth backward needs render_colors");
    if (N == 0) return HGSR_OK;
    HGSR_REQUIRE(v_means2d && v_conics && (cd.colors || cd.dc == 0) && cd.opac, "null pointer");
    hipStream_t s = as_stream(stream);
    const int64_t n = (int64_t)C * N;
    if (n_isects == 0) {  // nothing composited: every gradient is zero
        if (int st = memset_async(v_means2d, n * 2 * sizeof(float), s, "raster3d_bwd")) return st;
        if (int st = memset_async(v_conics, n * 3 * sizeof(float), s, "raster3d_bwd")) return st;
        if (cd.dc)
            if (int st = memset_async(cd.colors, (cd.col_shared ? N : n) * cd.dc * sizeof(float), s, "raster3d_bwd"))
                return st;
        if (cd.depths)
            if (int st = memset_async(cd.depths, n * sizeof(float), s, "raster3d_bwd")) return st;
        if (int st = memset_async(cd.opac, (cd.op_shared ? N : n) * sizeof(float), s, "raster3d_bwd")) return st;
        if (v_means2d_abs)
            if (int st = memset_async(v_means2d_abs, n * 2 * sizeof(float), s, "raster3d_bwd")) return st;
        return HGSR_OK;
    }
    HGSR_REQUIRE(means2d && conics && isect_offsets && flatten_ids && render_alphas && last_ids && v_render_colors &&
                     v_render_alphas && ws,
                 "null pointer");
    uint8_t* const flags = (uint8_t*)ws;
    float* const rows = (float*)((char*)ws + slot_flag_bytes(n_isects, kSlotWaves));
    char* const sbuf = (char*)rows + rows3_bytes(n_isects);
    if (!flags_zeroed)  // else hgsr_raster3d_fwd_packed cleared them (bwd_ws)
        if (int st = memset_async(flags, slot_flag_bytes(n_isects, kSlotWaves), s, "raster3d_bwd")) return st;
    // the forward's packed records when the caller kept them, else pack again
    Rec3* rec = (Rec3*)const_cast<void*>(fwd_ws);
    if (!rec) {
        rec = (Rec3*)(sbuf + grad_slot_bytes(n, true, n_isects));
        if (int st = pack3(C, N, D, means2d, conics, cs, rec, s)) return st;
    }
    // each (camera, Gaussian)'s gradient slots: the training forward packed them into the records
    // (fwd_slots: seg follows the records in fwd_ws), and only the big entries' piece list is left;
    // else from the tile rectangles (radii given) or the lists, the slot bases scattered into the
    // records' slot quads (Rec3::sl)
    GradSlots gs;
    if (fwd_ws && fwd_slots) {
        void* const slots = (char*)const_cast<void*>(fwd_ws) + rec_bytes(C, N);
        // the piece count the forward's scan cleared: zero for the first backward (the one the
        // forward's workspace went to, flags_zeroed); a later backward clears it again
        if (int st = launch_grad_pieces(n, (const int32_t*)slots, n_isects, sbuf, s, gs, slot_prefix_npieces(slots, n),
                                        flags_zeroed))
            return st;
    } else if (int st = launch_grad_slots(C, N, means2d, radii, tile_size, tile_w, tile_h, isect_offsets, flatten_ids,
                                          n_isects, sbuf, s, gs, reinterpret_cast<int2*>(&rec->sl),
                                          sizeof(Rec3) / sizeof(int2))) {
        return st;
    }
    const int64_t n_bins = (int64_t)C * tile_w * tile_h;
    const dim3 grid((unsigned)n_bins);
    unsigned long long* const pairs = timing_pair_counter("raster3d_bwd");
    // the mask buffer of the forward: its quadrant bits and its heaviest-first tile order
    const uint64_t* const qmask = qmask_words(qbuf, n_bins);
    const int64_t qstride = qbuf ? qmask_stride_of(qmask_bytes, n_bins) : 0;
    // the forward writes the order only for a non-empty view
    const int32_t* const order = (qbuf && HGSR_TILE_ORDER && n_isects > 0) ? tile_order_of(qbuf) : nullptr;
    // each tile's latest contributor + 1, written by the forward with the order
    const int32_t* const tile_end = (HGSR_BWD_ORDER && order) ? tile_end_of(const_cast<void*>(qbuf), n_bins) : nullptr;
    if (HGSR_BWD_ORDER && order) {
        // re-sort the tiles by the ranges the backward walks (up to each tile's latest contributor,
        // written by the forward) instead of by their whole bins
        void* const qb = const_cast<void*>(qbuf);
        if (int st = launch_tile_order(n_bins, isect_offsets, n_isects, nullptr, tile_order_of(qb), s,
                                       tile_end_of(qb, n_bins)))
            return st;
    }
    const bool abs = v_means2d_abs != nullptr;
#define LAUNCH_B(DD, AA)                                                                                       \
    {                                                                                                          \
        KernelTimer kt("raster3d_bwd", s);                                                                     \
        hipLaunchKernelGGL((raster3d_bwd_kernel<DD, AA>), grid, dim3(256), 0, s, C, width, height, tile_w,      \
                           tile_h, rec, backgrounds, bg_ch, ed_ch, render_colors, isect_offsets, n_isects,       \
                           flatten_ids, render_alphas, last_ids, v_render_colors, v_render_alphas, rows, flags,  \
                           n_isects, pairs, qmask, qstride, order, tile_end);                                  \
    }                                                                                                          \
    hipLaunchKernelGGL((reduce_pieces_kernel<12, 3, kRow3, kSlotWaves>), dim3(piece_grid(gs)), dim3(256), 0, s,   \
                       rows, flags, gs.seg, gs.pbase, gs.pieces, gs.npieces, gs.partial);                          \
    hipLaunchKernelGGL((split3_kernel<DD, AA>), dim3((unsigned)(((int64_t)N + 255) / 256)), dim3(256), 0, s, C, \
                       N, rows, flags, gs.seg, gs.pbase, gs.partial, cs.opac, cs.op_cstride, conics,               \
                       reinterpret_cast<float2*>(v_means2d), v_conics, cd, reinterpret_cast<float2*>(v_means2d_abs))
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

extern "C" int hgsr_raster3d_bwd(int C, int N, int D, const float* means2d, const float* conics,
                                 const float* colors, const float* opacities, const float* backgrounds,
                                 int width, int height, int tile_size, int tile_w, int tile_h,
                                 const int32_t* isect_offsets, int64_t n_isects, const int32_t* flatten_ids,
                                 const float* render_alphas, const int32_t* last_ids,
                                 const float* v_render_colors, const float* v_render_alphas, float* v_means2d,
                                 float* v_conics, float* v_colors, float* v_opacities, float* v_means2d_abs,
                                 const void* fwd_ws, void* ws, size_t ws_bytes, hgsr_stream_t stream) {
    const ChanSrc cs{colors, (int64_t)N * D, D, nullptr, opacities, (int64_t)N};
    const ChanDst cd{v_colors, false, D, nullptr, v_opacities, false};
    return raster3d_bwd_impl(C, N, D, means2d, conics, cs, backgrounds, D, -1, nullptr, width, height, tile_size,
                             tile_w, tile_h, isect_offsets, n_isects, flatten_ids, render_alphas, last_ids,
                             v_render_colors, v_render_alphas, v_means2d, v_conics, cd, v_means2d_abs, fwd_ws, ws,
                             ws_bytes, stream);
}

extern "C" int hgsr_raster3d_bwd_fused(int C, int N, int Dc, const float* means2d, const float* conics,
                                       const float* colors, int colors_shared, const float* depths,
                                       int expected_depth, const float* opacities, int opacities_shared,
                                       const float* backgrounds, int width, int height, int tile_size,
                                       int tile_w, int tile_h, const int32_t* isect_offsets, int64_t n_isects,
                                       const int32_t* flatten_ids, const float* render_colors,
                                       const float* render_alphas, const int32_t* last_ids,
                                       const float* v_render_colors, const float* v_render_alphas,
                                       float* v_means2d, float* v_conics, float* v_colors, float* v_depths,
                                       float* v_opacities, float* v_means2d_abs, const void* fwd_ws, void* ws,
                                       size_t ws_bytes, const void* qmask, size_t qmask_bytes, int ws_zeroed,
                                       const int32_t* radii, int fwd_slots, hgsr_stream_t stream) {
    HGSR_REQUIRE(Dc >= 0 && Dc <= 4 && (Dc > 0 || depths), "fused raster: 0..4 colour channels (got %d)", Dc);
    HGSR_REQUIRE(!qmask || qmask_bytes >= hgsr_raster3d_qmask_bytes(C, tile_w, tile_h, n_isects),
                 "raster3d_bwd_fused: quadrant-mask buffer too small");
    HGSR_REQUIRE(!(expected_depth && !depths), "expected_depth needs depths");
    HGSR_REQUIRE(!depths || v_depths, "null pointer");
    const int D = Dc + (depths ? 1 : 0);
    const ChanSrc cs{colors, colors_shared ? 0 : (int64_t)N * Dc, Dc, depths, opacities,
                     opacities_shared ? 0 : (int64_t)N};
    const ChanDst cd{v_colors, colors_shared != 0, Dc, depths ? v_depths : nullptr, v_opacities,
                     opacities_shared != 0};
    return raster3d_bwd_impl(C, N, D, means2d, conics, cs, backgrounds, Dc, expected_depth ? Dc : -1,
                             render_colors, width, height, tile_size, tile_w, tile_h, isect_offsets, n_isects,
                             flatten_ids, render_alphas, last_ids, v_render_colors, v_render_alphas, v_means2d,
                             v_conics, cd, v_means2d_abs, fwd_ws, ws, ws_bytes, stream, qmask, qmask_bytes,
                             ws_zeroed != 0, radii, fwd_slots != 0);
}
