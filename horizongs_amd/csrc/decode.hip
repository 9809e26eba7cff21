// K14: anchor -> neural-Gaussian decode, forward.
//
// Reference semantics: scene/lod_model.py:286-290 (LoD mask), scene/basic_model.py:297-371
// (generate_neural_gaussians) with the MLPs of scene/lod_model.py:67-84
// (Linear(F+vd -> F) -> ReLU -> Linear(F -> O) [-> Tanh for the opacity head]),
// appearance_dim = 0 and dist2level != 'progressive' (smooth_complement = 1).
//
// CDNA4 mapping
//  * one 256-lane workgroup per 64 visible anchors (grid-stride), each wave64 owning
//    16 anchors; the three MLPs' weights staged once per workgroup in LDS;
//  * both layers on exact-f32 MFMA (v_mfma_f32_16x16x4_f32), computed TRANSPOSED
//    (anchors are the N = 16 columns): the first layer's accumulator registers hold
//    H^T[hidden = 4g + r][anchor] (g = lane >> 4), which is directly the B operand of
//    the second layer's k-step r when the k order inside each 16-hidden group is
//    permuted to 4g + r -- absorbed by staging W2 with permuted columns, so no lane
//    movement between the layers;
//  * LDS strides chosen bank-conflict-free for the 16x4 fragment reads (kDecS, kDecYS);
//  * opacity > 0 compaction is order-preserving (anchor-major, then offset) with
//    wave ballots + a per-tile offset table from a count pass and a scan;
//  * the colour head (pure linear) is stored straight from the accumulators.
#include <stdlib.h>

#include <map>
#include <mutex>

#include "common.h"

namespace hgsr {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kDecTile = 64;      // visible anchors per workgroup iteration (4 waves x 16)
constexpr int kDecF = 32;         // feat_dim (every reference config)
constexpr int kDecS = 38;         // LDS row stride (floats) of W1 / W2 / X: conflict-free 16x4 fragment reads
constexpr int kDecYS = 20;        // LDS row stride of the Y^T tiles: conflict-free accumulator stores
// backward Y^T / dY^T / H^T stride: the MFMA fragment reads (rows i, columns 4kk+g) and the
// per-row sums (one row per lane) dominate there, both conflict-free at an odd stride
constexpr int kDecBS = 17;

// tanh to a few ulp for the opacity head: exp-based, and x itself below |x| < 2^-8 (error
// < x^3/3, keeps the sign and never rounds a positive input to 0, so the opacity > 0 mask
// is exactly the reference's)
__device__ __forceinline__ float tanh_fast(float x) {
    const float ax = fabsf(x);
    const float e = __expf(-2.0f * ax);
    const float t = (1.0f - e) * __builtin_amdgcn_rcpf(1.0f + e);
    return ax < 0.00390625f ? x : copysignf(t, x);
}
constexpr int kDecMaxRows = 368;  // W2 rows (opacity + cov + colour heads, padded to 16): SH2 x 10 offsets

struct MlpPtrs {
    const float* w1[3];  // [F, F+vd] (nn.Linear layout), heads: 0 opacity, 1 cov, 2 colour
    const float* b1[3];
    const float* w2[3];  // [O_h, F]
    const float* b2[3];
};

struct DecodeDims {
    int Av, vd, noff, cd;
    int O[3];     // outputs per head: noff, 7 noff, cd noff
    int T[3];     // 16-row tiles per head
    int row0[3];  // first W2 row of each head in LDS
    int rows;     // total padded W2 rows
};

static DecodeDims decode_dims(int Av, int vd, int noff, int cd) {
    DecodeDims d;
    d.Av = Av;
    d.vd = vd;
    d.noff = noff;
    d.cd = cd;
    d.O[0] = noff;
    d.O[1] = 7 * noff;
    d.O[2] = cd * noff;
    int r = 0;
    for (int h = 0; h < 3; ++h) {
        d.T[h] = (d.O[h] + 15) / 16;
        d.row0[h] = r;
        r += 16 * d.T[h];
    }
    d.rows = r;
    return d;
}

__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// LDS column of hidden unit h inside its 16-group, so that the second layer's
// k-step r reads 4 consecutive columns across the lane groups g: 4 (h % 4) + (h % 16) / 4
__device__ __forceinline__ int w2_col(int h) { return (h & ~15) | ((h & 3) << 2) | ((h & 15) >> 2); }

// LoD mask: dist = |anchor - cam| * res_scale; pred = log2(sd / dist) / log2(fork) + extra;
// mask = level <= clamp(floor(pred), 0, max_level).  Operation order as the reference.
__global__ __launch_bounds__(256) void lod_mask_kernel(int A, const float* __restrict__ anchor,
                                                       const int32_t* __restrict__ level,
                                                       const float* __restrict__ extra_level,
                                                       const float* __restrict__ cam, float res_scale,
                                                       float standard_dist, float log2_fork, int max_level,
                                                       uint8_t* __restrict__ mask) {
#pragma clang fp contract(off)
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= A) return;
    const float dx = anchor[i * 3] - cam[0], dy = anchor[i * 3 + 1] - cam[1], dz = anchor[i * 3 + 2] - cam[2];
    const float dist = sqrtf(dx * dx + dy * dy + dz * dz) * res_scale;
    const float pred = log2f(standard_dist / dist) / log2_fork + extra_level[i];
    const float fl = floorf(pred);
    int il = fl <= 0.f ? 0 : (fl >= (float)max_level ? max_level : (int)fl);
    mask[i] = level[i] <= il ? 1 : 0;
}

// ---------------------------------------------------------------- shared pieces
// LDS of the forward / count passes, sized per pass: W1R first-layer rows (96 = all
// three heads, 32 = opacity head only), W2R second-layer rows, YR pre-activation rows
template <int W1R, int W2R, int YR>
struct DecodeSmem {
    float w1[W1R * kDecS];
    float b1[W1R];
    float w2[W2R * kDecS];
    float b2[W2R];
    float x[4][16 * kDecS];    // per wave: X rows (feat | ob_view | 0)
    float y[4][YR * kDecYS];   // per wave: opacity / cov pre-activations Y^T[o][anchor]
    int pos[4][16 * 16];       // per wave: output row of (anchor, offset), -1 if dropped
    int wave_cnt[4];
};
using CountSmem = DecodeSmem<32, 16, 16>;

template <class S>
__device__ void stage_weights(S& sm, const MlpPtrs& mp, const DecodeDims& d, int w1_rows, int w2_rows) {
    const int K1 = kDecF + d.vd;
    for (int e = threadIdx.x; e < w1_rows * kDecS; e += 256) {
        const int h = e / kDecS, k = e - h * kDecS;
        const int head = h >> 5, hh = h & 31;
        sm.w1[e] = k < K1 ? mp.w1[head][hh * K1 + k] : 0.f;
    }
    for (int h = threadIdx.x; h < w1_rows; h += 256) sm.b1[h] = mp.b1[h >> 5][h & 31];
    for (int e = threadIdx.x; e < w2_rows * kDecF; e += 256) {
        const int row = e / kDecF, h = e - row * kDecF;
        int head = 0;
        while (head < 2 && row >= d.row0[head + 1]) ++head;
        const int o = row - d.row0[head];
        sm.w2[row * kDecS + w2_col(h)] = o < d.O[head] ? mp.w2[head][o * kDecF + h] : 0.f;
    }
    for (int row = threadIdx.x; row < w2_rows; row += 256) {
        int head = 0;
        while (head < 2 && row >= d.row0[head + 1]) ++head;
        const int o = row - d.row0[head];
        sm.b2[row] = o < d.O[head] ? mp.b2[head][o] : 0.f;
    }
}

// X rows of a wave's 16 anchors fetched into registers one tile ahead (software pipeline:
// the id loads, then the feat / anchor loads, are issued during the previous tile's MFMA
// work, so stage-in costs no exposed memory latency).  Lane l holds the id of anchor
// l & 15 (-1 past Av) and feat elements e = l + 64 j (row e >> 5, column e & 31).
struct XPrefetch {
    int id;
    float f[8];
    float ax, ay, az;  // lanes < 16: the anchor position (view direction)
};

__device__ __forceinline__ void x_issue_id(XPrefetch& p, const int32_t* __restrict__ vis_idx, int a0, int Av) {
    const int v = a0 + (threadIdx.x & 15);
    p.id = v < Av ? (vis_idx ? vis_idx[v] : v) : -1;
}

__device__ __forceinline__ void x_issue_data(XPrefetch& p, const float* __restrict__ feat,
                                             const float* __restrict__ anchor, int vd) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int id = __shfl(p.id, (lane >> 5) + 2 * j);
        p.f[j] = id >= 0 ? feat[(int64_t)id * kDecF + (lane & 31)] : 0.f;
    }
    const bool a = lane < 16 && p.id >= 0 && vd > 0;
    p.ax = a ? anchor[(int64_t)p.id * 3] : 0.f;
    p.ay = a ? anchor[(int64_t)p.id * 3 + 1] : 0.f;
    p.az = a ? anchor[(int64_t)p.id * 3 + 2] : 0.f;
}

// same LDS image as stage_x from the prefetched registers
// (lanes < 16 also return their anchor's view direction and distance for the backward)
__device__ __forceinline__ void x_store(const XPrefetch& p, float* sx, int vd, const float* __restrict__ cam,
                                        float (&ov)[3], float& dist) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int j = 0; j < 8; ++j) sx[((lane >> 5) + 2 * j) * kDecS + (lane & 31)] = p.f[j];
    ov[0] = ov[1] = ov[2] = 0.f;
    dist = 1.f;
    if (lane < 16) {
        if (p.id >= 0 && vd > 0) {
            const float dx = p.ax - cam[0], dy = p.ay - cam[1], dz = p.az - cam[2];
            dist = sqrtf(dx * dx + dy * dy + dz * dz);
            ov[0] = dx / dist;
            ov[1] = dy / dist;
            ov[2] = dz / dist;
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) sx[lane * kDecS + kDecF + k] = (k < 3 && vd > 0) ? ov[k] : 0.f;
    }
}

// first layer of head `head` (or all three): H^T tiles [16 hidden x 16 anchors], bias + ReLU
template <int KSTEPS, class S>
__device__ __forceinline__ f32x4 layer1_tile(const S& sm, const float* sx, int mt) {
    const int lane = threadIdx.x & 63, i = lane & 15, g = lane >> 4;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kk = 0; kk < KSTEPS; ++kk)
        acc = mfma4(sm.w1[(mt * 16 + i) * kDecS + 4 * kk + g], sx[i * kDecS + 4 * kk + g], acc);
#pragma unroll
    for (int r = 0; r < 4; ++r) acc[r] = fmaxf(acc[r] + sm.b1[mt * 16 + 4 * g + r], 0.f);
    return acc;
}

// second layer: Y^T tile [16 outputs x 16 anchors] of W2 rows [row, row + 16) from the
// head's two H^T tiles (k = 32 hidden in 8 k-steps, no lane movement)
template <class S>
__device__ __forceinline__ f32x4 layer2_tile(const S& sm, int row, f32x4 h0, f32x4 h1) {
    const int lane = threadIdx.x & 63, i = lane & 15, g = lane >> 4;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    const float* w = sm.w2 + (row + i) * kDecS + g;
#pragma unroll
    for (int r = 0; r < 4; ++r) acc = mfma4(w[4 * r], h0[r], acc);
#pragma unroll
    for (int r = 0; r < 4; ++r) acc = mfma4(w[16 + 4 * r], h1[r], acc);
#pragma unroll
    for (int r = 0; r < 4; ++r) acc[r] += sm.b2[row + 4 * g + r];
    return acc;
}

__device__ __forceinline__ int lanes_below_d(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
}

// opacity head of this wave's 16 anchors -> tanh values in sm.y rows [0, 16); returns
// the wave's kept count (and the ballot-ordered local position of every kept slot)
template <int KSTEPS, class S>
__device__ int opacity_head(S& sm, int wave, int a0, int Av, const DecodeDims& d, bool want_pos) {
    const int lane = threadIdx.x & 63, i = lane & 15, g = lane >> 4;
    const float* sx = sm.x[wave];
    const f32x4 h0 = layer1_tile<KSTEPS>(sm, sx, 0), h1 = layer1_tile<KSTEPS>(sm, sx, 1);
    const f32x4 y = layer2_tile(sm, d.row0[0], h0, h1);
    float* sy = sm.y[wave];
#pragma unroll
    for (int r = 0; r < 4; ++r) sy[(4 * g + r) * kDecYS + i] = tanh_fast(y[r]);
    // order-preserving keep positions over slots s = a * noff + k
    const int nslots = 16 * d.noff;
    int cnt = 0;
    for (int s0 = 0; s0 < nslots; s0 += 64) {
        const int s = s0 + lane;
        const int a = s / d.noff, k = s - a * d.noff;
        const bool keep = s < nslots && a0 + a < Av && sy[k * kDecYS + a] > 0.f;
        const uint64_t m = __ballot(keep);
        if (want_pos && s < nslots) sm.pos[wave][s] = keep ? cnt + lanes_below_d(m) : -1;
        cnt += __popcll(m);
    }
    return cnt;
}

// ---------------------------------------------------------------- count pass
template <int KSTEPS>
__global__ __launch_bounds__(256) void decode_count_kernel(DecodeDims d, MlpPtrs mp,
                                                           const int32_t* __restrict__ vis_idx,
                                                           const float* __restrict__ anchor,
                                                           const float* __restrict__ feat,
                                                           const float* __restrict__ cam,
                                                           int32_t* __restrict__ tile_cnt,
                                                           const int64_t* __restrict__ av_dev) {
    __shared__ CountSmem sm;
    if (av_dev) d.Av = (int)*av_dev;  // device-resident visible count (d.Av was the capacity)
    stage_weights(sm, mp, d, 32, 16);  // opacity head only
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int n_tiles = (d.Av + kDecTile - 1) / kDecTile;
    XPrefetch px;  // X rows one tile ahead
    if (blockIdx.x < (unsigned)n_tiles) {
        x_issue_id(px, vis_idx, blockIdx.x * kDecTile + wave * 16, d.Av);
        x_issue_data(px, feat, anchor, d.vd);
    }
    for (int t = blockIdx.x; t < n_tiles; t += gridDim.x) {
        __syncthreads();
        const int a0 = t * kDecTile + wave * 16;
        float ov[3], dist;
        x_store(px, sm.x[wave], d.vd, cam, ov, dist);
        const int tn = t + gridDim.x;
        if (tn < n_tiles) x_issue_id(px, vis_idx, tn * kDecTile + wave * 16, d.Av);
        __syncthreads();
        const int c = opacity_head<KSTEPS>(sm, wave, a0, d.Av, d, false);
        if (tn < n_tiles) x_issue_data(px, feat, anchor, d.vd);
        if (lane == 0) sm.wave_cnt[wave] = c;
        __syncthreads();
        if (threadIdx.x == 0) tile_cnt[t] = sm.wave_cnt[0] + sm.wave_cnt[1] + sm.wave_cnt[2] + sm.wave_cnt[3];
    }
}

// exclusive scan of the tile counts -> tile offsets; total = number of kept Gaussians
__global__ __launch_bounds__(1024) void decode_scan_kernel(int n, const int32_t* __restrict__ cnt,
                                                           int32_t* __restrict__ off, int64_t* __restrict__ total,
                                                           const int64_t* __restrict__ av_dev) {
    __shared__ int64_t s_sum[1024];
    if (av_dev) n = (int)((*av_dev + kDecTile - 1) / kDecTile);
    const int tid = threadIdx.x;
    const int per = (n + 1023) / 1024;
    const int b0 = min(tid * per, n), b1 = min(b0 + per, n);
    int64_t local = 0;
    for (int i = b0; i < b1; ++i) local += cnt[i];
    s_sum[tid] = local;
    __syncthreads();
    for (int dd = 1; dd < 1024; dd <<= 1) {
        const int64_t v = tid >= dd ? s_sum[tid - dd] : 0;
        __syncthreads();
        s_sum[tid] += v;
        __syncthreads();
    }
    int64_t run = s_sum[tid] - local;
    for (int i = b0; i < b1; ++i) {
        off[i] = (int32_t)run;
        run += cnt[i];
    }
    if (tid == 1023) total[0] = s_sum[1023];
}

// ---------------------------------------------------------------- forward
struct DecodeOut {
    float* xyz;      // [M,3]
    float* offsets;  // [M,3]
    float* color;    // [M,cd]
    float* opacity;  // [M]
    float* scaling;  // [M,3]
    float* rot;      // [M,4]
    uint8_t* mask;   // [Av*noff]
    int32_t* slot_row;  // [Av*noff] output row or -1 (kept for the backward)
};

template <int KSTEPS, int W2R, bool COLOR = true>
__global__ __launch_bounds__(256) void decode_fwd_kernel(DecodeDims d, MlpPtrs mp,
                                                         const int32_t* __restrict__ vis_idx,
                                                         const float* __restrict__ anchor,
                                                         const float* __restrict__ feat,
                                                         const float* __restrict__ offset,
                                                         const float* __restrict__ scaling_raw,
                                                         const float* __restrict__ cam,
                                                         const int32_t* __restrict__ tile_off, DecodeOut out) {
    __shared__ DecodeSmem<96, W2R, 80> sm;
    // without the colour head (decode_color_kernel writes it) only the opacity and cov rows
    stage_weights(sm, mp, d, 96, COLOR ? d.rows : d.row0[2]);
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, i = lane & 15, g = lane >> 4;
    const int n_tiles = (d.Av + kDecTile - 1) / kDecTile;
    const int noff = d.noff, cd = d.cd;
    XPrefetch px;  // X rows one tile ahead
    if (blockIdx.x < (unsigned)n_tiles) {
        x_issue_id(px, vis_idx, blockIdx.x * kDecTile + wave * 16, d.Av);
        x_issue_data(px, feat, anchor, d.vd);
    }
    constexpr int kSI = 3;  // 16 anchors x n_offsets <= 12 -> <= 192 slots = 3 per lane
    for (int t = blockIdx.x; t < n_tiles; t += gridDim.x) {
        __syncthreads();
        const int a0 = t * kDecTile + wave * 16;
        float ov[3], dist;
        x_store(px, sm.x[wave], d.vd, cam, ov, dist);
        const int cur_id = px.id;
        const int tn = t + gridDim.x;
        if (tn < n_tiles) x_issue_id(px, vis_idx, tn * kDecTile + wave * 16, d.Av);
        // per-slot operands of this tile (scaling_raw, offset, anchor position), issued now and
        // consumed after the MLPs
        float srw[kSI][6], ofs[kSI][3], anc[kSI][3];
#pragma unroll
        for (int it = 0; it < kSI; ++it) {
            const int sl = lane + 64 * it;
            const int a = sl / noff, k = sl - a * noff;
            const int aid = __shfl(cur_id, a < 16 ? a : 0);
            const bool live = sl < 16 * noff && a0 + a < d.Av;
            const int64_t id = live ? aid : 0;
#pragma unroll
            for (int q = 0; q < 6; ++q) srw[it][q] = live ? scaling_raw[id * 6 + q] : 0.f;
#pragma unroll
            for (int q = 0; q < 3; ++q) {
                ofs[it][q] = live ? offset[(id * noff + k) * 3 + q] : 0.f;
                anc[it][q] = live ? anchor[id * 3 + q] : 0.f;
            }
        }
        __syncthreads();
        const int c = opacity_head<KSTEPS>(sm, wave, a0, d.Av, d, true);
        if (tn < n_tiles) x_issue_data(px, feat, anchor, d.vd);
        if (lane == 0) sm.wave_cnt[wave] = c;
        __syncthreads();
        int base = tile_off[t];
        for (int w = 0; w < wave; ++w) base += sm.wave_cnt[w];
        int* pos = sm.pos[wave];
        const float* sy = sm.y[wave];
        // opacity + mask + slot rows
        for (int s = lane; s < 16 * noff; s += 64) {
            const int a = s / noff, k = s - a * noff;
            if (a0 + a >= d.Av) continue;
            const int p = pos[s] >= 0 ? base + pos[s] : -1;
            pos[s] = p;
            const int64_t slot = (int64_t)(a0 + a) * noff + k;
            out.mask[slot] = p >= 0;
            out.slot_row[slot] = p;
            if (p >= 0) out.opacity[p] = sy[k * kDecYS + a];
        }
        // hidden layer of the cov and colour heads
        const float* sx = sm.x[wave];
        const f32x4 hc0 = layer1_tile<KSTEPS>(sm, sx, 2), hc1 = layer1_tile<KSTEPS>(sm, sx, 3);
        // cov head -> LDS, then scaling / rotation / position per kept slot
        float* syw = sm.y[wave];
        for (int ot = 0; ot < d.T[1]; ++ot) {
            const f32x4 y = layer2_tile(sm, d.row0[1] + ot * 16, hc0, hc1);
#pragma unroll
            for (int r = 0; r < 4; ++r) syw[(ot * 16 + 4 * g + r) * kDecYS + i] = y[r];
        }
#pragma unroll
        for (int it = 0; it < kSI; ++it) {
            const int s = lane + 64 * it;
            if (s >= 16 * noff) continue;
            const int a = s / noff, k = s - a * noff;
            if (a0 + a >= d.Av) continue;
            const int p = pos[s];
            if (p < 0) continue;
            float cv[7];
#pragma unroll
            for (int q = 0; q < 7; ++q) cv[q] = syw[(7 * k + q) * kDecYS + a];
            const float* sr = srw[it];
#pragma unroll
            for (int q = 0; q < 3; ++q)
                out.scaling[(int64_t)p * 3 + q] = __expf(sr[3 + q]) * __builtin_amdgcn_rcpf(1.0f + __expf(-cv[q]));
            const float nrm = fmaxf(__builtin_amdgcn_sqrtf(cv[3] * cv[3] + cv[4] * cv[4] + cv[5] * cv[5] + cv[6] * cv[6]),
                                    1e-12f);
            const float inrm = __builtin_amdgcn_rcpf(nrm);
#pragma unroll
            for (int q = 0; q < 4; ++q) out.rot[(int64_t)p * 4 + q] = cv[3 + q] * inrm;
#pragma unroll
            for (int q = 0; q < 3; ++q) {
                const float o = ofs[it][q] * __expf(sr[q]);
                out.offsets[(int64_t)p * 3 + q] = o;
                out.xyz[(int64_t)p * 3 + q] = anc[it][q] + o;
            }
        }
        if (!COLOR) continue;
        // colour head (linear output), each tile transposed through the wave's (now free)
        // pre-activation buffer so a store covers 16 consecutive rows of 4 anchors (see
        // decode_color_kernel)
        const f32x4 hl0 = layer1_tile<KSTEPS>(sm, sx, 4), hl1 = layer1_tile<KSTEPS>(sm, sx, 5);
        for (int ot = 0; ot < d.T[2]; ++ot) {
            const f32x4 y = layer2_tile(sm, d.row0[2] + ot * 16, hl0, hl1);
#pragma unroll
            for (int r = 0; r < 4; ++r) syw[(4 * g + r) * kDecYS + i] = y[r];
            const int row = lane & 15, o = ot * 16 + row;
            const int k = o / cd;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int a = 4 * j + (lane >> 4);
                const float v = syw[row * kDecYS + a];
                if (o >= cd * noff || a0 + a >= d.Av) continue;
                const int p = pos[a * noff + k];
                if (p >= 0) out.color[(int64_t)p * cd + (o - k * cd)] = v;
            }
        }
    }
}

// (wave_lds_sync, common.h: the wave-level LDS ordering point; no workgroup barrier)

// Colour head alone, for models whose second layer exceeds the 128-row plan (SH colour
// heads: 27 x 10 outputs).  With every head's W2 in LDS the fused forward fits one workgroup
// per CU; split, the fused pass (opacity + cov, 128 rows) and this pass (the colour head's W1
// and W2 only, 61 KB) run two each.  The output rows of the kept slots come from slot_row,
// which the fused pass wrote; X rows are prefetched one tile ahead as there.
constexpr int kDecColRows = 272;  // colour W2 rows of this pass (17 tiles: SH2 x 10 offsets)
struct DecodeColorSmem {
    float w1[32 * kDecS];
    float b1[32];
    float w2[kDecColRows * kDecS];
    float b2[kDecColRows];
    float x[4][16 * kDecS];
    int pos[4][16 * 16];
    float ty[4][16 * 20];  // per wave: one output tile transposed for the stores (pitch 20: conflict-free)
};

template <int KSTEPS>
__global__ __launch_bounds__(256) void decode_color_kernel(DecodeDims d, MlpPtrs mp,
                                                           const int32_t* __restrict__ vis_idx,
                                                           const float* __restrict__ anchor,
                                                           const float* __restrict__ feat,
                                                           const float* __restrict__ cam,
                                                           const int32_t* __restrict__ slot_row,
                                                           float* __restrict__ color) {
    __shared__ DecodeColorSmem sm;
    const int K1 = kDecF + d.vd, O = d.O[2], rows = d.T[2] * 16;
    for (int e = threadIdx.x; e < 32 * kDecS; e += 256) {
        const int h = e / kDecS, k = e - h * kDecS;
        sm.w1[e] = k < K1 ? mp.w1[2][h * K1 + k] : 0.f;
    }
    if (threadIdx.x < 32) sm.b1[threadIdx.x] = mp.b1[2][threadIdx.x];
    for (int e = threadIdx.x; e < rows * kDecF; e += 256) {
        const int row = e / kDecF, h = e - row * kDecF;
        sm.w2[row * kDecS + w2_col(h)] = row < O ? mp.w2[2][row * kDecF + h] : 0.f;
    }
    for (int row = threadIdx.x; row < rows; row += 256) sm.b2[row] = row < O ? mp.b2[2][row] : 0.f;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, i = lane & 15, g = lane >> 4;
    const int n_tiles = (d.Av + kDecTile - 1) / kDecTile;
    const int noff = d.noff, cd = d.cd;
    XPrefetch px;
    if (blockIdx.x < (unsigned)n_tiles) {
        x_issue_id(px, vis_idx, blockIdx.x * kDecTile + wave * 16, d.Av);
        x_issue_data(px, feat, anchor, d.vd);
    }
    __syncthreads();  // weights staged
    float* sx = sm.x[wave];
    int* pos = sm.pos[wave];
    for (int t = blockIdx.x; t < n_tiles; t += gridDim.x) {
        wave_lds_sync();  // this wave's previous tile is done with its x / pos arrays
        const int a0 = t * kDecTile + wave * 16;
        float ov[3], dist;
        x_store(px, sx, d.vd, cam, ov, dist);
        for (int sl = lane; sl < 16 * noff; sl += 64) {
            const int a = sl / noff;
            pos[sl] = a0 + a < d.Av ? slot_row[(int64_t)a0 * noff + sl] : -1;
        }
        const int tn = t + gridDim.x;
        if (tn < n_tiles) x_issue_id(px, vis_idx, tn * kDecTile + wave * 16, d.Av);
        wave_lds_sync();
        const f32x4 h0 = layer1_tile<KSTEPS>(sm, sx, 0), h1 = layer1_tile<KSTEPS>(sm, sx, 1);
        if (tn < n_tiles) x_issue_data(px, feat, anchor, d.vd);
        // each tile goes out through the wave's transpose buffer: a store instruction then covers
        // 16 consecutive rows (a slot's consecutive colour values) of 4 anchors -- 64-B runs --
        // instead of 4 rows of 16 anchors (64 scattered words)
        float* const ty = sm.ty[wave];
        for (int ot = 0; ot < d.T[2]; ++ot) {
            const f32x4 y = layer2_tile(sm, ot * 16, h0, h1);
#pragma unroll
            for (int r = 0; r < 4; ++r) ty[(4 * g + r) * 20 + i] = y[r];
            const int row = lane & 15, o = ot * 16 + row;
            const int k = o / cd;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int a = 4 * j + (lane >> 4);
                const float v = ty[row * 20 + a];
                if (o >= cd * noff || a0 + a >= d.Av) continue;
                const int p = pos[a * noff + k];
                if (p >= 0) color[(int64_t)p * cd + (o - k * cd)] = v;
            }
        }
    }
}

// ---------------------------------------------------------------- backward

// Developer instrumentation (variant builds with -DHGSR_DECODE_PROF only): per-head, per-phase
// shader-clock totals of the backward; every boundary drains the wave's memory counters so a
// phase is charged the latency of the loads it issued.
#ifdef HGSR_DECODE_PROF
__device__ unsigned long long g_dprof[3][16];
#define DPROF_INIT uint64_t _tp = __builtin_amdgcn_s_memtime();
#define DPROF_T(k)                                                                  \
    do {                                                                            \
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");                 \
        const uint64_t _t = __builtin_amdgcn_s_memtime();                           \
        if ((threadIdx.x & 63) == 0) atomicAdd(&g_dprof[HEAD][k], (unsigned long long)(_t - _tp)); \
        _tp = _t;                                                                   \
    } while (0)
#else
#define DPROF_INIT
#define DPROF_T(k)
#endif

// One launch per (head, chunk of <= 5 output tiles): the colour head of an SH model
// has 17 tiles, whose dW2 accumulators would not fit registers in one pass.  Every
// launch recomputes its head's hidden layer, forms dY from the output gradients,
// and adds its share of dH = W2^T dY (ReLU-masked), dX = W1^T dH (-> d feat, d anchor
// through ob_view), dW2 = dY H^T and dW1 = dH X^T.  Weight gradients accumulate in
// registers over the launch's grid-stride tiles and are flushed as per-wave partials
// that decode_wgrad_reduce_kernel sums in a fixed order (deterministic).
constexpr int kBwdChunk = 5;  // output tiles per launch

// the backward only needs 1 - tanh^2 (absolute accuracy of tanh suffices): exp-based
__device__ __forceinline__ float fast_tanh(float x) {
    const float e = __expf(-2.0f * fabsf(x));
    return copysignf((1.0f - e) * __builtin_amdgcn_rcpf(1.0f + e), x);
}

struct DecodeGrads {
    const float* g_xyz;      // [M,3]
    const float* g_offsets;  // [M,3] nullable
    const float* g_color;    // [M,cd] nullable
    const float* g_opacity;  // [M] nullable
    const float* g_scaling;  // [M,3] nullable
    const float* g_rot;      // [M,4] nullable
    float* d_anchor;         // [A,3] accumulated (+=), nullable
    float* d_feat;           // [A,F] accumulated (+=)
    float* d_offset;         // [A,noff,3] written by the cov launch
    float* d_scaling;        // [A,6] accumulated (+=)
};

// LDS of a backward launch, sized per head: R = second-layer rows of a chunk,
// YR = recomputed pre-activation rows (0 for the linear colour head)
template <int R, int YR>
struct DecodeBwdSmem {
    float w1[32 * kDecS];
    float b1[32];
    float w2[YR * kDecS];  // YR >= R rows: the cov head stages (and recomputes) all of its rows
    float b2[YR];
    float x[4][16 * kDecS];
    float dy[4][YR * kDecBS];  // recomputed pre-activations Y^T, overwritten in place by dY^T[o][anchor]
    float h[4][32 * kDecBS];                 // H^T, then dH^T [hidden][anchor]
};

// partial layout per wave: dW2 chunk [nt*16][32] | db2 chunk [nt*16] | dW1 [32][48] | db1 [32]
__host__ __device__ inline int bwd_partial_floats(int nt) { return nt * 16 * 32 + nt * 16 + 32 * 48 + 32; }

template <int KSTEPS, int HEAD, int NT>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(HEAD == 0 ? 3 : 2, 8))) void decode_bwd_kernel(DecodeDims d, MlpPtrs mp, int t0, int nt,
                                                         const int32_t* __restrict__ vis_idx,
                                                         const float* __restrict__ anchor,
                                                         const float* __restrict__ feat,
                                                         const float* __restrict__ offset,
                                                         const float* __restrict__ scaling_raw,
                                                         const float* __restrict__ cam,
                                                         const int32_t* __restrict__ slot_row, DecodeGrads gr,
                                                         float* __restrict__ partials) {
    constexpr int R = NT * 16;                     // NT >= nt: accumulators sized to the chunk
    constexpr int RY = HEAD == 1 ? 5 * 16 : R;     // cov: all rows (a slot's 7 outputs straddle tiles)
    __shared__ DecodeBwdSmem<R, RY> sm;
    constexpr int head = HEAD;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, i = lane & 15, g = lane >> 4;
    const int K1 = kDecF + d.vd;
    const int noff = d.noff, cd = d.cd;
    const int o0 = t0 * 16, O = d.O[head], rows = nt * 16;
    // rows of W2 / Y staged in LDS: the whole head for cov (chunk rows start at co), else the chunk
    const int srow0 = head == 1 ? 0 : o0, srows = head == 1 ? d.T[1] * 16 : rows, co = head == 1 ? o0 : 0;
    // stage this head's layer-1 weights and the chunk of layer-2 rows (permuted columns)
    for (int e = threadIdx.x; e < 32 * kDecS; e += 256) {
        const int h = e / kDecS, k = e - h * kDecS;
        sm.w1[e] = k < K1 ? mp.w1[head][h * K1 + k] : 0.f;
    }
    if (threadIdx.x < 32) sm.b1[threadIdx.x] = mp.b1[head][threadIdx.x];
    for (int e = threadIdx.x; e < srows * kDecF; e += 256) {
        const int row = e / kDecF, h = e - row * kDecF;
        const int o = srow0 + row;
        sm.w2[row * kDecS + w2_col(h)] = o < O ? mp.w2[head][o * kDecF + h] : 0.f;
    }
    for (int row = threadIdx.x; row < srows; row += 256)
        sm.b2[row] = srow0 + row < O ? mp.b2[head][srow0 + row] : 0.f;
    f32x4 aw2[NT][2], aw1[2][3];
#pragma unroll
    for (int a = 0; a < NT; ++a) aw2[a][0] = aw2[a][1] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int a = 0; a < 2; ++a) aw1[a][0] = aw1[a][1] = aw1[a][2] = f32x4{0.f, 0.f, 0.f, 0.f};
    double ab2[2] = {0.0, 0.0}, ab1 = 0.0;  // bias sums over many anchors: f64
    float* sx = sm.x[wave];
    float* sdy = sm.dy[wave];
    float* sy = sdy;  // every slot reads its own Y entries before writing its dY there
    float* sh = sm.h[wave];
    const int n_tiles = (d.Av + kDecTile - 1) / kDecTile;
    __syncthreads();  // weights staged
    DPROF_INIT
    // Every per-tile LDS array (x, Y / dY, H / dH, per-anchor sums) belongs to one wave, so
    // the waves of a block run their tiles independently: a wave's LDS operations complete
    // in order, and the waits below only keep the compiler from reordering across phases.
    // software pipeline (one tile ahead): X rows of the next tile; this tile's slot rows,
    // output-gradient gathers and the old values of the accumulated input gradients are
    // issued before the MFMA phases that hide their latency
    XPrefetch px;
    if (blockIdx.x < (unsigned)n_tiles) {
        x_issue_id(px, vis_idx, blockIdx.x * kDecTile + wave * 16, d.Av);
        x_issue_data(px, feat, anchor, d.vd);
    }
    // slots of the opacity / cov heads: lane (anchor i, group g) takes offsets k = g + 4 it,
    // it < 3 (n_offsets <= 12), so an anchor's slot sums reduce across the 4 lane groups with
    // two cross-lane adds instead of LDS float atomics (3 cycles per lane each on the CU)
    constexpr int kSI = 3;
    constexpr int kCI = NT * 4;  // colour head: rows * 16 / 64 (anchor, output) pairs per lane
    for (int t = blockIdx.x; t < n_tiles; t += gridDim.x) {
        wave_lds_sync();  // this wave's previous tile is done with its LDS arrays
        const int a0 = t * kDecTile + wave * 16;
        float my_ov[3], my_dist;
        x_store(px, sx, d.vd, cam, my_ov, my_dist);
        const int cur_id = px.id;  // lane i (= lane & 15): id of anchor i of this tile, -1 past Av
        const int tn = t + gridDim.x;
        if (tn < n_tiles) x_issue_id(px, vis_idx, tn * kDecTile + wave * 16, d.Av);
        // old values of the accumulated input gradients of this tile (d feat rows of anchor i,
        // columns kt*16 + 4g + r; d anchor / d scaling_raw on lanes < 16)
        float old_feat[2][4], old_anc[3] = {0.f, 0.f, 0.f}, old_sc[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kt = 0; kt < 2; ++kt)
#pragma unroll
            for (int r = 0; r < 4; ++r)
                old_feat[kt][r] = cur_id >= 0 ? gr.d_feat[(int64_t)cur_id * kDecF + kt * 16 + 4 * g + r] : 0.f;
        const bool anc_lane = lane < 16 && cur_id >= 0 && gr.d_anchor && (d.vd > 0 || (head == 1 && t0 == 0));
        if (anc_lane)
#pragma unroll
            for (int q = 0; q < 3; ++q) old_anc[q] = gr.d_anchor[(int64_t)cur_id * 3 + q];
        if (head == 1 && t0 == 0 && lane < 16 && cur_id >= 0)
#pragma unroll
            for (int q = 0; q < 6; ++q) old_sc[q] = gr.d_scaling[(int64_t)cur_id * 6 + q];
        // slot rows of this tile's (anchor, offset) slots
        int sp[kSI], cp[kCI];
#pragma unroll
        for (int it = 0; it < kSI; ++it) {
            const int k = g + 4 * it;
            sp[it] = (head < 2 && k < noff && cur_id >= 0) ? slot_row[(int64_t)(a0 + i) * noff + k] : -1;
        }
#pragma unroll
        for (int it = 0; it < kCI; ++it) {
            const int e = lane + 64 * it, ol = e >> 4, a = e & 15, o = o0 + ol;
            const int k = o / cd;
            cp[it] = (head == 2 && gr.g_color && ol < rows && o < O && a0 + a < d.Av)
                         ? slot_row[(int64_t)(a0 + a) * noff + k] : -1;
        }
        wave_lds_sync();
        DPROF_T(0);
        // hidden layer of this head (rows 0..31 of sm.w1)
        f32x4 h0 = {0.f, 0.f, 0.f, 0.f}, h1 = h0;
#pragma unroll
        for (int kk = 0; kk < KSTEPS; ++kk) {
            h0 = mfma4(sm.w1[i * kDecS + 4 * kk + g], sx[i * kDecS + 4 * kk + g], h0);
            h1 = mfma4(sm.w1[(16 + i) * kDecS + 4 * kk + g], sx[i * kDecS + 4 * kk + g], h1);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            h0[r] = fmaxf(h0[r] + sm.b1[4 * g + r], 0.f);
            h1[r] = fmaxf(h1[r] + sm.b1[16 + 4 * g + r], 0.f);
            sh[(4 * g + r) * kDecBS + i] = h0[r];
            sh[(16 + 4 * g + r) * kDecBS + i] = h1[r];
        }
        // the next tile's X rows (its ids have arrived) and this tile's output-gradient gathers
        if (tn < n_tiles) x_issue_data(px, feat, anchor, d.vd);
        float gop[kSI], gcol[kCI];
        float gsc[kSI][3], grt[kSI][4], gxy[kSI][3], gof[kSI][3], ofs[kSI][3], srw[6];
#pragma unroll
        for (int it = 0; it < kSI; ++it) {
            const int k = g + 4 * it;
            const int64_t p = sp[it] < 0 ? 0 : sp[it];
            const bool live = sp[it] >= 0;
            gop[it] = (head == 0 && live && gr.g_opacity) ? gr.g_opacity[p] : 0.f;
            if (head == 1) {
                const int64_t id = cur_id < 0 ? 0 : cur_id;
#pragma unroll
                for (int q = 0; q < 3; ++q) {
                    gsc[it][q] = (live && gr.g_scaling) ? gr.g_scaling[p * 3 + q] : 0.f;
                    gxy[it][q] = (live && gr.g_xyz && t0 == 0) ? gr.g_xyz[p * 3 + q] : 0.f;
                    gof[it][q] = (live && gr.g_offsets && t0 == 0) ? gr.g_offsets[p * 3 + q] : 0.f;
                    ofs[it][q] = (live && t0 == 0) ? offset[(id * noff + k) * 3 + q] : 0.f;
                }
#pragma unroll
                for (int q = 0; q < 4; ++q) grt[it][q] = (live && gr.g_rot) ? gr.g_rot[p * 4 + q] : 0.f;
            }
        }
        if (head == 1)  // the anchor's raw scaling, once per lane (all its slots share it)
#pragma unroll
            for (int q = 0; q < 6; ++q) srw[q] = cur_id >= 0 ? scaling_raw[(int64_t)cur_id * 6 + q] : 0.f;
#pragma unroll
        for (int it = 0; it < kCI; ++it) {
            const int e = lane + 64 * it, o = o0 + (e >> 4);
            const int c = o - (o / cd) * cd;
            gcol[it] = cp[it] >= 0 ? gr.g_color[(int64_t)cp[it] * cd + c] : 0.f;
        }
        DPROF_T(1);
        // recompute the pre-activations the derivative needs
        if (head < 2) {
            for (int ot = 0; ot < srows / 16; ++ot) {
                f32x4 y = {0.f, 0.f, 0.f, 0.f};
                const float* w = sm.w2 + (ot * 16 + i) * kDecS + g;
#pragma unroll
                for (int r = 0; r < 4; ++r) y = mfma4(w[4 * r], h0[r], y);
#pragma unroll
                for (int r = 0; r < 4; ++r) y = mfma4(w[16 + 4 * r], h1[r], y);
#pragma unroll
                for (int r = 0; r < 4; ++r) sy[(ot * 16 + 4 * g + r) * kDecBS + i] = y[r] + sm.b2[ot * 16 + 4 * g + r];
            }
        }
        DPROF_T(2);
        // dY^T for the chunk, in place over Y^T for the opacity / cov heads: every slot writes
        // all of its rows (zeros when dropped or absent), padding rows are zeroed separately
        if (head == 2) {
#pragma unroll
            for (int it = 0; it < kCI; ++it) {
                const int e = lane + 64 * it;
                if ((e >> 4) < rows) sdy[(e >> 4) * kDecBS + (e & 15)] = gcol[it];
            }
        } else {
            const int used = head == 0 ? noff : 7 * noff;
            for (int e = lane; e < (srows - used) * 16; e += 64) sdy[(used + (e >> 4)) * kDecBS + (e & 15)] = 0.f;
        }
        // per-anchor sums of this lane's slots (cov head): d scaling_raw 0..5, d anchor 0..2
        float asum[9] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        if (head == 0) {
#pragma unroll
            for (int it = 0; it < kSI; ++it) {
                const int k = g + 4 * it;
                if (k >= noff) continue;
                float v = 0.f;
                if (sp[it] >= 0 && gr.g_opacity) {
                    const float th = fast_tanh(sy[k * kDecBS + i]);
                    v = gop[it] * (1.0f - th * th);
                }
                sdy[k * kDecBS + i] = v;
            }
        } else if (head == 1) {
#pragma unroll
            for (int it = 0; it < kSI; ++it) {
                const int a = i, k = g + 4 * it;
                if (k >= noff) continue;
                const int64_t id = cur_id;
                const int p = sp[it];
                float cv[7], dv[7];
#pragma unroll
                for (int q = 0; q < 7; ++q) {
                    cv[q] = sy[(7 * k + q) * kDecBS + a];
                    dv[q] = 0.f;
                }
                if (p < 0) {
#pragma unroll
                    for (int q = 0; q < 7; ++q) sdy[(7 * k + q) * kDecBS + a] = 0.f;
                    if (id >= 0 && t0 == 0) {
                        float* dof = gr.d_offset + (id * noff + k) * 3;
                        dof[0] = dof[1] = dof[2] = 0.f;
                    }
                    continue;
                }
                // scaling = exp(sr[3:6]) * sigmoid(cv[0:3])
                if (gr.g_scaling) {
#pragma unroll
                    for (int q = 0; q < 3; ++q) {
                        const float es = __expf(srw[3 + q]), sg = __builtin_amdgcn_rcpf(1.0f + __expf(-cv[q]));
                        const float gs = gsc[it][q];
                        dv[q] = gs * es * sg * (1.0f - sg);
                        asum[3 + q] += gs * es * sg;
                    }
                }
                // rot = v / max(|v|, 1e-12)
                if (gr.g_rot) {
                    const float n2 = cv[3] * cv[3] + cv[4] * cv[4] + cv[5] * cv[5] + cv[6] * cv[6];
                    if (n2 > 1e-24f) {  // |v| > 1e-12
                        const float inv = __builtin_amdgcn_rsqf(n2);
                        float dot = 0.f;
#pragma unroll
                        for (int q = 0; q < 4; ++q) dot += cv[3 + q] * inv * grt[it][q];
#pragma unroll
                        for (int q = 0; q < 4; ++q) dv[3 + q] = (grt[it][q] - cv[3 + q] * inv * dot) * inv;
                    } else {
#pragma unroll
                        for (int q = 0; q < 4; ++q) dv[3 + q] = grt[it][q] * 1e12f;
                    }
                }
#pragma unroll
                for (int q = 0; q < 7; ++q) sdy[(7 * k + q) * kDecBS + a] = dv[q];
                if (t0 != 0) continue;  // the position / offset chain belongs to the first cov chunk
                // xyz = anchor + offset * exp(sr[0:3]); offsets_out = offset * exp(sr[0:3])
                float* dof = gr.d_offset + (id * noff + k) * 3;
#pragma unroll
                for (int q = 0; q < 3; ++q) {
                    const float gx = gxy[it][q];
                    const float gt = gx + gof[it][q];
                    const float es = __expf(srw[q]);
                    dof[q] = gt * es;
                    asum[q] += gt * ofs[it][q] * es;
                    asum[6 + q] += gx;
                }
            }
            // the anchor's slot sums: its 4 lane groups g (offsets g + 4 it) combined
            if (t0 == 0)
#pragma unroll
                for (int q = 0; q < 9; ++q) {
                    asum[q] += __shfl_xor(asum[q], 16);
                    asum[q] += __shfl_xor(asum[q], 32);
                }
        }
        DPROF_T(3);
        // per-anchor d scaling_raw / d anchor of the cov head (xyz and scaling outputs); the
        // d anchor sum joins the view-direction term of dX below (one store per tile)
        float anc_add[3] = {0.f, 0.f, 0.f};
        if (head == 1 && t0 == 0) {
            if (lane < 16 && cur_id >= 0) {
#pragma unroll
                for (int q = 0; q < 6; ++q) gr.d_scaling[(int64_t)cur_id * 6 + q] = old_sc[q] + asum[q];
#pragma unroll
                for (int q = 0; q < 3; ++q) anc_add[q] = asum[6 + q];
                if (gr.d_anchor && d.vd == 0)
#pragma unroll
                    for (int q = 0; q < 3; ++q) gr.d_anchor[(int64_t)cur_id * 3 + q] = old_anc[q] + anc_add[q];
            }
        }
        DPROF_T(4);
        // dW2 += dY H^T (k = anchors), db2 += row sums of dY
#pragma unroll
        for (int ot = 0; ot < NT; ++ot) {
            if (ot < nt) {  // static indices: the accumulators stay in registers
#pragma unroll
                for (int ht = 0; ht < 2; ++ht) {
#pragma unroll
                    for (int kk = 0; kk < 4; ++kk)
                        aw2[ot][ht] = mfma4(sdy[(co + ot * 16 + i) * kDecBS + 4 * kk + g],
                                            sh[(ht * 16 + i) * kDecBS + 4 * kk + g], aw2[ot][ht]);
                }
            }
        }
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const int ol = lane + 64 * q;
            if (ol < rows) {
                float sum = 0.f;
#pragma unroll
                for (int a = 0; a < 16; ++a) sum += sdy[(co + ol) * kDecBS + a];
                ab2[q] += sum;
            }
        }
        DPROF_T(5);
        // dH = W2^T dY, masked by ReLU; then stored transposed for dW1
        f32x4 d0 = {0.f, 0.f, 0.f, 0.f}, d1 = d0;
        for (int kk = 0; kk < rows / 4; ++kk) {
            const int o = co + 4 * kk + g;
            const float b = sdy[o * kDecBS + i];
            d0 = mfma4(sm.w2[o * kDecS + w2_col(i)], b, d0);
            d1 = mfma4(sm.w2[o * kDecS + w2_col(16 + i)], b, d1);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            d0[r] = h0[r] > 0.f ? d0[r] : 0.f;
            d1[r] = h1[r] > 0.f ? d1[r] : 0.f;
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            sh[(4 * g + r) * kDecBS + i] = d0[r];
            sh[(16 + 4 * g + r) * kDecBS + i] = d1[r];
        }
        DPROF_T(6);
        // dW1 += dH X^T (k = anchors), db1 += row sums of dH
#pragma unroll
        for (int ht = 0; ht < 2; ++ht)
#pragma unroll
            for (int kt = 0; kt < 3; ++kt) {
                if (kt * 16 >= K1) break;
#pragma unroll
                for (int kk = 0; kk < 4; ++kk)
                    aw1[ht][kt] = mfma4(sh[(ht * 16 + i) * kDecBS + 4 * kk + g], sx[(4 * kk + g) * kDecS + kt * 16 + i],
                                        aw1[ht][kt]);
            }
        if (lane < 32) {
            float sum = 0.f;
#pragma unroll
            for (int a = 0; a < 16; ++a) sum += sh[lane * kDecBS + a];
            ab1 += sum;
        }
        DPROF_T(7);
        // dX = W1^T dH -> d feat (k < 32), d ob_view (k = 32..34) -> d anchor.  The MFMAs run
        // with the whole wave (an MFMA consumes every lane's operands whatever EXEC says);
        // only the stores are predicated on the anchor being present.
        const bool present = cur_id >= 0;
#pragma unroll
        for (int kt = 0; kt < 3; ++kt) {
            if (kt * 16 >= K1) break;
            f32x4 dx = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int r = 0; r < 4; ++r) dx = mfma4(sm.w1[(4 * g + r) * kDecS + kt * 16 + i], d0[r], dx);
#pragma unroll
            for (int r = 0; r < 4; ++r) dx = mfma4(sm.w1[(16 + 4 * g + r) * kDecS + kt * 16 + i], d1[r], dx);
            if (!present) continue;
            if (kt < 2) {
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    gr.d_feat[(int64_t)cur_id * kDecF + kt * 16 + 4 * g + r] = old_feat[kt][r] + dx[r];
            } else if (g == 0 && gr.d_anchor) {
                const float dot = my_ov[0] * dx[0] + my_ov[1] * dx[1] + my_ov[2] * dx[2];
#pragma unroll
                for (int q = 0; q < 3; ++q)
                    gr.d_anchor[(int64_t)cur_id * 3 + q] = (old_anc[q] + anc_add[q]) + (dx[q] - my_ov[q] * dot) / my_dist;
            }
        }
        DPROF_T(8);
    }
    DPROF_T(9);
    // the four waves' weight-gradient partials summed in LDS in wave order (deterministic),
    // one partial per workgroup for decode_wgrad_sum_kernel
    __syncthreads();  // every wave is done with its tile arrays: the LDS is reused
    float* red = reinterpret_cast<float*>(&sm);
    static_assert(sizeof(sm) >= sizeof(float) * (R * 32 + R + 32 * 48 + 32), "LDS too small for the combine");
    for (int w = 0; w < 4; ++w) {
        if (wave == w) {
            auto put = [&](int idx, float v) { red[idx] = w == 0 ? v : red[idx] + v; };
#pragma unroll
            for (int ot = 0; ot < NT; ++ot) {
                if (ot < nt) {
#pragma unroll
                    for (int ht = 0; ht < 2; ++ht)
#pragma unroll
                        for (int r = 0; r < 4; ++r) put((ot * 16 + 4 * g + r) * 32 + ht * 16 + i, aw2[ot][ht][r]);
                }
            }
#pragma unroll
            for (int q = 0; q < 2; ++q)
                if (lane + 64 * q < rows) put(rows * 32 + lane + 64 * q, (float)ab2[q]);
#pragma unroll
            for (int ht = 0; ht < 2; ++ht)
#pragma unroll
                for (int kt = 0; kt < 3; ++kt)
#pragma unroll
                    for (int r = 0; r < 4; ++r)
                        put(rows * 33 + (ht * 16 + 4 * g + r) * 48 + kt * 16 + i, aw1[ht][kt][r]);
            if (lane < 32) put(rows * 33 + 32 * 48 + lane, (float)ab1);
        }
        __syncthreads();
    }
    const int pf = bwd_partial_floats(nt);
    float* out = partials + (int64_t)blockIdx.x * pf;
    for (int e = threadIdx.x; e < pf; e += 256) out[e] = red[e];
}

// ---------------------------------------------------------------- colour head backward, one launch
// An SH colour head (c4: 27 x 10 = 270 outputs, 17 tiles) used to take four chunked launches of
// decode_bwd_kernel, each re-staging X, recomputing the hidden layer and doing the dW1 / dX /
// d feat work again for its 5 tiles (a fixed ~68 us per launch at c4).  Here one launch covers
// every output row: the workgroup's four waves share their 64 anchors' hidden layer H (LDS) and
// walk the rows in chunks of 64 (one 16-row tile per wave):
//   * each wave gathers dY (the colour gradients of the kept slots, zero for dropped ones) of
//     its own 16 anchors for the chunk's rows into LDS, and the chunk's W2 rows are staged;
//   * dW2 of the wave's tile accumulates over all 64 anchors (K = anchors, H from LDS) -- so
//     every wave keeps <= 5 tiles of dW2 accumulators, as in the chunked launches;
//   * dH of the wave's own anchors accumulates over the chunk's rows (W2^T dY).
// After the last chunk each wave finishes its anchors as decode_bwd_kernel does (ReLU mask,
// dW1, dX -> d feat / d anchor, one read-modify-write of d feat instead of four).  dW2 rows
// are owned by one wave each and go straight to the workgroup's partial; dW1 / db1 are summed
// over the waves in wave order (deterministic).  Fragment reads use padded strides (one base
// register + immediate offsets per pattern): ydt at 68 floats per anchor row is conflict-free
// for the dH fragment and 2-way for the dW2 one; hs / w2c at 32 are 2-way.
constexpr int kColBwdTilesPerWave = 5;  // <= 20 output tiles (320 rows)
constexpr int kYdtS = 68;               // ydt row stride (floats)

struct DecodeColBwdSmem {
    float w1[32 * kDecS];
    float b1[32];
    float x[4][16 * kDecS];
    float ydt[64 * kYdtS];  // the chunk's dY: [anchor][row]; after the chunks: dH^T scratch, reduction
    float hs[64 * 32];      // H of the tile's anchors: [anchor][hidden]
    float w2c[64 * 32];     // the chunk's W2 rows: [row][hidden]
    int slot[64 * 12];      // slot rows of the tile's (anchor, offset) pairs
};

#ifndef HGSR_COLBWD_WAVES
#define HGSR_COLBWD_WAVES 2  // waves / SIMD: 234 VGPRs, no spills (at 3 it spills ~170: 0.864 vs 0.803 ms at c4)
#endif
template <int KSTEPS>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(HGSR_COLBWD_WAVES, 8))) void decode_bwd_color_kernel(DecodeDims d, MlpPtrs mp,
                                                                  const int32_t* __restrict__ vis_idx,
                                                                  const float* __restrict__ anchor,
                                                                  const float* __restrict__ feat,
                                                                  const float* __restrict__ cam,
                                                                  const int32_t* __restrict__ slot_row,
                                                                  DecodeGrads gr, float* __restrict__ partials) {
    constexpr int NTW = kColBwdTilesPerWave;
    __shared__ DecodeColBwdSmem sm;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, i = lane & 15, g = lane >> 4;
    const int K1 = kDecF + d.vd, noff = d.noff, cd = d.cd, O = d.O[2], T = d.T[2];
    const int n_chunks = (T + 3) / 4;
    const float* gcol = gr.g_color;  // non-null: the host skips a colour head without gradients
    for (int e = threadIdx.x; e < 32 * kDecS; e += 256) {
        const int h = e / kDecS, k = e - h * kDecS;
        sm.w1[e] = k < K1 ? mp.w1[2][h * K1 + k] : 0.f;
    }
    if (threadIdx.x < 32) sm.b1[threadIdx.x] = mp.b1[2][threadIdx.x];
    f32x4 aw2[NTW][2], aw1[2][3];
#pragma unroll
    for (int c = 0; c < NTW; ++c) aw2[c][0] = aw2[c][1] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int a = 0; a < 2; ++a) aw1[a][0] = aw1[a][1] = aw1[a][2] = f32x4{0.f, 0.f, 0.f, 0.f};
    double ab2[NTW], ab1 = 0.0;
#pragma unroll
    for (int c = 0; c < NTW; ++c) ab2[c] = 0.0;
    float* sx = sm.x[wave];
    const int n_tiles = (d.Av + kDecTile - 1) / kDecTile;
    XPrefetch px;
    if (blockIdx.x < (unsigned)n_tiles) {
        x_issue_id(px, vis_idx, blockIdx.x * kDecTile + wave * 16, d.Av);
        x_issue_data(px, feat, anchor, d.vd);
    }
    __syncthreads();  // W1 staged
    for (int t = blockIdx.x; t < n_tiles; t += gridDim.x) {
        const int A0 = t * kDecTile;     // the workgroup's 64 anchors
        float my_ov[3], my_dist;
        x_store(px, sx, d.vd, cam, my_ov, my_dist);
        const int cur_id = px.id;  // lane i: id of anchor i of this wave, -1 past Av
        for (int e = threadIdx.x; e < kDecTile * noff; e += 256)
            sm.slot[e] = A0 + e / noff < d.Av ? slot_row[(int64_t)A0 * noff + e] : -1;
        const int tn = t + gridDim.x;
        if (tn < n_tiles) x_issue_id(px, vis_idx, tn * kDecTile + wave * 16, d.Av);
        float old_feat[2][4], old_anc[3] = {0.f, 0.f, 0.f};
#pragma unroll
        for (int kt = 0; kt < 2; ++kt)
#pragma unroll
            for (int r = 0; r < 4; ++r)
                old_feat[kt][r] = cur_id >= 0 ? gr.d_feat[(int64_t)cur_id * kDecF + kt * 16 + 4 * g + r] : 0.f;
        const bool anc_lane = lane < 16 && cur_id >= 0 && gr.d_anchor && d.vd > 0;
        if (anc_lane)
#pragma unroll
            for (int q = 0; q < 3; ++q) old_anc[q] = gr.d_anchor[(int64_t)cur_id * 3 + q];
        wave_lds_sync();
        // hidden layer of this wave's anchors, published to the workgroup as H[anchor][hidden]
        f32x4 h0 = {0.f, 0.f, 0.f, 0.f}, h1 = h0;
#pragma unroll
        for (int kk = 0; kk < KSTEPS; ++kk) {
            h0 = mfma4(sm.w1[i * kDecS + 4 * kk + g], sx[i * kDecS + 4 * kk + g], h0);
            h1 = mfma4(sm.w1[(16 + i) * kDecS + 4 * kk + g], sx[i * kDecS + 4 * kk + g], h1);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            h0[r] = fmaxf(h0[r] + sm.b1[4 * g + r], 0.f);
            h1[r] = fmaxf(h1[r] + sm.b1[16 + 4 * g + r], 0.f);
            sm.hs[(wave * 16 + i) * 32 + 4 * g + r] = h0[r];
            sm.hs[(wave * 16 + i) * 32 + 16 + 4 * g + r] = h1[r];
        }
        if (tn < n_tiles) x_issue_data(px, feat, anchor, d.vd);
        __syncthreads();  // H and the slot table published (every wave is past its last tile)
        f32x4 d0 = {0.f, 0.f, 0.f, 0.f}, d1 = d0;  // dH[hidden 4g + r (+16)][own anchor i]
        // chunk c works on aw2[0] / ab2[0], then the accumulators rotate by one (a rolled loop:
        // unrolled, the compiler hoists every chunk's fragment reads and spills); NTW rotations
        // per tile in all, so aw2[c] belongs to chunk c again after the tile
#pragma nounroll
        for (int c = 0; c < NTW; ++c) {
            if (c < n_chunks) {
            {
                // dY of this wave's anchors, rows [64 c, 64 c + 64): lane = row (a slot's colours
                // are contiguous, so a wave's loads cover whole slot rows)
                const int o = 64 * c + lane;
                const bool orow = o < O;
                const int k = orow ? o / cd : 0, ch = o - k * cd;
                // branch-free: a dropped slot (or a padding row) loads the first colour, then 0
                float v[16];
                const int* srow = sm.slot + wave * 16 * noff + k;
#pragma unroll
                for (int j = 0; j < 16; ++j) {
                    const int p = srow[j * noff];
                    const float x = gcol[(int64_t)(p > 0 ? p : 0) * cd + (orow ? ch : 0)];
                    v[j] = (orow & (p >= 0)) ? x : 0.f;
                }
                // the chunk's W2 rows: thread -> row tid / 4, 8 columns
                const int rr = threadIdx.x >> 2, hc = 8 * (threadIdx.x & 3), oo = 64 * c + rr;
                float w[8];
#pragma unroll
                for (int q = 0; q < 8; ++q) w[q] = oo < O ? mp.w2[2][oo * kDecF + hc + q] : 0.f;
#pragma unroll
                for (int j = 0; j < 16; ++j) sm.ydt[(wave * 16 + j) * kYdtS + lane] = v[j];
                *reinterpret_cast<float4*>(&sm.w2c[rr * 32 + hc]) = make_float4(w[0], w[1], w[2], w[3]);
                *reinterpret_cast<float4*>(&sm.w2c[rr * 32 + hc + 4]) = make_float4(w[4], w[5], w[6], w[7]);
            }
            __syncthreads();
            // dH of this wave's anchors over the chunk's rows: dH[h][a] += sum_r W2[r][h] dY[r][a]
            {
                const float* yb = sm.ydt + (wave * 16 + i) * kYdtS + g;
                const float* wb = sm.w2c + g * 32 + i;
#pragma unroll
                for (int kk = 0; kk < 16; ++kk) {
                    const float b = yb[4 * kk];
                    d0 = mfma4(wb[kk * 128], b, d0);
                    d1 = mfma4(wb[kk * 128 + 16], b, d1);
                }
            }
            // dW2 of this wave's tile (4 c + wave) over the 64 anchors, db2 partial row sums
            if (4 * c + wave < T) {
                float sum = 0.f;
                const float* ya = sm.ydt + g * kYdtS + wave * 16 + i;
                const float* hb = sm.hs + g * 32 + i;
#pragma unroll
                for (int kk = 0; kk < 16; ++kk) {
                    const float a = ya[4 * kk * kYdtS];
                    sum += a;
                    aw2[0][0] = mfma4(a, hb[kk * 128], aw2[0][0]);
                    aw2[0][1] = mfma4(a, hb[kk * 128 + 16], aw2[0][1]);
                }
                ab2[0] += sum;
            }
            __syncthreads();  // the chunk's ydt / w2c / hs reads are done before they are rewritten
            }
            const f32x4 r0 = aw2[0][0], r1 = aw2[0][1];
            const double rb = ab2[0];
#pragma unroll
            for (int q = 0; q + 1 < NTW; ++q) {
                aw2[q][0] = aw2[q + 1][0];
                aw2[q][1] = aw2[q + 1][1];
                ab2[q] = ab2[q + 1];
            }
            aw2[NTW - 1][0] = r0;
            aw2[NTW - 1][1] = r1;
            ab2[NTW - 1] = rb;
        }
        // ReLU mask, then dH^T through this wave's scratch (the chunk buffer, free now) for dW1
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            d0[r] = h0[r] > 0.f ? d0[r] : 0.f;
            d1[r] = h1[r] > 0.f ? d1[r] : 0.f;
        }
        float* sh = sm.ydt + wave * (32 * kDecBS);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            sh[(4 * g + r) * kDecBS + i] = d0[r];
            sh[(16 + 4 * g + r) * kDecBS + i] = d1[r];
        }
        wave_lds_sync();
#pragma unroll
        for (int ht = 0; ht < 2; ++ht)
#pragma unroll
            for (int kt = 0; kt < 3; ++kt) {
                if (kt * 16 >= K1) break;
#pragma unroll
                for (int kk = 0; kk < 4; ++kk)
                    aw1[ht][kt] = mfma4(sh[(ht * 16 + i) * kDecBS + 4 * kk + g], sx[(4 * kk + g) * kDecS + kt * 16 + i],
                                        aw1[ht][kt]);
            }
        if (lane < 32) {
            float sum = 0.f;
#pragma unroll
            for (int a = 0; a < 16; ++a) sum += sh[lane * kDecBS + a];
            ab1 += sum;
        }
        // dX = W1^T dH -> d feat (k < 32), d ob_view (k = 32..34) -> d anchor
        const bool present = cur_id >= 0;
#pragma unroll
        for (int kt = 0; kt < 3; ++kt) {
            if (kt * 16 >= K1) break;
            f32x4 dx = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int r = 0; r < 4; ++r) dx = mfma4(sm.w1[(4 * g + r) * kDecS + kt * 16 + i], d0[r], dx);
#pragma unroll
            for (int r = 0; r < 4; ++r) dx = mfma4(sm.w1[(16 + 4 * g + r) * kDecS + kt * 16 + i], d1[r], dx);
            if (!present) continue;
            if (kt < 2) {
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    gr.d_feat[(int64_t)cur_id * kDecF + kt * 16 + 4 * g + r] = old_feat[kt][r] + dx[r];
            } else if (g == 0 && gr.d_anchor) {
                const float dot = my_ov[0] * dx[0] + my_ov[1] * dx[1] + my_ov[2] * dx[2];
#pragma unroll
                for (int q = 0; q < 3; ++q)
                    gr.d_anchor[(int64_t)cur_id * 3 + q] = old_anc[q] + (dx[q] - my_ov[q] * dot) / my_dist;
            }
        }
    }
    // partial of this workgroup, layout of bwd_partial_floats(T): dW2 [rows][32] | db2 [rows] |
    // dW1 [32][48] | db1 [32].  dW2 / db2 rows belong to one wave each: stored directly.
    const int rows = T * 16;
    float* out = partials + (int64_t)blockIdx.x * bwd_partial_floats(T);
#pragma unroll
    for (int c = 0; c < NTW; ++c) {
        const int tt = 4 * c + wave;
        if (tt >= T) continue;
#pragma unroll
        for (int ht = 0; ht < 2; ++ht)
#pragma unroll
            for (int r = 0; r < 4; ++r) out[(tt * 16 + 4 * g + r) * 32 + ht * 16 + i] = aw2[c][ht][r];
        double s2 = ab2[c];
        s2 += __shfl_xor(s2, 16);
        s2 += __shfl_xor(s2, 32);
        if (g == 0) out[rows * 32 + tt * 16 + i] = (float)s2;
    }
    __syncthreads();  // the chunk buffer is reused for the dW1 / db1 sum
    float* red = sm.ydt;
    static_assert(sizeof(sm.ydt) >= sizeof(float) * (32 * 48 + 32), "LDS too small for the combine");
    for (int w = 0; w < 4; ++w) {
        if (wave == w) {
            auto put = [&](int idx, float v) { red[idx] = w == 0 ? v : red[idx] + v; };
#pragma unroll
            for (int ht = 0; ht < 2; ++ht)
#pragma unroll
                for (int kt = 0; kt < 3; ++kt)
#pragma unroll
                    for (int r = 0; r < 4; ++r) put((ht * 16 + 4 * g + r) * 48 + kt * 16 + i, aw1[ht][kt][r]);
            if (lane < 32) put(32 * 48 + lane, (float)ab1);
        }
        __syncthreads();
    }
    for (int e = threadIdx.x; e < 32 * 48 + 32; e += 256) out[rows * 33 + e] = red[e];
}

// sum the per-wave partials of one launch into the weight gradients (+=), in two
// fixed-order levels: decode_wgrad_sum_kernel folds groups of partials (f64 sums),
// decode_wgrad_reduce_kernel folds the groups and scatters into the gradient tensors
constexpr int kRedGroups = 32;

__global__ __launch_bounds__(256) void decode_wgrad_sum_kernel(int n_parts, int pf, const float* __restrict__ partials,
                                                               double* __restrict__ level2) {
    const int e = blockIdx.x * 256 + threadIdx.x;
    if (e >= pf) return;
    const int per = (n_parts + kRedGroups - 1) / kRedGroups;
    const int q0 = blockIdx.y * per, q1 = min(q0 + per, n_parts);
    double acc = 0.0;
    for (int q = q0; q < q1; ++q) acc += partials[(int64_t)q * pf + e];
    level2[(int64_t)blockIdx.y * pf + e] = acc;
}

__global__ __launch_bounds__(256) void decode_wgrad_reduce_kernel(int nt, int o0, int O, int K1,
                                                                  const double* __restrict__ level2,
                                                                  float* __restrict__ dw2, float* __restrict__ db2,
                                                                  float* __restrict__ dw1, float* __restrict__ db1) {
    const int pf = bwd_partial_floats(nt);
    const int e = blockIdx.x * 256 + threadIdx.x;
    if (e >= pf) return;
    double acc = 0.0;
    for (int q = 0; q < kRedGroups; ++q) acc += level2[(int64_t)q * pf + e];
    const float sum = (float)acc;
    const int rows = nt * 16;
    if (e < rows * 32) {
        const int o = o0 + e / 32, h = e % 32;
        if (o < O) dw2[o * 32 + h] += sum;
    } else if (e < rows * 33) {
        const int o = o0 + e - rows * 32;
        if (o < O) db2[o] += sum;
    } else if (e < rows * 33 + 32 * 48) {
        const int q = e - rows * 33, h = q / 48, k = q % 48;
        if (k < K1) dw1[h * K1 + k] += sum;
    } else {
        db1[e - rows * 33 - 32 * 48] += sum;
    }
}

}  // namespace hgsr

using namespace hgsr;

extern "C" int hgsr_lod_mask(int A, const float* anchor, const int32_t* level, const float* extra_level,
                             const float* cam_center, float res_scale, float standard_dist, float log2_fork,
                             int max_level, uint8_t* mask, hgsr_stream_t stream) {
    HGSR_REQUIRE(A >= 0 && max_level >= 0, "bad dims");
    if (A == 0) return HGSR_OK;
    HGSR_REQUIRE(anchor && level && extra_level && cam_center && mask, "null pointer");
    hipLaunchKernelGGL(lod_mask_kernel, dim3((A + 255) / 256), dim3(256), 0, as_stream(stream), A, anchor, level,
                       extra_level, cam_center, res_scale, standard_dist, log2_fork, max_level, mask);
    return check_launch("lod_mask");
}

static int check_decode(int Av, int F, int vd, int noff, int cd, const DecodeDims& d) {
    HGSR_REQUIRE(Av >= 0, "bad dims");
    HGSR_REQUIRE(F == kDecF, "decode: feat_dim must be %d (got %d)", kDecF, F);
    HGSR_REQUIRE(vd == 0 || vd == 3, "decode: view_dim must be 0 or 3 (got %d)", vd);
    // 16 anchors x n_offsets slots per wave tile, 3 per lane; the cov head (7 x n_offsets rows) fits
    // 5 output tiles: n_offsets <= 11 (every reference config: 5 or 10)
    HGSR_REQUIRE(noff >= 1 && noff <= 11, "decode: n_offsets must be 1..11 (got %d)", noff);
    HGSR_REQUIRE(cd >= 1 && cd % 3 == 0, "decode: color_dim must be a positive multiple of 3 (got %d)", cd);
    HGSR_REQUIRE(d.rows <= kDecMaxRows, "decode: %d second-layer rows exceed the LDS plan (%d)", d.rows, kDecMaxRows);
    HGSR_REQUIRE(d.T[1] <= 5, "decode: n_offsets too large for the cov head plan");
    return HGSR_OK;
}

static int decode_grid(int Av) {
    const int n_tiles = (Av + kDecTile - 1) / kDecTile;
    return n_tiles < 1024 ? (n_tiles > 0 ? n_tiles : 1) : 1024;
}

// Workgroups of one decode launch (grid-stride over 64-anchor tiles): what an MI355X holds
// resident at once (the kernel's occupancy per CU x 256 CUs), so the grid-stride tiles run in
// one round (1024 workgroups of the 3-per-CU opacity-head backward left a second round a third
// full).  The CU count is the MI355X's constant, not the device's: the backward's weight
// gradients are summed over per-workgroup partials, so the grid fixes their summation order,
// and a grid that depended on the device (a partitioned GPU, another SKU) would change their
// last bits from machine to machine.  The occupancy is a property of the compiled gfx950 code.
constexpr int kGridCUs = 256;
static int grid_resident(const void* kernel, int Av) {
    static std::mutex mu;
    static std::map<const void*, int> cache;  // kernel -> resident workgroups
    int resident = 0;
    {
        std::lock_guard<std::mutex> lk(mu);
        auto it = cache.find(kernel);
        if (it != cache.end()) {
            resident = it->second;
        } else {
            int per_cu = 0;
            if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, 256, 0) != hipSuccess) per_cu = 0;
            resident = per_cu * kGridCUs;
            cache[kernel] = resident;
        }
    }
    const int g = decode_grid(Av);  // the backward's workspace bound
    return resident > 0 && resident < g ? resident : g;
}

static MlpPtrs mlp_ptrs(const float* const* w) {
    MlpPtrs mp;
    for (int h = 0; h < 3; ++h) {
        mp.w1[h] = w[4 * h];
        mp.b1[h] = w[4 * h + 1];
        mp.w2[h] = w[4 * h + 2];
        mp.b2[h] = w[4 * h + 3];
    }
    return mp;
}

extern "C" size_t hgsr_decode_ws_bytes(int Av) {
    const size_t n_tiles = ((size_t)Av + kDecTile - 1) / kDecTile + 1;
    return ((n_tiles * 4 + 255) & ~(size_t)255) * 2 + 256;
}

extern "C" int hgsr_decode_count(int Av, int F, int view_dim, int n_offsets, int color_dim,
                                 const int32_t* vis_idx, const float* anchor, const float* feat,
                                 const float* cam_center, const float* const* mlp, void* ws, size_t ws_bytes,
                                 int64_t* total, const int64_t* av_dev, hgsr_stream_t stream) {
    const DecodeDims d = decode_dims(Av, view_dim, n_offsets, color_dim);
    if (int st = check_decode(Av, F, view_dim, n_offsets, color_dim, d)) return st;
    HGSR_REQUIRE(ws_bytes >= hgsr_decode_ws_bytes(Av), "decode workspace too small");
    HGSR_REQUIRE(mlp && ws && total, "null pointer");
    hipStream_t s = as_stream(stream);
    if (Av == 0) return memset_async(total, sizeof(int64_t), s, "decode_count");
    HGSR_REQUIRE(anchor && feat && cam_center, "null pointer");
    for (int q = 0; q < 12; ++q) HGSR_REQUIRE(mlp[q], "null MLP pointer %d", q);
    const MlpPtrs mp = mlp_ptrs(mlp);
    const int n_tiles = (Av + kDecTile - 1) / kDecTile;
    // tile offsets first (decode_fwd finds them at the workspace start whatever Av it is given),
    // tile counts after them
    int32_t* off = (int32_t*)ws;
    int32_t* cnt = (int32_t*)((char*)ws + (((size_t)(n_tiles + 1) * 4 + 255) & ~(size_t)255));
    KernelTimer kt("decode_count", s);
    if (view_dim == 3)
        hipLaunchKernelGGL(decode_count_kernel<9>, dim3(grid_resident(reinterpret_cast<const void*>(&decode_count_kernel<9>), Av)), dim3(256), 0, s, d, mp, vis_idx, anchor,
                           feat, cam_center, cnt, av_dev);
    else
        hipLaunchKernelGGL(decode_count_kernel<8>, dim3(grid_resident(reinterpret_cast<const void*>(&decode_count_kernel<8>), Av)), dim3(256), 0, s, d, mp, vis_idx, anchor,
                           feat, cam_center, cnt, av_dev);
    if (int st = check_launch("decode_count")) return st;
    hipLaunchKernelGGL(decode_scan_kernel, dim3(1), dim3(1024), 0, s, n_tiles, cnt, off, total, av_dev);
    return check_launch("decode_scan");
}

extern "C" int hgsr_decode_fwd(int Av, int F, int view_dim, int n_offsets, int color_dim, const int32_t* vis_idx,
                               const float* anchor, const float* feat, const float* offset, const float* scaling_raw,
                               const float* cam_center, const float* const* mlp, float* xyz, float* offsets_out,
                               float* color, float* opacity, float* scaling, float* rot, uint8_t* mask,
                               int32_t* slot_row, void* ws, size_t ws_bytes, hgsr_stream_t stream) {
    const DecodeDims d = decode_dims(Av, view_dim, n_offsets, color_dim);
    if (int st = check_decode(Av, F, view_dim, n_offsets, color_dim, d)) return st;
    HGSR_REQUIRE(ws_bytes >= hgsr_decode_ws_bytes(Av), "decode workspace too small");
    if (Av == 0) return HGSR_OK;
    HGSR_REQUIRE(mlp && ws && anchor && feat && offset && scaling_raw && cam_center && mask && slot_row,
                 "null pointer");
    for (int q = 0; q < 12; ++q) HGSR_REQUIRE(mlp[q], "null MLP pointer %d", q);
    const MlpPtrs mp = mlp_ptrs(mlp);
    const int32_t* off = (const int32_t*)ws;  // written by hgsr_decode_count's scan
    DecodeOut out{xyz, offsets_out, color, opacity, scaling, rot, mask, slot_row};
    hipStream_t s = as_stream(stream);
    KernelTimer kt("decode_fwd", s);
#define LAUNCH_DF(KS, R)                                                                                      \
    hipLaunchKernelGGL((decode_fwd_kernel<KS, R>), dim3(grid_resident(reinterpret_cast<const void*>(&decode_fwd_kernel<KS, R>), Av)), dim3(256), 0, s, d, mp, vis_idx, anchor, \
                       feat, offset, scaling_raw, cam_center, off, out)
    // LDS sized to the model: RGB heads fit 128 second-layer rows (2 workgroups per CU); an SH
    // colour head of up to 272 rows runs as its own pass after the opacity / cov pass (2
    // workgroups per CU each instead of 1 for all 368 rows at once)
    if (d.rows <= 128) {
        if (view_dim == 3) LAUNCH_DF(9, 128);
        else LAUNCH_DF(8, 128);
    } else if (d.row0[2] <= 128 && d.T[2] * 16 <= kDecColRows) {
        if (view_dim == 3)
            hipLaunchKernelGGL((decode_fwd_kernel<9, 128, false>), dim3(grid_resident(reinterpret_cast<const void*>(&decode_fwd_kernel<9, 128, false>), Av)), dim3(256), 0, s, d, mp,
                               vis_idx, anchor, feat, offset, scaling_raw, cam_center, off, out);
        else
            hipLaunchKernelGGL((decode_fwd_kernel<8, 128, false>), dim3(grid_resident(reinterpret_cast<const void*>(&decode_fwd_kernel<8, 128, false>), Av)), dim3(256), 0, s, d, mp,
                               vis_idx, anchor, feat, offset, scaling_raw, cam_center, off, out);
        if (int st = check_launch("decode_fwd")) return st;
        if (view_dim == 3)
            hipLaunchKernelGGL(decode_color_kernel<9>, dim3(grid_resident(reinterpret_cast<const void*>(&decode_color_kernel<9>), Av)), dim3(256), 0, s, d, mp, vis_idx, anchor,
                               feat, cam_center, slot_row, color);
        else
            hipLaunchKernelGGL(decode_color_kernel<8>, dim3(grid_resident(reinterpret_cast<const void*>(&decode_color_kernel<8>), Av)), dim3(256), 0, s, d, mp, vis_idx, anchor,
                               feat, cam_center, slot_row, color);
    } else {
        if (view_dim == 3) LAUNCH_DF(9, kDecMaxRows);
        else LAUNCH_DF(8, kDecMaxRows);
    }
#undef LAUNCH_DF
    return check_launch("decode_fwd");
}

static int bwd_grid(int Av) {
    const int n_tiles = (Av + kDecTile - 1) / kDecTile;
    return n_tiles < 1024 ? (n_tiles > 0 ? n_tiles : 1) : 1024;
}


// partials: 4 per workgroup of a chunked launch, or 1 (all rows) of the one-launch colour head
static size_t bwd_part_floats_max() {
    const size_t a = 4 * (size_t)bwd_partial_floats(kBwdChunk), b = bwd_partial_floats(4 * kColBwdTilesPerWave);
    return a > b ? a : b;
}

extern "C" size_t hgsr_decode_bwd_ws_bytes(int Av) {
    const size_t parts = ((size_t)bwd_grid(Av) * bwd_part_floats_max() * sizeof(float) + 255) & ~(size_t)255;
    const size_t pf = bwd_partial_floats(4 * kColBwdTilesPerWave) > bwd_partial_floats(kBwdChunk)
                          ? bwd_partial_floats(4 * kColBwdTilesPerWave) : bwd_partial_floats(kBwdChunk);
    return parts + (size_t)kRedGroups * pf * sizeof(double);
}

// the SH colour head's backward form: 1 (default) one launch (decode_bwd_color_kernel), 0 the
// chunked launches it replaced (kept for the tests that compare the two); returns the previous
static int g_color_one = 1;
extern "C" int hgsr_decode_set_color_bwd(int one) {
    const int old = g_color_one;
    if (one >= 0) g_color_one = one != 0;
    return old;
}

extern "C" int hgsr_decode_bwd(int Av, int F, int view_dim, int n_offsets, int color_dim, const int32_t* vis_idx,
                               const float* anchor, const float* feat, const float* offset, const float* scaling_raw,
                               const float* cam_center, const float* const* mlp, const int32_t* slot_row,
                               const float* g_xyz, const float* g_offsets, const float* g_color,
                               const float* g_opacity, const float* g_scaling, const float* g_rot, float* d_anchor,
                               float* d_feat, float* d_offset, float* d_scaling, float* const* d_mlp, int head_mask,
                               void* ws, size_t ws_bytes, hgsr_stream_t stream) {
    const DecodeDims d = decode_dims(Av, view_dim, n_offsets, color_dim);
    if (int st = check_decode(Av, F, view_dim, n_offsets, color_dim, d)) return st;
    HGSR_REQUIRE(ws_bytes >= hgsr_decode_bwd_ws_bytes(Av), "decode_bwd workspace too small");
    if (Av == 0) return HGSR_OK;
    HGSR_REQUIRE(mlp && d_mlp && ws && anchor && feat && offset && scaling_raw && cam_center && slot_row && d_feat &&
                     d_offset && d_scaling,
                 "null pointer");
    for (int q = 0; q < 12; ++q) HGSR_REQUIRE(mlp[q] && d_mlp[q], "null MLP pointer %d", q);
    const MlpPtrs mp = mlp_ptrs(mlp);
    const DecodeGrads gr{g_xyz, g_offsets, g_color, g_opacity, g_scaling, g_rot, d_anchor, d_feat, d_offset, d_scaling};
    hipStream_t s = as_stream(stream);
    int grid = bwd_grid(Av);
    float* partials = (float*)ws;
    double* level2 = (double*)((char*)ws + (((size_t)grid * bwd_part_floats_max() * sizeof(float) + 255) & ~(size_t)255));
    // an SH colour head (more tiles than one chunked launch holds) in one launch:
    // decode_bwd_color_kernel; hgsr_decode_set_color_bwd(0) keeps the chunked launches (tests)
    const bool col_one = g_color_one != 0;
    const int K1 = kDecF + view_dim;
    KernelTimer kt("decode_bwd", s);
    // the cov head first: after it d_offset, d_scaling and the cov weights are final, so a
    // caller (multi-GPU) can start reducing them while the opacity and colour heads run
    static const int kOrder[3] = {1, 0, 2};
    const int mask = head_mask ? head_mask : 7;
    for (int hi = 0; hi < 3; ++hi) {
        const int head = kOrder[hi];
        if (!((mask >> head) & 1)) continue;
        // up to 5 output tiles per launch (the cov head in one launch; measured: splitting it
        // into 3 + 2 tiles gains nothing, its time is the per-tile work, not the accumulators)
        if (head == 2 && col_one && d.T[2] > kBwdChunk && d.T[2] <= 4 * kColBwdTilesPerWave) {
            if (!g_color) continue;  // no colour gradient: every term of this head is zero
            const int nt = d.T[2];
            if (view_dim == 3) {
                grid = grid_resident(reinterpret_cast<const void*>(&decode_bwd_color_kernel<9>), Av);
                hipLaunchKernelGGL(decode_bwd_color_kernel<9>, dim3(grid), dim3(256), 0, s, d, mp, vis_idx, anchor,
                                   feat, cam_center, slot_row, gr, partials);
            } else {
                grid = grid_resident(reinterpret_cast<const void*>(&decode_bwd_color_kernel<8>), Av);
                hipLaunchKernelGGL(decode_bwd_color_kernel<8>, dim3(grid), dim3(256), 0, s, d, mp, vis_idx, anchor,
                                   feat, cam_center, slot_row, gr, partials);
            }
            if (int st = check_launch("decode_bwd")) return st;
            const int pf = bwd_partial_floats(nt);
            hipLaunchKernelGGL(decode_wgrad_sum_kernel, dim3((pf + 255) / 256, kRedGroups), dim3(256), 0, s, grid,
                               pf, partials, level2);
            if (int st = check_launch("decode_wgrad_sum")) return st;
            hipLaunchKernelGGL(decode_wgrad_reduce_kernel, dim3((pf + 255) / 256), dim3(256), 0, s, nt, 0, d.O[2], K1,
                               level2, d_mlp[4 * 2 + 2], d_mlp[4 * 2 + 3], d_mlp[4 * 2], d_mlp[4 * 2 + 1]);
            if (int st = check_launch("decode_wgrad_reduce")) return st;
            continue;
        }
        const int chunk = kBwdChunk;
        for (int t0 = 0; t0 < d.T[head]; t0 += chunk) {
            const int nt = d.T[head] - t0 < chunk ? d.T[head] - t0 : chunk;
#define LAUNCH_DB(KS, HD, NTT)                                                                                 \
    do {                                                                                                       \
        grid = grid_resident(reinterpret_cast<const void*>(&decode_bwd_kernel<KS, HD, NTT>), Av);          \
        hipLaunchKernelGGL((decode_bwd_kernel<KS, HD, NTT>), dim3(grid), dim3(256), 0, s, d, mp, t0, nt, vis_idx,   \
                           anchor, feat, offset, scaling_raw, cam_center, slot_row, gr, partials);              \
    } while (0)
#define LAUNCH_DB_NT(KS, HD) \
    do {                                                               \
        if (nt <= 1) LAUNCH_DB(KS, HD, 1);                             \
        else if (nt <= 2) LAUNCH_DB(KS, HD, 2);                        \
        else if (nt <= 3) LAUNCH_DB(KS, HD, 3);                        \
        else LAUNCH_DB(KS, HD, 5);                                     \
    } while (0)
            if (view_dim == 3) {
                if (head == 0) LAUNCH_DB(9, 0, 1);
                else if (head == 1) LAUNCH_DB_NT(9, 1);
                else LAUNCH_DB_NT(9, 2);
            } else {
                if (head == 0) LAUNCH_DB(8, 0, 1);
                else if (head == 1) LAUNCH_DB_NT(8, 1);
                else LAUNCH_DB_NT(8, 2);
            }
#undef LAUNCH_DB_NT
#undef LAUNCH_DB
            if (int st = check_launch("decode_bwd")) return st;
            const int pf = bwd_partial_floats(nt);
            hipLaunchKernelGGL(decode_wgrad_sum_kernel, dim3((pf + 255) / 256, kRedGroups), dim3(256), 0, s, grid,
                               pf, partials, level2);
            if (int st = check_launch("decode_wgrad_sum")) return st;
            hipLaunchKernelGGL(decode_wgrad_reduce_kernel, dim3((pf + 255) / 256), dim3(256), 0, s, nt, t0 * 16,
                               d.O[head], K1, level2, d_mlp[4 * head + 2], d_mlp[4 * head + 3], d_mlp[4 * head],
                               d_mlp[4 * head + 1]);
            if (int st = check_launch("decode_wgrad_reduce")) return st;
        }
    }
    return HGSR_OK;
}

#ifdef HGSR_DECODE_PROF
extern "C" int hgsr_debug_decode_prof(unsigned long long* out, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_dprof), sizeof(unsigned long long) * 48) != hipSuccess) return -2;
    if (reset) {
        static const unsigned long long z[48] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_dprof), z, sizeof(z)) != hipSuccess) return -2;
    }
    return 0;
}
#endif
