// K15: fused training loss: masked L1 + D-SSIM, the scale regulariser
// and the alpha regularisers of reference train.py:153-178 with utils/loss_utils.py:17-60
// (Gaussian window 11, sigma 1.5, zero padding, C1 = 0.01^2, C2 = 0.03^2).
//
//   x = image * mask, y = gt * mask (mask [H,W] broadcast over channels, nullable)
//   loss = (1 - l) * mean|x - y| + l * (1 - mean SSIM(x, y)) + l_dreg * mean_i prod_j s_ij
//        + l_sky * mean(-(1 - mask) log(1 - a)) + l_ent * mean(-a log a),  a = clamp(alpha, 1e-6, 1 - 1e-6)
//
// CDNA4 mapping: one 256-lane workgroup per 16x16 pixel tile, all channels of a group of
// NC (3 for RGB) at once.  The tile plus its 5-pixel halo is staged in LDS, the 11-tap
// window is applied separably: a horizontal pass producing two adjacent columns per lane
// (12 LDS reads for 2 outputs) and a vertical pass producing four rows per lane from a
// 14-row register window, i.e. ~4x fewer LDS reads than one output per lane.  The forward
// writes the three per-pixel derivative maps the SSIM gradient needs,
//   dS/dx(q) = G*(S_mu1 - 2 mu1 S_s11 - mu2 S_s12)(q) + 2 x(q) G*S_s11(q) + y(q) G*S_s12(q),
// and the backward filters them the same way.  The scale regulariser rides along: tile
// block b also reduces Gaussians [b*per, (b+1)*per).  Per-tile partial sums are reduced
// in a fixed order in f64 (deterministic).
#include "common.h"

namespace hgsr {

constexpr int kLT = 32;            // tile edge (1024 pixels per 256-lane workgroup)
constexpr int kLR = 5;             // window radius
constexpr int kLH = kLT + 2 * kLR;  // 42: tile + halo
constexpr int kLP = kLH + 1;       // staged row pitch (43: 4 rows x 8 column quads hit 32 banks)
constexpr int kHP = kLT + 1;       // filtered row pitch (33: same for the quad writes)
constexpr int kLS = (kLH * kLH + 255) / 256;  // 7 staged positions per lane
constexpr int kLQ4 = kLT / 4;      // column / row quads per tile edge
constexpr int kLC = 3;             // channels held in registers (the loss is defined on RGB)
constexpr int kLossOuts = 9;       // loss, l1, ssim, sky, entropy, scale_reg, normal, distortion, inv_depth
constexpr int kLQ = 8;  // partial sums per tile: l1, ssim, sky, entropy, scale-prod, normal, distortion, inv-depth

// utils/loss_utils.py:20-22 window, exp(-(x - 5)^2 / (2 * 1.5^2)) normalised, rounded to
// fp32; compile-time literals so the unrolled filters carry them as instruction constants
// (no SGPRs).  check_window() verifies them against the f64 formula at first use.
constexpr float kWin[11] = {0x1.0d956cp-10f, 0x1.f1fe02p-8f, 0x1.26eb18p-5f, 0x1.bff0fep-4f,
                            0x1.b43c40p-3f,  0x1.106560p-2f, 0x1.b43c40p-3f, 0x1.bff0fep-4f,
                            0x1.26eb18p-5f,  0x1.f1fe02p-8f, 0x1.0d956cp-10f};

// a [C,H,W] image with arbitrary element strides (contiguous CHW, or the channels-last
// [H,W,C] render output viewed through permute(2,0,1) without a copy)
struct Img {
    const float* p;
    int64_t sc, sy, sx;
    __device__ __forceinline__ int64_t at(int c, int y, int x) const { return c * sc + y * sy + x * sx; }
};

struct ScaleReg {  // scale regulariser operand: scaling [n, k] contiguous (nullable)
    const float* s;
    int64_t n;
    int k;
};

// per-pixel terms of train.py:180-202 (all nullable): normal consistency (2DGS),
// distortion, inverse-depth L1.  Strided views like Img; gradients use the same strides.
struct LossAux {
    const float* nrm;  // render_normals [3,H,W]
    int64_t ns[3];
    const float* nfd;  // render_normals_from_depth [3,H,W] (times alpha.detach() here)
    int64_t fs[3];
    const float* dist;  // render_distort [H,W]
    int64_t dst[2];
    const float* depth;  // render_depth [H,W]
    int64_t dps[2];
    const float* mono;   // mono inverse depth [H,W] contiguous
    const float* dmask;  // depth mask [H,W] contiguous (nullable = 1)
    float* g_nrm;
    float* g_nfd;
    float* g_dist;
    float* g_depth;
};

struct LossLam {
    float dssim, sky, ent, dreg, normal, dist, depth;
};

// the aux terms' per-pixel values {normal error * mask, distortion * mask, |invD - mono| * dmask}
__device__ __forceinline__ void aux_terms(const LossAux& ax, const float* __restrict__ alpha,
                                          const float* __restrict__ mask, int W, int y, int x, float (&t)[3]) {
    const int64_t p = (int64_t)y * W + x;
    const float mk = mask ? mask[p] : 1.f;
    t[0] = t[1] = t[2] = 0.f;
    if (ax.nrm) {
        const float a = alpha ? alpha[p] : 1.f;
        float dot = 0.f;
#pragma unroll
        for (int c = 0; c < 3; ++c)
            dot += ax.nrm[c * ax.ns[0] + y * ax.ns[1] + x * ax.ns[2]] *
                   (ax.nfd[c * ax.fs[0] + y * ax.fs[1] + x * ax.fs[2]] * a);
        t[0] = (1.f - dot) * mk;
    }
    if (ax.dist) t[1] = ax.dist[y * ax.dst[0] + x * ax.dst[1]] * mk;
    if (ax.depth) {
        const float d = ax.depth[y * ax.dps[0] + x * ax.dps[1]];
        const float inv = d > 0.f ? 1.f / d : 0.f;
        t[2] = fabsf((inv - ax.mono[p]) * (ax.dmask ? ax.dmask[p] : 1.f));
    }
}

__device__ __forceinline__ float row_prod(const float* __restrict__ s, int k) {
    float p = s[0];
    for (int j = 1; j < k; ++j) p *= s[j];
    return p;
}

__device__ __forceinline__ float block_sum(float v, float* red) {
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d);
    const int wave = threadIdx.x >> 6;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[wave] = v;
    __syncthreads();
    return red[0] + red[1] + red[2] + red[3];
}

// staged position i of this lane: LDS index, image coordinates, inside-image flag
__device__ __forceinline__ bool stage_pos(int i, int H, int W, int x0, int y0, int& lds, int& yy, int& xx) {
    const int e = threadIdx.x + 256 * i;
    const int r = e / kLH, q = e - r * kLH;
    lds = e < kLH * kLH ? r * kLP + q : -1;
    yy = y0 + r;
    xx = x0 + q;
    return e < kLH * kLH && yy >= 0 && yy < H && xx >= 0 && xx < W;
}

// keeps the compiler from hoisting every LDS read of a filter pass to the top (which
// costs ~60 live VGPRs and halves occupancy); LDS latency is hidden by the other waves
__device__ __forceinline__ void sched_fence() { asm volatile("" ::: "memory"); }

// horizontal pass over NM staged maps: (row, column quad) items, 14-sample scatter form
// (each sample feeds up to four outputs, so only the accumulators stay live); map m of
// item (r, q4) -> hout[m][r * kHP + 4 q4 + o].  PROD adds x^2, y^2, xy of maps 0 and 1.
template <int NM, bool PROD>
__device__ __forceinline__ void hpass(const float* const (&in)[NM], float* const (&hout)[PROD ? 5 : NM]) {
    constexpr int NO = PROD ? 5 : NM;
    for (int item = threadIdx.x; item < kLH * kLQ4; item += 256) {
        const int q4 = item & (kLQ4 - 1), r = item / kLQ4;
        float acc[4][NO] = {};
#pragma unroll
        for (int t = 0; t < 14; ++t) {
            sched_fence();
            float v[NO];
#pragma unroll
            for (int m = 0; m < NM; ++m) v[m] = in[m][r * kLP + 4 * q4 + t];
            if constexpr (PROD) {
                v[2] = v[0] * v[0];
                v[3] = v[1] * v[1];
                v[4] = v[0] * v[1];
            }
#pragma unroll
            for (int o = 0; o < 4; ++o) {
                if (t - o < 0 || t - o > 10) continue;
#pragma unroll
                for (int m = 0; m < NO; ++m) acc[o][m] += kWin[t - o] * v[m];
            }
        }
#pragma unroll
        for (int o = 0; o < 4; ++o)
#pragma unroll
            for (int m = 0; m < NO; ++m) hout[m][r * kHP + 4 * q4 + o] = acc[o][m];
    }
}

// vertical pass: lane (column tx, row quad qd) filters 14 rows of each map into 4 outputs
template <int NO>
__device__ __forceinline__ void vpass(float* const (&h)[NO], int tx, int qd, float (&acc)[NO][4]) {
#pragma unroll
    for (int m = 0; m < NO; ++m)
#pragma unroll
        for (int o = 0; o < 4; ++o) acc[m][o] = 0.f;
#pragma unroll
    for (int t = 0; t < 14; ++t) {
        sched_fence();
#pragma unroll
        for (int m = 0; m < NO; ++m) {
            const float v = h[m][(4 * qd + t) * kHP + tx];
#pragma unroll
            for (int o = 0; o < 4; ++o)
                if (t - o >= 0 && t - o <= 10) acc[m][o] += kWin[t - o] * v;
        }
    }
}

struct LossFwdSmem {
    float x[kLH * kLP];
    float y[kLH * kLP];
    float h[5][kLH * kHP];  // horizontally filtered mu1, mu2, x^2, y^2, xy
    float red[4];
};

// SSIM at one pixel from the five filtered moments, with the derivative-map terms
struct SsimPix {
    float S, dm0, ds11, ds12;
};

__device__ __forceinline__ SsimPix ssim_pix(float mu1, float mu2, float ex2, float ey2, float exy) {
    const float C1 = 0.01f * 0.01f, C2 = 0.03f * 0.03f;
    const float mu1_sq = mu1 * mu1, mu2_sq = mu2 * mu2, mu12 = mu1 * mu2;
    const float s11 = ex2 - mu1_sq, s22 = ey2 - mu2_sq, s12 = exy - mu12;
    const float A1 = 2.f * mu12 + C1, A2 = 2.f * s12 + C2;
    const float B1 = mu1_sq + mu2_sq + C1, B2 = s11 + s22 + C2;
    const float rB1 = __builtin_amdgcn_rcpf(B1), rB2 = __builtin_amdgcn_rcpf(B2);
    const float inv = rB1 * rB2;
    SsimPix o;
    o.S = A1 * A2 * inv;
    const float dmu1 = 2.f * mu2 * A2 * inv - 2.f * mu1 * o.S * rB1;
    o.ds11 = -o.S * rB2;
    o.ds12 = 2.f * A1 * inv;
    o.dm0 = dmu1 - 2.f * mu1 * o.ds11 - mu2 * o.ds12;
    return o;
}

// forward: SSIM statistics + derivative maps, L1, alpha / aux terms, scale products;
// per-tile partials, layout [kLQ][n_tiles].  Channels are processed one at a time with
// the next channel's window already in flight in registers (LDS-only barriers keep it so).
__global__ __launch_bounds__(256, 3) void loss_fwd_kernel(int C, int H, int W, Img img, Img gt,
                                                       const float* __restrict__ mask,
                                                       const float* __restrict__ alpha, ScaleReg sr, LossAux ax,
                                                       float* __restrict__ dmaps, float* __restrict__ partials) {
    __shared__ LossFwdSmem sm;
    const int tiles_x = (W + kLT - 1) / kLT;
    // logical tile = XCD-contiguous remap of the dispatch index: the tiles of one XCD are a band
    // of neighbours, so the 5-px halos they share are L2 hits of that XCD, not HBM re-reads
    const int blk = xcd_remap(blockIdx.x, gridDim.x);
    const int bx = blk % tiles_x, by = blk / tiles_x;
    const int x0 = bx * kLT - kLR, y0 = by * kLT - kLR;
    const int64_t HW = (int64_t)H * W;
    const int tid = threadIdx.x;
    // the whole window for every channel is loaded up front: a pixel's channels are read
    // together (channels-last renders are not re-fetched once per channel)
    float nx[kLC][kLS], ny[kLC][kLS], nm[kLS];
#pragma unroll
    for (int i = 0; i < kLS; ++i) {
        int l, yy, xx;
        const bool in = stage_pos(i, H, W, x0, y0, l, yy, xx);
#pragma unroll
        for (int c = 0; c < kLC; ++c) {
            const bool ok = in && c < C;
            nx[c][i] = ok ? img.p[(unsigned)(c * img.sc + yy * img.sy + xx * img.sx)] : 0.f;
            ny[c][i] = ok ? gt.p[(unsigned)(c * gt.sc + yy * gt.sy + xx * gt.sx)] : 0.f;
        }
        nm[i] = (in && mask) ? mask[(unsigned)(yy * W + xx)] : 1.f;
    }
    // per-pixel alpha / aux terms and this block's share of the scale products
    float sky = 0.f, ent = 0.f, aux[3] = {0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < kLT * kLT / 256; ++j) {
        const int pl = tid + 256 * j;
        const int px = bx * kLT + (pl & (kLT - 1)), py = by * kLT + pl / kLT;
        if (px >= W || py >= H) continue;
        const int64_t p = (int64_t)py * W + px;
        if (alpha) {
            const float o = fminf(fmaxf(alpha[p], 1e-6f), 1.f - 1e-6f);
            const float sk = mask ? mask[p] : 1.f;
            sky += -(1.f - sk) * logf(1.f - o);
            ent += -o * logf(o);
        }
        float t[3];
        aux_terms(ax, alpha, mask, W, py, px, t);
#pragma unroll
        for (int q = 0; q < 3; ++q) aux[q] += t[q];
    }
    float dreg = 0.f;
    if (sr.s) {
        const int64_t per = (sr.n + gridDim.x - 1) / gridDim.x;
        const int64_t g0 = (int64_t)blk * per, g1 = min(sr.n, g0 + per);
        for (int64_t g = g0 + tid; g < g1; g += 256) dreg += row_prod(sr.s + g * sr.k, sr.k);
    }
    const int tx = tid & (kLT - 1), qd = tid / kLT;  // vertical pass: column, row quad
    const int vx = bx * kLT + tx;
    float l1 = 0.f, ss = 0.f;
#pragma unroll
    for (int c = 0; c < kLC; ++c) {
        if (c >= C) break;
        lds_barrier();  // previous channel's passes are done with sm.x / sm.h
#pragma unroll
        for (int i = 0; i < kLS; ++i) {
            int l, yy, xx;
            stage_pos(i, H, W, x0, y0, l, yy, xx);
            if (l >= 0) {
                sm.x[l] = nx[c][i] * nm[i];
                sm.y[l] = ny[c][i] * nm[i];
            }
        }
        lds_barrier();
        {
            const float* const in[2] = {sm.x, sm.y};
            float* const ho[5] = {sm.h[0], sm.h[1], sm.h[2], sm.h[3], sm.h[4]};
            hpass<2, true>(in, ho);
        }
        lds_barrier();
        float acc[5][4];
        {
            float* const hh[5] = {sm.h[0], sm.h[1], sm.h[2], sm.h[3], sm.h[4]};
            vpass<5>(hh, tx, qd, acc);
        }
#pragma unroll
        for (int o = 0; o < 4; ++o) {
            const int ty = 4 * qd + o, py = by * kLT + ty;
            if (vx >= W || py >= H) continue;
            const SsimPix sp2 = ssim_pix(acc[0][o], acc[1][o], acc[2][o], acc[3][o], acc[4][o]);
            const int64_t p = (int64_t)c * HW + (int64_t)py * W + vx;
            dmaps[p] = sp2.dm0;
            dmaps[(int64_t)C * HW + p] = sp2.ds11;
            dmaps[2 * (int64_t)C * HW + p] = sp2.ds12;
            ss += sp2.S;
            const int li = (ty + kLR) * kLP + tx + kLR;
            l1 += fabsf(sm.x[li] - sm.y[li]);
        }
    }
    l1 = block_sum(l1, sm.red);
    ss = block_sum(ss, sm.red);
    sky = block_sum(sky, sm.red);
    ent = block_sum(ent, sm.red);
    dreg = block_sum(dreg, sm.red);
#pragma unroll
    for (int q = 0; q < 3; ++q) aux[q] = block_sum(aux[q], sm.red);
    if (tid == 0) {
        const int64_t nt = gridDim.x;
        partials[blk] = l1;
        partials[nt + blk] = ss;
        partials[2 * nt + blk] = sky;
        partials[3 * nt + blk] = ent;
        partials[4 * nt + blk] = dreg;
#pragma unroll
        for (int q = 0; q < 3; ++q) partials[(5 + q) * nt + blk] = aux[q];
    }
}

// fixed-order f64 reduction of the tile partials -> [loss, l1, ssim, sky, entropy, scale_reg, normal,
// distortion, inv_depth]
__global__ __launch_bounds__(256) void loss_reduce_kernel(int n_tiles, int C, int64_t HW, int64_t n_sc,
                                                          LossLam lam, const float* __restrict__ partials,
                                                          float* __restrict__ out) {
    __shared__ double s[kLQ][256];
    double a[kLQ] = {};
    for (int t = threadIdx.x; t < n_tiles; t += 256)
#pragma unroll
        for (int q = 0; q < kLQ; ++q) a[q] += partials[(int64_t)q * n_tiles + t];
#pragma unroll
    for (int q = 0; q < kLQ; ++q) s[q][threadIdx.x] = a[q];
    __syncthreads();
    for (int d = 128; d > 0; d >>= 1) {
        if (threadIdx.x < d)
#pragma unroll
            for (int q = 0; q < kLQ; ++q) s[q][threadIdx.x] += s[q][threadIdx.x + d];
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        const double n = (double)C * (double)HW;
        const double l1 = s[0][0] / n, ssim = s[1][0] / n, sky = s[2][0] / (double)HW, ent = s[3][0] / (double)HW;
        const double dreg = n_sc > 0 ? s[4][0] / (double)n_sc : 0.0;  // train.py:163-166: 0 when empty
        const double nrm = s[5][0] / (double)HW, dist = s[6][0] / (double)HW, dep = s[7][0] / (double)HW;
        const double loss = (1.0 - lam.dssim) * l1 + lam.dssim * (1.0 - ssim) + lam.dreg * dreg + lam.sky * sky +
                            lam.ent * ent + lam.normal * nrm + lam.dist * dist + lam.depth * dep;
        out[0] = (float)loss;
        out[1] = (float)l1;
        out[2] = (float)ssim;
        out[3] = (float)sky;
        out[4] = (float)ent;
        out[5] = (float)dreg;
        out[6] = (float)nrm;
        out[7] = (float)dist;
        out[8] = (float)dep;
    }
}

struct LossBwdSmem {
    float m[3][kLH * kLP];  // staged derivative maps
    float h[3][kLH * kHP];  // horizontally filtered
};

struct LossCoef {
    float l1, ss, sky, ent, dreg, nrm, dist, dep;
};

// upstream gradients of the nine 0-dim outputs: one device pointer each, NULL = zero
// (autograd hands None for outputs the loss graph does not use: no zero tensors built)
struct GradOuts {
    const float* p[kLossOuts];
};

__device__ __forceinline__ LossCoef loss_coef(const GradOuts& go, int C, int64_t HW, int64_t n_sc,
                                              const LossLam& lam) {
    float g[kLossOuts];
#pragma unroll
    for (int i = 0; i < kLossOuts; ++i) g[i] = go.p[i] ? *go.p[i] : 0.f;
    const float g0 = g[0];
    const float n = (float)C * (float)HW, hw = (float)HW;
    LossCoef k;
    k.l1 = (g0 * (1.f - lam.dssim) + g[1]) / n;
    k.ss = (g[2] - g0 * lam.dssim) / n;
    k.sky = (g0 * lam.sky + g[3]) / hw;
    k.ent = (g0 * lam.ent + g[4]) / hw;
    k.dreg = n_sc > 0 ? (g0 * lam.dreg + g[5]) / (float)n_sc : 0.f;
    k.nrm = (g0 * lam.normal + g[6]) / hw;
    k.dist = (g0 * lam.dist + g[7]) / hw;
    k.dep = (g0 * lam.depth + g[8]) / hw;
    return k;
}

// per-pixel gradients of the alpha and aux terms (and the zero trailing channels)
__device__ __forceinline__ void pixel_grads(const LossCoef& k, const LossAux& ax, const float* __restrict__ alpha,
                                            const float* __restrict__ mask, float* __restrict__ g_img, const Img& gi,
                                            int C, int extra_ch, float* __restrict__ g_alpha, int W, int py, int px) {
    const int64_t pp = (int64_t)py * W + px;
    const float mk = mask ? mask[pp] : 1.f;
    if (g_alpha) {
        float ga = 0.f;
        if (alpha) {
            const float a = alpha[pp];
            const bool pass = a >= 1e-6f && a <= 1.f - 1e-6f;  // clamp passes the gradient inside
            const float o = fminf(fmaxf(a, 1e-6f), 1.f - 1e-6f);
            const float d_sky = (1.f - mk) / (1.f - o);
            const float d_ent = -(logf(o) + 1.f);
            ga = pass ? k.sky * d_sky + k.ent * d_ent : 0.f;
        }
        g_alpha[pp] = ga;
    }
    if (ax.nrm) {  // d/dn = -mask nfd a, d/dnfd = -mask n a (alpha detached, train.py:183)
        const float a = alpha ? alpha[pp] : 1.f;
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            const int64_t in = c * ax.ns[0] + py * ax.ns[1] + px * ax.ns[2];
            const int64_t iF = c * ax.fs[0] + py * ax.fs[1] + px * ax.fs[2];
            const float n = ax.nrm[in], f = ax.nfd[iF];
            if (ax.g_nrm) ax.g_nrm[in] = -k.nrm * mk * f * a;
            if (ax.g_nfd) ax.g_nfd[iF] = -k.nrm * mk * n * a;
        }
    }
    if (ax.dist && ax.g_dist) ax.g_dist[py * ax.dst[0] + px * ax.dst[1]] = k.dist * mk;
    if (ax.depth && ax.g_depth) {
        const int64_t id = py * ax.dps[0] + px * ax.dps[1];
        const float d = ax.depth[id];
        float g = 0.f;
        if (d > 0.f) {
            const float dm = ax.dmask ? ax.dmask[pp] : 1.f;
            const float e = (1.f / d - ax.mono[pp]) * dm;
            const float sg = e > 0.f ? 1.f : (e < 0.f ? -1.f : 0.f);
            g = k.dep * sg * dm * (-1.f / (d * d));
        }
        ax.g_depth[id] = g;
    }
}

// backward: d loss / d image (and d alpha, d scaling, aux); same channel pipeline as the forward
__global__ __launch_bounds__(256, 3) void loss_bwd_kernel(int C, int H, int W, Img img, Img gt,
                                                       const float* __restrict__ mask,
                                                       const float* __restrict__ alpha, ScaleReg sr, LossAux ax,
                                                       LossLam lam, const float* __restrict__ dmaps,
                                                       GradOuts g_out, float* __restrict__ g_img,
                                                       int extra_ch, float* __restrict__ g_alpha,
                                                       float* __restrict__ g_scaling) {
    __shared__ LossBwdSmem sm;
    const int tid = threadIdx.x;
    const int tiles_x = (W + kLT - 1) / kLT;
    const int blk = xcd_remap(blockIdx.x, gridDim.x);  // as in loss_fwd_kernel
    const int bx = blk % tiles_x, by = blk / tiles_x;
    const int x0 = bx * kLT - kLR, y0 = by * kLT - kLR;
    const int64_t HW = (int64_t)H * W;
    const int tx = tid & (kLT - 1), qd = tid / kLT;
    const int vx = bx * kLT + tx;
    float nd[3][kLS];
    auto fetch = [&](int c) {  // planar derivative maps: one channel ahead
#pragma unroll
        for (int i = 0; i < kLS; ++i) {
            int l, yy, xx;
            const bool in = stage_pos(i, H, W, x0, y0, l, yy, xx);
#pragma unroll
            for (int m = 0; m < 3; ++m)
                nd[m][i] = in ? dmaps[((int64_t)m * C + c) * HW + (unsigned)(yy * W + xx)] : 0.f;
        }
    };
    fetch(0);
    // this lane's four output pixels, every channel read together (channels-last renders)
    float cx[kLC][4], cy[kLC][4], gimg[kLC][4];
#pragma unroll
    for (int o = 0; o < 4; ++o) {
        const int vy = by * kLT + 4 * qd + o;
        const bool in = vx < W && vy < H;
#pragma unroll
        for (int c = 0; c < kLC; ++c) {
            const bool ok = in && c < C;
            cx[c][o] = ok ? img.p[(unsigned)(c * img.sc + vy * img.sy + vx * img.sx)] : 0.f;
            cy[c][o] = ok ? gt.p[(unsigned)(c * gt.sc + vy * gt.sy + vx * gt.sx)] : 0.f;
            gimg[c][o] = 0.f;
        }
    }
    const LossCoef k = loss_coef(g_out, C, HW, sr.n, lam);
    Img gi = img;
    gi.p = g_img;
#pragma unroll
    for (int j = 0; j < kLT * kLT / 256; ++j) {
        const int pl = tid + 256 * j;
        const int px = bx * kLT + (pl & (kLT - 1)), py = by * kLT + pl / kLT;
        if (px < W && py < H) pixel_grads(k, ax, alpha, mask, g_img, gi, C, extra_ch, g_alpha, W, py, px);
    }
    if (g_scaling) {  // d mean_i prod_j s_ij / d s_ij = prod_{l != j} s_il / n
        const int64_t per = (sr.n + gridDim.x - 1) / gridDim.x;
        const int64_t g0 = (int64_t)blk * per, g1 = min(sr.n, g0 + per);
        for (int64_t g = g0 + tid; g < g1; g += 256) {
            const float* s = sr.s + g * sr.k;
            for (int j = 0; j < sr.k; ++j) {
                float p = 1.f;
                for (int l = 0; l < sr.k; ++l)
                    if (l != j) p *= s[l];
                g_scaling[g * sr.k + j] = k.dreg * p;
            }
        }
    }
    float vmk[4];
#pragma unroll
    for (int o = 0; o < 4; ++o) {
        const int vy = by * kLT + 4 * qd + o;
        vmk[o] = (mask && vx < W && vy < H) ? mask[(int64_t)vy * W + vx] : 1.f;
    }
#pragma unroll
    for (int c = 0; c < kLC; ++c) {
        if (c >= C) break;
        lds_barrier();
#pragma unroll
        for (int i = 0; i < kLS; ++i) {
            int l, yy, xx;
            stage_pos(i, H, W, x0, y0, l, yy, xx);
            if (l >= 0)
#pragma unroll
                for (int m = 0; m < 3; ++m) sm.m[m][l] = nd[m][i];
        }
        if (c + 1 < C) fetch(c + 1);
        lds_barrier();
        {
            const float* const in[3] = {sm.m[0], sm.m[1], sm.m[2]};
            float* const ho[3] = {sm.h[0], sm.h[1], sm.h[2]};
            hpass<3, false>(in, ho);
        }
        lds_barrier();
        float acc[3][4];
        {
            float* const hh[3] = {sm.h[0], sm.h[1], sm.h[2]};
            vpass<3>(hh, tx, qd, acc);
        }
#pragma unroll
        for (int o = 0; o < 4; ++o) {
            const float x = cx[c][o] * vmk[o], y = cy[c][o] * vmk[o];
            const float d = x - y;
            const float sgn = d > 0.f ? 1.f : (d < 0.f ? -1.f : 0.f);
            gimg[c][o] = (k.l1 * sgn + k.ss * (acc[0][o] + 2.f * x * acc[1][o] + y * acc[2][o])) * vmk[o];
        }
    }
    // all channels of a pixel written together (plus the zero trailing channels)
#pragma unroll
    for (int o = 0; o < 4; ++o) {
        const int vy = by * kLT + 4 * qd + o;
        if (vx >= W || vy >= H) continue;
#pragma unroll
        for (int c = 0; c < kLC; ++c)
            if (c < C) g_img[(unsigned)(c * img.sc + vy * img.sy + vx * img.sx)] = gimg[c][o];
        for (int c = C; c < C + extra_ch; ++c) g_img[(unsigned)(c * img.sc + vy * img.sy + vx * img.sx)] = 0.f;
    }
}

static bool check_window() {
    double g[11], s = 0.0;
    for (int k = 0; k < 11; ++k) {
        g[k] = exp(-(double)((k - 5) * (k - 5)) / (2.0 * 1.5 * 1.5));
        s += g[k];
    }
    for (int k = 0; k < 11; ++k)
        if ((float)(g[k] / s) != kWin[k]) return false;
    return true;
}

}  // namespace hgsr

using namespace hgsr;

static int loss_tiles(int H, int W) { return ((W + kLT - 1) / kLT) * ((H + kLT - 1) / kLT); }

static size_t loss_maps_bytes(int C, int H, int W) {
    return ((size_t)3 * C * H * W * sizeof(float) + 255) & ~(size_t)255;
}

extern "C" size_t hgsr_loss_ws_bytes(int C, int H, int W) {
    return loss_maps_bytes(C, H, W) + (size_t)loss_tiles(H, W) * kLQ * sizeof(float);
}

static int check_strides(const int64_t* st, const char* what, int C, int H, int W) {
    HGSR_REQUIRE(st == nullptr || (st[0] >= 0 && st[1] >= 0 && st[2] >= 0), "negative %s strides", what);
    const int64_t sc = st ? st[0] : (int64_t)H * W, sy = st ? st[1] : W, sx = st ? st[2] : 1;
    HGSR_REQUIRE((C - 1) * sc + (int64_t)(H - 1) * sy + (int64_t)(W - 1) * sx < ((int64_t)1 << 31),
                 "%s spans >= 2^31 elements", what);
    return HGSR_OK;
}

static Img make_img(const float* p, const int64_t* st, int H, int W) {
    if (!st) return Img{p, (int64_t)H * W, W, 1};
    return Img{p, st[0], st[1], st[2]};
}

static int check_scale_reg(int64_t n_sc, int k_sc, const float* scaling, float lam_dreg) {
    HGSR_REQUIRE(n_sc >= 0 && (n_sc == 0 || (k_sc >= 1 && scaling)), "bad scaling operand (n=%lld k=%d)",
                 (long long)n_sc, k_sc);
    (void)lam_dreg;  // an absent or empty scaling contributes 0 (train.py:163-166)
    return HGSR_OK;
}

static int make_terms(const hgsr_loss_terms* t, const hgsr_loss_aux_grads* g, int H, int W, LossLam& lam,
                      LossAux& ax) {
    HGSR_REQUIRE(t, "null loss terms");
    lam = LossLam{t->lambda_dssim, t->lambda_sky_opa, t->lambda_entropy, t->lambda_dreg,
                  t->lambda_normal, t->lambda_dist, t->lambda_depth};
    HGSR_REQUIRE(!t->normals == !t->normals_from_depth, "normal term needs normals and normals_from_depth");
    HGSR_REQUIRE(t->lambda_normal == 0.f || t->normals, "lambda_normal needs normals");
    HGSR_REQUIRE(t->lambda_dist == 0.f || t->distort, "lambda_dist needs distort");
    HGSR_REQUIRE(!t->depth == !t->mono_invdepth, "depth term needs depth and mono_invdepth");
    HGSR_REQUIRE(t->lambda_depth == 0.f || t->depth, "lambda_depth needs depth");
    ax = LossAux{};
    ax.nrm = t->normals;
    ax.nfd = t->normals_from_depth;
    const int64_t def3[3] = {(int64_t)H * W, W, 1}, def2[2] = {W, 1};
    for (int k = 0; k < 3; ++k) {
        ax.ns[k] = t->normals_strides[k] ? t->normals_strides[k] : def3[k];
        ax.fs[k] = t->nfd_strides[k] ? t->nfd_strides[k] : def3[k];
    }
    ax.dist = t->distort;
    ax.depth = t->depth;
    for (int k = 0; k < 2; ++k) {
        ax.dst[k] = t->distort_strides[k] ? t->distort_strides[k] : def2[k];
        ax.dps[k] = t->depth_strides[k] ? t->depth_strides[k] : def2[k];
    }
    ax.mono = t->mono_invdepth;
    ax.dmask = t->depth_mask;
    if (g) {
        ax.g_nrm = g->g_normals;
        ax.g_nfd = g->g_normals_from_depth;
        ax.g_dist = g->g_distort;
        ax.g_depth = g->g_depth;
    }
    return HGSR_OK;
}

extern "C" int hgsr_loss_fwd(int C, int H, int W, const float* image, const int64_t* image_strides,
                             const float* gt, const int64_t* gt_strides, const float* mask,
                             const float* alpha, const float* scaling, int64_t n_scaling, int k_scaling,
                             const hgsr_loss_terms* terms, float* out, void* ws, size_t ws_bytes,
                             hgsr_stream_t stream) {
    HGSR_REQUIRE(C >= 1 && C <= kLC && H > 0 && W > 0, "bad dims (C must be 1..3)");
    HGSR_REQUIRE(image && gt && out && ws, "null pointer");
    static const bool win_ok = check_window();
    HGSR_REQUIRE(win_ok, "SSIM window constants disagree with utils/loss_utils.py's formula");
    HGSR_REQUIRE(ws_bytes >= hgsr_loss_ws_bytes(C, H, W), "loss workspace too small");
    LossLam lam;
    LossAux ax;
    if (int st = make_terms(terms, nullptr, H, W, lam, ax)) return st;
    HGSR_REQUIRE(alpha || (lam.sky == 0.f && lam.ent == 0.f), "alpha terms need alpha");
    if (int st = check_strides(image_strides, "image", C, H, W)) return st;
    if (int st = check_strides(gt_strides, "gt", C, H, W)) return st;
    if (int st = check_scale_reg(n_scaling, k_scaling, scaling, lam.dreg)) return st;
    hipStream_t s = as_stream(stream);
    float* dmaps = (float*)ws;
    float* partials = (float*)((char*)ws + loss_maps_bytes(C, H, W));
    const int nt = loss_tiles(H, W);
    const Img im = make_img(image, image_strides, H, W), gm = make_img(gt, gt_strides, H, W);
    const ScaleReg sr{n_scaling > 0 ? scaling : nullptr, n_scaling, k_scaling};
    {
        KernelTimer kt("loss_fwd", s);
        hipLaunchKernelGGL(loss_fwd_kernel, dim3(nt), dim3(256), 0, s, C, H, W, im, gm, mask, alpha, sr, ax, dmaps,
                           partials);
    }
    if (int st = check_launch("loss_fwd")) return st;
    hipLaunchKernelGGL(loss_reduce_kernel, dim3(1), dim3(256), 0, s, nt, C, (int64_t)H * W, n_scaling, lam,
                       partials, out);
    return check_launch("loss_reduce");
}

extern "C" int hgsr_loss_bwd(int C, int H, int W, const float* image, const int64_t* image_strides,
                             const float* gt, const int64_t* gt_strides, const float* mask,
                             const float* alpha, const float* scaling, int64_t n_scaling, int k_scaling,
                             const hgsr_loss_terms* terms, const float* const* g_outs, float* g_image,
                             int extra_channels,
                             float* g_alpha, float* g_scaling, const hgsr_loss_aux_grads* aux_grads,
                             const void* ws, size_t ws_bytes, hgsr_stream_t stream) {
    HGSR_REQUIRE(C >= 1 && C <= kLC && H > 0 && W > 0, "bad dims (C must be 1..3)");
    HGSR_REQUIRE(image && gt && g_outs && g_image && ws, "null pointer");
    GradOuts go;
    for (int i = 0; i < kLossOuts; ++i) go.p[i] = g_outs[i];
    HGSR_REQUIRE(ws_bytes >= hgsr_loss_ws_bytes(C, H, W), "loss workspace too small");
    LossLam lam;
    LossAux ax;
    if (int st = make_terms(terms, aux_grads, H, W, lam, ax)) return st;
    if (int st = check_strides(image_strides, "image", C, H, W)) return st;
    if (int st = check_strides(gt_strides, "gt", C, H, W)) return st;
    if (int st = check_scale_reg(n_scaling, k_scaling, scaling, lam.dreg)) return st;
    HGSR_REQUIRE(extra_channels >= 0, "negative extra_channels");
    hipStream_t s = as_stream(stream);
    const Img im = make_img(image, image_strides, H, W), gm = make_img(gt, gt_strides, H, W);
    const ScaleReg sr{n_scaling > 0 ? scaling : nullptr, n_scaling, k_scaling};
    float* gsc = n_scaling > 0 ? g_scaling : nullptr;
    KernelTimer kt("loss_bwd", s);
    hipLaunchKernelGGL(loss_bwd_kernel, dim3(loss_tiles(H, W)), dim3(256), 0, s, C, H, W, im, gm, mask, alpha, sr,
                       ax, lam, (const float*)ws, go, g_image, extra_channels, g_alpha, gsc);
    return check_launch("loss_bwd");
}
