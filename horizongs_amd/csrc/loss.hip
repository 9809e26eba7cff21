// K15: fused training loss: masked L1 + D-SSIM and the alpha
// regularisers of reference train.py:153-178 with utils/loss_utils.py:17-60
// (Gaussian window 11, sigma 1.5, zero padding, C1 = 0.01^2, C2 = 0.03^2).
//
//   x = image * mask, y = gt * mask (mask [H,W] broadcast over channels, nullable)
//   loss = (1 - l) * mean|x - y| + l * (1 - mean SSIM(x, y))
//        + l_sky * mean(-(1 - mask) log(1 - a)) + l_ent * mean(-a log a),  a = clamp(alpha, 1e-6, 1 - 1e-6)
//
// CDNA4 mapping: one 256-lane workgroup per 16x16 pixel tile; the tile plus its 5-pixel
// halo is staged in LDS and the 11x11 window is applied separably (horizontal pass into
// LDS, vertical pass in registers) for the five moments.  The forward also writes the
// three per-pixel derivative maps the SSIM gradient needs,
//   dS/dx(q) = G*(S_mu1 - 2 mu1 S_s11 - mu2 S_s12)(q) + 2 x(q) G*S_s11(q) + y(q) G*S_s12(q),
// and the backward pass filters them the same way; everything is HBM-streaming, with
// per-tile partial sums reduced in a fixed order (deterministic).
#include "common.h"

namespace hgsr {

constexpr int kLT = 16;            // tile edge
constexpr int kLR = 5;             // window radius
constexpr int kLH = kLT + 2 * kLR;  // 26: tile + halo

struct LossWin {
    float w[11];
};

// a [C,H,W] image with arbitrary element strides (contiguous CHW, or the channels-last
// [H,W,C] render output viewed through permute(2,0,1) without a copy)
struct Img {
    const float* p;
    int64_t sc, sy, sx;
    __device__ __forceinline__ int64_t at(int c, int y, int x) const { return c * sc + y * sy + x * sx; }
};

__device__ __forceinline__ float masked(Img img, const float* __restrict__ mask, int c, int H, int W, int yy, int xx) {
    if (yy < 0 || yy >= H || xx < 0 || xx >= W) return 0.f;  // conv2d zero padding
    const float v = img.p[img.at(c, yy, xx)];
    return mask ? v * mask[(int64_t)yy * W + xx] : v;
}

__device__ __forceinline__ float block_sum(float v, float* red) {
    // wave sum via DPP/shuffles, then 4 waves through LDS
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d);
    const int wave = threadIdx.x >> 6;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[wave] = v;
    __syncthreads();
    return red[0] + red[1] + red[2] + red[3];
}

// forward: SSIM map statistics + derivative maps, L1, alpha terms; per-tile partials
// partial layout per tile: [sum |x-y|, sum S, sum sky, sum entropy]
__global__ __launch_bounds__(256) void loss_fwd_kernel(int C, int H, int W, Img img, Img gt,
                                                       const float* __restrict__ mask,
                                                       const float* __restrict__ alpha, LossWin win,
                                                       float* __restrict__ dmaps, float* __restrict__ partials) {
    __shared__ float s_x[kLH][kLH + 1], s_y[kLH][kLH + 1];
    __shared__ float s_h[5][kLH][kLT + 1];
    __shared__ float s_red[4];
    const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
    const int tiles_x = (W + kLT - 1) / kLT;
    const int bx = blockIdx.x % tiles_x, by = blockIdx.x / tiles_x;
    const int x0 = bx * kLT - kLR, y0 = by * kLT - kLR;
    const int px = bx * kLT + tx, py = by * kLT + ty;
    const bool inside = px < W && py < H;
    const int64_t HW = (int64_t)H * W;
    float l1 = 0.f, ss = 0.f;
    for (int c = 0; c < C; ++c) {
        __syncthreads();
        for (int e = threadIdx.x; e < kLH * kLH; e += 256) {
            const int r = e / kLH, q = e - r * kLH;
            s_x[r][q] = masked(img, mask, c, H, W, y0 + r, x0 + q);
            s_y[r][q] = masked(gt, mask, c, H, W, y0 + r, x0 + q);
        }
        __syncthreads();
        // horizontal pass: 26 rows x 16 output columns x 5 moments
        for (int e = threadIdx.x; e < kLH * kLT; e += 256) {
            const int r = e / kLT, q = e - r * kLT;
            float m1 = 0.f, m2 = 0.f, a = 0.f, b = 0.f, xy = 0.f;
#pragma unroll
            for (int k = 0; k < 11; ++k) {
                const float xv = s_x[r][q + k], yv = s_y[r][q + k], w = win.w[k];
                m1 += w * xv;
                m2 += w * yv;
                a += w * xv * xv;
                b += w * yv * yv;
                xy += w * xv * yv;
            }
            s_h[0][r][q] = m1;
            s_h[1][r][q] = m2;
            s_h[2][r][q] = a;
            s_h[3][r][q] = b;
            s_h[4][r][q] = xy;
        }
        __syncthreads();
        float mu1 = 0.f, mu2 = 0.f, ex2 = 0.f, ey2 = 0.f, exy = 0.f;
#pragma unroll
        for (int k = 0; k < 11; ++k) {
            const float w = win.w[k];
            mu1 += w * s_h[0][ty + k][tx];
            mu2 += w * s_h[1][ty + k][tx];
            ex2 += w * s_h[2][ty + k][tx];
            ey2 += w * s_h[3][ty + k][tx];
            exy += w * s_h[4][ty + k][tx];
        }
        if (inside) {
            const float C1 = 0.01f * 0.01f, C2 = 0.03f * 0.03f;
            const float mu1_sq = mu1 * mu1, mu2_sq = mu2 * mu2, mu12 = mu1 * mu2;
            const float s11 = ex2 - mu1_sq, s22 = ey2 - mu2_sq, s12 = exy - mu12;
            const float A1 = 2.f * mu12 + C1, A2 = 2.f * s12 + C2;
            const float B1 = mu1_sq + mu2_sq + C1, B2 = s11 + s22 + C2;
            const float inv = 1.0f / (B1 * B2);
            const float S = A1 * A2 * inv;
            const float dmu1 = 2.f * mu2 * A2 * inv - 2.f * mu1 * S / B1;
            const float ds11 = -S / B2;
            const float ds12 = 2.f * A1 * inv;
            const int64_t p = (int64_t)c * HW + (int64_t)py * W + px;
            dmaps[p] = dmu1 - 2.f * mu1 * ds11 - mu2 * ds12;
            dmaps[(int64_t)C * HW + p] = ds11;
            dmaps[2 * (int64_t)C * HW + p] = ds12;
            ss += S;
            l1 += fabsf(s_x[ty + kLR][tx + kLR] - s_y[ty + kLR][tx + kLR]);
        }
    }
    float sky = 0.f, ent = 0.f;
    if (alpha && inside) {
        const int64_t p = (int64_t)py * W + px;
        const float o = fminf(fmaxf(alpha[p], 1e-6f), 1.f - 1e-6f);
        const float sk = mask ? mask[p] : 1.f;
        sky = -(1.f - sk) * logf(1.f - o);
        ent = -o * logf(o);
    }
    l1 = block_sum(l1, s_red);
    ss = block_sum(ss, s_red);
    sky = block_sum(sky, s_red);
    ent = block_sum(ent, s_red);
    if (threadIdx.x == 0) {
        float* o = partials + (int64_t)blockIdx.x * 4;
        o[0] = l1;
        o[1] = ss;
        o[2] = sky;
        o[3] = ent;
    }
}

// fixed-order f64 reduction of the tile partials -> [loss, l1, ssim, sky, entropy]
__global__ __launch_bounds__(256) void loss_reduce_kernel(int n_tiles, int C, int64_t HW, float lam_dssim,
                                                          float lam_sky, float lam_ent,
                                                          const float* __restrict__ partials, float* __restrict__ out) {
    __shared__ double s[4][256];
    double a[4] = {0.0, 0.0, 0.0, 0.0};
    for (int t = threadIdx.x; t < n_tiles; t += 256)
#pragma unroll
        for (int q = 0; q < 4; ++q) a[q] += partials[(int64_t)t * 4 + q];
#pragma unroll
    for (int q = 0; q < 4; ++q) s[q][threadIdx.x] = a[q];
    __syncthreads();
    for (int d = 128; d > 0; d >>= 1) {
        if (threadIdx.x < d)
#pragma unroll
            for (int q = 0; q < 4; ++q) s[q][threadIdx.x] += s[q][threadIdx.x + d];
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        const double n = (double)C * (double)HW;
        const double l1 = s[0][0] / n, ssim = s[1][0] / n, sky = s[2][0] / (double)HW, ent = s[3][0] / (double)HW;
        const double loss = (1.0 - lam_dssim) * l1 + lam_dssim * (1.0 - ssim) + lam_sky * sky + lam_ent * ent;
        out[0] = (float)loss;
        out[1] = (float)l1;
        out[2] = (float)ssim;
        out[3] = (float)sky;
        out[4] = (float)ent;
    }
}

// backward: d loss / d image (and d alpha), scaled by the upstream scalar gradient
__global__ __launch_bounds__(256) void loss_bwd_kernel(int C, int H, int W, Img img, Img gt,
                                                       const float* __restrict__ mask,
                                                       const float* __restrict__ alpha, LossWin win, float lam_dssim,
                                                       float lam_sky, float lam_ent,
                                                       const float* __restrict__ dmaps,
                                                       const float* __restrict__ g_out, float* __restrict__ g_img,
                                                       int extra_ch, float* __restrict__ g_alpha) {
    __shared__ float s_m[3][kLH][kLH + 1];
    __shared__ float s_h[3][kLH][kLT + 1];
    const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
    const int tiles_x = (W + kLT - 1) / kLT;
    const int bx = blockIdx.x % tiles_x, by = blockIdx.x / tiles_x;
    const int x0 = bx * kLT - kLR, y0 = by * kLT - kLR;
    const int px = bx * kLT + tx, py = by * kLT + ty;
    const bool inside = px < W && py < H;
    const int64_t HW = (int64_t)H * W;
    // upstream gradients of [loss, l1, ssim, sky, entropy] folded into per-term coefficients
    const float g0 = g_out[0], g1 = g_out[1], g2 = g_out[2], g3 = g_out[3], g4 = g_out[4];
    const float n = (float)C * (float)HW;
    const float k_l1 = (g0 * (1.f - lam_dssim) + g1) / n, k_ss = (g2 - g0 * lam_dssim) / n;
    const float k_sky = (g0 * lam_sky + g3) / (float)HW, k_ent = (g0 * lam_ent + g4) / (float)HW;
    const int64_t pp = (int64_t)py * W + px;
    const float mk = (mask && inside) ? mask[pp] : 1.f;
    for (int c = 0; c < C; ++c) {
        __syncthreads();
        for (int e = threadIdx.x; e < kLH * kLH; e += 256) {
            const int r = e / kLH, q = e - r * kLH;
            const int yy = y0 + r, xx = x0 + q;
            const bool in = yy >= 0 && yy < H && xx >= 0 && xx < W;
            const int64_t p = (int64_t)c * HW + (int64_t)yy * W + xx;
#pragma unroll
            for (int m = 0; m < 3; ++m) s_m[m][r][q] = in ? dmaps[(int64_t)m * C * HW + p] : 0.f;
        }
        __syncthreads();
        for (int e = threadIdx.x; e < kLH * kLT; e += 256) {
            const int r = e / kLT, q = e - r * kLT;
            float v[3] = {0.f, 0.f, 0.f};
#pragma unroll
            for (int k = 0; k < 11; ++k)
#pragma unroll
                for (int m = 0; m < 3; ++m) v[m] += win.w[k] * s_m[m][r][q + k];
#pragma unroll
            for (int m = 0; m < 3; ++m) s_h[m][r][q] = v[m];
        }
        __syncthreads();
        if (!inside) continue;
        float ga = 0.f, gb = 0.f, gc = 0.f;
#pragma unroll
        for (int k = 0; k < 11; ++k) {
            const float w = win.w[k];
            ga += w * s_h[0][ty + k][tx];
            gb += w * s_h[1][ty + k][tx];
            gc += w * s_h[2][ty + k][tx];
        }
        const float x = img.p[img.at(c, py, px)] * mk, y = gt.p[gt.at(c, py, px)] * mk;
        const float d = x - y;
        const float sgn = d > 0.f ? 1.f : (d < 0.f ? -1.f : 0.f);
        const float gx = k_l1 * sgn + k_ss * (ga + 2.f * x * gb + y * gc);
        g_img[img.at(c, py, px)] = gx * mk;
    }
    // trailing image channels the loss does not read (e.g. the ED channel of RGB+ED)
    if (inside)
        for (int c = C; c < C + extra_ch; ++c) g_img[img.at(c, py, px)] = 0.f;
    if (g_alpha && inside) {
        float ga = 0.f;
        if (alpha) {
            const float a = alpha[pp];
            const bool pass = a >= 1e-6f && a <= 1.f - 1e-6f;  // clamp passes the gradient inside
            const float o = fminf(fmaxf(a, 1e-6f), 1.f - 1e-6f);
            const float sk = mask ? mask[pp] : 1.f;
            const float d_sky = (1.f - sk) / (1.f - o);
            const float d_ent = -(logf(o) + 1.f);
            ga = pass ? k_sky * d_sky + k_ent * d_ent : 0.f;
        }
        g_alpha[pp] = ga;
    }
}

static LossWin gaussian_window() {
    // utils/loss_utils.py:20-22: exp(-(x - 5)^2 / (2 * 1.5^2)), normalised; f64 then rounded
    LossWin w;
    double g[11], s = 0.0;
    for (int k = 0; k < 11; ++k) {
        g[k] = exp(-(double)((k - 5) * (k - 5)) / (2.0 * 1.5 * 1.5));
        s += g[k];
    }
    for (int k = 0; k < 11; ++k) w.w[k] = (float)(g[k] / s);
    return w;
}

}  // namespace hgsr

using namespace hgsr;

static int loss_tiles(int H, int W) { return ((W + kLT - 1) / kLT) * ((H + kLT - 1) / kLT); }

extern "C" size_t hgsr_loss_ws_bytes(int C, int H, int W) {
    const size_t maps = ((size_t)3 * C * H * W * sizeof(float) + 255) & ~(size_t)255;
    return maps + (size_t)loss_tiles(H, W) * 4 * sizeof(float);
}

static int check_strides(const int64_t* st, const char* what) {
    HGSR_REQUIRE(st == nullptr || (st[0] >= 0 && st[1] >= 0 && st[2] >= 0), "negative %s strides", what);
    return HGSR_OK;
}

static Img make_img(const float* p, const int64_t* st, int H, int W) {
    if (!st) return Img{p, (int64_t)H * W, W, 1};
    return Img{p, st[0], st[1], st[2]};
}

extern "C" int hgsr_loss_fwd(int C, int H, int W, const float* image, const int64_t* image_strides,
                             const float* gt, const int64_t* gt_strides, const float* mask,
                             const float* alpha, float lambda_dssim, float lambda_sky_opa, float lambda_entropy,
                             float* out, void* ws, size_t ws_bytes, hgsr_stream_t stream) {
    HGSR_REQUIRE(C >= 1 && H > 0 && W > 0, "bad dims");
    HGSR_REQUIRE(image && gt && out && ws, "null pointer");
    HGSR_REQUIRE(ws_bytes >= hgsr_loss_ws_bytes(C, H, W), "loss workspace too small");
    HGSR_REQUIRE(alpha || (lambda_sky_opa == 0.f && lambda_entropy == 0.f), "alpha terms need alpha");
    if (int st = check_strides(image_strides, "image")) return st;
    if (int st = check_strides(gt_strides, "gt")) return st;
    hipStream_t s = as_stream(stream);
    float* dmaps = (float*)ws;
    float* partials = (float*)((char*)ws + (((size_t)3 * C * H * W * sizeof(float) + 255) & ~(size_t)255));
    const int nt = loss_tiles(H, W);
    {
        KernelTimer kt("loss_fwd", s);
        hipLaunchKernelGGL(loss_fwd_kernel, dim3(nt), dim3(256), 0, s, C, H, W, make_img(image, image_strides, H, W),
                           make_img(gt, gt_strides, H, W), mask, alpha,
                           gaussian_window(), dmaps, partials);
    }
    if (int st = check_launch("loss_fwd")) return st;
    hipLaunchKernelGGL(loss_reduce_kernel, dim3(1), dim3(256), 0, s, nt, C, (int64_t)H * W, lambda_dssim,
                       lambda_sky_opa, lambda_entropy, partials, out);
    return check_launch("loss_reduce");
}

extern "C" int hgsr_loss_bwd(int C, int H, int W, const float* image, const int64_t* image_strides,
                             const float* gt, const int64_t* gt_strides, const float* mask,
                             const float* alpha, float lambda_dssim, float lambda_sky_opa, float lambda_entropy,
                             const float* g_out, float* g_image, int extra_channels, float* g_alpha,
                             const void* ws, size_t ws_bytes, hgsr_stream_t stream) {
    HGSR_REQUIRE(C >= 1 && H > 0 && W > 0, "bad dims");
    HGSR_REQUIRE(image && gt && g_out && g_image && ws, "null pointer");
    HGSR_REQUIRE(ws_bytes >= hgsr_loss_ws_bytes(C, H, W), "loss workspace too small");
    if (int st = check_strides(image_strides, "image")) return st;
    if (int st = check_strides(gt_strides, "gt")) return st;
    HGSR_REQUIRE(extra_channels >= 0, "negative extra_channels");
    hipStream_t s = as_stream(stream);
    KernelTimer kt("loss_bwd", s);
    hipLaunchKernelGGL(loss_bwd_kernel, dim3(loss_tiles(H, W)), dim3(256), 0, s, C, H, W,
                       make_img(image, image_strides, H, W), make_img(gt, gt_strides, H, W), mask, alpha,
                       gaussian_window(), lambda_dssim, lambda_sky_opa, lambda_entropy, (const float*)ws, g_out,
                       g_image, extra_channels, g_alpha);
    return check_launch("loss_bwd");
}
