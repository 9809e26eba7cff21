// Explicit (merged-scene) Gaussians, the c5 path: reference render() with pc.explicit_gs
// (gaussian_renderer/render.py:22-25) =
//   set_gs_mask          <- scene/lod_model.py:292-296 (the LoD level test of set_anchor_mask,
//                           on the explicit Gaussians' centres)
//   generate_explicit_gaussians <- scene/basic_model.py:373-383 (boolean-mask gathers of
//                           xyz, cat(features_dc, features_rest), opacity, scaling, rotation)
// as one ordered stream compaction:
//   explicit_count   one 256-lane workgroup per 1024 Gaussians: the LoD mask (or a given
//                    visibility mask), written as bytes, and the block's kept count;
//   explicit_scan    one workgroup: exclusive scan of the block counts -> block bases and
//                    the total (the one host read, as the reference's mask indexing has);
//   explicit_gather  per block: the kept source rows in order (ballot + mbcnt ranks) staged
//                    in LDS, then every attribute copied with consecutive lanes on
//                    consecutive output floats (coalesced writes; a row's columns are
//                    contiguous reads), the colour rows assembled from dc + rest;
//   explicit_scatter the backward: every source row's gradient = its output row's, or 0
//                    when it was dropped (overwrite; no zero fill, no atomics).
// HBM-bound: read 4 B mask + the kept rows, write the kept rows (+ 4 B index per row).
#include "common.h"

namespace hgsr {

constexpr int kExBlock = 1024;  // Gaussians per workgroup (256 lanes x 4)

struct ExLod {
    const int32_t* level;       // [N]
    const float* extra_level;   // [N]
    const float* cam;           // [3]
    float res_scale, standard_dist, log2_fork;
    int max_level;
};

__device__ __forceinline__ bool ex_lod(const float* __restrict__ xyz, int64_t i, const ExLod& L) {
#pragma clang fp contract(off)
    const float dx = xyz[i * 3] - L.cam[0], dy = xyz[i * 3 + 1] - L.cam[1], dz = xyz[i * 3 + 2] - L.cam[2];
    const float dist = sqrtf(dx * dx + dy * dy + dz * dz) * L.res_scale;
    const float pred = log2f(L.standard_dist / dist) / L.log2_fork + L.extra_level[i];
    const float fl = floorf(pred);
    const int il = fl <= 0.f ? 0 : (fl >= (float)L.max_level ? L.max_level : (int)fl);
    return L.level[i] <= il;
}

__global__ __launch_bounds__(256) void explicit_count_kernel(int64_t N, const float* __restrict__ xyz, ExLod L,
                                                             const uint8_t* __restrict__ vis_in,
                                                             uint8_t* __restrict__ mask,
                                                             int32_t* __restrict__ block_cnt) {
    __shared__ int s_cnt[4];
    const int64_t b0 = (int64_t)blockIdx.x * kExBlock;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    int cnt = 0;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int64_t i = b0 + r * 256 + threadIdx.x;
        bool keep = false;
        if (i < N) {
            keep = vis_in ? vis_in[i] != 0 : ex_lod(xyz, i, L);
            if (!vis_in) mask[i] = keep ? 1 : 0;  // a given visibility mask is used in place
        }
        cnt += __popcll(__ballot(keep));
    }
    if (lane == 0) s_cnt[wave] = cnt;
    __syncthreads();
    if (threadIdx.x == 0) block_cnt[blockIdx.x] = s_cnt[0] + s_cnt[1] + s_cnt[2] + s_cnt[3];
}

// exclusive scan of nb block counts in one workgroup: each of the 1024 lanes walks nb / 1024 counts
// serially (host check nb <= 2^20, i.e. <= 2^30 Gaussians; 10M Gaussians -> 9,766 blocks, 10 per lane)
__global__ __launch_bounds__(1024) void explicit_scan_kernel(int nb, const int32_t* __restrict__ cnt,
                                                             int64_t* __restrict__ base,
                                                             int64_t* __restrict__ total) {
    __shared__ int64_t s_part[1024];
    const int per = (nb + 1023) / 1024;
    const int t = threadIdx.x;
    int64_t sum = 0;
    for (int k = 0; k < per; ++k) {
        const int j = t * per + k;
        if (j < nb) sum += cnt[j];
    }
    s_part[t] = sum;
    __syncthreads();
    for (int off = 1; off < 1024; off <<= 1) {  // Hillis-Steele over the 1024 partials
        const int64_t v = t >= off ? s_part[t - off] : 0;
        __syncthreads();
        s_part[t] += v;
        __syncthreads();
    }
    int64_t run = t > 0 ? s_part[t - 1] : 0;
    for (int k = 0; k < per; ++k) {
        const int j = t * per + k;
        if (j < nb) {
            base[j] = run;
            run += cnt[j];
        }
    }
    if (t == 1023) *total = s_part[1023];
}

struct ExSrc {
    const float* xyz;     // [N,3]
    const float* f_dc;    // [N,1,3]
    const float* f_rest;  // [N,K-1,3] (nullable when K == 1)
    const float* opac;    // [N,1]
    const float* scale;   // [N,3]
    const float* rot;     // [N,4]
    int K;                // SH coefficients per colour row
};

struct ExDst {
    float* xyz;
    float* color;  // [M,K,3]
    float* opac;
    float* scale;
    float* rot;
    int32_t* index;  // [M] source row of each output row
};

// kept source rows of this block, in order, into LDS; returns the kept count.  Block order
// = round r (256 Gaussians each) major, then wave, then lane: ranks from the 16 per-(round,
// wave) ballot counts and mbcnt.
__device__ __forceinline__ int ex_block_rows(int64_t N, const uint8_t* __restrict__ mask, int64_t b0, int32_t* rows) {
    __shared__ int s_wave[16];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    bool keep[4];
    uint64_t bal[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int64_t i = b0 + r * 256 + threadIdx.x;
        keep[r] = i < N && mask[i] != 0;
        bal[r] = __ballot(keep[r]);
        if (lane == 0) s_wave[r * 4 + wave] = __popcll(bal[r]);
    }
    __syncthreads();
    int run = 0, pre[4] = {0, 0, 0, 0};
#pragma unroll
    for (int q = 0; q < 16; ++q) {
        if ((q & 3) == wave) pre[q >> 2] = run;
        run += s_wave[q];
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int rank = pre[r] + __builtin_amdgcn_mbcnt_hi((uint32_t)(bal[r] >> 32),
                                                            __builtin_amdgcn_mbcnt_lo((uint32_t)bal[r], 0));
        if (keep[r]) rows[rank] = (int32_t)(r * 256 + threadIdx.x);
    }
    __syncthreads();
    return run;
}

__global__ __launch_bounds__(256) void explicit_gather_kernel(int64_t N, const uint8_t* __restrict__ mask,
                                                              const int64_t* __restrict__ block_base, ExSrc s,
                                                              ExDst d) {
    __shared__ int32_t s_rows[kExBlock];
    const int64_t b0 = (int64_t)blockIdx.x * kExBlock;
    const int n = ex_block_rows(N, mask, b0, s_rows);
    if (n == 0) return;
    const int64_t o0 = block_base[blockIdx.x];
    const int tid = threadIdx.x;
    for (int e = tid; e < n; e += 256) d.index[o0 + e] = (int32_t)(b0 + s_rows[e]);
    // consecutive lanes -> consecutive output floats of each attribute
    auto copy = [&](const float* src, float* dst, int w) {
        const int tot = n * w;
        for (int e = tid; e < tot; e += 256) {
            const int r = e / w, c = e - r * w;
            dst[(o0 + r) * w + c] = src[(b0 + s_rows[r]) * w + c];
        }
    };
    copy(s.xyz, d.xyz, 3);
    copy(s.opac, d.opac, 1);
    copy(s.scale, d.scale, 3);
    copy(s.rot, d.rot, 4);
    const int wc = 3 * s.K, wr = wc - 3;
    const int tot = n * wc;
    for (int e = tid; e < tot; e += 256) {
        const int r = e / wc, c = e - r * wc;
        const int64_t src = b0 + s_rows[r];
        d.color[(o0 + r) * wc + c] = c < 3 ? s.f_dc[src * 3 + c] : s.f_rest[src * wr + (c - 3)];
    }
}

// backward: grad of every source row (overwrite) = grad of its output row or 0
struct ExGradIn {
    const float* xyz;
    const float* color;
    const float* opac;
    const float* scale;
    const float* rot;
};

struct ExGradOut {
    float* xyz;
    float* f_dc;
    float* f_rest;
    float* opac;
    float* scale;
    float* rot;
};

__global__ __launch_bounds__(256) void explicit_scatter_kernel(int64_t N, int K, const uint8_t* __restrict__ mask,
                                                               const int64_t* __restrict__ block_base, ExGradIn g,
                                                               ExGradOut v) {
    __shared__ int32_t s_rows[kExBlock];
    __shared__ int32_t s_out[kExBlock];  // output row of each source row of the block, -1 if dropped
    const int64_t b0 = (int64_t)blockIdx.x * kExBlock;
    for (int e = threadIdx.x; e < kExBlock; e += 256) s_out[e] = -1;
    const int n = ex_block_rows(N, mask, b0, s_rows);
    for (int e = threadIdx.x; e < n; e += 256) s_out[s_rows[e]] = e;
    __syncthreads();
    const int64_t o0 = block_base[blockIdx.x];
    const int64_t m = min((int64_t)kExBlock, N - b0);
    auto scatter = [&](const float* src, float* dst, int w) {
        if (!dst) return;
        const int64_t tot = m * w;
        for (int64_t e = threadIdx.x; e < tot; e += 256) {
            const int r = (int)(e / w), c = (int)(e - (int64_t)r * w);
            const int o = s_out[r];
            dst[(b0 + r) * w + c] = (o >= 0 && src) ? src[(o0 + o) * w + c] : 0.f;
        }
    };
    scatter(g.xyz, v.xyz, 3);
    scatter(g.opac, v.opac, 1);
    scatter(g.scale, v.scale, 3);
    scatter(g.rot, v.rot, 4);
    const int wc = 3 * K, wr = wc - 3;
    const int64_t tot = m * wc;
    for (int64_t e = threadIdx.x; e < tot; e += 256) {
        const int r = (int)(e / wc), c = (int)(e - (int64_t)r * wc);
        const int o = s_out[r];
        const float val = (o >= 0 && g.color) ? g.color[(o0 + o) * wc + c] : 0.f;
        if (c < 3) {
            if (v.f_dc) v.f_dc[(b0 + r) * 3 + c] = val;
        } else if (v.f_rest) {
            v.f_rest[(b0 + r) * wr + (c - 3)] = val;
        }
    }
}

// kept indices of a mask, in order (the compaction of explicit_gather without the rows)
__global__ __launch_bounds__(256) void mask_index_kernel(int64_t N, const uint8_t* __restrict__ mask,
                                                         const int64_t* __restrict__ block_base,
                                                         int32_t* __restrict__ index) {
    __shared__ int32_t s_rows[kExBlock];
    const int64_t b0 = (int64_t)blockIdx.x * kExBlock;
    const int n = ex_block_rows(N, mask, b0, s_rows);
    const int64_t o0 = block_base[blockIdx.x];
    for (int e = threadIdx.x; e < n; e += 256) index[o0 + e] = (int32_t)(b0 + s_rows[e]);
}

}  // namespace hgsr

using namespace hgsr;

static int64_t ex_blocks(int64_t N) { return (N + kExBlock - 1) / kExBlock; }

extern "C" size_t hgsr_explicit_ws_bytes(int64_t N) {
    const int64_t nb = ex_blocks(N);
    return (size_t)(nb * (int64_t)sizeof(int32_t) + 255) / 256 * 256 + (size_t)nb * sizeof(int64_t);
}

extern "C" int hgsr_explicit_count(int64_t N, const float* xyz, const int32_t* level, const float* extra_level,
                                   const float* cam_center, float res_scale, float standard_dist, float log2_fork,
                                   int max_level, const uint8_t* visible, uint8_t* mask, void* ws, size_t ws_bytes,
                                   int64_t* total, hgsr_stream_t stream) {
    HGSR_REQUIRE(N >= 0 && N < (1ll << 31), "explicit: N must be < 2^31 (got %lld)", (long long)N);
    HGSR_REQUIRE(ws_bytes >= hgsr_explicit_ws_bytes(N), "explicit: workspace too small");
    HGSR_REQUIRE(total && ws && (mask || visible), "null pointer");
    HGSR_REQUIRE(visible || (xyz && level && extra_level && cam_center && max_level >= 0),
                 "explicit: give a visibility mask or the LoD inputs");
    const int64_t nb = ex_blocks(N);
    HGSR_REQUIRE(nb <= (1 << 20), "explicit: too many Gaussians for the single-workgroup scan");
    hipStream_t s = as_stream(stream);
    if (N == 0) return memset_async(total, sizeof(int64_t), s, "explicit_count");
    int32_t* cnt = (int32_t*)ws;
    int64_t* base = (int64_t*)((char*)ws + (nb * (int64_t)sizeof(int32_t) + 255) / 256 * 256);
    const ExLod L{level, extra_level, cam_center, res_scale, standard_dist, log2_fork, max_level};
    hipLaunchKernelGGL(explicit_count_kernel, dim3((unsigned)nb), dim3(256), 0, s, N, xyz, L, visible, mask, cnt);
    hipLaunchKernelGGL(explicit_scan_kernel, dim3(1), dim3(1024), 0, s, (int)nb, cnt, base, total);
    return check_launch("explicit_count");
}

extern "C" int hgsr_explicit_gather(int64_t N, int K, const uint8_t* mask, const float* xyz, const float* f_dc,
                                    const float* f_rest, const float* opacity, const float* scaling,
                                    const float* rotation, const void* ws, size_t ws_bytes, float* out_xyz,
                                    float* out_color, float* out_opacity, float* out_scaling, float* out_rotation,
                                    int32_t* out_index, hgsr_stream_t stream) {
    HGSR_REQUIRE(N >= 0 && K >= 1, "bad dims");
    HGSR_REQUIRE(ws_bytes >= hgsr_explicit_ws_bytes(N), "explicit: workspace too small");
    if (N == 0) return HGSR_OK;
    HGSR_REQUIRE(mask && xyz && f_dc && (f_rest || K == 1) && opacity && scaling && rotation && ws, "null pointer");
    HGSR_REQUIRE(out_xyz && out_color && out_opacity && out_scaling && out_rotation && out_index, "null pointer");
    const int64_t nb = ex_blocks(N);
    const int64_t* base = (const int64_t*)((const char*)ws + (nb * (int64_t)sizeof(int32_t) + 255) / 256 * 256);
    const ExSrc src{xyz, f_dc, f_rest, opacity, scaling, rotation, K};
    const ExDst dst{out_xyz, out_color, out_opacity, out_scaling, out_rotation, out_index};
    KernelTimer kt("explicit_gather", as_stream(stream));
    hipLaunchKernelGGL(explicit_gather_kernel, dim3((unsigned)nb), dim3(256), 0, as_stream(stream), N, mask, base,
                       src, dst);
    return check_launch("explicit_gather");
}

extern "C" int hgsr_explicit_scatter(int64_t N, int K, const uint8_t* mask, const void* ws, size_t ws_bytes,
                                     const float* g_xyz, const float* g_color, const float* g_opacity,
                                     const float* g_scaling, const float* g_rotation, float* v_xyz, float* v_f_dc,
                                     float* v_f_rest, float* v_opacity, float* v_scaling, float* v_rotation,
                                     hgsr_stream_t stream) {
    HGSR_REQUIRE(N >= 0 && K >= 1, "bad dims");
    HGSR_REQUIRE(ws_bytes >= hgsr_explicit_ws_bytes(N), "explicit: workspace too small");
    if (N == 0) return HGSR_OK;
    HGSR_REQUIRE(mask && ws, "null pointer");
    const int64_t nb = ex_blocks(N);
    const int64_t* base = (const int64_t*)((const char*)ws + (nb * (int64_t)sizeof(int32_t) + 255) / 256 * 256);
    const ExGradIn g{g_xyz, g_color, g_opacity, g_scaling, g_rotation};
    const ExGradOut v{v_xyz, v_f_dc, K > 1 ? v_f_rest : nullptr, v_opacity, v_scaling, v_rotation};
    hipLaunchKernelGGL(explicit_scatter_kernel, dim3((unsigned)nb), dim3(256), 0, as_stream(stream), N, K, mask,
                       base, g, v);
    return check_launch("explicit_scatter");
}

extern "C" int hgsr_mask_index(int64_t N, const uint8_t* mask, const void* ws, size_t ws_bytes, int32_t* index,
                               hgsr_stream_t stream) {
    HGSR_REQUIRE(N >= 0, "bad dims");
    HGSR_REQUIRE(ws_bytes >= hgsr_explicit_ws_bytes(N), "mask_index: workspace too small");
    if (N == 0) return HGSR_OK;
    HGSR_REQUIRE(mask && ws && index, "null pointer");
    const int64_t nb = ex_blocks(N);
    const int64_t* base = (const int64_t*)((const char*)ws + (nb * (int64_t)sizeof(int32_t) + 255) / 256 * 256);
    hipLaunchKernelGGL(mask_index_kernel, dim3((unsigned)nb), dim3(256), 0, as_stream(stream), N, mask, base, index);
    return check_launch("mask_index");
}
