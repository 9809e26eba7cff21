// K16: densification on device.
//
//  * training_statis   <- scene/basic_model.py:96-144: one lane per (visible anchor, slot),
//                         whole anchors per workgroup (deterministic, no atomics): opacity
//                         mean/max per anchor, visit count, per-slot grad-norm / radius /
//                         opacity / denominator updates for the selected, visible slots;
//  * voxel dedup       <- scene/basic_model.py:179-190 get_remove_duplicates: the O(M*A)
//                         broadcast compare becomes an open-addressing hash set of the
//                         existing anchors' voxel coordinates (64-bit packed keys,
//                         linear probing, atomicCAS insert) queried once per candidate;
//  * segment max       <- torch_scatter.scatter_max(src, index, dim=0)[0] as used by
//                         scene/lod_model.py:559 (order-free float max via int atomics);
//  * weed_out          <- scene/lod_model.py:236-249: per candidate, the fraction of
//                         training cameras whose LoD level admits it (cameras in LDS).
// All entry points are asynchronous; none allocates.
#include "common.h"

namespace hgsr {

// ------------------------------------------------------------ training_statis
struct StatisIn {
    const int32_t* vis_idx;   // [Av] anchor id of each visible anchor (ascending, = nonzero(visible_mask))
    const uint8_t* sel;       // [Av*noff] selection mask (decode opacity > 0)
    const int32_t* sel_rank;  // [Av*noff] exclusive prefix of sel = row in the decoded outputs
    const uint8_t* filt;      // [M] visibility filter (radii > 0)
    const float* grad;        // [M,2] viewspace grad (means2d.grad)
    const float* opacity;     // [M]
    const int32_t* radii;     // [M] (max mode only)
};

struct StatisState {
    float* anchor_opacity_accum;  // [A]
    float* anchor_demon;          // [A]
    float* offset_gradient_accum;  // [A*noff]
    float* offset_denom;           // [A*noff]
    float* max_radii2D;            // [A*noff] (max mode)
    float* offset_opacity_accum;   // [A*noff] (max mode)
};

// One lane per (visible anchor, slot): a workgroup holds kStatAnch whole anchors (kStatAnch *
// n_offsets lanes), so the selection bytes / ranks, the Gaussian gathers and the per-slot
// accumulators are read and written by consecutive lanes (a lane per anchor walking its
// slots touched every cache line n_offsets times).  Each slot's accumulators are written by
// exactly one lane; the per-anchor opacity sum and count go through LDS and are formed by the
// anchor's slot-0 lane in slot order (the arithmetic of a sequential walk: deterministic).
constexpr int kStatMaxOff = 16;
constexpr int kStatAnch = 32;  // anchors per workgroup (<= 512 lanes)
__global__ __launch_bounds__(kStatAnch * kStatMaxOff) void training_statis_kernel(
    int Av, int noff, float half_w, float half_h, int pruning_max, int growing_max, StatisIn in, StatisState st) {
    __shared__ float s_o[kStatAnch * kStatMaxOff];
    __shared__ uint8_t s_sel[kStatAnch * kStatMaxOff];
    const int t = threadIdx.x, la = t / noff, k = t - la * noff;
    const int a = blockIdx.x * kStatAnch + la;
    const bool lane_ok = la < kStatAnch && a < Av;
    const int64_t j = (int64_t)a * noff + k;
    const int64_t id = lane_ok ? in.vis_idx[a] : 0;
    const bool sel = lane_ok && in.sel[j];
    const int64_t mk = sel ? in.sel_rank[j] : 0;
    const int64_t gslot = id * noff + k;
    const float o = sel ? in.opacity[mk] : 0.f;
    const bool flt = sel && in.filt[mk];
    const float gx = flt ? in.grad[mk * 2] : 0.f, gy = flt ? in.grad[mk * 2 + 1] : 0.f;
    const float acc = flt ? st.offset_gradient_accum[gslot] : 0.f;
    const float den = flt ? st.offset_denom[gslot] : 0.f;
    const float mr = (flt && growing_max) ? st.max_radii2D[gslot] : 0.f;
    const float oa = (flt && growing_max) ? st.offset_opacity_accum[gslot] : 0.f;
    const float rad = (flt && growing_max) ? (float)in.radii[mk] : 0.f;
    if (flt) {
        // grad[:, 0] *= W/2, grad[:, 1] *= H/2, then the 2-norm (basic_model.py:128-131)
        const float sx = gx * half_w, sy = gy * half_h;
        const float gn = sqrtf(sx * sx + sy * sy);
        if (growing_max) {
            st.offset_gradient_accum[gslot] = fmaxf(acc, fabsf(gn));
            st.max_radii2D[gslot] = fmaxf(mr, rad);
            st.offset_opacity_accum[gslot] = oa + o;
        } else {
            st.offset_gradient_accum[gslot] = acc + gn;
        }
        st.offset_denom[gslot] = den + 1.f;
    }
    s_o[t] = o;
    s_sel[t] = sel;
    __syncthreads();
    if (!lane_ok || k != 0) return;
    const float a_old = st.anchor_opacity_accum[id], d_old = st.anchor_demon[id];
    float osum = 0.f;
    int cnt = 0;
    for (int q = 0; q < noff; ++q) {
        if (!s_sel[t + q]) continue;
        osum += s_o[t + q];
        ++cnt;
    }
    if (pruning_max) {
        st.anchor_opacity_accum[id] = fmaxf(a_old, fabsf(osum));
    } else {
        st.anchor_opacity_accum[id] = a_old + (cnt > 0 ? osum / (float)cnt : 0.f);  // clamp(count, 1); 0 if empty
    }
    st.anchor_demon[id] = d_old + 1.f;
}

// ------------------------------------------------------------ voxel hash set
constexpr uint64_t kHashEmpty = ~0ull;
constexpr int kCoordBits = 21;
constexpr int32_t kCoordMax = (1 << (kCoordBits - 1)) - 1;

__device__ __forceinline__ bool pack_voxel(const int32_t* c, uint64_t& key) {
    const int32_t x = c[0], y = c[1], z = c[2];
    if (x < -kCoordMax || x > kCoordMax || y < -kCoordMax || y > kCoordMax || z < -kCoordMax || z > kCoordMax)
        return false;
    const uint64_t m = (1ull << kCoordBits) - 1;
    key = ((uint64_t)(x + kCoordMax) & m) | (((uint64_t)(y + kCoordMax) & m) << kCoordBits) |
          (((uint64_t)(z + kCoordMax) & m) << (2 * kCoordBits));
    return true;
}

__device__ __forceinline__ uint64_t mix64(uint64_t k) {  // splitmix64 finaliser
    k ^= k >> 30;
    k *= 0xbf58476d1ce4e5b9ull;
    k ^= k >> 27;
    k *= 0x94d049bb133111ebull;
    k ^= k >> 31;
    return k;
}

__global__ __launch_bounds__(256) void voxel_clear_kernel(int64_t cap, uint64_t* __restrict__ table) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < cap) table[i] = kHashEmpty;
}

__global__ __launch_bounds__(256) void voxel_insert_kernel(int64_t n, const int32_t* __restrict__ coords,
                                                           int64_t cap, uint64_t* __restrict__ table,
                                                           int32_t* __restrict__ overflow) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    uint64_t key;
    if (!pack_voxel(coords + i * 3, key)) {
        atomicOr(overflow, 1);
        return;
    }
    uint64_t h = mix64(key) & (uint64_t)(cap - 1);
    for (int64_t probe = 0; probe < cap; ++probe) {
        const uint64_t prev = atomicCAS((unsigned long long*)&table[h], (unsigned long long)kHashEmpty,
                                        (unsigned long long)key);
        if (prev == kHashEmpty || prev == key) return;
        h = (h + 1) & (uint64_t)(cap - 1);
    }
    atomicOr(overflow, 2);  // table full (cannot happen at load factor <= 1/2)
}

__global__ __launch_bounds__(256) void voxel_query_kernel(int64_t n, const int32_t* __restrict__ coords, int64_t cap,
                                                          const uint64_t* __restrict__ table,
                                                          uint8_t* __restrict__ found,
                                                          int32_t* __restrict__ overflow) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    uint64_t key;
    if (!pack_voxel(coords + i * 3, key)) {
        atomicOr(overflow, 1);
        found[i] = 0;
        return;
    }
    uint64_t h = mix64(key) & (uint64_t)(cap - 1);
    uint8_t hit = 0;
    for (int64_t probe = 0; probe < cap; ++probe) {
        const uint64_t v = table[h];
        if (v == key) {
            hit = 1;
            break;
        }
        if (v == kHashEmpty) break;
        h = (h + 1) & (uint64_t)(cap - 1);
    }
    found[i] = hit;
}

// ------------------------------------------------------------ segment max
__device__ __forceinline__ void atomic_max_f32(float* addr, float v) {
    // order-free: non-negative floats order like ints, negative ones reversed like uints
    if (v >= 0.f)
        atomicMax(reinterpret_cast<int*>(addr), __float_as_int(v));
    else
        atomicMin(reinterpret_cast<unsigned int*>(addr), __float_as_uint(v));
}

__global__ __launch_bounds__(256) void fill_f32_kernel(int64_t n, float v, float* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n) out[i] = v;
}

__global__ __launch_bounds__(256) void scatter_max_kernel(int64_t n, int F, const float* __restrict__ src,
                                                          const int64_t* __restrict__ index, int64_t n_out,
                                                          float* __restrict__ out) {
    const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (e >= n * F) return;
    const int64_t r = e / F, f = e - r * F;
    const int64_t o = index[r];
    if (o < 0 || o >= n_out) return;
    atomic_max_f32(out + o * F + f, src[e]);
}

__global__ __launch_bounds__(256) void unfilled_to_zero_kernel(int64_t n, float* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n && __float_as_uint(out[i]) == 0xff800000u) out[i] = 0.f;  // torch_scatter fills empty rows with 0
}

// ------------------------------------------------------------ weed_out
// map_to_int_level (basic_model.py:192-210): 0 floor, 1 round (half to even), 2 ceil,
// 3 progressive (floor(clamp(pred + 1, 0.9999, cur + 0.9999)))
__device__ __forceinline__ int int_level(float pred, int mode, int cur) {
    if (mode == 3) return (int)floorf(fminf(fmaxf(pred + 1.0f, 0.9999f), (float)cur + 0.9999f));
    const float r = mode == 0 ? floorf(pred) : (mode == 1 ? rintf(pred) : ceilf(pred));
    return min(max((int)r, 0), cur);
}

constexpr int kWeedCams = 2048;  // cameras staged per LDS pass

__global__ __launch_bounds__(256) void weed_out_kernel(int64_t n, const float* __restrict__ pos,
                                                       const int32_t* __restrict__ levels, int n_cams,
                                                       const float* __restrict__ cams, float standard_dist,
                                                       float log2_fork, int max_level, int mode, float ratio,
                                                       uint8_t* __restrict__ mask) {
    __shared__ float4 s_cam[kWeedCams];
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const bool live = i < n;
    const float px = live ? pos[i * 3] : 0.f, py = live ? pos[i * 3 + 1] : 0.f, pz = live ? pos[i * 3 + 2] : 0.f;
    const int lv = live ? levels[i] : 0;
    int count = 0;
    for (int c0 = 0; c0 < n_cams; c0 += kWeedCams) {
        const int nc = min(kWeedCams, n_cams - c0);
        __syncthreads();
        for (int c = threadIdx.x; c < nc; c += 256)
            s_cam[c] = make_float4(cams[(c0 + c) * 4], cams[(c0 + c) * 4 + 1], cams[(c0 + c) * 4 + 2],
                                   cams[(c0 + c) * 4 + 3]);
        __syncthreads();
        for (int c = 0; c < nc; ++c) {
            const float4 cm = s_cam[c];
            const float dx = px - cm.x, dy = py - cm.y, dz = pz - cm.z;
            const float dist = sqrtf(dx * dx + dy * dy + dz * dz) * cm.w;
            const float pred = log2f(standard_dist / dist) / log2_fork;
            count += lv <= int_level(pred, mode, max_level) ? 1 : 0;
        }
    }
    // visible_count / len(cam_infos) > weed_ratio (lod_model.py:245-246)
    if (live) mask[i] = ((float)count / (float)n_cams) > ratio ? 1 : 0;
}

}  // namespace hgsr

using namespace hgsr;

static unsigned blocks_for(int64_t n) { return (unsigned)((n + 255) / 256); }

extern "C" int hgsr_training_statis(int Av, int n_offsets, int width, int height, int pruning_max, int growing_max,
                                    const int32_t* vis_idx, const uint8_t* selection, const int32_t* selection_rank,
                                    const uint8_t* visibility_filter, const float* viewspace_grad,
                                    const float* opacity, const int32_t* radii, float* anchor_opacity_accum,
                                    float* anchor_demon, float* offset_gradient_accum, float* offset_denom,
                                    float* max_radii2D, float* offset_opacity_accum, hgsr_stream_t stream) {
    HGSR_REQUIRE(Av >= 0 && n_offsets > 0 && width > 0 && height > 0, "bad dims");
    HGSR_REQUIRE(n_offsets <= kStatMaxOff, "training_statis: n_offsets must be <= %d (got %d)", kStatMaxOff, n_offsets);
    if (Av == 0) return HGSR_OK;
    HGSR_REQUIRE(vis_idx && selection && selection_rank && visibility_filter && viewspace_grad && opacity &&
                     anchor_opacity_accum && anchor_demon && offset_gradient_accum && offset_denom,
                 "null pointer");
    HGSR_REQUIRE(!growing_max || (radii && max_radii2D && offset_opacity_accum), "max growing needs radii/max/opacity");
    const StatisIn in{vis_idx, selection, selection_rank, visibility_filter, viewspace_grad, opacity, radii};
    const StatisState st{anchor_opacity_accum, anchor_demon, offset_gradient_accum, offset_denom, max_radii2D,
                         offset_opacity_accum};
    KernelTimer kt("training_statis", as_stream(stream));
    hipLaunchKernelGGL(training_statis_kernel, dim3((Av + kStatAnch - 1) / kStatAnch), dim3(kStatAnch * n_offsets), 0,
                       as_stream(stream), Av, n_offsets, 0.5f * (float)width, 0.5f * (float)height, pruning_max,
                       growing_max, in, st);
    return check_launch("training_statis");
}

static int64_t voxel_capacity(int64_t n) {
    int64_t cap = 64;
    while (cap < 2 * n) cap <<= 1;
    return cap;
}

extern "C" size_t hgsr_voxel_dedup_ws_bytes(int64_t n_grid) { return (size_t)voxel_capacity(n_grid) * 8 + 256; }

extern "C" int hgsr_voxel_dedup(int64_t n_grid, const int32_t* grid_coords, int64_t n_cand, const int32_t* cand_coords,
                                uint8_t* found, int32_t* overflow, void* ws, size_t ws_bytes, hgsr_stream_t stream) {
    HGSR_REQUIRE(n_grid >= 0 && n_cand >= 0, "bad sizes");
    HGSR_REQUIRE(ws_bytes >= hgsr_voxel_dedup_ws_bytes(n_grid), "voxel dedup workspace too small");
    HGSR_REQUIRE(overflow && ws && (n_grid == 0 || grid_coords) && (n_cand == 0 || (cand_coords && found)),
                 "null pointer");
    hipStream_t s = as_stream(stream);
    if (int st = memset_async(overflow, 4, s, "voxel_dedup")) return st;
    const int64_t cap = voxel_capacity(n_grid);
    uint64_t* table = (uint64_t*)ws;
    hipLaunchKernelGGL(voxel_clear_kernel, dim3(blocks_for(cap)), dim3(256), 0, s, cap, table);
    if (n_grid > 0)
        hipLaunchKernelGGL(voxel_insert_kernel, dim3(blocks_for(n_grid)), dim3(256), 0, s, n_grid, grid_coords, cap,
                           table, overflow);
    if (n_cand > 0)
        hipLaunchKernelGGL(voxel_query_kernel, dim3(blocks_for(n_cand)), dim3(256), 0, s, n_cand, cand_coords, cap,
                           table, found, overflow);
    return check_launch("voxel_dedup");
}

extern "C" int hgsr_scatter_max(int64_t n, int F, const float* src, const int64_t* index, int64_t n_out, float* out,
                                hgsr_stream_t stream) {
    HGSR_REQUIRE(n >= 0 && F > 0 && n_out >= 0, "bad sizes");
    HGSR_REQUIRE((n == 0 || (src && index)) && (n_out == 0 || out), "null pointer");
    hipStream_t s = as_stream(stream);
    if (n_out == 0) return HGSR_OK;
    hipLaunchKernelGGL(fill_f32_kernel, dim3(blocks_for(n_out * F)), dim3(256), 0, s, n_out * F, -INFINITY, out);
    if (n > 0)
        hipLaunchKernelGGL(scatter_max_kernel, dim3(blocks_for(n * F)), dim3(256), 0, s, n, F, src, index, n_out, out);
    hipLaunchKernelGGL(unfilled_to_zero_kernel, dim3(blocks_for(n_out * F)), dim3(256), 0, s, n_out * F, out);
    return check_launch("scatter_max");
}

extern "C" int hgsr_weed_out(int64_t n, const float* positions, const int32_t* levels, int n_cams,
                             const float* cam_infos, float standard_dist, float fork, int street_levels,
                             int dist2level_mode, float weed_ratio, uint8_t* mask, hgsr_stream_t stream) {
    HGSR_REQUIRE(n >= 0 && n_cams > 0 && fork > 1.f && street_levels >= 1, "bad args");
    HGSR_REQUIRE(dist2level_mode >= 0 && dist2level_mode <= 3, "dist2level mode must be 0..3");
    if (n == 0) return HGSR_OK;
    HGSR_REQUIRE(positions && levels && cam_infos && mask, "null pointer");
    hipLaunchKernelGGL(weed_out_kernel, dim3(blocks_for(n)), dim3(256), 0, as_stream(stream), n, positions, levels,
                       n_cams, cam_infos, standard_dist, log2f(fork), street_levels - 1, dist2level_mode, weed_ratio,
                       mask);
    return check_launch("weed_out");
}
