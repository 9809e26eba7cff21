// Shared helpers for the hgsr HIP kernels (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "../../include/hgsr.h"

namespace hgsr {

void set_error(const char* fmt, ...);

// Optional HIP-event timing of the main kernel of an entry point (timing.hip).
bool timing_on();
int timing_begin(const char* name, hipStream_t s);
void timing_end(int id, hipStream_t s);
// measurement only: device counter the raster backward adds its visited (pixel, Gaussian)
// pairs to while `kernel` is being timed (nullptr otherwise)
unsigned long long* timing_pair_counter(const char* kernel);
struct KernelTimer {
    int id;
    hipStream_t s;
    KernelTimer(const char* name, hipStream_t st) : id(timing_on() ? timing_begin(name, st) : -1), s(st) {}
    ~KernelTimer() { timing_end(id, s); }
};

// The pair counters are spread over kPairSlots 128-B lines (two counters per workgroup
// slot) so the per-tile atomics of the timed kernel never queue on one L2 channel; the
// readout sums the slots.
constexpr int kPairSlots = 256;
__device__ __forceinline__ unsigned long long* pair_slot(unsigned long long* base, int which) {
    return base + ((int)(blockIdx.x & (kPairSlots - 1)) * 2 + which) * 16;
}

// Returns HGSR_ELAUNCH (and records the HIP error) if the last launch failed.
int check_launch(const char* what);

constexpr int kTile = 16;          // gsplat default tile_size; one 256-lane workgroup per tile
constexpr int kTilePixels = 256;
constexpr int kWave = 64;

#define HGSR_REQUIRE(cond, ...)            \
    do {                                   \
        if (!(cond)) {                     \
            ::hgsr::set_error(__VA_ARGS__); \
            return HGSR_EINVAL;            \
        }                                  \
    } while (0)

inline int memset_async(void* p, size_t n, hipStream_t s, const char* what) {
    hipError_t e = hipMemsetAsync(p, 0, n, s);
    if (e != hipSuccess) {
        set_error("%s: hipMemsetAsync failed: %s", what, hipGetErrorString(e));
        return HGSR_ELAUNCH;
    }
    return HGSR_OK;
}

inline hipStream_t as_stream(hgsr_stream_t s) { return reinterpret_cast<hipStream_t>(s); }

// Bijective XCD-aware remap of a 1-D grid: the dispatcher deals workgroups
// round-robin over the 8 XCDs (b and b+8 share one), so give XCD x a contiguous
// run of work items (neighbouring tiles share Gaussians through that XCD's L2).
// Speed only: correctness never depends on placement.
__device__ __forceinline__ int xcd_remap(int b, int nwg) {
    const int xcd = b & 7;
    const int idx = b >> 3;
    const int q = nwg >> 3, r = nwg & 7;
    return xcd * q + (xcd < r ? xcd : r) + idx;
}

// the raster kernels' tile of workgroup blockIdx.x: its XCD band's slot, through the
// heaviest-first order when one was computed (order == nullptr: band order)
__device__ __forceinline__ int raster_bin(const int32_t* __restrict__ order) {
    const int slot = xcd_remap(blockIdx.x, gridDim.x);
    return order ? order[slot] : slot;
}

template <int CTRL>
__device__ __forceinline__ float dpp(float x) {  // lane-shuffled copy of x (bound_ctrl: 0 for invalid)
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), CTRL, 0xF, 0xF, false));
}

// Full 64-lane sum with DPP row ops; the total lands in lane 63.
__device__ __forceinline__ float wave_sum_to_lane63(float v) {
    int x;
    x = __builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xB1, 0xF, 0xF, false);  // quad_perm [1,0,3,2]
    v += __int_as_float(x);
    x = __builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x4E, 0xF, 0xF, false);  // quad_perm [2,3,0,1]
    v += __int_as_float(x);
    x = __builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x124, 0xF, 0xF, false); // row_ror:4
    v += __int_as_float(x);
    x = __builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x128, 0xF, 0xF, false); // row_ror:8
    v += __int_as_float(x);
    x = __builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x142, 0xA, 0xF, false); // row_bcast:15
    v += __int_as_float(x);
    x = __builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x143, 0xC, 0xF, false); // row_bcast:31
    v += __int_as_float(x);
    return v;
}

// Workgroup barrier that only orders LDS: waits for this wave's LDS operations
// (lgkmcnt) but NOT for outstanding global loads/stores/atomics.  __syncthreads()
// would drain vmcnt(0) -- i.e. stall every wave on the float atomics it just
// issued -- which dominated the raster backward (SQ_WAIT_ANY ~47 % of wave cycles).
// Valid only where no global-memory value written by one wave is read by another
// wave of the workgroup across the barrier.
// Quadrant masks (raster forward -> backward, 3DGS and 2DGS): bit r of array w says whether
// record r of a tile's list (r = isect index - tile start) passed wave w's quadrant culling
// in the forward (the same test the backward would repeat).  A tile's bits
// start at word qmask_word0(start, bin) = ceil(start / 64) + bin + 2 and it writes only the
// ceil(n / 64) words holding its n records, so no two tiles share a word; the backward may
// read up to two words before a tile's first.  One array of qstride words per quadrant.
__host__ __device__ __forceinline__ int64_t qmask_word0(int64_t start, int64_t bin) {
    return (start + 63) / 64 + bin + 2;
}
__host__ __device__ __forceinline__ int64_t qmask_stride(int64_t n_isects, int64_t n_bins) {
    return (n_isects + 63) / 64 + n_bins + 4;
}
// The caller-sized quadrant-mask buffer (hgsr_raster3d_qmask_bytes) starts with the tiles'
// dispatch order (tile_order_kernel, one int32 per (camera, tile) bin, 256-B aligned), then
// the 4 arrays of 64-bit words.  Forward and backward derive both from the same buffer,
// which may be sized for a capacity above n_isects.
inline size_t tile_list_bytes(int64_t n_bins) { return ((size_t)n_bins * sizeof(int32_t) + 255) & ~(size_t)255; }
// [order | per-tile trimmed end (the 3DGS forward's latest contributor + 1, for the backward's order)]
inline size_t tile_order_bytes(int64_t n_bins) { return 2 * tile_list_bytes(n_bins); }
inline int64_t qmask_stride_of(size_t qmask_bytes, int64_t n_bins) {
    const size_t ob = tile_order_bytes(n_bins);
    return qmask_bytes > ob ? (int64_t)((qmask_bytes - ob) / (4 * sizeof(uint64_t))) : 0;
}
inline uint64_t* qmask_words(void* buf, int64_t n_bins) {
    return buf ? reinterpret_cast<uint64_t*>(static_cast<char*>(buf) + tile_order_bytes(n_bins)) : nullptr;
}
inline const uint64_t* qmask_words(const void* buf, int64_t n_bins) {
    return buf ? reinterpret_cast<const uint64_t*>(static_cast<const char*>(buf) + tile_order_bytes(n_bins)) : nullptr;
}
inline int32_t* tile_order_of(void* buf) { return static_cast<int32_t*>(buf); }
inline int32_t* tile_end_of(void* buf, int64_t n_bins) {
    return reinterpret_cast<int32_t*>(static_cast<char*>(buf) + tile_list_bytes(n_bins));
}
inline const int32_t* tile_order_of(const void* buf) { return static_cast<const int32_t*>(buf); }

// Heaviest-first dispatch order of the raster tiles (core.hip): within each XCD's contiguous
// band of bins (xcd_remap), the bins sorted by intersection count, largest first, so the
// long tiles start early and the grid does not end on a few stragglers.  order[slot] = bin.
#ifndef HGSR_TILE_ORDER
#define HGSR_TILE_ORDER 1
#endif
// tile_end (nullable): order by the trimmed range [start, min(end, tile_end)) instead of the whole bin
int launch_tile_order(int64_t n_bins, const int32_t* offsets, int64_t n_isects, const int64_t* info, int32_t* order,
                      hipStream_t s, const int32_t* tile_end = nullptr);
// The raster backwards' tiles ordered by the ranges they walk -- up to each tile's latest
// contributor, written by the forward into the mask buffer -- rather than by whole-bin counts
// (c2 raster3d_bwd 0.542 -> 0.529 ms on the camera set, 0.551 -> 0.514 on the fixed view,
// gpurun_out/r05s17/ab_bo)
#ifndef HGSR_BWD_ORDER
#define HGSR_BWD_ORDER 1
#endif

// Gradient slots of the raster backwards (isect.hip): (camera, Gaussian) o owns the slots
// [seg[o], seg[o + 1]), one per tile of its rectangle in row-major order; its slot at tile (x, y)
// is slot[o].x + y slot[o].y + x.  Each slot e has kSlotWaves partial rows (one per wave of the
// tile's workgroup) and flags[kSlotWaves e + w] != 0 iff wave w wrote row (e, w) in this launch
// (both raster backwards).
constexpr int kSlotWaves = 4;
// A (camera, Gaussian) with more than kBigSlots slots (a footprint over kBigSlots tiles: close
// views put Gaussians over the whole screen, 8,160 tiles at 1080p) is reduced in pieces of
// kPieceSlots slots, one wave each (reduce_pieces), instead of by the wave that owns it: a wave
// walking 8,160 slots alone held the whole reduction's tail (split3 0.28 ms at c2).
#ifndef HGSR_BIG_SLOTS
#define HGSR_BIG_SLOTS 32
#endif
constexpr int kBigSlots = HGSR_BIG_SLOTS;
constexpr int kPieceSlots = 128;
constexpr int kPieceFloats = 20;  // floats per piece partial (>= the rows' used values, 16-B aligned)
struct GradSlots {
    int32_t* seg;     // [C N + 1]
    int2* slot;       // [C N] with element stride sstride (the dense array, or the 3DGS records' slot quads)
    int64_t sstride;
    int32_t* pbase;   // [C N]: first piece of a big entry, -1 for the others
    int32_t* pieces;  // [piece capacity]: the entry of each piece (order of no consequence)
    int32_t* npieces; // [1]: pieces listed
    float* partial;   // [piece capacity][kPieceFloats]: each piece's fixed-order sum
    int64_t cap;      // piece capacity
};
// piece capacity for n_isects slots: sum over big entries of ceil(slots / kPieceSlots)
inline int64_t piece_capacity(int64_t n_isects) { return n_isects / kPieceSlots + n_isects / (kBigSlots + 1) + 4; }
// reduce_pieces_kernel's grid: 4 waves per workgroup striding over the device-side piece count
inline unsigned piece_grid(const GradSlots& g) {
    const int64_t w = (g.cap + 3) / 4;
    return (unsigned)(w < 2048 ? (w > 0 ? w : 1) : 2048);
}
// gsplat isect_tiles rectangle; identical float ops to oracle/hgsr_oracle.c tile_rect.  For a
// power-of-two tile size (gsplat's 16) x / tile_size is x times the exact reciprocal, bit for
// bit, so the correctly rounded division sequence is only run for other sizes.
__device__ __forceinline__ void tile_rect(float mx, float my, int32_t radius, int tile_size, int tw,
                                          int th, int& x0, int& y0, int& x1, int& y1) {
#pragma clang fp contract(off)
    const float ts = (float)tile_size;
    float tr, tx, ty;
    if ((tile_size & (tile_size - 1)) == 0) {
        const float inv = __int_as_float(0x7F000000 - __float_as_int(ts));  // 2^-k exactly
        tr = (float)radius * inv;
        tx = mx * inv;
        ty = my * inv;
    } else {
        tr = (float)radius / ts;
        tx = mx / ts;
        ty = my / ts;
    }
    const float fx0 = floorf(tx - tr), fy0 = floorf(ty - tr), fx1 = ceilf(tx + tr), fy1 = ceilf(ty + tr);
    x0 = fx0 <= 0.f ? 0 : (fx0 >= (float)tw ? tw : (int)fx0);
    y0 = fy0 <= 0.f ? 0 : (fy0 >= (float)th ? th : (int)fy0);
    x1 = fx1 <= 0.f ? 0 : (fx1 >= (float)tw ? tw : (int)fx1);
    y1 = fy1 <= 0.f ? 0 : (fy1 >= (float)th ? th : (int)fy1);
}

// a (camera, Gaussian)'s tile rectangle from its projection (isect_tiles'): its area, corner and width
struct RectFromRadii {
    const float2* m;
    const int32_t* r;
    int ts, tw, th;
    __device__ __forceinline__ int operator()(int64_t o, int& x0, int& y0, int& w) const {
        const int32_t rad = r[o];
        if (rad <= 0) {
            x0 = y0 = w = 0;
            return 0;
        }
        const float2 mm = m[o];
        int x1, y1;
        tile_rect(mm.x, mm.y, rad, ts, tw, th, x0, y0, x1, y1);
        w = x1 - x0;
        return (y1 - y0) * w;
    }
};

// the same areas, already counted by hgsr_isect_count (its tiles_per_gauss): 4 B an entry read
// instead of 12 B and a rectangle (the slot prefix's row sums; the corner is not needed there)
struct AreaFromCounts {
    const int32_t* a;
    __device__ __forceinline__ int operator()(int64_t o, int& x0, int& y0, int& w) const {
        x0 = y0 = w = 0;
        return a[o];
    }
};

constexpr int kSlotRow = 256;  // entries per element of the slot-area prefix (one workgroup row)
// the forward's slot prefix (hgsr_raster3d_pack_fused with radii): seg [CN + 1], the row prefix
// [CN / kSlotRow + 1], then the backward's piece count (cleared by the forward's scan)
size_t slot_prefix_bytes(int64_t CN);
int32_t* slot_prefix_npieces(void* buf, int64_t CN);
// row area sums + their exclusive scan into buf (seg[CN] = the total); pack3 finishes seg.
// areas (nullable): the entries' areas as hgsr_isect_count counted them (else from r)
int launch_slot_prefix(int64_t CN, const RectFromRadii& r, void* buf, hipStream_t s, const int32_t* areas = nullptr);
// the big entries' piece list from a finished seg (launch_grad_slots' buffer layout in buf)
// npieces (nullable): the piece count's location, already zero when npieces_zeroed (else cleared here)
int launch_grad_pieces(int64_t CN, const int32_t* seg, int64_t n_isects, void* buf, hipStream_t s, GradSlots& out,
                       int32_t* npieces = nullptr, bool npieces_zeroed = false);
// bytes of launch_grad_slots' buffer (from_lists: the rectangles are found from the lists)
size_t grad_slot_bytes(int64_t CN, bool from_lists, int64_t n_isects);
// radii != nullptr: rectangles from means2d / radii (isect_tiles'); else from the sorted lists.
// slot_dst (nullable): where the slot bases go, element o at slot_dst[o * sstride] (the 3DGS
// records' slot quads); else the dense array in buf
int launch_grad_slots(int C, int N, const float* means2d, const int32_t* radii, int tile_size, int tw, int th,
                      const int32_t* offsets, const int32_t* flatten_ids, int64_t n_isects, void* buf,
                      hipStream_t s, GradSlots& out, int2* slot_dst = nullptr, int64_t sstride = 1);
// the flags and partial rows of a backward workspace: flags first, so a forward that only
// knows the intersection capacity can clear them (hgsr_raster{3,2}d_fwd_packed bwd_ws)
inline size_t slot_flag_bytes(int64_t n_isects, int ways) { return ((size_t)n_isects * ways + 255) & ~(size_t)255; }

// LDS ordering between the lanes of ONE wave (a wave's LDS operations complete in issue order;
// this keeps the compiler from moving LDS accesses across it)
__device__ __forceinline__ void wave_lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// The splits' fixed-order sum of gradient slots, for one wave owning the nloc (1..64)
// (camera, Gaussian) entries [ib, ib + nloc), whose slots are contiguous and ascending.  Each slot
// has WAYS partial rows of ROWF floats (the first NV used, R4 float4) and WAYS flag bytes (row
// (e, w) written iff flags[WAYS e + w] != 0).  Entries over kBigSlots slots were reduced in pieces
// (reduce_pieces_kernel, pbase >= 0); the wave walks the other entries' slots 64 at a time:
//   * lane s takes slot cs + s: its flagged rows, loaded together through a range-checked buffer
//     descriptor (an unflagged way passes an out-of-range offset and reads zero without touching
//     memory; the loads are never skipped, so the compiler's wait counts stay exact) and summed
//     in way order in registers -- the next chunk's flags already in flight;
//   * the slot sums are parked in LDS ([slot][NV], float4 runs) and each entry's lane adds its
//     own slots' sums in slot order.
// (Measured against this at c2, split3 0.130 ms: a compacted-list variant -- ballot per way, every
// lane loading a useful quarter row -- 0.147 ms, its list and parking costing more than the loads
// it coalesced (gpurun_out/r06probe, probe builds since removed); four lanes per row with the ways summed by DPP row shifts
// 0.172 ms at 166 VGPRs (gpurun_out/r06probe3).)  No atomics anywhere: the result depends only on the inputs.
// LDS per wave: reduce_slots_floats() floats.
template <int NV>
constexpr int reduce_slots_floats() {
    return 64 * 4 * ((NV + 3) / 4);
}
// wave-wide minimum, returned as a scalar (readfirstlane: the compiler then knows it is uniform)
__device__ __forceinline__ int32_t wave_min_i32(int32_t v) {
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) v = min(v, __shfl_xor(v, d));
    return __builtin_amdgcn_readfirstlane(v);
}
constexpr int kBufWord3 = 0x00020000;  // gfx9 raw buffer descriptor word 3 (32-bit data, range-checked)
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ float4 buf_load4(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    // (an explicitly typed result: through `auto` and v[k] the compiler kept one dword of four)
    const u32x4_t v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 0);
    return make_float4(__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z), __uint_as_float(v.w));
}
template <int NV, int R4, int ROWF, int WAYS, int UNR>
__device__ __forceinline__ void reduce_slots(const float* __restrict__ rows, const uint8_t* __restrict__ flags,
                                             const int32_t* __restrict__ seg, const int32_t* __restrict__ pbase,
                                             const float* __restrict__ partial, int64_t ib, int nloc, float* s_scr,
                                             float (&out)[NV]) {
    static_assert(WAYS >= 1 && WAYS <= 4 && NV <= 4 * R4 && R4 <= 8, "slot rows");
    constexpr int V4 = (NV + 3) / 4;      // float4 per parked slot sum
    constexpr uint32_t kOOB = 0x7fffffffu;  // out-of-range buffer offset: reads zero
    float4* const s_sum = reinterpret_cast<float4*>(s_scr);  // [64 slots][V4]
    const int lane = threadIdx.x & 63;
    const bool live = lane < nloc;
    const int32_t pb = live ? pbase[ib + lane] : -1;
    const int32_t sl = live ? seg[ib + lane] : 0, sh = live ? seg[ib + lane + 1] : 0;
    // a big entry's slots were reduced in pieces: the walker skips them
    const int32_t lo_e = pb < 0 ? sl : 0, hi_e = pb < 0 ? sh : 0;
    const int32_t E1 = __builtin_amdgcn_readfirstlane(seg[ib + nloc]);
    constexpr int32_t kNone = 0x7fffffff;
    // flags of slots [0, E1) through a range-checked descriptor: beyond E1 (or no chunk) reads zero
    const __amdgpu_buffer_rsrc_t frs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint8_t*>(flags), (short)0, (int)(E1 * WAYS), kBufWord3);
    auto fl = [&](int32_t cs) -> uint32_t {
        const uint32_t off = cs != kNone ? (uint32_t)(cs + lane) * WAYS : kOOB;
        return WAYS == 4 ? (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(frs, (int)off, 0, 0)
                         : (uint32_t)__builtin_amdgcn_raw_buffer_load_b8(frs, (int)off, 0, 0);
    };
    // the next chunk: 64 slots from the next slot any entry of this wave still needs.  The
    // entries' slot ranges ascend with the lane, so that is the first lane still needing one
    // (a ballot and a readlane: no cross-lane reduction)
    auto first_from = [&](uint64_t m, int32_t floor_cs) -> int32_t {
        if (m == 0) return kNone;
        const int l = (int)__builtin_ctzll(m);
        return max(__builtin_amdgcn_readlane(lo_e, l), floor_cs);
    };
#pragma unroll
    for (int k = 0; k < NV; ++k) out[k] = 0.f;
    int32_t cs = first_from(__ballot(lo_e < hi_e), 0);
    uint32_t f = cs != kNone ? fl(cs) : 0u;
    while (cs != kNone) {
        const int32_t cn = first_from(__ballot(hi_e > cs + 64), cs + 64);
        const __amdgpu_buffer_rsrc_t rrs = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<float*>(rows) + (int64_t)cs * WAYS * ROWF, (short)0, 64 * WAYS * ROWF * 4, kBufWord3);
        // slot cs + lane: its flagged rows in way order
        float4 x[WAYS][V4];
#pragma unroll
        for (int w = 0; w < WAYS; ++w) {
            const bool has = (f >> (8 * w)) & 0xffu;
#pragma unroll
            for (int r = 0; r < V4; ++r) {
                const uint32_t off = has ? (uint32_t)(((lane * WAYS + w) * ROWF + 4 * r) * 4) : kOOB;
                x[w][r] = buf_load4(rrs, off);
            }
        }
        f = cn != kNone ? fl(cn) : 0u;  // the next chunk's flags, behind this chunk's rows
#pragma unroll
        for (int r = 0; r < V4; ++r) {
            float4 a = x[0][r];
#pragma unroll
            for (int w = 1; w < WAYS; ++w)
                a = make_float4(a.x + x[w][r].x, a.y + x[w][r].y, a.z + x[w][r].z, a.w + x[w][r].w);
            s_sum[lane * V4 + r] = a;
        }
        wave_lds_sync();
        // this entry's slots of the chunk, in order; UNR slots' reads issued together
        const int32_t lo = max(lo_e, cs) - cs, hi = min(hi_e, cs + 64) - cs;
        for (int32_t y = lo; y < hi; y += UNR) {
            float4 t[UNR][V4];
#pragma unroll
            for (int u = 0; u < UNR; ++u)
#pragma unroll
                for (int r = 0; r < V4; ++r)
                    t[u][r] = y + u < hi ? s_sum[(y + u) * V4 + r] : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
            for (int u = 0; u < UNR; ++u)
                if (y + u < hi)
#pragma unroll
                    for (int r = 0; r < V4; ++r) {
                        const float t4[4] = {t[u][r].x, t[u][r].y, t[u][r].z, t[u][r].w};
#pragma unroll
                        for (int c = 0; c < 4; ++c)
                            if (4 * r + c < NV) out[4 * r + c] += t4[c];
                    }
        }
        wave_lds_sync();
        cs = cn;
    }
    // the big entries (a few per wave at most): the whole wave sums each one's piece partials,
    // lane j taking piece j (64 per round, one load latency each), with the fixed DPP tree; a lane
    // walking an 8,160-tile entry's 64 pieces alone held the kernel's tail
    uint64_t bigm = __ballot(pb >= 0);
    while (bigm) {
        const int l = (int)__builtin_ctzll(bigm);
        bigm &= bigm - 1;
        const int32_t pbl = __builtin_amdgcn_readlane(pb, l);
        const int32_t e0 = __builtin_amdgcn_readlane(sl, l), e1 = __builtin_amdgcn_readlane(sh, l);
        const int32_t np = (e1 - e0 + kPieceSlots - 1) / kPieceSlots;
        float tot[NV];
#pragma unroll
        for (int k = 0; k < NV; ++k) tot[k] = 0.f;
        for (int32_t j0 = 0; j0 < np; j0 += 64) {
            const int32_t j = j0 + lane;
            float v[4 * ((NV + 3) / 4)];
#pragma unroll
            for (int r = 0; r < (NV + 3) / 4; ++r) {
                const float4 y = j < np ? reinterpret_cast<const float4*>(partial + (int64_t)(pbl + j) * kPieceFloats)[r]
                                        : make_float4(0.f, 0.f, 0.f, 0.f);
                v[4 * r] = y.x; v[4 * r + 1] = y.y; v[4 * r + 2] = y.z; v[4 * r + 3] = y.w;
            }
#pragma unroll
            for (int k = 0; k < NV; ++k)
                tot[k] += __int_as_float(__builtin_amdgcn_readlane(__float_as_int(wave_sum_to_lane63(v[k])), 63));
        }
        if (lane == l)
#pragma unroll
            for (int k = 0; k < NV; ++k) out[k] = tot[k];
    }
}

// One wave per piece of a big entry's slots (listed by launch_grad_slots): lane l sums slots
// s0 + l and s0 + 64 + l (each slot's flagged rows in way order), then a fixed DPP tree over the
// 64 lanes; partial[k] = the piece's NV sums.  Grid-stride over the device-side piece count.
template <int NV, int R4, int ROWF, int WAYS>
__global__ __launch_bounds__(256) void reduce_pieces_kernel(const float* __restrict__ rows,
                                                            const uint8_t* __restrict__ flags,
                                                            const int32_t* __restrict__ seg,
                                                            const int32_t* __restrict__ pbase,
                                                            const int32_t* __restrict__ pieces,
                                                            const int32_t* __restrict__ npieces,
                                                            float* __restrict__ partial) {
    static_assert(kPieceSlots == 128 && NV <= kPieceFloats, "piece shape");
    const int lane = threadIdx.x & 63;
    const int n = *npieces;
    const int nw = gridDim.x * 4;
    for (int k = blockIdx.x * 4 + (threadIdx.x >> 6); k < n; k += nw) {
        const int32_t o = pieces[k];
        const int32_t j = k - pbase[o];
        const int32_t s0 = seg[o] + j * kPieceSlots, s1 = min(seg[o + 1], s0 + kPieceSlots);
        float4 acc[R4];
#pragma unroll
        for (int r = 0; r < R4; ++r) acc[r] = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int m = 0; m < 2; ++m) {
            const int32_t e = s0 + 64 * m + lane;
            const uint32_t f = e < s1 ? (WAYS == 4 ? reinterpret_cast<const uint32_t*>(flags)[e] : (uint32_t)flags[e]) : 0u;
#pragma unroll
            for (int w = 0; w < WAYS; ++w)
                if ((f >> (8 * w)) & 0xffu) {
                    const float4* rp = reinterpret_cast<const float4*>(rows + ((int64_t)e * WAYS + w) * ROWF);
#pragma unroll
                    for (int r = 0; r < R4; ++r) {
                        const float4 y = rp[r];
                        acc[r] = make_float4(acc[r].x + y.x, acc[r].y + y.y, acc[r].z + y.z, acc[r].w + y.w);
                    }
                }
        }
        float v[4 * R4];
#pragma unroll
        for (int r = 0; r < R4; ++r) {
            v[4 * r] = wave_sum_to_lane63(acc[r].x);
            v[4 * r + 1] = wave_sum_to_lane63(acc[r].y);
            v[4 * r + 2] = wave_sum_to_lane63(acc[r].z);
            v[4 * r + 3] = wave_sum_to_lane63(acc[r].w);
        }
        if (lane == 63) {
            float4* pp = reinterpret_cast<float4*>(partial + (int64_t)k * kPieceFloats);
#pragma unroll
            for (int r = 0; r < R4; ++r) pp[r] = make_float4(v[4 * r], v[4 * r + 1], v[4 * r + 2], v[4 * r + 3]);
        }
    }
}

// count floats from src to LDS dst (16-B aligned) as float4 runs when src allows
__device__ __forceinline__ void stage_floats(const float* __restrict__ src, int count, float* dst) {
    int done = 0;
    if ((reinterpret_cast<uintptr_t>(src) & 15) == 0) {
        const int n4 = count >> 2;
        const float4* s4 = reinterpret_cast<const float4*>(src);
        for (int q = threadIdx.x; q < n4; q += 256) *reinterpret_cast<float4*>(dst + 4 * q) = s4[q];
        done = n4 << 2;
    }
    for (int e = done + threadIdx.x; e < count; e += 256) dst[e] = src[e];
}

// count floats from LDS src (16-B aligned) to dst as float4 runs when dst allows
__device__ __forceinline__ void unstage_floats(const float* src, int count, float* __restrict__ dst) {
    int done = 0;
    if ((reinterpret_cast<uintptr_t>(dst) & 15) == 0) {
        const int n4 = count >> 2;
        float4* d4 = reinterpret_cast<float4*>(dst);
        for (int q = threadIdx.x; q < n4; q += 256) d4[q] = *reinterpret_cast<const float4*>(src + 4 * q);
        done = n4 << 2;
    }
    for (int e = done + threadIdx.x; e < count; e += 256) dst[e] = src[e];
}

// A grid-wide memset folded into a kernel that is not HBM-bound (the raster forwards clear
// the backward's accumulator rows): workgroup b of the grid clears its share
// [b n4 / nwg, (b+1) n4 / nwg) of the n4 float4s.  Called after the kernel's last load, so
// no later vmcnt wait covers these stores.
__device__ __forceinline__ void zero_share(float4* __restrict__ p, int64_t n4) {
    if (!p) return;
    const int64_t nwg = gridDim.x, b = blockIdx.x;
    const int64_t a = b * n4 / nwg, z = (b + 1) * n4 / nwg;
    for (int64_t q = a + threadIdx.x; q < z; q += blockDim.x) p[q] = make_float4(0.f, 0.f, 0.f, 0.f);
}

// LDS-DMA of 16 B per lane (global_load_lds_dwordx4): per-lane source, LDS destination = the
// wave-uniform base + 16 B x lane.  HGSR_ASM_DMA issues it as inline asm, so the compiler's wait
// insertion does not know an LDS-DMA is outstanding: with the builtin it puts s_waitcnt vmcnt(0)
// in front of LDS reads it cannot prove disjoint from the destination, which waits for the
// prefetch itself and for every outstanding gradient atomic of the wave.  Callers order the
// DMA themselves (s_waitcnt vmcnt(0) and a barrier before the destination is read, and before
// the workgroup ends).
#ifndef HGSR_ASM_DMA
#define HGSR_ASM_DMA 1
#endif
__device__ __forceinline__ void lds_dma16(const void* src, void* lds_dst) {
#if HGSR_ASM_DMA
    const uint32_t base = (uint32_t)__builtin_amdgcn_readfirstlane(
        (int)(uint32_t)(uintptr_t)(__attribute__((address_space(3))) void*)lds_dst);
    // m0 is a reserved register the compiler does not let a clobber list name; none of the kernels
    // that call this reads m0 anywhere else (their listings hold no other m0 access)
    asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dwordx4 %0, off" : : "v"(src), "s"(base) : "memory");
#else
    __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)src,
                                     (void __attribute__((address_space(3)))*)lds_dst, 16, 0, 0);
#endif
}

// Wait-site attribution hooks (scripts/micro/wait_probe.py builds the library with
// -DHGSR_PROBE_WAIT=1 into its own directory; in the product build they compile to nothing).
// HGSR_WP_MARK(k) adds the shader-clock cycles since the previous mark to the wave's site k;
// HGSR_WP_FLUSH() adds the wave's sites into the kernel's device-global sums (vector atomics).
#ifndef HGSR_PROBE_WAIT
#define HGSR_PROBE_WAIT 0
#endif
#if HGSR_PROBE_WAIT
#define HGSR_WP_DECL(acc)                                   \
    unsigned long long wp_acc_[8] = {0, 0, 0, 0, 0, 0, 0, 0}; \
    unsigned long long wp_t_ = __builtin_amdgcn_s_memtime();  \
    unsigned long long* const wp_dst_ = (acc)
#define HGSR_WP_MARK(k)                                               \
    {                                                                 \
        const unsigned long long t_ = __builtin_amdgcn_s_memtime();   \
        wp_acc_[k] += t_ - wp_t_;                                     \
        wp_t_ = t_;                                                   \
    }
#define HGSR_WP_FLUSH()                                                                  \
    if ((threadIdx.x & 63) == 0) {                                                       \
        for (int k_ = 0; k_ < 8; ++k_) atomicAdd(wp_dst_ + k_, wp_acc_[k_]);              \
        atomicAdd(wp_dst_ + 8, 1ull);                                                    \
    }
#else
#define HGSR_WP_DECL(acc)
#define HGSR_WP_MARK(k)
#define HGSR_WP_FLUSH()
#endif

__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}


// Where a raster call's channels come from.  gsplat's rasterize_to_pixels takes
// colors [C,N,D] and opacities [C,N]; rasterization() itself concatenates the depth
// and repeats shared colours/opacities over cameras, which the fused entry points do
// here instead: channel k < dc is colors[c*col_cstride + g*dc + k] (col_cstride 0 =
// shared over cameras), channel dc is depths[c*N + g] when depths != nullptr.
struct ChanSrc {
    const float* colors;
    int64_t col_cstride;
    int dc;
    const float* depths;
    const float* opac;
    int64_t op_cstride;
};

// Where a backward's channel gradients go (mirror of ChanSrc): v_colors has the
// layout of the colours (shared ones are summed over cameras), v_depths [C,N]
// (nullable), v_opac has the layout of the opacities.
struct ChanDst {
    float* colors;
    bool col_shared;
    int dc;
    float* depths;
    float* opac;
    bool op_shared;
};

}  // namespace hgsr
