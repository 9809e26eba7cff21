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
struct GradSlots {
    int32_t* seg;  // [C N + 1]
    int2* slot;    // [C N]
};
// bytes of launch_grad_slots' buffer (from_lists: the rectangles are found from the lists)
size_t grad_slot_bytes(int64_t CN, bool from_lists);
// radii != nullptr: rectangles from means2d / radii (isect_tiles'); else from the sorted lists
int launch_grad_slots(int C, int N, const float* means2d, const int32_t* radii, int tile_size, int tw, int th,
                      const int32_t* offsets, const int32_t* flatten_ids, int64_t n_isects, void* buf,
                      hipStream_t s, GradSlots& out);
// the flags and partial rows of a backward workspace: flags first, so a forward that only
// knows the intersection capacity can clear them (hgsr_raster{3,2}d_fwd_packed bwd_ws)
inline size_t slot_flag_bytes(int64_t n_isects, int ways) { return ((size_t)n_isects * ways + 255) & ~(size_t)255; }

// LDS ordering between the lanes of ONE wave (a wave's LDS operations complete in issue order;
// this keeps the compiler from moving LDS accesses across it)
__device__ __forceinline__ void wave_lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// The splits' fixed-order sum of gradient slots, for one wave owning the nloc (1..64)
// (camera, Gaussian) entries [ib, ib + nloc): the wave walks their contiguous slot range 64 slots
// at a time.  Each slot has WAYS partial rows of ROWF floats (the first NV used, R4 float4) and
// WAYS flag bytes; LPR consecutive lanes read one row (one coalesced request per row, 64 / LPR
// rows per load instruction, all of a chunk's loads issued before any is summed), sum the slot's
// flagged rows in way order and park the sums in the wave's LDS area; then each entry's lane adds
// its own slots' sums in slot order, the next chunk's flags already in flight.  No atomics: the
// result depends only on the inputs.
template <int NV, int R4, int ROWF, int WAYS>
__device__ __forceinline__ void reduce_slots(const float* __restrict__ rows, const uint8_t* __restrict__ flags,
                                             const int32_t* __restrict__ seg, int64_t ib, int nloc,
                                             float (*s_v)[65], float (&out)[NV]) {
    static_assert(WAYS == 1 || WAYS == 4, "slot ways");
    static_assert(R4 <= 8 && NV <= 4 * R4, "row shape");
    constexpr int LPR = R4 <= 4 ? 4 : 8;  // lanes per row
    constexpr int SPI = 64 / LPR;         // slots per load instruction
    constexpr int G = LPR;                // slot groups per 64-slot chunk
    constexpr int GB = 4;                 // slot groups whose loads are issued together
    const int lane = threadIdx.x & 63;
    const int q = lane & (LPR - 1), sl = lane / LPR;
    const bool live = lane < nloc;
    const int32_t lo_e = live ? seg[ib + lane] : 0, hi_e = live ? seg[ib + lane + 1] : 0;
    const int32_t E0 = __builtin_amdgcn_readfirstlane(lo_e), E1 = seg[ib + nloc];
    auto fl = [&](int32_t e) -> uint32_t {
        if (e >= E1) return 0u;
        return WAYS == 4 ? reinterpret_cast<const uint32_t*>(flags)[e] : (uint32_t)flags[e];
    };
#pragma unroll
    for (int k = 0; k < NV; ++k) out[k] = 0.f;
    uint32_t fc = fl(E0 + lane);  // flags of slot cs + lane
    for (int32_t cs = E0; cs < E1; cs += 64) {
        const uint32_t fcur = fc;
        fc = fl(cs + 64 + lane);  // the next chunk's, in flight while this one is summed
#pragma unroll
        for (int g0 = 0; g0 < G; g0 += GB) {
            float4 x[GB][WAYS];
#pragma unroll
            for (int gb = 0; gb < GB; ++gb) {
                const int s = (g0 + gb) * SPI + sl;
                const uint32_t f = (uint32_t)__shfl((int)fcur, s);
#pragma unroll
                for (int w = 0; w < WAYS; ++w) {
                    x[gb][w] = make_float4(0.f, 0.f, 0.f, 0.f);
                    if (q < R4 && ((f >> (8 * w)) & 0xffu))
                        x[gb][w] = reinterpret_cast<const float4*>(rows + ((int64_t)(cs + s) * WAYS + w) * ROWF)[q];
                }
            }
#pragma unroll
            for (int gb = 0; gb < GB; ++gb) {
                float4 a = x[gb][0];
#pragma unroll
                for (int w = 1; w < WAYS; ++w)
                    a = make_float4(a.x + x[gb][w].x, a.y + x[gb][w].y, a.z + x[gb][w].z, a.w + x[gb][w].w);
                const int s = (g0 + gb) * SPI + sl;
                const float av[4] = {a.x, a.y, a.z, a.w};
#pragma unroll
                for (int c = 0; c < 4; ++c)
                    if (q < R4 && 4 * q + c < NV) s_v[4 * q + c][s] = av[c];
            }
        }
        wave_lds_sync();
        const int32_t lo = max(lo_e, cs), hi = min(hi_e, cs + 64);
        for (int32_t y = lo; y < hi; ++y)
#pragma unroll
            for (int k = 0; k < NV; ++k) out[k] += s_v[k][y - cs];
        wave_lds_sync();
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

__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

template <int CTRL>
__device__ __forceinline__ float dpp(float x) {  // lane-shuffled copy of x (bound_ctrl: 0 for invalid)
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), CTRL, 0xF, 0xF, false));
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
