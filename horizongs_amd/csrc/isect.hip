// K5/K6/K7: tile intersection, depth sort and tile offsets.
//
// gsplat emits one 64-bit key per (Gaussian, covered tile) in Gaussian-major
// order, radix-sorts all of them (46 bits at 1080p: 6 HBM passes over 12 B/isect)
// and then scans the sorted keys for tile boundaries.  Here the tile is known
// at emission time, so the work is re-shaped as a bucket sort:
//
//   1. isect_count  : per-block LDS histogram of (camera, tile) bins, written as
//                     a dense [blocks][bins] matrix (no global atomics);
//   2. isect_colscan: per-bin exclusive prefix over blocks (coalesced across bins,
//                     two levels over chunks of 64 block rows);
//   3. isect_binscan: exclusive scan over bins -> isect_offsets (= gsplat
//                     isect_offset_encode) and {n_isects, largest bin};
//   4. isect_emit   : each block scatters 8-byte (depth_bits<<32 | flatten_id)
//                     keys into its pre-reserved slice of every bin (LDS cursors);
//   5. tile_sort    : one workgroup per bin sorts its keys in LDS (bitonic; bins
//                     over 2048 keys: LDS-sorted chunks + in-workgroup merge path)
//                     and writes isect_ids / flatten_ids.
// Keys inside a bin are unique ((depth, id) pairs), so ANY correct sort yields
// exactly the order of gsplat's stable radix sort: depth ascending, ties in
// Gaussian-major emission order.  Integer outputs are bit-identical.
#include <stdlib.h>

#include "common.h"

namespace hgsr {

// the histogram / cursors take <= 60 KiB of LDS per block, plus the 4,104-B BigQ: 65,544 B at most
// (isect_lds_bytes), above 64 KiB -- gfx950 allows 160 KiB per workgroup (static_assert below)
constexpr int kLdsBins = 15360;
constexpr int kSortCap = 2048;    // keys sorted entirely in LDS by one 256-lane workgroup
constexpr int kIsectBatch = 8;    // Gaussians per lane whose loads are issued together (count / emit)

__host__ __device__ inline int nbits64(int64_t v) {
    int b = 0;
    while (v > 0) { ++b; v >>= 1; }
    return b;
}

// camera of flattened index o (< 2^31 by the entry checks): 32-bit division, none for o < N
__device__ __forceinline__ int cam_of(int64_t o, int N) {
    return o < N ? 0 : (int)((uint32_t)o / (uint32_t)N);
}

// Large footprints (close street views put Gaussians hundreds of pixels wide on screen): a lane
// walking a 30 x 30-tile rectangle alone keeps its whole wave for 900 iterations while the other
// lanes' rectangles hold a few tiles.  Rectangles above kBigRect tiles are therefore queued in
// LDS (kBigQ per block; a full queue falls back to the lane) and walked by the whole block after
// the per-lane pass: key j of the block's queued keys goes to thread j mod 256, its entry found
// by binary search over the entries' key prefixes.  Count and emit do this identically, so a
// block's (bin, key count) pairs -- all the emission needs to agree on -- are unchanged.
#ifndef HGSR_BIGRECT
#define HGSR_BIGRECT 12
#endif
constexpr int kBigRect = HGSR_BIGRECT;
constexpr int kBigQ = 256;
struct BigQ {
    unsigned long long ctr;  // (entries << 32) | keys, one 64-bit LDS atomic per push
    int o[kBigQ];            // flattened (camera, Gaussian) index
    int start[kBigQ];        // first key of the entry in the block's queued-key order
    int x0y0[kBigQ];         // x0 | y0 << 16
    int wh[kBigQ];           // width | height << 16
};
// the dynamic LDS of count / emit: n_bins int counters, then the queue (16-B aligned)
__host__ __device__ inline size_t isect_lds_bytes(int n_bins) {
    return (((size_t)n_bins * 4 + 15) & ~(size_t)15) + sizeof(BigQ);
}
static_assert(((size_t)kLdsBins * 4 + 15) / 16 * 16 + sizeof(BigQ) <= 160 * 1024, "count / emit LDS over gfx950's 160 KiB");
__device__ __forceinline__ BigQ* bigq_of(int* s, int n_bins) {
    return reinterpret_cast<BigQ*>(reinterpret_cast<char*>(s) + (((size_t)n_bins * 4 + 15) & ~(size_t)15));
}
// queue a rectangle; false when the queue is full (the caller walks it itself)
__device__ __forceinline__ bool bigq_push(BigQ* q, int o, int x0, int y0, int w, int h) {
    const unsigned long long old = atomicAdd(&q->ctr, (1ull << 32) | (unsigned long long)(w * h));
    const int e = (int)(old >> 32);
    if (e >= kBigQ) return false;  // (the counter keeps counting; entries past kBigQ are ignored)
    q->o[e] = o;
    q->start[e] = (int)(old & 0xffffffffu);
    q->x0y0[e] = x0 | (y0 << 16);
    q->wh[e] = w | (h << 16);
    return true;
}
// after a barrier: call f(o, x, y) for every tile of every queued rectangle, keys spread evenly
// over the block's threads
template <typename F>
__device__ __forceinline__ void bigq_walk(const BigQ* q, F&& f) {
    const int n = min((int)(q->ctr >> 32), kBigQ);
    if (n == 0) return;
    const int total = q->start[n - 1] + (q->wh[n - 1] & 0xffff) * (q->wh[n - 1] >> 16);
    for (int j = threadIdx.x; j < total; j += blockDim.x) {
        int lo = 0, hi = n - 1;  // the last entry starting at or before j
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (q->start[mid] <= j) lo = mid;
            else hi = mid - 1;
        }
        const int t = j - q->start[lo], w = q->wh[lo] & 0xffff;
        const int dy = t / w;
        f(q->o[lo], (q->x0y0[lo] & 0xffff) + (t - dy * w), (q->x0y0[lo] >> 16) + dy);
    }
}

struct IsectGeom {
    int64_t CN;
    int n_tiles, n_bins;
    int per_block;  // Gaussians per block (stage 1/4 partition)
    int n_blocks;
    bool lds;       // dense per-block histogram path
};

static IsectGeom isect_geom(int C, int N, int tw, int th) {
    IsectGeom g;
    g.CN = (int64_t)C * N;
    g.n_tiles = tw * th;
    g.n_bins = C * g.n_tiles;
    g.lds = g.n_bins <= kLdsBins;
    // bound the [blocks][bins] matrix to ~16M entries (64 MiB)
    int64_t per = 2048;
    if (g.lds) {
        const int64_t need = (g.CN * (int64_t)g.n_bins + (16ll << 20) - 1) / (16ll << 20);
        if (need > per) per = (need + 255) / 256 * 256;
    }
    g.per_block = (int)per;
    g.n_blocks = (int)((g.CN + per - 1) / per);
    if (g.n_blocks < 1) g.n_blocks = 1;
    return g;
}

// ---------------------------------------------------------------- stage 1
__global__ __launch_bounds__(256) void isect_count_lds_kernel(
    int64_t CN, int N, int per_block, const float2* __restrict__ means2d,
    const int32_t* __restrict__ radii, int tile_size, int tw, int th, int n_tiles, int n_bins,
    int32_t* __restrict__ tiles_per_gauss, int32_t* __restrict__ blockhist) {
    extern __shared__ __attribute__((aligned(16))) int s_hist[];
    BigQ* const bq = bigq_of(s_hist, n_bins);
    for (int i = threadIdx.x; i < n_bins; i += 256) s_hist[i] = 0;
    if (threadIdx.x == 0) bq->ctr = 0;
    __syncthreads();
    const int blk = xcd_remap(blockIdx.x, gridDim.x);  // the same block <-> Gaussian range map as the emit
    const int64_t g0 = (int64_t)blk * per_block;
    const int64_t g1 = min(g0 + per_block, CN);
    // kIsectBatch Gaussians per lane per round, all loads issued before any is used
    for (int64_t ob = g0 + threadIdx.x; ob < g1; ob += 256 * kIsectBatch) {
        int32_t r[kIsectBatch];
        float2 m[kIsectBatch];
#pragma unroll
        for (int k = 0; k < kIsectBatch; ++k) {
            const int64_t o = ob + 256 * k;
            r[k] = o < g1 ? radii[o] : 0;
            m[k] = o < g1 ? means2d[o] : make_float2(0.f, 0.f);
        }
#pragma unroll
        for (int k = 0; k < kIsectBatch; ++k) {
            const int64_t o = ob + 256 * k;
            if (o >= g1) break;
            if (r[k] <= 0) {
                tiles_per_gauss[o] = 0;
                continue;
            }
            int x0, y0, x1, y1;
            tile_rect(m[k].x, m[k].y, r[k], tile_size, tw, th, x0, y0, x1, y1);
            const int area = (y1 - y0) * (x1 - x0);
            tiles_per_gauss[o] = area;
            if (area > kBigRect && bigq_push(bq, (int)o, x0, y0, x1 - x0, y1 - y0)) continue;
            const int base = cam_of(o, N) * n_tiles;
            for (int y = y0; y < y1; ++y)
                for (int x = x0; x < x1; ++x) atomicAdd(&s_hist[base + y * tw + x], 1);
        }
    }
    __syncthreads();
    bigq_walk(bq, [&](int o, int x, int y) { atomicAdd(&s_hist[cam_of(o, N) * n_tiles + y * tw + x], 1); });
    __syncthreads();
    int32_t* row = blockhist + (int64_t)blk * n_bins;
    for (int i = threadIdx.x; i < n_bins; i += 256) row[i] = s_hist[i];
}

__global__ __launch_bounds__(256) void isect_count_global_kernel(
    int64_t CN, int N, const float2* __restrict__ means2d, const int32_t* __restrict__ radii,
    int tile_size, int tw, int th, int n_tiles, int32_t* __restrict__ tiles_per_gauss,
    int32_t* __restrict__ totals) {
    const int64_t o = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (o >= CN) return;
    const int32_t r = radii[o];
    if (r <= 0) {
        tiles_per_gauss[o] = 0;
        return;
    }
    const float2 m = means2d[o];
    int x0, y0, x1, y1;
    tile_rect(m.x, m.y, r, tile_size, tw, th, x0, y0, x1, y1);
    tiles_per_gauss[o] = (y1 - y0) * (x1 - x0);
    const int base = cam_of(o, N) * n_tiles;
    for (int y = y0; y < y1; ++y)
        for (int x = x0; x < x1; ++x) atomicAdd(&totals[base + y * tw + x], 1);
}

// ---------------------------------------------------------------- stage 2
// Per-bin exclusive prefix over the block rows, in two levels so that enough
// workgroups run: (a) each (bin, chunk of kColRows rows) is scanned in place and
// its total written to chunk_pre[chunk][bin]; (b) per bin, the chunk totals are
// scanned in place into chunk offsets and the bin total.  The emit adds
// chunk_pre[row / kColRows] to its row's prefix.
constexpr int kColRows = 64;

__global__ __launch_bounds__(256) void isect_colscan_kernel(int n_blocks, int n_bins,
                                                            int32_t* __restrict__ blockhist,
                                                            int32_t* __restrict__ chunk_pre) {
    const int bin = blockIdx.x * 256 + threadIdx.x;
    if (bin >= n_bins) return;
    const int b0 = blockIdx.y * kColRows, b1 = min(b0 + kColRows, n_blocks);
    int32_t run = 0;
    int b = b0;
    for (; b + 8 <= b1; b += 8) {
        int32_t v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = blockhist[(int64_t)(b + k) * n_bins + bin];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            blockhist[(int64_t)(b + k) * n_bins + bin] = run;
            run += v[k];
        }
    }
    for (; b < b1; ++b) {
        const int32_t v = blockhist[(int64_t)b * n_bins + bin];
        blockhist[(int64_t)b * n_bins + bin] = run;
        run += v;
    }
    chunk_pre[(int64_t)blockIdx.y * n_bins + bin] = run;
}

__global__ __launch_bounds__(256) void isect_chunkscan_kernel(int n_chunks, int n_bins,
                                                              int32_t* __restrict__ chunk_pre,
                                                              int32_t* __restrict__ totals) {
    const int bin = blockIdx.x * 256 + threadIdx.x;
    if (bin >= n_bins) return;
    int32_t run = 0;
    for (int c = 0; c < n_chunks; ++c) {
        const int32_t v = chunk_pre[(int64_t)c * n_bins + bin];
        chunk_pre[(int64_t)c * n_bins + bin] = run;
        run += v;
    }
    totals[bin] = run;
}

// ---------------------------------------------------------------- stage 3
// single-workgroup exclusive scan over bins (n_bins <= C * tiles; a few 10^4)
__global__ __launch_bounds__(1024) void isect_binscan_kernel(int n_bins, const int32_t* __restrict__ totals,
                                                             int32_t* __restrict__ offsets,
                                                             int64_t* __restrict__ info) {
    // thread t owns bins [t*per, t*per + per): its sum and max, then an in-wave shuffle scan
    // and one cross-wave step through LDS (two barriers instead of a 10-level LDS scan)
    __shared__ int64_t s_wsum[16];
    __shared__ int s_wmax[16];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int per = (n_bins + 1023) / 1024;
    const int b0 = min(tid * per, n_bins), b1 = min(b0 + per, n_bins);
    int64_t local = 0;
    int mx = 0;
#pragma unroll 8
    for (int i = b0; i < b1; ++i) {
        const int v = totals[i];
        local += v;
        mx = max(mx, v);
    }
    int64_t inc = local;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int64_t o = __shfl_up(inc, d);
        if (lane >= d) inc += o;
    }
    int wm = mx;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) wm = max(wm, __shfl_xor(wm, d));
    if (lane == 63) {
        s_wsum[wave] = inc;
        s_wmax[wave] = wm;
    }
    __syncthreads();
    int64_t wpre = 0, total = 0;
    int gmax = 0;
#pragma unroll
    for (int w = 0; w < 16; ++w) {
        const int64_t ws = s_wsum[w];
        wpre += w < wave ? ws : 0;
        total += ws;
        gmax = max(gmax, s_wmax[w]);
    }
    int64_t run = wpre + inc - local;
    for (int i = b0; i < b1; ++i) {
        offsets[i] = (int32_t)run;
        run += totals[i];
    }
    if (tid == 0) {
        info[0] = total;
        info[1] = gmax;
    }
}

// ---------------------------------------------------------------- stage 4
// Deferred count (info != nullptr): the emission was sized by the host from a capacity
// (cap keys, bins up to mb_cap) before it read the count; info = {n_isects, largest bin,
// overflow}.  Every block tests the capacity itself, block 0 publishes the verdict in
// info[2] for the sort and raster kernels that follow on the stream, and an overflowed
// emission writes nothing (the host re-runs it at the exact size).
__device__ __forceinline__ bool emit_overflow(int64_t* info, int64_t cap, int64_t mb_cap) {
    if (!info) return false;
    const bool ovf = info[0] > cap || info[1] > mb_cap;
    if (blockIdx.x == 0 && threadIdx.x == 0) info[2] = ovf ? 1 : 0;
    return ovf;
}

__global__ __launch_bounds__(256) void isect_emit_lds_kernel(
    int64_t CN, int N, int per_block, const float2* __restrict__ means2d,
    const int32_t* __restrict__ radii, const float* __restrict__ depths, int tile_size, int tw,
    int th, int n_tiles, int n_bins, const int32_t* __restrict__ offsets,
    const int32_t* __restrict__ blockhist, const int32_t* __restrict__ chunk_pre, uint64_t* __restrict__ keys,
    int phases, int64_t* __restrict__ info, int64_t cap, int64_t mb_cap) {
    extern __shared__ __attribute__((aligned(16))) int s_cur[];
    if (emit_overflow(info, cap, mb_cap)) return;
    BigQ* const bq = bigq_of(s_cur, n_bins);
    if (threadIdx.x == 0) bq->ctr = 0;
    // Logical block = XCD-contiguous remap of the dispatch index: the blocks resident on one
    // XCD hold consecutive slices of every bin, so their scattered 8-B key writes to a bin
    // land in adjacent addresses of the same L2 and leave it as whole lines.
    const int blk = xcd_remap(blockIdx.x, gridDim.x);
    const int32_t* row = blockhist + (int64_t)blk * n_bins;
    const int32_t* cpre = chunk_pre + (int64_t)(blk / kColRows) * n_bins;
    for (int i = threadIdx.x; i < n_bins; i += 256) s_cur[i] = offsets[i] + cpre[i] + row[i];
    __syncthreads();
    const int64_t g0 = (int64_t)blk * per_block;
    const int64_t g1 = min(g0 + per_block, CN);
    for (int64_t ob = g0 + threadIdx.x; ob < g1; ob += 256 * kIsectBatch) {
        int32_t r[kIsectBatch];
        float2 m[kIsectBatch];
        float d[kIsectBatch];
#pragma unroll
        for (int k = 0; k < kIsectBatch; ++k) {
            const int64_t o = ob + 256 * k;
            r[k] = o < g1 ? radii[o] : 0;
            m[k] = o < g1 ? means2d[o] : make_float2(0.f, 0.f);
            d[k] = o < g1 ? depths[o] : 0.f;
        }
        // Phases over bands of tile rows: every block of an XCD emits into the same band at
        // the same time, so the partially written key lines the XCD's L2 must hold until
        // their 16 keys (from 16 neighbouring blocks) arrive are 1 / phases of all bins --
        // they merge in L2 instead of leaving as partial-line writes.
        // rectangles once (an empty one for culled / out-of-range Gaussians), clipped per phase
        int rx0[kIsectBatch], ry0[kIsectBatch], rx1[kIsectBatch], ry1[kIsectBatch];
#pragma unroll
        for (int k = 0; k < kIsectBatch; ++k) {
            const int64_t o = ob + 256 * k;
            if (o < g1 && r[k] > 0) {
                tile_rect(m[k].x, m[k].y, r[k], tile_size, tw, th, rx0[k], ry0[k], rx1[k], ry1[k]);
                const int w = rx1[k] - rx0[k], h = ry1[k] - ry0[k];
                // a large rectangle goes to the block's queue (walked by every thread below)
                if (w * h > kBigRect && bigq_push(bq, (int)o, rx0[k], ry0[k], w, h)) rx0[k] = rx1[k] = 0;
            } else {
                rx0[k] = ry0[k] = rx1[k] = ry1[k] = 0;
            }
        }
        for (int ph = 0; ph < phases; ++ph) {
            const int ylo = (int)((int64_t)ph * th / phases), yhi = (int)((int64_t)(ph + 1) * th / phases);
#pragma unroll
            for (int k = 0; k < kIsectBatch; ++k) {
                const int y0 = max(ry0[k], ylo), y1 = min(ry1[k], yhi);
                if (y0 >= y1) continue;
                const int64_t o = ob + 256 * k;
                const uint64_t key = ((uint64_t)__float_as_uint(d[k]) << 32) | (uint32_t)o;
                const int base = cam_of(o, N) * n_tiles;
                for (int y = y0; y < y1; ++y)
                    for (int x = rx0[k]; x < rx1[k]; ++x) {
                        const int pos = atomicAdd(&s_cur[base + y * tw + x], 1);
                        keys[pos] = key;
                    }
            }
        }
    }
    __syncthreads();
    bigq_walk(bq, [&](int o, int x, int y) {
        const uint64_t key = ((uint64_t)__float_as_uint(depths[o]) << 32) | (uint32_t)o;
        keys[atomicAdd(&s_cur[cam_of(o, N) * n_tiles + y * tw + x], 1)] = key;
    });
}

__global__ __launch_bounds__(256) void isect_emit_global_kernel(
    int64_t CN, int N, const float2* __restrict__ means2d, const int32_t* __restrict__ radii,
    const float* __restrict__ depths, int tile_size, int tw, int th, int n_tiles,
    int32_t* __restrict__ cursor, uint64_t* __restrict__ keys, int64_t* __restrict__ info, int64_t cap,
    int64_t mb_cap) {
    if (emit_overflow(info, cap, mb_cap)) return;
    const int64_t o = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (o >= CN) return;
    const int32_t r = radii[o];
    if (r <= 0) return;
    const float2 m = means2d[o];
    int x0, y0, x1, y1;
    tile_rect(m.x, m.y, r, tile_size, tw, th, x0, y0, x1, y1);
    const uint64_t key = ((uint64_t)__float_as_uint(depths[o]) << 32) | (uint32_t)o;
    const int base = cam_of(o, N) * n_tiles;
    for (int y = y0; y < y1; ++y)
        for (int x = x0; x < x1; ++x) keys[atomicAdd(&cursor[base + y * tw + x], 1)] = key;
}

// ---------------------------------------------------------------- stage 5
// Bitonic sort of 256*E keys held E per thread (thread t owns elements t*E..t*E+E-1),
// in the "flip" form where every comparator is ascending: merge level K opens with
// the mirror stage (i <-> i ^ (K-1)) and continues with i <-> i ^ J for J = K/4..1.
// Padding keys (~0) start in the suffix and a comparator never moves one down, so
// a wave whose elements are all padding skips every stage except the cross-wave
// LDS exchanges it must still feed.  Partners inside a thread are registers; inside
// a wave they arrive by DPP / ds_swizzle / v_permlane32_swap (no LDS memory); only
// partners in another wave go through LDS (lane-contiguous, conflict-free layout).
// The network is unrolled at compile time.
// (mov_dpp, not update_dpp with an old value: no v_mov initialising the destination first)
template <int M>
__device__ __forceinline__ uint32_t lane_xor32(uint32_t x) {
    if constexpr (M == 1) return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0xB1, 0xF, 0xF, true);  // quad_perm [1,0,3,2]
    else if constexpr (M == 2) return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x4E, 0xF, 0xF, true);  // quad_perm [2,3,0,1]
    else if constexpr (M == 3) return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x1B, 0xF, 0xF, true);  // quad_perm [3,2,1,0]
    else if constexpr (M == 4) return (uint32_t)__builtin_amdgcn_ds_swizzle((int)x, 0x1F | (4 << 10));
    else if constexpr (M == 7) return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x141, 0xF, 0xF, true);  // row_half_mirror
    else if constexpr (M == 8) return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x128, 0xF, 0xF, true);  // row_ror:8
    else if constexpr (M == 15) return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x140, 0xF, 0xF, true);  // row_mirror
    else if constexpr (M == 16) return (uint32_t)__builtin_amdgcn_ds_swizzle((int)x, 0x1F | (16 << 10));
    else if constexpr (M == 31) return (uint32_t)__builtin_amdgcn_ds_swizzle((int)x, 0x1F | (31 << 10));
    else if constexpr (M == 32) {
        const auto r = __builtin_amdgcn_permlane32_swap(x, x, false, false);
        return (threadIdx.x & 32) ? r[0] : r[1];
    } else {
        static_assert(M == 63, "in-wave partner mask");
        return lane_xor32<31>(lane_xor32<32>(x));
    }
}

template <int M>
__device__ __forceinline__ uint64_t lane_xor64(uint64_t x) {
    const uint32_t lo = lane_xor32<M>((uint32_t)x), hi = lane_xor32<M>((uint32_t)(x >> 32));
    return ((uint64_t)hi << 32) | lo;
}

template <int M, typename K>
__device__ __forceinline__ K lane_xor(K x) {
    if constexpr (sizeof(K) == 8) return lane_xor64<M>(x);
    else return lane_xor32<M>(x);
}

// The network is written for 64-bit (depth, id) keys and for 32-bit (truncated depth, local
// index) keys (K); unique keys in both cases.
// cross-thread stage: partner thread t ^ M, partner slot r (FLIP: E-1-r); the lower
// thread of the pair (t & LOWBIT == 0) keeps the minimum.
template <typename K, int E, int M, int LOWBIT, bool FLIP>
__device__ __forceinline__ void thread_stage(K (&v)[E], K* __restrict__ s, bool active) {
    const int t = threadIdx.x;
    const bool keep_min = (t & LOWBIT) == 0;
    K p[E];
    if constexpr (M >= 64) {
        lds_barrier();  // earlier reads of s are done
#pragma unroll
        for (int r = 0; r < E; ++r) s[r * 256 + t] = v[r];
        lds_barrier();
        if (!active) return;
#pragma unroll
        for (int r = 0; r < E; ++r) p[r] = s[(FLIP ? E - 1 - r : r) * 256 + (t ^ M)];
    } else {
        if (!active) return;
#pragma unroll
        for (int r = 0; r < E; ++r) p[r] = lane_xor<M>(v[FLIP ? E - 1 - r : r]);
    }
#pragma unroll
    for (int r = 0; r < E; ++r) v[r] = ((v[r] < p[r]) == keep_min) ? v[r] : p[r];
}

// in-thread stage over aligned groups of G slots: FLIP pairs r <-> r ^ (G-1), else r <-> r + G/2
template <typename K, int E, int G, bool FLIP>
__device__ __forceinline__ void reg_stage(K (&v)[E], bool active) {
    if (!active) return;
#pragma unroll
    for (int r = 0; r < E; ++r) {
        if (r & (G / 2)) continue;
        const int q = FLIP ? (r ^ (G - 1)) : (r + G / 2);
        const K a = v[r], b = v[q];
        const bool keep = a < b;
        v[r] = keep ? a : b;
        v[q] = keep ? b : a;
    }
}

template <typename K, int E, int L, int J>
__device__ __forceinline__ void half_stages(K (&v)[E], K* s, bool active) {
    if constexpr (J >= 1) {
        if constexpr (J >= E) thread_stage<K, E, J / E, J / E, false>(v, s, active);
        else reg_stage<K, E, 2 * J, false>(v, active);
        half_stages<K, E, L, J / 2>(v, s, active);
    }
}

template <typename K, int E, int L>
__device__ __forceinline__ void merge_levels(K (&v)[E], K* s, bool active) {
    if constexpr (L <= 256 * E) {
        if constexpr (L <= E) reg_stage<K, E, L, true>(v, active);
        else thread_stage<K, E, L / E - 1, L / (2 * E), true>(v, s, active);
        half_stages<K, E, L, L / 4>(v, s, active);
        merge_levels<K, E, 2 * L>(v, s, active);
    }
}

template <typename K, int E>
__device__ __forceinline__ void bitonic_regs(K (&v)[E], K* __restrict__ s, int n) {
    // a wave holds elements [wave*64*E, (wave+1)*64*E)
    const bool active = (int)(threadIdx.x >> 6) * 64 * E < n;
    merge_levels<K, E, 2>(v, s, active);
    lds_barrier();
}

// back to lane-contiguous order through LDS so the global stores coalesce; the
// row pitch of 260 keys keeps the transposed reads within two-way bank sharing
constexpr int kSortPitch = 260;
template <typename K, int E>
__device__ __forceinline__ void untranspose(K (&v)[E], K* s) {
    const int t = threadIdx.x;
#pragma unroll
    for (int r = 0; r < E; ++r) s[r * kSortPitch + t] = v[r];
    lds_barrier();
#pragma unroll
    for (int r = 0; r < E; ++r) {
        const int i = r * 256 + t;
        v[r] = s[(i % E) * kSortPitch + i / E];
    }
    lds_barrier();
}

// inverse of untranspose: lane-contiguous element i = r*256 + t -> thread i/E, slot i%E
template <typename K, int E>
__device__ __forceinline__ void to_blocked(K (&v)[E], K* s) {
    const int t = threadIdx.x;
#pragma unroll
    for (int r = 0; r < E; ++r) {
        const int i = r * 256 + t;
        s[(i % E) * kSortPitch + i / E] = v[r];
    }
    lds_barrier();
#pragma unroll
    for (int r = 0; r < E; ++r) v[r] = s[r * kSortPitch + t];
    lds_barrier();
}

// load n <= 256*E keys (any order: the input is unsorted) lane-contiguously,
// padding with ~0, and sort them; thread t ends holding sorted elements t*E..t*E+E-1
template <int E>
__device__ __forceinline__ void sort_chunk(const uint64_t* src, int n, uint64_t* s, uint64_t (&v)[E]) {
    const int t = threadIdx.x;
#pragma unroll
    for (int r = 0; r < E; ++r) {
        const int i = r * 256 + t;
        v[r] = i < n ? src[i] : ~0ull;
    }
    // the network wants the padding in the suffix of the blocked order t*E + r
    to_blocked<uint64_t, E>(v, s);
    bitonic_regs<uint64_t, E>(v, s, n);
}

template <int E>
__device__ __forceinline__ void sort_and_emit(const uint64_t* keys, int n, uint64_t* s, int64_t hi,
                                              int64_t* __restrict__ isect_ids, int32_t* __restrict__ flatten_ids) {
    uint64_t v[E];
    sort_chunk<E>(keys, n, s, v);
    untranspose<uint64_t, E>(v, s);
    const int t = threadIdx.x;
#pragma unroll
    for (int r = 0; r < E; ++r) {
        const int i = r * 256 + t;
        if (i < n) {
            isect_ids[i] = hi | (int64_t)(v[r] >> 32);
            flatten_ids[i] = (int32_t)(uint32_t)v[r];
        }
    }
}

// Bins of 257..2048 keys: sort 32-bit keys (quantised depth : 20 bits | local index : 11
// bits, see depth_q) -- half the compare / select work of the 64-bit network -- gather the
// full keys in that order and repair the runs of equal quantised depth with odd-even
// transposition passes (the keys inside such a run are in emission order).  Two passes fixed
// every bin of the c2 scene already with a fixed depth >> 10 (scripts/sim_sort_fixup.py); a bin
// still unsorted after them (many equal depths) is sorted again by the 64-bit network, so the
// result is always the exact order.
constexpr int kFixPasses = 2;

// pair (thread t's last, thread t+1's first): t keeps the smaller, t+1 the larger
template <int E>
__device__ __forceinline__ void oe_boundary(uint64_t (&w)[E], uint64_t* sb) {
    const int t = threadIdx.x;
    sb[t] = w[E - 1];
    sb[256 + t] = w[0];
    lds_barrier();
    const uint64_t nf = t < 255 ? sb[256 + t + 1] : ~0ull;
    const uint64_t pl = t > 0 ? sb[t - 1] : 0ull;
    lds_barrier();
    w[E - 1] = w[E - 1] < nf ? w[E - 1] : nf;
    w[0] = w[0] > pl ? w[0] : pl;
}

// the fix-up passes over the gathered full keys (thread t holds sorted slots t*E..t*E+E-1);
// true when every thread's keys are then in exact order (one workgroup-wide vote)
template <int E>
__device__ __forceinline__ bool fix_runs(uint64_t (&w)[E], uint64_t* sb) {
    static_assert(E % 2 == 0, "blocked pairs");
    const int t = threadIdx.x;
#pragma unroll
    for (int pass = 0; pass < kFixPasses; ++pass) {
#pragma unroll
        for (int r = 0; r < E; r += 2) {
            const uint64_t a = w[r], b = w[r + 1];
            w[r] = a < b ? a : b;
            w[r + 1] = a < b ? b : a;
        }
#pragma unroll
        for (int r = 1; r + 1 < E; r += 2) {
            const uint64_t a = w[r], b = w[r + 1];
            w[r] = a < b ? a : b;
            w[r + 1] = a < b ? b : a;
        }
        oe_boundary<E>(w, sb);
    }
    bool ok = true;
#pragma unroll
    for (int r = 0; r + 1 < E; ++r) ok &= w[r] <= w[r + 1];
    sb[256 + t] = w[0];
    lds_barrier();
    ok &= t == 255 || w[E - 1] <= sb[256 + t + 1];
    return __syncthreads_and(ok);
}

template <int E>
__device__ __forceinline__ void emit_sorted(uint64_t (&w)[E], int n, uint64_t* smem, int64_t hi,
                                            int64_t* __restrict__ isect_ids, int32_t* __restrict__ flatten_ids) {
    const int t = threadIdx.x;
    untranspose<uint64_t, E>(w, smem);
#pragma unroll
    for (int r = 0; r < E; ++r) {
        const int i = r * 256 + t;
        if (i < n) {
            if (isect_ids) isect_ids[i] = hi | (int64_t)(w[r] >> 32);
            flatten_ids[i] = (int32_t)(uint32_t)w[r];
        }
    }
}

// Per-bin depth quantiser of the 32-bit keys: (depth bits - the bin's minimum) >> shift, the
// smallest shift that fits 20 bits, so two keys of a bin tie only where their depths agree to
// within 2^shift ulps (the fixed depth bits >> 10 tied long runs in bins whose depths span a
// narrow range).  20 bits keep every real key below the ~0 padding.
struct DepthQ {
    uint32_t lo;
    int shift;
};
template <int IB = 11>
__device__ __forceinline__ DepthQ depth_q(uint32_t mn, uint32_t mx) {
    __shared__ uint32_t s_red[8];
    // wave min / max over the network's in-wave lane exchanges (DPP / swizzle / permlane)
    mn = min(mn, lane_xor32<1>(mn)), mx = max(mx, lane_xor32<1>(mx));
    mn = min(mn, lane_xor32<2>(mn)), mx = max(mx, lane_xor32<2>(mx));
    mn = min(mn, lane_xor32<4>(mn)), mx = max(mx, lane_xor32<4>(mx));
    mn = min(mn, lane_xor32<8>(mn)), mx = max(mx, lane_xor32<8>(mx));
    mn = min(mn, lane_xor32<16>(mn)), mx = max(mx, lane_xor32<16>(mx));
    mn = min(mn, lane_xor32<32>(mn)), mx = max(mx, lane_xor32<32>(mx));
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        s_red[w] = mn;
        s_red[4 + w] = mx;
    }
    lds_barrier();
    mn = min(min(s_red[0], s_red[1]), min(s_red[2], s_red[3]));
    mx = max(max(s_red[4], s_red[5]), max(s_red[6], s_red[7]));
    const uint32_t span = mx - mn;
    const int bits = span ? 32 - __clz((int)span) : 0;
    constexpr int DB = 31 - IB;  // depth bits: every real key stays below the ~0 padding
    return {mn, bits > DB ? bits - DB : 0};
}

template <int IB = 11>
__device__ __forceinline__ uint32_t key32(uint64_t k, int i, DepthQ q) {
    return ((((uint32_t)(k >> 32) - q.lo) >> q.shift) << IB) | (uint32_t)i;
}

template <int E>
__device__ __forceinline__ void sort32_and_emit(const uint64_t* keys, int n, uint64_t* smem, int64_t hi,
                                                int64_t* __restrict__ isect_ids, int32_t* __restrict__ flatten_ids) {
    constexpr int NF = 256 * E > 2048 ? 256 * E : 2048;    // full keys held (2048 up to E = 8)
    constexpr int IB = NF > 2048 ? 12 : 11;                 // local index bits of the 32-bit key
    uint64_t* full = smem;                                  // [NF] full keys by local index
    uint32_t* s32 = reinterpret_cast<uint32_t*>(smem + NF);  // 32-bit network scratch
    const int t = threadIdx.x;
    uint64_t kk[E];
    uint32_t mn = ~0u, mx = 0u;
#pragma unroll
    for (int r = 0; r < E; ++r) {
        const int i = r * 256 + t;
        if (i < n) {
            kk[r] = keys[i];
            full[i] = kk[r];
            mn = min(mn, (uint32_t)(kk[r] >> 32));
            mx = max(mx, (uint32_t)(kk[r] >> 32));
        }
    }
    const DepthQ q = depth_q<IB>(mn, mx);
    uint32_t v[E];
#pragma unroll
    for (int r = 0; r < E; ++r) {
        const int i = r * 256 + t;
        v[r] = i < n ? key32<IB>(kk[r], i, q) : ~0u;
    }
    to_blocked<uint32_t, E>(v, s32);  // its barriers also publish full[]
    bitonic_regs<uint32_t, E>(v, s32, n);
    uint64_t w[E];
#pragma unroll
    for (int r = 0; r < E; ++r) w[r] = v[r] == ~0u ? ~0ull : full[v[r] & ((1u << IB) - 1u)];
    // boundary exchange in the network scratch (its last reads were before bitonic_regs' barrier)
    if (!fix_runs<E>(w, reinterpret_cast<uint64_t*>(s32)))
        bitonic_regs<uint64_t, E>(w, smem, n);  // rare: many equal depths
    emit_sorted<E>(w, n, smem, hi, isect_ids, flatten_ids);
}

// Bins of 1025..1280 keys (90 % of the c2 bins hold 1025-1254): a 1024-key network (4 keys
// per thread) and a 256 * EB-key one (EB per thread) instead of one padded 2048-key
// network (8 per thread), then a merge by co-ranking -- each key's output slot is its index in
// its own run plus its lower bound in the other run (binary search in LDS; the 32-bit keys are
// unique) -- and the same full-key gather and fix-up passes, 6 slots per thread.  The 32-bit
// order is the E = 8 path's exactly; a bin the fix-up leaves unsorted takes the E = 8 path.
// (EB = 2 for 1281..1536 keys: no gain over the E = 8 path on the anchor scene's bins, 0.083 ms
// either way once the quantised keys stopped the fallbacks; not dispatched.)
template <int EB>
__device__ __forceinline__ void sort32_split_and_emit(const uint64_t* keys, int n, uint64_t* smem, int64_t hi,
                                                      int64_t* __restrict__ isect_ids,
                                                      int32_t* __restrict__ flatten_ids) {
    constexpr int E = 6, NB = 256 * EB;
    uint64_t* full = smem;
    uint32_t* s32 = reinterpret_cast<uint32_t*>(smem + 2048);
    const int t = threadIdx.x;
    const int nb = n - 1024;  // 1..NB
    uint64_t ka[4], kb[EB];
    uint32_t mn = ~0u, mx = 0u;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int i = r * 256 + t;
        ka[r] = keys[i];
        full[i] = ka[r];
        mn = min(mn, (uint32_t)(ka[r] >> 32));
        mx = max(mx, (uint32_t)(ka[r] >> 32));
    }
#pragma unroll
    for (int r = 0; r < EB; ++r) {
        const int j = r * 256 + t;
        if (j < nb) {
            kb[r] = keys[1024 + j];
            full[1024 + j] = kb[r];
            mn = min(mn, (uint32_t)(kb[r] >> 32));
            mx = max(mx, (uint32_t)(kb[r] >> 32));
        }
    }
    const DepthQ q = depth_q(mn, mx);
    uint32_t a[4], b[EB];
#pragma unroll
    for (int r = 0; r < 4; ++r) a[r] = key32(ka[r], r * 256 + t, q);
#pragma unroll
    for (int r = 0; r < EB; ++r) b[r] = r * 256 + t < nb ? key32(kb[r], 1024 + r * 256 + t, q) : ~0u;
    to_blocked<uint32_t, 4>(a, s32);
    bitonic_regs<uint32_t, 4>(a, s32, 1024);
    if constexpr (EB > 1) to_blocked<uint32_t, EB>(b, s32);  // (E = 1: blocked order is lane order)
    bitonic_regs<uint32_t, EB>(b, s32, nb);
    uint32_t* sA = s32;         // run A, sorted [1024]
    uint32_t* sB = s32 + 1024;  // run B, sorted [NB] (~0 padded)
#pragma unroll
    for (int r = 0; r < 4; ++r) sA[4 * t + r] = a[r];
#pragma unroll
    for (int r = 0; r < EB; ++r) sB[EB * t + r] = b[r];
    lds_barrier();
    int pa[4], pb[EB];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        int lo = 0;
#pragma unroll
        for (int step = NB / 2; step >= 1; step >>= 1) lo += sB[lo + step - 1] < a[r] ? step : 0;
        lo += sB[lo] < a[r];  // lo reaches NB only when every B key is smaller
        pa[r] = 4 * t + r + lo;
    }
#pragma unroll
    for (int r = 0; r < EB; ++r) {
        int lo = 0;
#pragma unroll
        for (int step = 512; step >= 1; step >>= 1) lo += sA[lo + step - 1] < b[r] ? step : 0;
        lo += sA[lo] < b[r];
        pb[r] = EB * t + r + lo;
    }
    lds_barrier();  // every search is done before the merged order overwrites the runs
    uint32_t* sM = s32;  // merged [n]
#pragma unroll
    for (int r = 0; r < 4; ++r) sM[pa[r]] = a[r];
#pragma unroll
    for (int r = 0; r < EB; ++r)
        if (EB * t + r < nb) sM[pb[r]] = b[r];
    lds_barrier();
    uint64_t w[E];
#pragma unroll
    for (int r = 0; r < E; ++r) {
        const int i = t * E + r;
        w[r] = i < n ? full[sM[i] & 2047u] : ~0ull;
    }
    lds_barrier();  // the fix-up's boundary exchange reuses the merged array's space
    if (!fix_runs<E>(w, reinterpret_cast<uint64_t*>(s32))) {
        sort32_and_emit<8>(keys, n, smem, hi, isect_ids, flatten_ids);  // rare: many equal depths
        return;
    }
    emit_sorted<E>(w, n, smem, hi, isect_ids, flatten_ids);
}

// merge sorted runs A=[0,la), B=[la,la+lb) of src into dst (unique keys)
__device__ void merge_runs(const uint64_t* __restrict__ src, uint64_t* __restrict__ dst, int la, int lb) {
    constexpr int E = 8;
    const uint64_t* A = src;
    const uint64_t* B = src + la;
    const int total = la + lb;
    for (int base = threadIdx.x * E; base < total; base += 256 * E) {
        int lo = max(0, base - lb), hi = min(base, la);
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (A[mid] < B[base - mid - 1]) lo = mid + 1;
            else hi = mid;
        }
        int i = lo, j = base - lo;
        const int cnt = min(E, total - base);
        for (int e = 0; e < cnt; ++e) {
            const bool takeA = j >= lb || (i < la && A[i] < B[j]);
            dst[base + e] = takeA ? A[i++] : B[j++];
        }
    }
}

// BIG = false: the bins of <= kSortCap keys (24.6 KB of LDS); BIG = true: the larger ones,
// launched only when some bin exceeds kSortCap (anchor scenes: 1M anchors put most bins just
// above 2048), with the LDS for a 4096-key sort (49 KB: 4096 full keys + the 32-bit network's
// scratch) so those bins sort in LDS instead of by chunk merges through global memory.
template <bool BIG>
__global__ __launch_bounds__(256) void tile_sort_kernel(int n_bins, int n_tiles, int tile_bits,
                                                        const int32_t* __restrict__ offsets,
                                                        int64_t n_isects, uint64_t* __restrict__ keys,
                                                        uint64_t* __restrict__ tmp,
                                                        int64_t* __restrict__ isect_ids,
                                                        int32_t* __restrict__ flatten_ids,
                                                        const int64_t* __restrict__ info) {
    // 64-bit network scratch, or (32-bit path) the full keys + the 32-bit network's scratch
    __shared__ uint64_t s_keys[BIG ? 4096 + 8 * kSortPitch : 2048 + 4 * kSortPitch];
    if (info && info[2]) return;  // deferred count over capacity: nothing was emitted
    const int bin = blockIdx.x;
    const int64_t start = offsets[bin];
    const int64_t end = bin + 1 < n_bins ? (int64_t)offsets[bin + 1] : (info ? info[0] : n_isects);
    const int n = (int)(end - start);
    if (n <= 0 || (n <= kSortCap) == BIG) return;
    const int cam = bin / n_tiles, tile = bin - cam * n_tiles;
    const int64_t hi = ((int64_t)cam << (32 + tile_bits)) | ((int64_t)tile << 32);
    if constexpr (!BIG) {
        if (n <= 256) sort_and_emit<1>(keys + start, n, s_keys, hi, isect_ids + start, flatten_ids + start);
        else if (n <= 512) sort32_and_emit<2>(keys + start, n, s_keys, hi, isect_ids + start, flatten_ids + start);
        else if (n <= 1024) sort32_and_emit<4>(keys + start, n, s_keys, hi, isect_ids + start, flatten_ids + start);
        else if (n <= 1280) sort32_split_and_emit<1>(keys + start, n, s_keys, hi, isect_ids + start, flatten_ids + start);
        else sort32_and_emit<8>(keys + start, n, s_keys, hi, isect_ids + start, flatten_ids + start);
        return;
    } else if (n <= 2 * kSortCap) {
        sort32_and_emit<16>(keys + start, n, s_keys, hi, isect_ids + start, flatten_ids + start);
        return;
    }
    // larger bins: LDS-sorted chunks, then merge passes ping-ponging keys <-> tmp
    uint64_t* a = keys + start;
    uint64_t* b = tmp + start;
    for (int c0 = 0; c0 < n; c0 += kSortCap) {
        const int cn = min(kSortCap, n - c0);
        uint64_t v[8];
        sort_chunk<8>(a + c0, cn, s_keys, v);
        untranspose<uint64_t, 8>(v, s_keys);
#pragma unroll
        for (int r = 0; r < 8; ++r) {
            const int i = r * 256 + threadIdx.x;
            if (i < cn) a[c0 + i] = v[r];
        }
    }
    __syncthreads();
    for (int L = kSortCap; L < n; L <<= 1) {
        for (int p = 0; p < n; p += 2 * L) {
            const int la = min(L, n - p);
            const int lb = max(0, min(L, n - p - la));
            merge_runs(a + p, b + p, la, lb);
        }
        __syncthreads();
        uint64_t* t = a;
        a = b;
        b = t;
    }
    for (int i = threadIdx.x; i < n; i += 256) {
        const uint64_t k = a[i];
        isect_ids[start + i] = hi | (int64_t)(k >> 32);
        flatten_ids[start + i] = (int32_t)(uint32_t)k;
    }
}

// ---------------------------------------------------------------- gsplat-order emission / offsets
__global__ __launch_bounds__(256) void isect_emit_unsorted_kernel(
    int64_t CN, int N, const float2* __restrict__ means2d, const int32_t* __restrict__ radii,
    const float* __restrict__ depths, int tile_size, int tw, int th, int tile_bits,
    const int64_t* __restrict__ cum, int64_t* __restrict__ isect_ids, int32_t* __restrict__ flatten_ids) {
    const int64_t o = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (o >= CN) return;
    const int32_t r = radii[o];
    if (r <= 0) return;
    const float2 m = means2d[o];
    int x0, y0, x1, y1;
    tile_rect(m.x, m.y, r, tile_size, tw, th, x0, y0, x1, y1);
    int64_t cur = o == 0 ? 0 : cum[o - 1];
    const int64_t cid = o / N;
    const int64_t denc = (int64_t)(int32_t)__float_as_int(depths[o]) & 0xFFFFFFFFll;
    for (int y = y0; y < y1; ++y)
        for (int x = x0; x < x1; ++x) {
            const int64_t tile_id = (int64_t)y * tw + x;
            isect_ids[cur] = (cid << (32 + tile_bits)) | (tile_id << 32) | denc;
            flatten_ids[cur] = (int32_t)o;
            ++cur;
        }
}

__global__ __launch_bounds__(256) void offset_encode_kernel(int64_t n_isects, const int64_t* __restrict__ ids,
                                                            int C, int n_tiles, int tile_bits,
                                                            int32_t* __restrict__ offsets) {
    const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (idx >= n_isects) return;
    const int64_t mask = (1ll << tile_bits) - 1;
    const int64_t cur = ids[idx] >> 32;
    const int64_t id_cur = (cur >> tile_bits) * n_tiles + (cur & mask);
    if (idx == 0)
        for (int64_t i = 0; i < id_cur + 1; ++i) offsets[i] = 0;
    if (idx == n_isects - 1)
        for (int64_t i = id_cur + 1; i < (int64_t)C * n_tiles; ++i) offsets[i] = (int32_t)n_isects;
    if (idx > 0) {
        const int64_t prev = ids[idx - 1] >> 32;
        const int64_t id_prev = (prev >> tile_bits) * n_tiles + (prev & mask);
        if (id_prev == id_cur) return;
        for (int64_t i = id_prev + 1; i < id_cur + 1; ++i) offsets[i] = (int32_t)idx;
    }
}

__global__ void copy_i32_kernel(int n, const int32_t* __restrict__ a, int32_t* __restrict__ b) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i < n) b[i] = a[i];
}

// ---------------------------------------------------------------- gradient slots
// The raster backwards give every (tile-list entry, wave) partial sum its own slot row instead
// of adding it into a per-Gaussian row with float atomics (whose order -- hence whose last bits
// -- changes from launch to launch); the splits then sum each Gaussian's slots in one fixed
// order, so two launches give bit-identical gradients.  Slot e of flattened (camera, Gaussian)
// o's tile (x, y) is seg[o] + (y - y0) w + (x - x0): the tile's rank in o's rectangle in
// gsplat's emission order (row-major over the rectangle, isect_tiles), seg = the exclusive
// prefix of the rectangles' areas (tiles_per_gauss).  A Gaussian's slots are contiguous and
// slot[o] = {seg[o] - y0 w - x0, w} gives e = slot.x + y slot.y + x in one multiply-add.
// The rectangles come from means2d / radii (the same tile_rect the emission ran), or -- for
// rasterize_to_pixels called on bare lists -- from each Gaussian's first and last tile in the
// lists (a rectangle's corners are its smallest and largest row-major tile index).
constexpr int kSlotPer = 2048;  // (camera, Gaussian) entries per slot_write block: 256 threads x 8 rows

struct RectFromTiles {
    const int32_t* tmin;  // per-camera row-major tile index, INT32_MAX when o has no entry
    const int32_t* tmax;
    int tw;
    __device__ __forceinline__ int operator()(int64_t o, int& x0, int& y0, int& w) const {
        const int32_t a = tmin[o], b = tmax[o];
        if (a > b) {
            x0 = y0 = w = 0;
            return 0;
        }
        y0 = a / tw;
        x0 = a - y0 * tw;
        const int y1 = b / tw + 1, x1 = b - (y1 - 1) * tw + 1;
        w = x1 - x0;
        return (y1 - y0) * w;
    }
};

// stage A: the area total of each row of kSlotRow entries
template <typename R>
__global__ __launch_bounds__(256) void slot_sum_kernel(int64_t CN, R rect, int32_t* __restrict__ bsum) {
    const int64_t o = (int64_t)blockIdx.x * kSlotRow + threadIdx.x;
    int s = 0;
    {
        int x0, y0, w;
        if (o < CN) s = rect(o, x0, y0, w);
    }
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) s += __shfl_xor(s, d);
    __shared__ int ws[4];
    if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) bsum[blockIdx.x] = ws[0] + ws[1] + ws[2] + ws[3];
}

// stage B: one workgroup, exclusive scan of the row totals in place; seg[CN] = the total; the
// piece count cleared for stage C (nullable)
__global__ __launch_bounds__(1024) void slot_scan_kernel(int nb, int32_t* __restrict__ bsum,
                                                         int32_t* __restrict__ seg_end, int32_t* __restrict__ npieces) {
    __shared__ int32_t s_w[16];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int per = (nb + 1023) / 1024;
    const int b0 = min(tid * per, nb), b1 = min(b0 + per, nb);
    // up to 8 rows per thread (8,192 rows = 2M entries) held in registers: their loads issued
    // together, one memory round trip instead of one per row
    constexpr int kR = 8;
    int32_t r[kR];
    int32_t local = 0;
    if (per <= kR) {
#pragma unroll
        for (int k = 0; k < kR; ++k) r[k] = b0 + k < b1 ? bsum[b0 + k] : 0;
#pragma unroll
        for (int k = 0; k < kR; ++k) local += r[k];
    } else {
        for (int i = b0; i < b1; ++i) local += bsum[i];
    }
    int32_t inc = local;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int32_t o = __shfl_up(inc, d);
        if (lane >= d) inc += o;
    }
    if (lane == 63) s_w[wave] = inc;
    __syncthreads();
    int32_t pre = 0, total = 0;
#pragma unroll
    for (int w = 0; w < 16; ++w) {
        pre += w < wave ? s_w[w] : 0;
        total += s_w[w];
    }
    int32_t run = pre + inc - local;
    if (per <= kR) {
#pragma unroll
        for (int k = 0; k < kR; ++k)
            if (b0 + k < b1) {
                bsum[b0 + k] = run;
                run += r[k];
            }
    } else {
        for (int i = b0; i < b1; ++i) {
            const int32_t v = bsum[i];
            bsum[i] = run;
            run += v;
        }
    }
    if (tid == 0) {
        *seg_end = total;
        if (npieces) *npieces = 0;
    }
}

// stage C: per block of eight rows, the exclusive prefix of the areas (a block-wide scan over
// each coalesced row o0 + 256 k + tid) plus the row's offset -> seg and slot of every entry, and
// the big entries' piece list.  FROM_SEG: the areas are seg's differences (seg written by
// pack3's slot pass) and only the piece list is made
template <typename R, bool FROM_SEG>
__global__ __launch_bounds__(256) void slot_write_kernel(int64_t CN, R rect, const int32_t* __restrict__ bpre,
                                                         int32_t* __restrict__ seg, int2* __restrict__ slot,
                                                         int64_t sstride, int32_t* __restrict__ pbase,
                                                         int32_t* __restrict__ pieces,
                                                         int32_t* __restrict__ npieces, int64_t piece_cap) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int64_t o0 = (int64_t)blockIdx.x * kSlotPer + tid;
    int area[8], sa[8], x0[8], y0[8], w[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const int64_t o = o0 + 256 * k;
        if (FROM_SEG) {
            x0[k] = y0[k] = w[k] = 0;
            area[k] = o < CN ? seg[o + 1] - seg[o] : 0;
        } else {
            area[k] = o < CN ? rect(o, x0[k], y0[k], w[k]) : 0;
        }
    }
    __shared__ int s_w[8][4];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        int inc = area[k];
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const int o = __shfl_up(inc, d);
            if (lane >= d) inc += o;
        }
        if (lane == 63) s_w[k][wave] = inc;
        sa[k] = inc - area[k];  // exclusive within the wave
    }
    // the block's big entries' pieces: one list reservation per block (where in the list is of no
    // consequence: each piece is reduced on its own and an entry sums its pieces in piece order)
    int npk[8], tnp = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        npk[k] = area[k] > kBigSlots ? (area[k] + kPieceSlots - 1) / kPieceSlots : 0;
        tnp += npk[k];
    }
    int pinc = tnp;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int o = __shfl_up(pinc, d);
        if (lane >= d) pinc += o;
    }
    __shared__ int s_p[4], s_pbase;
    if (lane == 63) s_p[wave] = pinc;
    __syncthreads();
    const int ptot = s_p[0] + s_p[1] + s_p[2] + s_p[3];
    if (tid == 0 && ptot > 0) s_pbase = atomicAdd(npieces, ptot);
    __syncthreads();
    int pnext = 0;
    if (ptot > 0) {
        pnext = s_pbase + pinc - tnp;
#pragma unroll
        for (int v = 0; v < 4; ++v) pnext += v < wave ? s_p[v] : 0;
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const int64_t o = o0 + 256 * k;
        if (!FROM_SEG && o < CN) {
            int pre = bpre[blockIdx.x * (kSlotPer / kSlotRow) + k];
#pragma unroll
            for (int v = 0; v < 4; ++v) pre += v < wave ? s_w[k][v] : 0;
            const int e = pre + sa[k];
            seg[o] = e;
            slot[o * sstride] = make_int2(e - y0[k] * w[k] - x0[k], w[k]);
        }
        if (o < CN) {
            int32_t pb = -1;
            if (npk[k] > 0) {
                pb = pnext;
                pnext += npk[k];
                if (pb + npk[k] <= piece_cap)
                    for (int j = 0; j < npk[k]; ++j) pieces[pb + j] = (int32_t)o;
                else
                    pb = -1;  // (cannot happen within piece_capacity; the walker then takes it)
            }
            pbase[o] = pb;
        }
    }
}

// bare lists: each entry's first and last tile (row-major index within its camera)
__global__ __launch_bounds__(256) void slot_minmax_kernel(int n_tiles, const int32_t* __restrict__ offsets,
                                                          int64_t n_isects, int n_bins,
                                                          const int32_t* __restrict__ flatten_ids,
                                                          int32_t* __restrict__ tmin, int32_t* __restrict__ tmax) {
    const int bin = blockIdx.x;
    const int32_t start = offsets[bin];
    const int32_t end = bin == n_bins - 1 ? (int32_t)n_isects : offsets[bin + 1];
    const int tile = bin % n_tiles;
    for (int32_t p = start + threadIdx.x; p < end; p += 256) {
        const int32_t o = flatten_ids[p];
        atomicMin(&tmin[o], tile);
        atomicMax(&tmax[o], tile);
    }
}

__global__ void fill_i32_kernel(int64_t n, int32_t* __restrict__ p, int32_t v) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n) p[i] = v;
}

}  // namespace hgsr

static size_t align256_(size_t x) { return (x + 255) & ~(size_t)255; }

size_t hgsr::grad_slot_bytes(int64_t CN, bool from_lists, int64_t n_isects) {
    const int64_t nb = (CN + kSlotRow - 1) / kSlotRow, pc = piece_capacity(n_isects);
    size_t b = align256_((size_t)(CN + 1) * 4) + align256_((size_t)CN * 8) + align256_((size_t)(nb + 1) * 4);
    b += align256_((size_t)CN * 4) + align256_((size_t)pc * 4) + 256 + align256_((size_t)pc * kPieceFloats * 4);
    if (from_lists) b += 2 * align256_((size_t)CN * 4);
    return b;
}

int hgsr::launch_grad_slots(int C, int N, const float* means2d, const int32_t* radii, int tile_size, int tw, int th,
                            const int32_t* offsets, const int32_t* flatten_ids, int64_t n_isects, void* buf,
                            hipStream_t s, GradSlots& out, int2* slot_dst, int64_t sstride) {
    const int64_t CN = (int64_t)C * N;
    const int64_t nb = (CN + kSlotRow - 1) / kSlotRow;  // rows of the area prefix
    const int64_t nblk = (CN + kSlotPer - 1) / kSlotPer;  // slot_write blocks
    char* p = (char*)buf;
    out.seg = (int32_t*)p;
    p += align256_((size_t)(CN + 1) * 4);
    out.slot = slot_dst ? slot_dst : (int2*)p;
    out.sstride = slot_dst ? sstride : 1;
    p += align256_((size_t)CN * 8);
    int32_t* bsum = (int32_t*)p;
    p += align256_((size_t)(nb + 1) * 4);
    out.cap = piece_capacity(n_isects);
    out.pbase = (int32_t*)p;
    p += align256_((size_t)CN * 4);
    out.pieces = (int32_t*)p;
    p += align256_((size_t)out.cap * 4);
    out.npieces = (int32_t*)p;
    p += 256;
    out.partial = (float*)p;
    p += align256_((size_t)out.cap * kPieceFloats * 4);
    HGSR_REQUIRE(nb < (1ll << 31), "too many Gaussians for the gradient slots");
    if (CN == 0) {
        if (int st = memset_async(out.npieces, 4, s, "grad_slots")) return st;
        return memset_async(out.seg, 4, s, "grad_slots");
    }
    const dim3 grid((unsigned)nblk), rows((unsigned)nb);
    if (radii) {
        HGSR_REQUIRE(means2d, "null pointer");
        const RectFromRadii r{reinterpret_cast<const float2*>(means2d), radii, tile_size, tw, th};
        hipLaunchKernelGGL(slot_sum_kernel<RectFromRadii>, rows, dim3(256), 0, s, CN, r, bsum);
        hipLaunchKernelGGL(slot_scan_kernel, dim3(1), dim3(1024), 0, s, (int)nb, bsum, out.seg + CN, out.npieces);
        hipLaunchKernelGGL((slot_write_kernel<RectFromRadii, false>), grid, dim3(256), 0, s, CN, r, bsum, out.seg, out.slot,
                           out.sstride, out.pbase, out.pieces, out.npieces, out.cap);
    } else {
        HGSR_REQUIRE(offsets && (n_isects == 0 || flatten_ids), "null pointer");
        int32_t* tmin = (int32_t*)p;
        int32_t* tmax = (int32_t*)(p + align256_((size_t)CN * 4));
        const dim3 g1((unsigned)((CN + 255) / 256));
        hipLaunchKernelGGL(fill_i32_kernel, g1, dim3(256), 0, s, CN, tmin, (int32_t)0x7fffffff);
        hipLaunchKernelGGL(fill_i32_kernel, g1, dim3(256), 0, s, CN, tmax, (int32_t)-1);
        const int n_bins = C * tw * th;
        if (n_isects > 0)
            hipLaunchKernelGGL(slot_minmax_kernel, dim3(n_bins), dim3(256), 0, s, tw * th, offsets, n_isects, n_bins,
                               flatten_ids, tmin, tmax);
        const RectFromTiles r{tmin, tmax, tw};
        hipLaunchKernelGGL(slot_sum_kernel<RectFromTiles>, rows, dim3(256), 0, s, CN, r, bsum);
        hipLaunchKernelGGL(slot_scan_kernel, dim3(1), dim3(1024), 0, s, (int)nb, bsum, out.seg + CN, out.npieces);
        hipLaunchKernelGGL((slot_write_kernel<RectFromTiles, false>), grid, dim3(256), 0, s, CN, r, bsum, out.seg, out.slot,
                           out.sstride, out.pbase, out.pieces, out.npieces, out.cap);
    }
    return check_launch("grad_slots");
}

size_t hgsr::slot_prefix_bytes(int64_t CN) {
    return align256_((size_t)(CN + 1) * 4) + align256_((size_t)((CN + kSlotRow - 1) / kSlotRow + 1) * 4) + 256;
}

int32_t* hgsr::slot_prefix_npieces(void* buf, int64_t CN) {
    return (int32_t*)((char*)buf + align256_((size_t)(CN + 1) * 4) +
                      align256_((size_t)((CN + kSlotRow - 1) / kSlotRow + 1) * 4));
}

int hgsr::launch_slot_prefix(int64_t CN, const RectFromRadii& r, void* buf, hipStream_t s, const int32_t* areas) {
    int32_t* const seg = (int32_t*)buf;
    int32_t* const bpre = (int32_t*)((char*)buf + align256_((size_t)(CN + 1) * 4));
    const int64_t nb = (CN + kSlotRow - 1) / kSlotRow;
    HGSR_REQUIRE(nb < (1ll << 31), "too many Gaussians for the gradient slots");
    if (CN == 0) return memset_async(seg, 4, s, "slot_prefix");
    if (areas)
        hipLaunchKernelGGL(slot_sum_kernel<AreaFromCounts>, dim3((unsigned)nb), dim3(256), 0, s, CN,
                           AreaFromCounts{areas}, bpre);
    else
        hipLaunchKernelGGL(slot_sum_kernel<RectFromRadii>, dim3((unsigned)nb), dim3(256), 0, s, CN, r, bpre);
    // (the scan also clears the backward's piece count, kept here with the prefix)
    hipLaunchKernelGGL(slot_scan_kernel, dim3(1), dim3(1024), 0, s, (int)nb, bpre, seg + CN,
                       slot_prefix_npieces(buf, CN));
    return check_launch("slot_prefix");
}

int hgsr::launch_grad_pieces(int64_t CN, const int32_t* seg, int64_t n_isects, void* buf, hipStream_t s,
                             GradSlots& out, int32_t* npieces, bool npieces_zeroed) {
    // the layout of launch_grad_slots' buffer (grad_slot_bytes), seg and slot held elsewhere
    const int64_t nb = (CN + kSlotRow - 1) / kSlotRow, nblk = (CN + kSlotPer - 1) / kSlotPer;
    char* p = (char*)buf;
    out.seg = const_cast<int32_t*>(seg);
    out.slot = nullptr;
    out.sstride = 0;
    p += align256_((size_t)(CN + 1) * 4) + align256_((size_t)CN * 8) + align256_((size_t)(nb + 1) * 4);
    out.cap = piece_capacity(n_isects);
    out.pbase = (int32_t*)p;
    p += align256_((size_t)CN * 4);
    out.pieces = (int32_t*)p;
    p += align256_((size_t)out.cap * 4);
    out.npieces = npieces ? npieces : (int32_t*)p;
    p += 256;
    out.partial = (float*)p;
    if (!(npieces && npieces_zeroed))
        if (int st = memset_async(out.npieces, 4, s, "grad_pieces")) return st;
    if (CN == 0) return HGSR_OK;
    const RectFromRadii none{nullptr, nullptr, 0, 0, 0};
    hipLaunchKernelGGL((slot_write_kernel<RectFromRadii, true>), dim3((unsigned)nblk), dim3(256), 0, s, CN, none,
                       (const int32_t*)nullptr, out.seg, (int2*)nullptr, (int64_t)0, out.pbase, out.pieces,
                       out.npieces, out.cap);
    return check_launch("grad_pieces");
}

using namespace hgsr;

static size_t align256(size_t x) { return align256_(x); }

extern "C" size_t hgsr_isect_ws1_bytes(int C, int N, int tile_w, int tile_h) {
    const IsectGeom g = isect_geom(C, N, tile_w, tile_h);
    size_t b = align256((size_t)g.n_bins * 4);  // totals (or global counters)
    b += align256((size_t)g.n_bins * 4);        // cursors (global path)
    if (g.lds) {
        b += align256((size_t)g.n_blocks * g.n_bins * 4);
        b += align256((size_t)((g.n_blocks + kColRows - 1) / kColRows) * g.n_bins * 4);  // chunk prefixes
    }
    return b;
}

extern "C" size_t hgsr_isect_ws2_bytes(int64_t n_isects, int64_t max_bin) {
    size_t b = align256((size_t)n_isects * 8);
    if (max_bin > kSortCap) b += align256((size_t)n_isects * 8);
    return b;
}

struct Ws1 {
    int32_t* totals;
    int32_t* cursor;
    int32_t* blockhist;
    int32_t* chunk_pre;
};
static Ws1 carve_ws1(const IsectGeom& g, void* ws) {
    Ws1 w;
    char* p = (char*)ws;
    w.totals = (int32_t*)p;
    p += align256((size_t)g.n_bins * 4);
    w.cursor = (int32_t*)p;
    p += align256((size_t)g.n_bins * 4);
    w.blockhist = g.lds ? (int32_t*)p : nullptr;
    w.chunk_pre = g.lds ? (int32_t*)(p + align256((size_t)g.n_blocks * g.n_bins * 4)) : nullptr;
    return w;
}

extern "C" int hgsr_isect_count(int C, int N, const float* means2d, const int32_t* radii, int tile_size,
                                int tile_w, int tile_h, int32_t* tiles_per_gauss, int32_t* isect_offsets,
                                int64_t* info, void* ws1, size_t ws1_bytes, hgsr_stream_t stream) {
    HGSR_REQUIRE(C >= 1 && N >= 0 && tile_size > 0 && tile_w > 0 && tile_h > 0, "bad dims");
    HGSR_REQUIRE((int64_t)C * tile_w * tile_h < (1ll << 30), "too many tiles");
    HGSR_REQUIRE((int64_t)C * N < (1ll << 31), "C*N exceeds int32 flatten ids");
    HGSR_REQUIRE(ws1_bytes >= hgsr_isect_ws1_bytes(C, N, tile_w, tile_h), "isect ws1 too small");
    HGSR_REQUIRE(isect_offsets && info && ws1 && (N == 0 || (means2d && radii && tiles_per_gauss)), "null pointer");
    const IsectGeom g = isect_geom(C, N, tile_w, tile_h);
    const Ws1 w = carve_ws1(g, ws1);
    hipStream_t s = as_stream(stream);
    if (g.lds) {
        if (g.CN > 0) {
            KernelTimer kt("isect_count", s);
            hipLaunchKernelGGL(isect_count_lds_kernel, dim3(g.n_blocks), dim3(256), isect_lds_bytes(g.n_bins), s, g.CN, N,
                               g.per_block, reinterpret_cast<const float2*>(means2d), radii, tile_size, tile_w,
                               tile_h, g.n_tiles, g.n_bins, tiles_per_gauss, w.blockhist);
            if (int st = check_launch("isect_count")) return st;
            const int n_chunks = (g.n_blocks + kColRows - 1) / kColRows;
            hipLaunchKernelGGL(isect_colscan_kernel, dim3((g.n_bins + 255) / 256, n_chunks), dim3(256), 0, s,
                               g.n_blocks, g.n_bins, w.blockhist, w.chunk_pre);
            hipLaunchKernelGGL(isect_chunkscan_kernel, dim3((g.n_bins + 255) / 256), dim3(256), 0, s, n_chunks,
                               g.n_bins, w.chunk_pre, w.totals);
        } else {
            if (int st = memset_async(w.totals, (size_t)g.n_bins * 4, s, "isect_count")) return st;
        }
    } else {
        if (int st = memset_async(w.totals, (size_t)g.n_bins * 4, s, "isect_count")) return st;
        if (g.CN > 0)
            hipLaunchKernelGGL(isect_count_global_kernel, dim3((unsigned)((g.CN + 255) / 256)), dim3(256), 0, s,
                               g.CN, N, reinterpret_cast<const float2*>(means2d), radii, tile_size, tile_w,
                               tile_h, g.n_tiles, tiles_per_gauss, w.totals);
    }
    if (int st = check_launch("isect_count")) return st;
    hipLaunchKernelGGL(isect_binscan_kernel, dim3(1), dim3(1024), 0, s, g.n_bins, w.totals, isect_offsets, info);
    return check_launch("isect_binscan");
}

// bands of tile rows emitted one after another (4 bands let each XCD's L2 merge
// the key lines; more bands trade the write amplification against time, r03_emit_phase_sweep)
static int emit_phases(int tile_h) {
    constexpr int p = 4;
    return p < tile_h ? p : (tile_h > 0 ? tile_h : 1);
}

extern "C" int hgsr_isect_emit_sorted(int C, int N, const float* means2d, const int32_t* radii,
                                      const float* depths, int tile_size, int tile_w, int tile_h,
                                      const int32_t* isect_offsets, int64_t n_isects, int64_t max_bin,
                                      int64_t* isect_ids, int32_t* flatten_ids, void* ws1, size_t ws1_bytes,
                                      void* ws2, size_t ws2_bytes, int64_t* isect_info, hgsr_stream_t stream) {
    // isect_info (nullable): deferred count -- n_isects / max_bin are then capacities and the
    // device-resident count decides (emit_overflow)
    HGSR_REQUIRE(C >= 1 && N >= 0 && tile_size > 0 && tile_w > 0 && tile_h > 0, "bad dims");
    HGSR_REQUIRE(ws1_bytes >= hgsr_isect_ws1_bytes(C, N, tile_w, tile_h), "isect ws1 too small");
    HGSR_REQUIRE(ws2_bytes >= hgsr_isect_ws2_bytes(n_isects, max_bin), "isect ws2 too small");
    if (n_isects == 0) return HGSR_OK;
    HGSR_REQUIRE(means2d && radii && depths && isect_offsets && isect_ids && flatten_ids && ws1 && ws2,
                 "null pointer");
    const IsectGeom g = isect_geom(C, N, tile_w, tile_h);
    const Ws1 w = carve_ws1(g, ws1);
    uint64_t* keys = (uint64_t*)ws2;
    uint64_t* tmp = max_bin > kSortCap ? (uint64_t*)((char*)ws2 + align256((size_t)n_isects * 8)) : nullptr;
    hipStream_t s = as_stream(stream);
    if (g.lds) {
        KernelTimer kt("isect_emit", s);
        hipLaunchKernelGGL(isect_emit_lds_kernel, dim3(g.n_blocks), dim3(256), isect_lds_bytes(g.n_bins), s, g.CN, N,
                           g.per_block, reinterpret_cast<const float2*>(means2d), radii, depths, tile_size,
                           tile_w, tile_h, g.n_tiles, g.n_bins, isect_offsets, w.blockhist, w.chunk_pre, keys,
                           emit_phases(tile_h), isect_info, n_isects, max_bin);
    } else {
        hipLaunchKernelGGL(copy_i32_kernel, dim3((g.n_bins + 255) / 256), dim3(256), 0, s, g.n_bins,
                           isect_offsets, w.cursor);
        hipLaunchKernelGGL(isect_emit_global_kernel, dim3((unsigned)((g.CN + 255) / 256)), dim3(256), 0, s, g.CN,
                           N, reinterpret_cast<const float2*>(means2d), radii, depths, tile_size, tile_w, tile_h,
                           g.n_tiles, w.cursor, keys, isect_info, n_isects, max_bin);
    }
    if (int st = check_launch("isect_emit")) return st;
    KernelTimer kt("tile_sort", s);
    hipLaunchKernelGGL(tile_sort_kernel<false>, dim3(g.n_bins), dim3(256), 0, s, g.n_bins, g.n_tiles,
                       nbits64(g.n_tiles), isect_offsets, n_isects, keys, tmp, isect_ids, flatten_ids, isect_info);
    if (max_bin > kSortCap)
        hipLaunchKernelGGL(tile_sort_kernel<true>, dim3(g.n_bins), dim3(256), 0, s, g.n_bins, g.n_tiles,
                           nbits64(g.n_tiles), isect_offsets, n_isects, keys, tmp, isect_ids, flatten_ids,
                           isect_info);
    return check_launch("tile_sort");
}

extern "C" int hgsr_isect_emit_unsorted(int C, int N, const float* means2d, const int32_t* radii,
                                        const float* depths, int tile_size, int tile_w, int tile_h,
                                        const int64_t* cum_tiles, int64_t* isect_ids, int32_t* flatten_ids,
                                        hgsr_stream_t stream) {
    HGSR_REQUIRE(C >= 1 && N >= 0 && tile_size > 0 && tile_w > 0 && tile_h > 0, "bad dims");
    const int64_t CN = (int64_t)C * N;
    if (CN == 0) return HGSR_OK;
    HGSR_REQUIRE(means2d && radii && depths && cum_tiles && isect_ids && flatten_ids, "null pointer");
    hipLaunchKernelGGL(isect_emit_unsorted_kernel, dim3((unsigned)((CN + 255) / 256)), dim3(256), 0,
                       as_stream(stream), CN, N, reinterpret_cast<const float2*>(means2d), radii, depths,
                       tile_size, tile_w, tile_h, nbits64((int64_t)tile_w * tile_h), cum_tiles, isect_ids,
                       flatten_ids);
    return check_launch("isect_emit_unsorted");
}

extern "C" int hgsr_isect_offset_encode(int64_t n_isects, const int64_t* isect_ids, int C, int tile_w,
                                        int tile_h, int32_t* offsets, hgsr_stream_t stream) {
    HGSR_REQUIRE(C >= 1 && tile_w > 0 && tile_h > 0 && offsets, "bad args");
    hipStream_t s = as_stream(stream);
    const int n_tiles = tile_w * tile_h;
    if (n_isects == 0) {
        if (int st = memset_async(offsets, (size_t)C * n_tiles * 4, s, "offset_encode")) return st;
        return check_launch("offset_encode");
    }
    HGSR_REQUIRE(isect_ids, "null pointer");
    hipLaunchKernelGGL(offset_encode_kernel, dim3((unsigned)((n_isects + 255) / 256)), dim3(256), 0, s, n_isects,
                       isect_ids, C, n_tiles, nbits64(n_tiles), offsets);
    return check_launch("offset_encode");
}
