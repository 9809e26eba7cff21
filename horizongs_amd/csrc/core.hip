// Library status / error plumbing for the hgsr C ABI.
#include <stdarg.h>
#include <string.h>

#include "common.h"

namespace hgsr {

static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}

int check_launch(const char* what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_error("%s: kernel launch failed: %s", what, hipGetErrorString(e));
        return HGSR_ELAUNCH;
    }
    return HGSR_OK;
}

// ---------------------------------------------------------------- raster tile dispatch order
// One workgroup per XCD band (the slots xcd_remap gives XCD x: [x q + min(x, r), + q + (x < r))).
// A counting sort of the band's bins by intersection count, descending, over 1024 buckets of
// width 2^shift (shift: the smallest that fits the band's largest bin): ties and bins in one
// bucket go in atomic order, which only moves work between workgroups -- every result is
// independent of the order.
__global__ __launch_bounds__(1024) void tile_order_kernel(int64_t n_bins, const int32_t* __restrict__ offsets,
                                                          int64_t n_isects, const int64_t* __restrict__ info,
                                                          int32_t* __restrict__ order,
                                                          const int32_t* __restrict__ tile_end) {
    constexpr int NBK = 1024;
    __shared__ int hist[NBK];
    __shared__ int s_max[16];
    const int x = blockIdx.x, tid = threadIdx.x;
    const int64_t q = n_bins >> 3, r = n_bins & 7;
    const int64_t base = x * q + (x < r ? x : r), len = q + (x < r ? 1 : 0);
    const int64_t n = info ? info[0] : n_isects;
    const bool ovf = info && info[2];
    auto cnt = [&](int64_t b) {
        int64_t e = b == n_bins - 1 ? n : offsets[b + 1];
        if (tile_end) e = min(e, (int64_t)tile_end[b]);
        return (int)max((int64_t)0, e - (int64_t)offsets[b]);
    };
    int mx = 0;
    for (int64_t i = tid; i < len; i += 1024) mx = max(mx, cnt(base + i));
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) mx = max(mx, __shfl_xor(mx, d));
    if ((tid & 63) == 0) s_max[tid >> 6] = mx;
    hist[tid] = 0;
    __syncthreads();
    mx = 0;
#pragma unroll
    for (int w = 0; w < 16; ++w) mx = max(mx, s_max[w]);
    int shift = 0;
    while ((mx >> shift) >= NBK) ++shift;
    auto key = [&](int c) { return NBK - 1 - (c >> shift); };  // descending
    for (int64_t i = tid; i < len; i += 1024) atomicAdd(&hist[key(cnt(base + i))], 1);
    __syncthreads();
    // exclusive scan of the 1024 bucket sizes (one per thread): in-wave shuffle scan + wave totals
    const int v = hist[tid];
    int inc = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int o = __shfl_up(inc, d);
        if ((tid & 63) >= d) inc += o;
    }
    __syncthreads();
    if ((tid & 63) == 63) s_max[tid >> 6] = inc;
    __syncthreads();
    int wpre = 0;
    for (int w = 0; w < (tid >> 6); ++w) wpre += s_max[w];
    hist[tid] = wpre + inc - v;  // cursor of bucket tid
    __syncthreads();
    for (int64_t i = tid; i < len; i += 1024) {
        const int64_t b = base + i;
        const int pos = ovf ? (int)i : atomicAdd(&hist[key(cnt(b))], 1);
        order[base + pos] = (int32_t)b;
    }
}

int launch_tile_order(int64_t n_bins, const int32_t* offsets, int64_t n_isects, const int64_t* info, int32_t* order,
                      hipStream_t s, const int32_t* tile_end) {
    if (n_bins <= 0 || !order) return HGSR_OK;
    hipLaunchKernelGGL(tile_order_kernel, dim3(8), dim3(1024), 0, s, n_bins, offsets, n_isects, info, order, tile_end);
    return check_launch("tile_order");
}

}  // namespace hgsr

extern "C" int hgsr_version(void) { return 1; }
extern "C" const char* hgsr_last_error(void) { return hgsr::g_err; }
