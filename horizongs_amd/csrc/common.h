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
struct KernelTimer {
    int id;
    hipStream_t s;
    KernelTimer(const char* name, hipStream_t st) : id(timing_on() ? timing_begin(name, st) : -1), s(st) {}
    ~KernelTimer() { timing_end(id, s); }
};

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

}  // namespace hgsr
