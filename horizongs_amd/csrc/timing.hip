// Optional per-kernel HIP-event timing (bench.py uses it for the live roofline
// numbers; rocprofv3 gives the same durations from outside the process).
#include <mutex>
#include <string.h>
#include <string>
#include <vector>

#include "common.h"

namespace hgsr {

namespace {
struct Rec {
    const char* name;
    hipEvent_t a, b;
};
std::mutex g_mu;
bool g_on = false;
std::vector<hipEvent_t> g_pool;
std::vector<Rec> g_recs;
size_t g_next = 0;
constexpr size_t kMaxRecs = 1 << 16;
constexpr size_t kPrealloc = 256;  // events created by hgsr_timing_enable
std::string g_only;  // record only this kernel (empty = all)
// device counters of the timed raster bwd: [0] (pixel, Gaussian) pairs visited (gsplat's span),
// [1] lane-pairs stepped (compacted list entries x 64)
unsigned long long* g_pairs = nullptr;
constexpr size_t kPairBytes = (size_t)kPairSlots * 2 * 16 * sizeof(unsigned long long);
}  // namespace

bool timing_on() { return g_on; }

// the event pool is filled by reset / enable, outside the region being timed (creating
// events there costs host time inside it); called with g_mu held
static void prefill_pool() {
    while (g_pool.size() < kPrealloc) {
        hipEvent_t e;
        if (hipEventCreateWithFlags(&e, hipEventDisableSystemFence) != hipSuccess) break;
        g_pool.push_back(e);
    }
}

int timing_begin(const char* name, hipStream_t s) {
    std::lock_guard<std::mutex> lk(g_mu);
    if (!g_on || g_recs.size() >= kMaxRecs) return -1;
    if (!g_only.empty() && g_only != name) return -1;
    while (g_pool.size() < g_next + 2) {
        hipEvent_t e;
        // device-scope release only: a system-scope fence per record would stall the
        // stream (~25 us per event pair on MI355X) and distort the timed region
        if (hipEventCreateWithFlags(&e, hipEventDisableSystemFence) != hipSuccess) return -1;
        g_pool.push_back(e);
    }
    Rec r{name, g_pool[g_next], g_pool[g_next + 1]};
    g_next += 2;
    if (hipEventRecord(r.a, s) != hipSuccess) return -1;
    g_recs.push_back(r);
    return (int)g_recs.size() - 1;
}

unsigned long long* timing_pair_counter(const char* kernel) {
    std::lock_guard<std::mutex> lk(g_mu);
    if (!g_on || (!g_only.empty() && g_only != kernel)) return nullptr;
    if (!g_pairs) {
        if (hipMalloc(&g_pairs, kPairBytes) != hipSuccess) return nullptr;
        if (hipMemset(g_pairs, 0, kPairBytes) != hipSuccess) return nullptr;
    }
    return g_pairs;
}

// counter `which` summed over the workgroup slots (pair_slot in common.h)
static int read_pairs(int which, unsigned long long* out) {
    std::vector<unsigned long long> h(kPairBytes / sizeof(unsigned long long));
    if (hipDeviceSynchronize() != hipSuccess ||
        hipMemcpy(h.data(), g_pairs, kPairBytes, hipMemcpyDeviceToHost) != hipSuccess) {
        set_error("timing: pair counter read failed");
        return HGSR_ELAUNCH;
    }
    unsigned long long v = 0;
    for (int s = 0; s < kPairSlots; ++s) v += h[(s * 2 + which) * 16];
    *out = v;
    return HGSR_OK;
}

void timing_end(int id, hipStream_t s) {
    if (id < 0) return;
    std::lock_guard<std::mutex> lk(g_mu);
    (void)hipEventRecord(g_recs[id].b, s);
}

}  // namespace hgsr

using namespace hgsr;

extern "C" int hgsr_timing_enable(int on) {
    std::lock_guard<std::mutex> lk(g_mu);
    g_on = on != 0;
    if (g_on) prefill_pool();
    return HGSR_OK;
}

extern "C" int hgsr_timing_only(const char* kernel) {
    std::lock_guard<std::mutex> lk(g_mu);
    g_only = kernel ? kernel : "";
    return HGSR_OK;
}

extern "C" int hgsr_timing_pairs(unsigned long long* out, int reset) {
    std::lock_guard<std::mutex> lk(g_mu);
    unsigned long long v = 0;
    // a reset allocates the counters now: their synchronous hipMalloc / hipMemset must not
    // fall inside the timed steps (the first counted launch would drain the queue)
    if (!g_pairs && reset) {
        if (hipMalloc(&g_pairs, kPairBytes) != hipSuccess) return HGSR_ELAUNCH;
        if (hipMemset(g_pairs, 0, kPairBytes) != hipSuccess) return HGSR_ELAUNCH;
    }
    if (g_pairs) {
        if (int st = read_pairs(0, &v)) return st;
        if (reset && hipMemset(g_pairs, 0, kPairBytes) != hipSuccess) return HGSR_ELAUNCH;
    }
    if (out) *out = v;
    return HGSR_OK;
}

extern "C" int hgsr_timing_exec_pairs(unsigned long long* out) {
    std::lock_guard<std::mutex> lk(g_mu);
    unsigned long long v = 0;
    if (g_pairs)
        if (int st = read_pairs(1, &v)) return st;
    if (out) *out = v;
    return HGSR_OK;
}

extern "C" int hgsr_timing_reset(void) {
    std::lock_guard<std::mutex> lk(g_mu);
    g_recs.clear();
    g_next = 0;
    prefill_pool();
    return HGSR_OK;
}

extern "C" int hgsr_timing_query(const char* kernel, double* total_ms, int64_t* count) {
    std::lock_guard<std::mutex> lk(g_mu);
    double tot = 0.0;
    int64_t n = 0;
    for (const Rec& r : g_recs) {
        if (strcmp(r.name, kernel) != 0) continue;
        if (hipEventSynchronize(r.b) != hipSuccess) {
            set_error("timing: event sync failed");
            return HGSR_ELAUNCH;
        }
        float ms = 0.f;
        if (hipEventElapsedTime(&ms, r.a, r.b) != hipSuccess) {
            set_error("timing: elapsed time failed");
            return HGSR_ELAUNCH;
        }
        tot += ms;
        ++n;
    }
    if (total_ms) *total_ms = tot;
    if (count) *count = n;
    return HGSR_OK;
}
