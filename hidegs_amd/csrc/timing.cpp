// timing.cpp -- per-kernel device timing with hipEvents (hidegs_kernel_timing*).
//
// Used by bench.py to measure the average duration of individual kernels live, on the
// stream they are launched on, so a roofline fraction can be priced per kernel; rocprofv3
// summaries under profiles/ are the cross-check.  Off by default: a disabled timer costs
// one relaxed atomic load per launch.
#include <atomic>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "common.h"

namespace hidegs {
namespace {
std::atomic<bool> g_enabled{false};
std::mutex g_mu;
struct Pending {
    std::string name;
    hipEvent_t start, stop;
};
std::vector<Pending> g_pending;
struct Acc {
    double ms = 0.0;
    long long n = 0;
};
std::map<std::string, Acc> g_acc;

void resolve_locked()
{
    for (auto& p : g_pending) {
        float ms = 0.f;
        if (hipEventSynchronize(p.stop) == hipSuccess && hipEventElapsedTime(&ms, p.start, p.stop) == hipSuccess) {
            Acc& a = g_acc[p.name];
            a.ms += ms;
            a.n += 1;
        }
        (void)hipEventDestroy(p.start);
        (void)hipEventDestroy(p.stop);
    }
    g_pending.clear();
}
}  // namespace

bool kernel_timing_enabled() { return g_enabled.load(std::memory_order_relaxed); }

// Timing-only events: no system-scope fence when they are recorded.  A default event writes the
// L2 back and invalidates it at the record, which the measured interval then includes (the
// radix_scatter launch read 46.7 us this way against rocprofv3's 43.6 us); the host still waits
// for the stop event in hipEventSynchronize.
constexpr unsigned kTimerEventFlags = hipEventDisableSystemFence;

LaunchTimer::LaunchTimer(const char* n, hipStream_t s) : name(n), stream(s)
{
    if (hipEventCreateWithFlags(&start, kTimerEventFlags) != hipSuccess ||
        hipEventCreateWithFlags(&stop, kTimerEventFlags) != hipSuccess) {
        start = stop = nullptr;
        return;
    }
    (void)hipEventRecord(start, stream);
}

LaunchTimer::~LaunchTimer()
{
    if (!start) return;
    (void)hipEventRecord(stop, stream);
    std::lock_guard<std::mutex> g(g_mu);
    g_pending.push_back({name, start, stop});
}

}  // namespace hidegs

extern "C" {

void hidegs_kernel_timing(int enable) { hidegs::g_enabled.store(enable != 0); }

void hidegs_kernel_timing_reset(void)
{
    std::lock_guard<std::mutex> g(hidegs::g_mu);
    hidegs::resolve_locked();
    hidegs::g_acc.clear();
}

int hidegs_kernel_time(const char* name, double* total_ms, long long* launches)
{
    std::lock_guard<std::mutex> g(hidegs::g_mu);
    hidegs::resolve_locked();
    auto it = hidegs::g_acc.find(name ? name : "");
    if (total_ms) *total_ms = it == hidegs::g_acc.end() ? 0.0 : it->second.ms;
    if (launches) *launches = it == hidegs::g_acc.end() ? 0 : it->second.n;
    return it == hidegs::g_acc.end() ? -1 : 0;
}

}  // extern "C"
