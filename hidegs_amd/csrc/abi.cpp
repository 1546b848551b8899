// abi.cpp -- error channel, launch checks and the entry points of include/hidegs.h
// that are not built in this release.
//
// The rasterizer forward/backward and markVisible stay unbuilt: writing their kernels
// was refused in rounds 1 and 2 and the refusal binds ("Decisions in force").
// They fail loudly with HIDEGS_E_UNSUPPORTED; nothing falls back to a CPU path.
#include "common.h"

#include <atomic>
#include <mutex>

namespace hidegs {

namespace {
thread_local std::string g_last_error;
std::atomic<int> g_debug{0};
constexpr const char* kNotBuilt =
    "not built: the gfx950 rasterizer kernels are outside this release (DESIGN.md, 'Decisions in force')";
}  // namespace

void set_error(const std::string& msg) { g_last_error = msg; }
const std::string& last_error() { return g_last_error; }

bool debug_enabled() { return g_debug.load(std::memory_order_relaxed) != 0; }

int check_launch(const char* stage, hipStream_t stream, int debug)
{
    hipError_t e = hipGetLastError();
    if (e == hipSuccess && (debug || debug_enabled())) e = hipStreamSynchronize(stream);
    if (e != hipSuccess) return fail(HIDEGS_E_HIP, std::string(stage) + ": " + hipGetErrorString(e));
    return 0;
}

static int not_built(const char* fn) { return fail(HIDEGS_E_UNSUPPORTED, std::string(fn) + ": " + kNotBuilt); }

namespace {
std::once_flag g_async_once;
std::atomic<uint32_t*> g_async_host{nullptr};    // mapped, coherent pinned word
std::atomic<uint32_t*> g_async_device{nullptr};  // its device address (published after the host word)
}  // namespace

uint32_t* async_error_slot(hipStream_t stream)
{
    // not allocated yet and the stream is being captured into a graph: no pinned allocation inside a
    // capture (it may synchronise); that call goes without the asynchronous word
    if (!g_async_device.load(std::memory_order_acquire)) {
        hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
        if (hipStreamIsCapturing(stream, &st) != hipSuccess) (void)hipGetLastError();
        if (st != hipStreamCaptureStatusNone) return nullptr;
    }
    std::call_once(g_async_once, [] {
        void* h = nullptr;
        if (hipHostMalloc(&h, 64, hipHostMallocMapped | hipHostMallocPortable | hipHostMallocCoherent) != hipSuccess) {
            (void)hipGetLastError();
            return;
        }
        void* d = nullptr;
        if (hipHostGetDevicePointer(&d, h, 0) != hipSuccess) {
            (void)hipGetLastError();
            (void)hipHostFree(h);
            return;
        }
        __atomic_store_n(static_cast<uint32_t*>(h), 0u, __ATOMIC_SEQ_CST);
        g_async_host.store(static_cast<uint32_t*>(h), std::memory_order_release);
        g_async_device.store(static_cast<uint32_t*>(d), std::memory_order_release);
    });
    return g_async_device.load(std::memory_order_acquire);
}

uint32_t take_async_bits()
{
    // the word exists only once a sort asked for its slot; before that nothing can be pending
    uint32_t* h = g_async_host.load(std::memory_order_acquire);
    return h ? __atomic_exchange_n(h, 0u, __ATOMIC_SEQ_CST) : 0u;
}

int take_async_error(const char* what)
{
    const uint32_t err = take_async_bits();
    if (!err) return 0;
    return fail(HIDEGS_E_ASYNC, std::string(what) + ": not run -- an earlier sort's hot-tile partition queue failed (error " +
                                    std::to_string(err) + ((err & 1u) ? ", job slots exhausted" : "") +
                                    ((err & 4u) ? ", a worker gave up waiting" : "") +
                                    "): that sort's output is not sorted");
}

}  // namespace hidegs

extern "C" {

int hidegs_rasterize_forward(hidegs_alloc_fn, hidegs_alloc_fn, hidegs_alloc_fn, void*, int, int, int, const float*,
                             int, int, const int*, const int*, const float*, const int*, const float*, const float*,
                             const float*, const float*, const float*, const float*, float, const float*,
                             const float*, const float*, const float*, const float*, float, float, int, float*,
                             float*, int*, float*, float*, int, int*, int, void*, int* num_rendered)
{
    if (num_rendered) *num_rendered = 0;
    return hidegs::not_built("hidegs_rasterize_forward");
}

int hidegs_rasterize_backward(int, int, int, int, const float*, const float*, int, int, const int*, const int*,
                              const float*, const int*, const float*, const float*, const float*, const float*,
                              const float*, const float*, const float*, float, const float*, const float*,
                              const float*, const float*, float, float, const int*, float, char*, char*, char*,
                              const float*, const float*, const float*, const float*, float*, float*, float*, float*,
                              float*, float*, float*, float*, float*, int, int, void*)
{
    return hidegs::not_built("hidegs_rasterize_backward");
}

int hidegs_mark_visible(int, const float*, const float*, const float*, unsigned char*, void*)
{
    return hidegs::not_built("hidegs_mark_visible");
}

void hidegs_set_debug(int enable) { hidegs::g_debug.store(enable ? 1 : 0, std::memory_order_relaxed); }

const char* hidegs_last_error(void) { return hidegs::last_error().c_str(); }
const char* hidegs_version(void) { return "hidegs-abi 0.6 (gfx950: distCUDA2, scan, radix sort, tile sort + ranges, masked Adam, view-DP wire; HIDEGS_E_ASYNC)"; }

}  // extern "C"
