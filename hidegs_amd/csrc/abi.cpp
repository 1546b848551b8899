// abi.cpp -- error channel, launch checks and the entry points of include/hidegs.h
// that are not built in this release.
//
// The rasterizer forward/backward and markVisible stay unbuilt: writing their kernels
// was refused in rounds 1 and 2 and the refusal binds ("Decisions in force").
// They fail loudly with HIDEGS_E_UNSUPPORTED; nothing falls back to a CPU path.
#include "common.h"

#include <atomic>
#include <mutex>
#include <unordered_map>
#include <utility>

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
// One word per stream (a process-wide word reported thread A's failed sort on thread B's
// unrelated call and let a second failure overwrite the first's bits).  Streams past the table share
// the last word.  A stream handle that is destroyed and handed out again keeps its word.  A sort
// captured into a graph writes word 0 instead: the graph may be replayed on any stream, so that word
// is taken by the next call on ANY stream.
constexpr int kAsyncWords = 1024;
constexpr int kGraphWord = 0;
constexpr int kOverflowWord = kAsyncWords - 1;
std::once_flag g_async_once;
std::atomic<uint32_t*> g_async_host{nullptr};    // mapped, coherent pinned page of kAsyncWords words
std::atomic<uint32_t*> g_async_device{nullptr};  // its device address (published after the host page)
std::mutex g_slot_mutex;
std::unordered_map<hipStream_t, int> g_slot;  // stream -> word index, guarded by g_slot_mutex
int g_next_slot = kGraphWord + 1;

bool capturing(hipStream_t stream)
{
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(stream, &st) != hipSuccess) (void)hipGetLastError();
    return st != hipStreamCaptureStatusNone;
}

// The page, allocated by the first call from a stream that is not being captured (no pinned
// allocation inside a capture: it may synchronise).  Every entry point asks first, so a sort captured
// into a graph finds the page already there unless every earlier call was captured too.
void ensure_async_page(hipStream_t stream)
{
    if (g_async_device.load(std::memory_order_acquire) || capturing(stream)) return;
    std::call_once(g_async_once, [] {
        void* h = nullptr;
        const size_t bytes = kAsyncWords * sizeof(uint32_t);
        if (hipHostMalloc(&h, bytes, hipHostMallocMapped | hipHostMallocPortable | hipHostMallocCoherent) != hipSuccess) {
            (void)hipGetLastError();
            return;
        }
        void* d = nullptr;
        if (hipHostGetDevicePointer(&d, h, 0) != hipSuccess) {
            (void)hipGetLastError();
            (void)hipHostFree(h);
            return;
        }
        for (int i = 0; i < kAsyncWords; i++) __atomic_store_n(static_cast<uint32_t*>(h) + i, 0u, __ATOMIC_SEQ_CST);
        g_async_host.store(static_cast<uint32_t*>(h), std::memory_order_release);
        g_async_device.store(static_cast<uint32_t*>(d), std::memory_order_release);
    });
}

// `stream`'s word index; -1 if it has none and `create` is false (no sort ever reported to it).
int slot_of(hipStream_t stream, bool create)
{
    std::lock_guard<std::mutex> lock(g_slot_mutex);
    auto it = g_slot.find(stream);
    if (it != g_slot.end()) return it->second;
    if (!create) return -1;
    const int s = g_next_slot < kOverflowWord ? g_next_slot++ : kOverflowWord;
    g_slot.emplace(stream, s);
    return s;
}
}  // namespace

uint32_t* async_error_slot(hipStream_t stream)
{
    ensure_async_page(stream);
    uint32_t* d = g_async_device.load(std::memory_order_acquire);
    if (!d) return nullptr;
    return d + (capturing(stream) ? kGraphWord : slot_of(stream, true));
}

namespace {
// (bits of `stream`'s own word, bits of the graph word), both taken
std::pair<uint32_t, uint32_t> take_words(hipStream_t stream)
{
    uint32_t* h = g_async_host.load(std::memory_order_acquire);
    if (!h) return {0u, 0u};
    const int s = slot_of(stream, false);
    const uint32_t own = s < 0 ? 0u : __atomic_exchange_n(h + s, 0u, __ATOMIC_SEQ_CST);
    return {own, __atomic_exchange_n(h + kGraphWord, 0u, __ATOMIC_SEQ_CST)};
}
}  // namespace

uint32_t take_async_bits(hipStream_t stream)
{
    const auto w = take_words(stream);
    return w.first | w.second;
}

int take_async_error(const char* what, hipStream_t stream)
{
    ensure_async_page(stream);
    const auto w = take_words(stream);
    const uint32_t err = w.first | w.second;
    if (!err) return 0;
    const char* who = w.first ? "an earlier sort on this stream" : "a sort replayed from a graph (any stream)";
    return fail(HIDEGS_E_ASYNC, std::string(what) + ": not run -- " + who + " failed in its hot-tile "
                                    "partition queue (error " + std::to_string(err) +
                                    ((err & 1u) ? ", job slots exhausted" : "") +
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
