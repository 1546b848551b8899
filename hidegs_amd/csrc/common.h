// common.h -- shared plumbing of the C-ABI library: error channel, stream handle,
// scratch carving, launch checks and a few wave64 helpers.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include <string>

#include "../../include/hidegs.h"

namespace hidegs {

// Last error message of the calling thread (hidegs_last_error()).
void set_error(const std::string& msg);
const std::string& last_error();

inline int fail(int code, const std::string& msg)
{
    set_error(msg);
    return code;
}

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

// Checks the launch queue after kernels were enqueued; with debug != 0 it also
// synchronises the stream so an asynchronous fault is reported at its stage
// (the reference's CHECK_CUDA(..., debug), auxiliary.h:23-30).
int check_launch(const char* stage, hipStream_t stream, int debug);

// Library-wide debug mode (hidegs_set_debug): every launch check synchronises, and the sort reads
// back the partition queue's error word.
bool debug_enabled();

// Sticky partition-queue error word of the current device (primitives.hip); synchronises `stream`.
// Reads and clears it in one device-side exchange.
int queue_error(hipStream_t stream, int clear, uint32_t* flags);

// Asynchronous error words: one u32 per stream in a page of mapped, coherent pinned host memory.  A
// sort's last kernel ORs its partition queue's error bits into its stream's word (system-scope vector
// stores), so that the failure surfaces without a host synchronisation.  The page is allocated by the
// first entry-point call of any kind that does not come from a stream being captured into a graph.
// async_error_slot() returns the device address of `stream`'s word -- of the graph word when `stream`
// is being captured (a graph may be replayed on any stream) -- or NULL if the page does not exist (it
// could not be allocated, or every call so far came from a capturing stream; then only the debug mode
// and hidegs_queue_error report that call's queue errors).
uint32_t* async_error_slot(hipStream_t stream);
// Called first by every compute entry point: if `stream`'s word (or the graph word) is set it is taken
// (exchanged with 0) and turned into HIDEGS_E_ASYNC with its message, so a call on the stream of a failed
// sort (any call, after a failed graph replay), made once that sort's last kernel has run, fails loudly
// instead of running.
int take_async_error(const char* what, hipStream_t stream);
// `stream`'s word's bits and the graph word's, taken (exchanged with 0); 0 when none are pending.
uint32_t take_async_bits(hipStream_t stream);

// 256-byte aligned carving of one caller-provided scratch buffer.
constexpr size_t kAlign = 256;
inline size_t align_up(size_t n) { return (n + kAlign - 1) & ~(kAlign - 1); }

struct Carver {
    char* base;
    size_t used = 0;
    explicit Carver(void* b) : base(static_cast<char*>(b)) {}
    template <typename T>
    T* take(size_t count)
    {
        T* p = reinterpret_cast<T*>(base ? base + used : nullptr);
        used += align_up(count * sizeof(T));
        return p;
    }
};

// ---- wave64 helpers (device) --------------------------------------------------
constexpr int kWave = 64;

__device__ __forceinline__ int lane_id() { return __lane_id(); }

// Block b of nb -> a work index such that consecutive work indices run on one XCD: the dispatcher
// deals workgroups to the 8 XCDs round-robin (b, b+8, ... share an XCD's L2), so this hands each
// XCD a contiguous range of indices.
__device__ __forceinline__ int xcd_swizzle(int b, int nb)
{
    // consecutive leaf groups land on one XCD (blocks b, b+8, ... share an XCD's L2)
    const int per = nb / 8, rem = nb % 8, x = b % 8, k = b / 8;
    return (x < rem) ? x * (per + 1) + k : rem * (per + 1) + (x - rem) * per + k;
}

template <typename T>
__device__ __forceinline__ T wave_shfl_xor(T v, int m)
{
    return __shfl_xor(v, m, kWave);
}

// Inclusive prefix sum over the 64 lanes with DPP moves (row_shr within rows of 16, then the
// row_bcast:15 / row_bcast:31 carries of GFX9): VALU-latency steps instead of LDS-path shuffles.
// Every lane of the wave must be active.
__device__ __forceinline__ uint32_t wave_inclusive_scan_u32(uint32_t v)
{
    const int lane = lane_id(), rl = lane & 15;
    int x = (int)v, t;
    t = __builtin_amdgcn_mov_dpp(x, 0x111, 0xf, 0xf, false);  // row_shr:1
    if (rl >= 1) x += t;
    t = __builtin_amdgcn_mov_dpp(x, 0x112, 0xf, 0xf, false);  // row_shr:2
    if (rl >= 2) x += t;
    t = __builtin_amdgcn_mov_dpp(x, 0x114, 0xf, 0xf, false);  // row_shr:4
    if (rl >= 4) x += t;
    t = __builtin_amdgcn_mov_dpp(x, 0x118, 0xf, 0xf, false);  // row_shr:8
    if (rl >= 8) x += t;
    t = __builtin_amdgcn_mov_dpp(x, 0x142, 0xf, 0xf, false);  // row_bcast:15
    if ((lane & 31) >= 16) x += t;
    t = __builtin_amdgcn_mov_dpp(x, 0x143, 0xf, 0xf, false);  // row_bcast:31
    if (lane >= 32) x += t;
    return (uint32_t)x;
}

__device__ __forceinline__ float wave_max(float v)
{
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) v = fmaxf(v, __shfl_xor(v, m, kWave));
    return v;
}
__device__ __forceinline__ float wave_min(float v)
{
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) v = fminf(v, __shfl_xor(v, m, kWave));
    return v;
}
__device__ __forceinline__ float wave_sum(float v)
{
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, kWave);
    return v;
}
__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v)
{
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, kWave);
    return v;
}

}  // namespace hidegs

namespace hidegs {

// Per-kernel device timing (hidegs_kernel_timing in include/hidegs.h): when enabled, each
// launch made through HIDEGS_LAUNCH is bracketed by two hipEvents recorded on its stream;
// the durations are resolved and accumulated per kernel name when they are queried.
bool kernel_timing_enabled();
struct LaunchTimer {
    const char* name;
    hipStream_t stream;
    hipEvent_t start = nullptr, stop = nullptr;
    LaunchTimer(const char* n, hipStream_t s);
    ~LaunchTimer();
};

}  // namespace hidegs

#define HIDEGS_LAUNCH(NAME, KERNEL, GRID, BLOCK, SHMEM, STREAM, ...)                        \
    do {                                                                                   \
        if (::hidegs::kernel_timing_enabled()) {                                           \
            ::hidegs::LaunchTimer _t(NAME, STREAM);                                        \
            hipLaunchKernelGGL(KERNEL, GRID, BLOCK, SHMEM, STREAM, __VA_ARGS__);           \
        } else {                                                                           \
            hipLaunchKernelGGL(KERNEL, GRID, BLOCK, SHMEM, STREAM, __VA_ARGS__);           \
        }                                                                                  \
    } while (0)
