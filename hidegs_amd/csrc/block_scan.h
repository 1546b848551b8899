// block_scan.h -- workgroup-level scan helpers shared by the kernels of the library
// (256-thread workgroups of four wave64s).
#pragma once
#include "common.h"

namespace hidegs {
namespace {

constexpr int kScanBlock = 256;
constexpr int kScanWaves = kScanBlock / kWave;  // 4
constexpr int kScanItems = 16;
constexpr int kScanTile = kScanBlock * kScanItems;  // 4096

// Block-wide exclusive scan of one u32 per thread (W wave64s, 256 threads by default); returns
// the exclusive prefix and writes the block total to *total.  s_wave holds W entries.
template <int W = kScanWaves>
__device__ __forceinline__ uint32_t block_exclusive_scan(uint32_t v, uint32_t* s_wave, uint32_t* total)
{
    const int lane = lane_id();
    const int wave = threadIdx.x / kWave;
    const uint32_t inc = wave_inclusive_scan_u32(v);
    if (lane == kWave - 1) s_wave[wave] = inc;
    __syncthreads();
    uint32_t woff = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < W; w++) {
        uint32_t s = s_wave[w];
        if (w < wave) woff += s;
        tot += s;
    }
    *total = tot;
    __syncthreads();  // s_wave may be reused by the caller
    return woff + inc - v;
}

// Exclusive scan of `count` u32 in place by ONE workgroup (count is small: tiles).
__global__ __launch_bounds__(kScanBlock) void scan_small_kernel(uint32_t* __restrict__ data, int count,
                                                                uint32_t* __restrict__ total_out)
{
    __shared__ uint32_t s_wave[kScanWaves];
    uint32_t carry = 0;
    for (int base = 0; base < count; base += kScanTile) {
        uint32_t v[kScanItems];
        uint32_t sum = 0;
#pragma unroll
        for (int j = 0; j < kScanItems; j++) {
            int i = base + threadIdx.x * kScanItems + j;
            v[j] = (i < count) ? data[i] : 0u;
            sum += v[j];
        }
        uint32_t total;
        uint32_t pre = block_exclusive_scan(sum, s_wave, &total) + carry;
#pragma unroll
        for (int j = 0; j < kScanItems; j++) {
            int i = base + threadIdx.x * kScanItems + j;
            if (i < count) data[i] = pre;
            pre += v[j];
        }
        carry += total;
    }
    if (total_out && threadIdx.x == 0) *total_out = carry;
}

}  // namespace
}  // namespace hidegs
