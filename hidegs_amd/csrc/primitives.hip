// primitives.hip -- the binning primitives of Rasterizer::forward as gfx950 kernels:
//
//   hidegs_inclusive_scan_u32   <- cub::DeviceScan::InclusiveSum of tiles_touched
//                                  (rasterizer_impl.cu:171,321)
//   hidegs_sort_pairs_u64/_u32  <- cub::DeviceRadixSort::SortPairs over bits [begin, end)
//                                  (rasterizer_impl.cu:193-196,354-362; simple_knn.cu:211-214)
//   hidegs_identify_tile_ranges <- cudaMemsetAsync(ranges) + identifyTileRanges
//                                  (rasterizer_impl.cu:364-371,120-142)
//   hidegs_sort_tile_pairs      <- SortPairs + memset + identifyTileRanges as one call
//                                  (rasterizer_impl.cu:354-371)
//   hidegs_higher_msb           <- getHigherMsb (rasterizer_impl.cu:35-50)
//
// Design (MI355X-first, not a CUB restatement):
//  * Tiles of 4096 items per 256-thread workgroup (4 x wave64, 16 items per lane),
//    global traffic in 16-byte-per-lane vector loads where the layout allows.
//  * Scan: tile sums, then a rescan in which each workgroup adds up the sums before it
//    (two stream-ordered launches, no inter-workgroup hand-off inside a launch).
//  * Radix sort: LSD, 8-bit digits, per pass three launches:
//      1. tile histogram  (per-wave LDS histograms, digit-major counts[d][tile])
//      2. per-digit exclusive scan over tiles (one workgroup per digit)
//      3. scatter: stable ranks from wave64 ballot matching (8 ballots give the
//         set of lanes sharing a digit), per-wave running counters in LDS,
//         a local sort of the tile in LDS, then run-contiguous global stores.
//    Stability is by construction: item order inside a wave is (round, lane),
//    waves own consecutive 1024-item segments, tiles are ordered by the scan.
// No kernel depends on dispatch order or XCD placement.
#include "block_scan.h"
#include "common.h"

namespace hidegs {
int identify_tile_ranges(const uint64_t* keys, long long n, uint32_t* ranges, int num_tiles, hipStream_t stream);

namespace {

constexpr int kBlock = 256;
#ifndef HIDEGS_RADIX_ITEMS
#define HIDEGS_RADIX_ITEMS 16  // items per thread of a scan / radix tile (experiments: tools/build_variant.py)
#endif
constexpr int kItems = HIDEGS_RADIX_ITEMS;
constexpr int kTile = kBlock * kItems;       // 4096
constexpr int kWavesPerBlock = kBlock / kWave;  // 4
constexpr int kRadixBits = 8;
constexpr int kRadix = 1 << kRadixBits;     // 256

inline int ceil_div(long long a, long long b) { return (int)((a + b - 1) / b); }

// ============================== scan ===========================================

// Loads one tile of u32 (striped 16-byte loads) and leaves it in LDS.
__device__ __forceinline__ void load_tile_u32(const uint32_t* in, long long base, long long n,
                                              uint32_t* s_tile)
{
    const int t = threadIdx.x;
    if (base + kTile <= n && ((reinterpret_cast<uintptr_t>(in) & 15) == 0)) {
        const uint4* src = reinterpret_cast<const uint4*>(in + base);
#pragma unroll
        for (int j = 0; j < kItems / 4; j++) {
            uint4 v = src[j * kBlock + t];
            reinterpret_cast<uint4*>(s_tile)[j * kBlock + t] = v;
        }
    } else {
#pragma unroll
        for (int j = 0; j < kItems; j++) {
            long long i = base + j * kBlock + t;
            s_tile[j * kBlock + t] = (i < n) ? in[i] : 0u;
        }
    }
    __syncthreads();
}

__global__ __launch_bounds__(kBlock) void scan_reduce_kernel(const uint32_t* __restrict__ in, long long n,
                                                             uint32_t* __restrict__ tile_sums)
{
    __shared__ __attribute__((aligned(16))) uint32_t s_tile[kTile];
    __shared__ uint32_t s_wave[kWavesPerBlock];
    const long long base = (long long)blockIdx.x * kTile;
    load_tile_u32(in, base, n, s_tile);
    uint32_t sum = 0;
#pragma unroll
    for (int j = 0; j < kItems; j++) sum += s_tile[threadIdx.x * kItems + j];
    uint32_t total;
    block_exclusive_scan(sum, s_wave, &total);
    if (threadIdx.x == 0) tile_sums[blockIdx.x] = total;
}

// in and out may alias (in-place scan): each workgroup reads its whole tile before writing it.
// With `sums_raw` the workgroup adds up the tile sums before it itself (up to kOwnOffsetTiles
// tiles: a few loads per thread), which saves the separate scan of the tile sums; otherwise
// tile_offsets holds that exclusive scan.
constexpr int kOwnOffsetTiles = 4096;
__global__ __launch_bounds__(kBlock) void scan_downsweep_kernel(const uint32_t* in, long long n,
                                                                const uint32_t* __restrict__ tile_offsets,
                                                                int sums_raw, uint32_t* out)
{
    __shared__ __attribute__((aligned(16))) uint32_t s_tile[kTile];
    __shared__ uint32_t s_wave[kWavesPerBlock];
    const long long base = (long long)blockIdx.x * kTile;
    uint32_t tile_off;
    if (sums_raw) {
        uint32_t part = 0;
        for (int i = threadIdx.x; i < (int)blockIdx.x; i += kBlock) part += tile_offsets[i];
        block_exclusive_scan(part, s_wave, &tile_off);
    } else {
        tile_off = tile_offsets[blockIdx.x];
    }
    load_tile_u32(in, base, n, s_tile);
    uint32_t v[kItems];
    uint32_t sum = 0;
#pragma unroll
    for (int j = 0; j < kItems; j++) {
        v[j] = s_tile[threadIdx.x * kItems + j];
        sum += v[j];
    }
    uint32_t total;
    uint32_t run = block_exclusive_scan(sum, s_wave, &total) + tile_off;
#pragma unroll
    for (int j = 0; j < kItems; j++) {
        run += v[j];
        s_tile[threadIdx.x * kItems + j] = run;  // inclusive
    }
    __syncthreads();
    if (base + kTile <= n && ((reinterpret_cast<uintptr_t>(out) & 15) == 0)) {
        uint4* dst = reinterpret_cast<uint4*>(out + base);
#pragma unroll
        for (int j = 0; j < kItems / 4; j++) dst[j * kBlock + threadIdx.x] = reinterpret_cast<uint4*>(s_tile)[j * kBlock + threadIdx.x];
    } else {
#pragma unroll
        for (int j = 0; j < kItems; j++) {
            long long i = base + j * kBlock + threadIdx.x;
            if (i < n) out[i] = s_tile[j * kBlock + threadIdx.x];
        }
    }
}

// ============================== radix sort =====================================

template <typename K>
__device__ __forceinline__ uint32_t digit_of(K key, int shift, uint32_t mask)
{
    return (uint32_t)(key >> shift) & mask;
}

// Stable wave64 ranking of R rounds of items (round r, lane l = the wave's item r*64 + l,
// in input order).  cnt = this wave's 256 digit counters, zero on entry; on exit cnt[d] is
// the number of valid items with digit d and rank[r] the item's position among them.
// The lanes sharing a digit are found with one ballot per digit bit; bits outside `vary`
// are equal in every item (a caller's guarantee) and need none.  The lowest lane of each
// digit group bumps the counter (LDS ops of one wave retire in order, so the read precedes
// the write).
template <typename K, int R>
__device__ __forceinline__ void wave_rank(const K (&k)[R], const bool (&ok)[R], int shift, uint32_t mask,
                                          uint32_t* cnt, uint32_t (&rank)[R], uint32_t vary)
{
#pragma unroll
    for (int r = 0; r < R; r++) {
        const uint32_t d = digit_of(k[r], shift, mask);
        const uint64_t okb = __ballot(ok[r]);
        uint32_t mlo = (uint32_t)okb, mhi = (uint32_t)(okb >> 32);  // lanes with the same digit
#pragma unroll
        for (int b = 0; b < kRadixBits; b++) {
            if (!((vary >> b) & 1u)) continue;  // wave-uniform
            const uint32_t nb = ((d >> b) & 1u) - 1u;  // 0 when the bit is set, ~0 when clear
            const uint64_t bb = __ballot(nb == 0u);
            mlo &= nb ^ (uint32_t)bb;
            mhi &= nb ^ (uint32_t)(bb >> 32);
        }
        const uint32_t below = __builtin_amdgcn_mbcnt_hi(mhi, __builtin_amdgcn_mbcnt_lo(mlo, 0u));
        uint32_t old = 0;
        if (ok[r]) old = cnt[d];
        __builtin_amdgcn_wave_barrier();
        if (ok[r] && below == 0) cnt[d] = old + (uint32_t)(__popc(mlo) + __popc(mhi));
        __builtin_amdgcn_wave_barrier();
        rank[r] = old + below;
    }
}

// After every wave ranked (and a __syncthreads): thread d turns s_cnt[w][d] into the count of
// digit d in waves < w and returns the block's total for digit d.
__device__ __forceinline__ uint32_t digit_wave_prefix(uint32_t (*s_cnt)[kRadix])
{
    const int d = threadIdx.x;  // kBlock == kRadix
    uint32_t run = 0;
#pragma unroll
    for (int w = 0; w < kWavesPerBlock; w++) {
        const uint32_t c = s_cnt[w][d];
        s_cnt[w][d] = run;
        run += c;
    }
    return run;
}

// counts[d * ntiles + tile] = number of keys of tile `tile` whose digit is d.
template <typename K>
__global__ __launch_bounds__(kBlock) void radix_hist_kernel(const K* __restrict__ keys, long long n, int shift,
                                                            uint32_t mask, int ntiles, uint32_t* __restrict__ counts)
{
    __shared__ uint32_t s_hist[kWavesPerBlock][kRadix];
    const int t = threadIdx.x;
    const int wave = t / kWave;
    for (int i = t; i < kWavesPerBlock * kRadix; i += kBlock) (&s_hist[0][0])[i] = 0;
    __syncthreads();
    const long long base = (long long)blockIdx.x * kTile;
    K k[kItems];
    if (sizeof(K) == 8 && base + kTile <= n && (reinterpret_cast<uintptr_t>(keys) & 15) == 0) {
        // full tile: 16-byte loads, two keys each (the histogram does not care about item order)
        const ulonglong2* k2 = reinterpret_cast<const ulonglong2*>(keys + base);
#pragma unroll
        for (int j = 0; j < kItems / 2; j++) {
            const ulonglong2 p = k2[j * kBlock + t];
            k[2 * j] = (K)p.x;
            k[2 * j + 1] = (K)p.y;
        }
#pragma unroll
        for (int j = 0; j < kItems; j++) atomicAdd(&s_hist[wave][digit_of(k[j], shift, mask)], 1u);
    } else {
#pragma unroll
        for (int j = 0; j < kItems; j++) {
            long long i = base + j * kBlock + t;
            k[j] = (i < n) ? keys[i] : K(0);
        }
#pragma unroll
        for (int j = 0; j < kItems; j++) {
            long long i = base + j * kBlock + t;
            if (i < n) atomicAdd(&s_hist[wave][digit_of(k[j], shift, mask)], 1u);
        }
    }
    __syncthreads();
    for (int d = t; d < kRadix; d += kBlock) {
        uint32_t c = 0;
#pragma unroll
        for (int w = 0; w < kWavesPerBlock; w++) c += s_hist[w][d];
        counts[(long long)d * ntiles + blockIdx.x] = c;
    }
}

// One workgroup per digit: exclusive scan of counts[d][0..ntiles) in place; totals[d] = sum.
__global__ __launch_bounds__(kBlock) void radix_digit_scan_kernel(uint32_t* __restrict__ counts, int ntiles,
                                                                  uint32_t* __restrict__ totals)
{
    __shared__ uint32_t s_wave[kWavesPerBlock];
    uint32_t* row = counts + (long long)blockIdx.x * ntiles;
    uint32_t carry = 0;
    for (int base = 0; base < ntiles; base += kBlock * 4) {
        uint32_t v[4];
        uint32_t sum = 0;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            int i = base + threadIdx.x * 4 + j;
            v[j] = (i < ntiles) ? row[i] : 0u;
            sum += v[j];
        }
        uint32_t total;
        uint32_t pre = block_exclusive_scan(sum, s_wave, &total) + carry;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            int i = base + threadIdx.x * 4 + j;
            if (i < ntiles) row[i] = pre;
            pre += v[j];
        }
        carry += total;
    }
    if (threadIdx.x == 0) totals[blockIdx.x] = carry;
}

// Stable scatter of one tile.  LDS: one staging buffer of the tile's keys (values reuse it
// afterwards), per-wave digit counters -- 43 KB at 8 waves, 3 workgroups per CU.
// Global offsets: tile_prefix[d][tile] (per-digit exclusive scan over tiles) + exclusive scan
// of the digit totals.  (A single-pass decoupled look-back variant measured slower on MI355X:
// the chained tile-to-tile hand-off crosses the non-coherent per-XCD L2s at every hop.)
#ifndef HIDEGS_SCATTER_WAVES
#define HIDEGS_SCATTER_WAVES 8  // wave64s per scatter workgroup (the tile stays kTile pairs); 8 waves
                                // of 8 pairs each (66 VGPRs, 6 waves/SIMD) measured 2-3% faster than 4 of 16
#endif
constexpr int kSWaves = HIDEGS_SCATTER_WAVES;
constexpr int kSBlock = kSWaves * kWave;
constexpr int kSItems = kTile / kSBlock;  // pairs per thread
static_assert(kSBlock >= kRadix, "one thread per digit in the digit scans");

template <typename K>
__global__ __launch_bounds__(kSBlock) void radix_scatter_kernel(const K* __restrict__ keys_in,
                                                                const uint32_t* __restrict__ vals_in,
                                                                K* __restrict__ keys_out, uint32_t* __restrict__ vals_out,
                                                                long long n, int shift, uint32_t mask, int ntiles,
                                                                const uint32_t* __restrict__ tile_prefix,
                                                                const uint32_t* __restrict__ totals)
{
    __shared__ __attribute__((aligned(16))) K s_stage[kTile];  // keys by tile-local rank, then values
    __shared__ uint32_t s_cnt[kSWaves][kRadix];         // per-wave running counters
    __shared__ uint32_t s_start[kRadix];                // tile-local start of each digit run
    __shared__ uint32_t s_off[kRadix];                  // global position of tile-local position 0 of digit d
    __shared__ uint32_t s_wave[kSWaves];
    uint32_t* s_vals = reinterpret_cast<uint32_t*>(s_stage);

    const int t = threadIdx.x;
    const int lane = lane_id();
    const int wave = t / kWave;
    const bool digit_thread = t < kRadix;  // thread d owns digit d in the digit scans
    for (int i = t; i < kSWaves * kRadix; i += kSBlock) (&s_cnt[0][0])[i] = 0;
    const long long base = (long long)blockIdx.x * kTile;
    const long long seg = base + (long long)wave * (kSItems * kWave);  // this wave's items
    // this tile's global digit offsets, loaded now so their latency hides behind the ranking (digits
    // above `mask` read stale counts that no item uses)
    const uint32_t digit_total = digit_thread ? totals[t] : 0u;
    const uint32_t digit_prefix = digit_thread ? tile_prefix[(long long)t * ntiles + blockIdx.x] : 0u;

    K k[kSItems];
    uint32_t v[kSItems];
    bool ok[kSItems];
#pragma unroll
    for (int r = 0; r < kSItems; r++) {
        const long long i = seg + r * kWave + lane;
        ok[r] = i < n;
        k[r] = ok[r] ? keys_in[i] : K(0);
        v[r] = ok[r] ? vals_in[i] : 0u;
    }
    // the digits' global bases, scanned while the tile's loads are in flight (workgroup barriers
    // do not wait for global loads)
    uint32_t dummy;
    const uint32_t digit_base = block_exclusive_scan<kSWaves>(digit_total, s_wave, &dummy) + digit_prefix;
    uint32_t rank[kSItems];
    wave_rank<K, kSItems>(k, ok, shift, mask, s_cnt[wave], rank, mask);
    __syncthreads();

    uint32_t tile_count_d = 0;  // thread d: count of digit d in waves before each wave, in place
    if (digit_thread) {
#pragma unroll
        for (int w = 0; w < kSWaves; w++) {
            const uint32_t c = s_cnt[w][t];
            s_cnt[w][t] = tile_count_d;
            tile_count_d += c;
        }
    }
    const uint32_t start_d = block_exclusive_scan<kSWaves>(tile_count_d, s_wave, &dummy);
    if (digit_thread) {
        s_start[t] = start_d;
        s_off[t] = digit_base - start_d;
    }
    __syncthreads();
    uint32_t pos[kSItems];
#pragma unroll
    for (int r = 0; r < kSItems; r++) {
        if (ok[r]) {
            const uint32_t dd = digit_of(k[r], shift, mask);
            pos[r] = s_start[dd] + s_cnt[wave][dd] + rank[r];
            s_stage[pos[r]] = k[r];
        }
    }
    __syncthreads();
    const int count = (int)((n - base) < kTile ? (n - base) : kTile);
    uint32_t dst[kSItems];
#pragma unroll
    for (int j = 0; j < kSItems; j++) {  // keys, run-contiguous: position i = t + kSBlock j
        const int i = t + j * kSBlock;
        dst[j] = 0xffffffffu;
        if (i < count) {
            const K key = s_stage[i];
            dst[j] = s_off[digit_of(key, shift, mask)] + i;
            if (dst[j] < n) keys_out[dst[j]] = key;  // always true for consistent counts
        }
    }
    __syncthreads();  // every key read: the staging buffer takes the values
#pragma unroll
    for (int r = 0; r < kSItems; r++)
        if (ok[r]) s_vals[pos[r]] = v[r];
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kSItems; j++) {
        const int i = t + j * kSBlock;
        if (i < count && dst[j] < n) vals_out[dst[j]] = s_vals[i];
    }
}

// ============================== segmented sort =================================
//
// Keys whose bits [32, end_bit) are a small segment id -- the (tile | depth) keys of the
// binning stage -- are sorted in two stages with the same result as the LSD sort over
// [0, end_bit): (1) the LSD passes above over [32, end_bit) only, which partition the pairs
// stably by segment; (2) one workgroup per segment sorts it stably by the low 32 bits.
// Global traffic drops from 6 LSD passes to 2 plus one read/write of every pair.
//
// Stage (2) has three forms, chosen per segment (block-uniform):
//   bucket form  (<= kSegCap pairs, the common case): bucket by the top 10 varying low-key bits,
//                exact rank inside each bucket, LDS-staged in-place stores -- see segment_sort_kernel;
//   LSD form     (a bucket over kMaxBucket pairs: crowded depths): 8-bit LDS LSD passes over the
//                varying bits, two runs of <= kSegRun merged by rank;
//   global form  (> kSegCap pairs: a hot tile): 4 LSD passes through global memory.
#ifndef HIDEGS_SEG_BITS
#define HIDEGS_SEG_BITS 32  // experiments only (tools/build_variant.py): fewer bits give wrong orders
#endif
constexpr int kSegRun = 1024;            // pairs per LDS-sorted run
constexpr int kSegCap = 2 * kSegRun;     // largest segment sorted by segment_sort_kernel
constexpr int kRunItems = kSegRun / kBlock;  // run items per thread (rounds of 64 per wave)
constexpr int kSegItems = kSegCap / kBlock;  // segment items per thread

// LDS of one workgroup: two (low key, index-in-segment) buffers of one run plus ranking state.
struct SegShared {
    uint32_t k[2][kSegRun];
    uint16_t i[2][kSegRun];  // index in segment (< kSegCap)
    uint32_t cnt[kWavesPerBlock][kRadix];
    uint32_t start[kRadix];
    uint32_t wave[kWavesPerBlock];
};

// Stable LSD sort of the n <= kSegRun (k, i) pairs in buffer 0 by the key bits set in `diff`
// (8-bit digits; a digit that is constant over the segment is skipped).  Returns the buffer
// holding the result.  Wave w ranks items [w*C, w*C + C) in (round, lane) order.
__device__ __forceinline__ int lds_radix_sort(SegShared& sh, const uint32_t n, const uint32_t diff)
{
    const int t = threadIdx.x, lane = lane_id(), wave = t / kWave;
    const uint32_t C = ((n + kBlock - 1) / kBlock) * kWave;
    const int rounds = (int)(C / kWave);
    const uint32_t w0 = wave * C;
    int cur = 0;
    for (int shift = 0; shift < HIDEGS_SEG_BITS; shift += kRadixBits) {
        const uint32_t vary = (diff >> shift) & (kRadix - 1);
        if (vary == 0) continue;  // digit constant over the segment (block-uniform)
        for (int i = t; i < kWavesPerBlock * kRadix; i += kBlock) (&sh.cnt[0][0])[i] = 0;
        __syncthreads();
        uint32_t k[kRunItems], id[kRunItems], rank[kRunItems];
        bool ok[kRunItems];
#pragma unroll
        for (int q = 0; q < kRunItems; q++) {
            const uint32_t i = w0 + q * kWave + lane;
            ok[q] = q < rounds && i < n;
            k[q] = ok[q] ? sh.k[cur][i] : 0u;
            id[q] = ok[q] ? sh.i[cur][i] : 0u;
        }
        if (rounds == kRunItems) {
            wave_rank<uint32_t, kRunItems>(k, ok, shift, kRadix - 1, sh.cnt[wave], rank, vary);
        } else {  // rounds past `rounds` hold no item: skip their ranking (block-uniform)
#pragma unroll
            for (int q = 0; q < kRunItems; q++) {
                if (q < rounds) {
                    uint32_t kk[1] = {k[q]}, rr[1];
                    bool oo[1] = {ok[q]};
                    wave_rank<uint32_t, 1>(kk, oo, shift, kRadix - 1, sh.cnt[wave], rr, vary);
                    rank[q] = rr[0];
                }
            }
        }
        __syncthreads();
        const uint32_t tot = digit_wave_prefix(sh.cnt);
        uint32_t dummy;
        sh.start[t] = block_exclusive_scan(tot, sh.wave, &dummy);
        __syncthreads();
#pragma unroll
        for (int q = 0; q < kRunItems; q++) {
            if (ok[q]) {
                const uint32_t dd = digit_of(k[q], shift, kRadix - 1);
                const uint32_t pos = sh.start[dd] + sh.cnt[wave][dd] + rank[q];
                sh.k[cur ^ 1][pos] = k[q];
                sh.i[cur ^ 1][pos] = id[q];
            }
        }
        __syncthreads();
        cur ^= 1;
    }
    return cur;
}

// Number of the n sorted keys in a[] that are < key (or <= key when `inclusive`).
__device__ __forceinline__ uint32_t lds_rank(const uint32_t* a, uint32_t n, uint32_t key, bool inclusive)
{
    uint32_t lo = 0, len = n;
    while (len > 0) {
        const uint32_t half = len >> 1;
        const uint32_t v = a[lo + half];
        const bool go_right = inclusive ? (v <= key) : (v < key);
        lo = go_right ? lo + half + 1 : lo;
        len = go_right ? len - half - 1 : half;
    }
    return lo;
}

__device__ __forceinline__ void wave_and_or(uint32_t& a, uint32_t& o)
{
#pragma unroll
    for (int sh = 32; sh >= 1; sh >>= 1) {
        a &= __shfl_xor(a, sh, kWave);
        o |= __shfl_xor(o, sh, kWave);
    }
}

// LDS of the oversized-segment form.
struct BigShared {
    uint32_t cnt[kWavesPerBlock][kRadix];
    uint32_t hist[kRadix];
    uint32_t run[kRadix];  // running start of each digit within the segment
    uint32_t wave[kWavesPerBlock];
};

// A segment of more than kSegCap pairs (a hot tile): 4 stable LSD passes over the low 32 bits
// through global memory (keys/vals <-> alt within the segment's range), 2048 items per step (8 per
// thread keeps the kernel inside the bucket form's register budget), by the segment's own workgroup.
constexpr int kBigItems = 8;
__device__ __forceinline__ void segment_sort_global(uint64_t* __restrict__ keys, uint32_t* __restrict__ vals,
                                                    uint64_t* __restrict__ alt_k, uint32_t* __restrict__ alt_v,
                                                    const uint32_t begin, const uint32_t m, BigShared& sh)
{
    const int t = threadIdx.x;
    const int lane = lane_id();
    const int wave = t / kWave;
    for (int pass = 0; pass < 4; pass++) {
        const int shift = pass * kRadixBits;
        const uint64_t* sk = (pass & 1) ? alt_k : keys;
        const uint32_t* sv = (pass & 1) ? alt_v : vals;
        uint64_t* dk = (pass & 1) ? keys : alt_k;
        uint32_t* dv = (pass & 1) ? vals : alt_v;
        sh.hist[t] = 0;
        __syncthreads();
        for (uint32_t i = t; i < m; i += kBlock) atomicAdd(&sh.hist[digit_of(sk[begin + i], shift, kRadix - 1)], 1u);
        __syncthreads();
        uint32_t dummy;
        sh.run[t] = begin + block_exclusive_scan(sh.hist[t], sh.wave, &dummy);
        __syncthreads();
        for (uint32_t c0 = 0; c0 < m; c0 += (kBigItems * kBlock)) {
            for (int i = t; i < kWavesPerBlock * kRadix; i += kBlock) (&sh.cnt[0][0])[i] = 0;
            __syncthreads();
            uint64_t k[kBigItems];
            uint32_t v[kBigItems];
            bool ok[kBigItems];
            uint32_t rank[kBigItems];
            const uint32_t w0 = c0 + wave * (kBigItems * kWave);
#pragma unroll
            for (int q = 0; q < kBigItems; q++) {
                const uint32_t i = w0 + q * kWave + lane;
                ok[q] = i < m;
                k[q] = ok[q] ? sk[begin + i] : 0ull;
                v[q] = ok[q] ? sv[begin + i] : 0u;
            }
            wave_rank<uint64_t, kBigItems>(k, ok, shift, kRadix - 1, sh.cnt[wave], rank, kRadix - 1);
            __syncthreads();
            const uint32_t tot = digit_wave_prefix(sh.cnt);
            __syncthreads();
#pragma unroll
            for (int q = 0; q < kBigItems; q++) {
                if (ok[q]) {
                    const uint32_t dd = digit_of(k[q], shift, kRadix - 1);
                    const uint32_t dst = sh.run[dd] + sh.cnt[wave][dd] + rank[q];
                    if (dst < begin + m) {  // always, for a consistent segment; never outside it
                        dk[dst] = k[q];
                        dv[dst] = v[q];
                    }
                }
            }
            __syncthreads();
            sh.run[t] += tot;
            __syncthreads();
        }
    }
}

// LSD form of the per-segment sort (the fallback of segment_sort_kernel for segments whose
// depth bits crowd into a few buckets): run A (<= kSegRun) sorted in LDS, run B parked in registers
// and sorted after it, the two merged by rank; every item's high key half and value gathered by
// its index in the segment and written in place.  `diff` = the low key bits that vary.
__device__ __forceinline__ void segment_sort_lsd(uint64_t* __restrict__ keys, uint32_t* __restrict__ vals,
                                                 const uint32_t begin, const uint32_t m, const uint32_t diff,
                                                 SegShared& sh)
{
    const int t = threadIdx.x;
    const uint32_t na = m < (uint32_t)kSegRun ? m : (uint32_t)kSegRun, nb = m - na;
    uint32_t bk[kRunItems];
#pragma unroll
    for (int q = 0; q < kRunItems; q++) {
        const uint32_t i = t + q * kBlock;
        if (i < na) {
            sh.k[0][i] = (uint32_t)keys[begin + i];
            sh.i[0][i] = i;
        }
        bk[q] = i < nb ? (uint32_t)keys[begin + kSegRun + i] : 0u;
    }
    __syncthreads();
    const int ca = lds_radix_sort(sh, na, diff);

    // final (position, low key, index) of this thread's items: position t + 256 q
    uint32_t fk[kSegItems], fi[kSegItems], fp[kSegItems];
    bool fok[kSegItems];
    if (nb == 0) {
#pragma unroll
        for (int q = 0; q < kSegItems; q++) {
            const uint32_t i = t + q * kBlock;
            fok[q] = q < kRunItems && i < na;
            fp[q] = i;
            fk[q] = fok[q] ? sh.k[ca][i] : 0u;
            fi[q] = fok[q] ? sh.i[ca][i] : 0u;
        }
    } else {
        // park sorted run A in registers, sort run B, then merge by rank
        uint32_t ak[kRunItems], ai[kRunItems];
#pragma unroll
        for (int q = 0; q < kRunItems; q++) {
            ak[q] = sh.k[ca][t + q * kBlock];
            ai[q] = sh.i[ca][t + q * kBlock];
        }
        __syncthreads();
#pragma unroll
        for (int q = 0; q < kRunItems; q++) {
            const uint32_t i = t + q * kBlock;
            if (i < nb) {
                sh.k[0][i] = bk[q];
                sh.i[0][i] = kSegRun + i;
            }
        }
        __syncthreads();
        const int cb = lds_radix_sort(sh, nb, diff);
#pragma unroll
        for (int q = 0; q < kRunItems; q++) {
            sh.k[cb ^ 1][t + q * kBlock] = ak[q];
            sh.i[cb ^ 1][t + q * kBlock] = ai[q];
        }
        __syncthreads();
        // stable merge: an A item precedes every B item with an equal key (A indices are smaller)
#pragma unroll
        for (int q = 0; q < kRunItems; q++) {
            const uint32_t i = t + q * kBlock;
            fok[q] = true;
            fk[q] = ak[q];
            fi[q] = ai[q];
            fp[q] = i + lds_rank(sh.k[cb], nb, ak[q], false);
            const uint32_t j = i;
            fok[kRunItems + q] = j < nb;
            fk[kRunItems + q] = fok[kRunItems + q] ? sh.k[cb][j] : 0u;
            fi[kRunItems + q] = fok[kRunItems + q] ? sh.i[cb][j] : 0u;
            fp[kRunItems + q] = fok[kRunItems + q] ? j + lds_rank(sh.k[cb ^ 1], kSegRun, fk[kRunItems + q], true) : 0u;
        }
    }
    // gather each item's high key half and value by its index in the segment (the segment is
    // unmodified until every workgroup thread has gathered), then write in place
    uint32_t hi[kSegItems], v[kSegItems];
#pragma unroll
    for (int q = 0; q < kSegItems; q++) {
        if (fok[q]) {
            hi[q] = (uint32_t)(keys[begin + fi[q]] >> 32);
            v[q] = vals[begin + fi[q]];
        }
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < kSegItems; q++) {
        if (fok[q]) {
            keys[begin + fp[q]] = ((uint64_t)hi[q] << 32) | fk[q];
            vals[begin + fp[q]] = v[q];
        }
    }
}

// Bucket form (the common case).  The segment's top kBucketBits varying low-key bits pick a
// bucket; a counting pass (LDS atomics, any order) gives every bucket its place, and each item's
// place inside its bucket is its exact rank there by (key bits below the bucket digit, index in
// segment) -- one 32-bit compare per bucket member (the two fields fit 32 bits when the top
// varying bit is <= 30, as for the float bits of positive depths; otherwise the LSD form runs).  Equal keys are therefore ordered by their input
// index, which is the stable order; no ballots and three workgroup barriers in place of the LSD
// form's four per 8-bit pass.  Each item's key and value stay in registers from the load to the
// in-place store (every load of the segment precedes the first barrier).
constexpr int kBucketBits = 10;
constexpr int kBuckets = 1 << kBucketBits;
constexpr int kMaxBucket = 128;  // a fuller bucket sends the segment to the LSD form
constexpr int kIndexBits = 11;   // index in segment < kSegCap
#ifndef HIDEGS_SEG_WAVES
#define HIDEGS_SEG_WAVES 7  // waves per SIMD the register budget is set for (17 KB of LDS allows 9)
#endif

static_assert(kSegCap <= (1 << kIndexBits), "segment index must fit its field");

struct BucketShared {
    uint32_t comb[kSegCap];   // (key bits below the digit << kIndexBits) | index, grouped by bucket
    uint32_t start[kBuckets];
    uint32_t fill[kBuckets];  // histogram, then the running fill pointer (= bucket end after filling)
};
// after ranking, the whole struct stages the sorted segment: keys (u64) then values (u32) when
// they fit together (<= kSegRun pairs), else keys and values one after the other
static_assert(sizeof(BucketShared) >= kSegCap * sizeof(uint64_t), "staging of the keys");
static_assert(sizeof(BucketShared) >= kSegRun * (sizeof(uint64_t) + sizeof(uint32_t)), "staging of a run");

union SegLds {
    SegShared lsd;
    BucketShared bucket;
    BigShared big;
};

// Workgroup b sorts segment b in place by the low 32 key bits: the bucket form, its LSD fallback
// for crowded buckets, or (more than kSegCap pairs) the global form through alt_k / alt_v.
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(HIDEGS_SEG_WAVES))) void segment_sort_kernel(
    uint64_t* __restrict__ keys, uint32_t* __restrict__ vals, const uint2* __restrict__ ranges,
    uint64_t* __restrict__ alt_k, uint32_t* __restrict__ alt_v)
{
    __shared__ __attribute__((aligned(16))) SegLds lds;
    __shared__ uint32_t s_and[kWavesPerBlock], s_or[kWavesPerBlock], s_max[kWavesPerBlock];
    const int t = threadIdx.x, lane = lane_id(), wave = t / kWave;
    const uint2 r = ranges[blockIdx.x];
    const uint32_t begin = r.x, m = r.y - r.x;
    if (r.y <= r.x + 1) return;  // absent or single pair: already in place
    if (m > (uint32_t)kSegCap) {
        segment_sort_global(keys, vals, alt_k, alt_v, begin, m, lds.big);
        return;
    }
    uint64_t k[kSegItems];
    uint32_t v[kSegItems];
    uint32_t a = 0xffffffffu, o = 0;
#pragma unroll
    for (int q = 0; q < kSegItems; q++) {
        const uint32_t i = t + q * kBlock;
        if (i < m) {
            k[q] = keys[begin + i];
            v[q] = vals[begin + i];
            a &= (uint32_t)k[q];
            o |= (uint32_t)k[q];
        }
    }
    BucketShared& sh = lds.bucket;
    for (int i = t; i < kBuckets; i += kBlock) sh.fill[i] = 0u;
    wave_and_or(a, o);
    if (lane == 0) {
        s_and[wave] = a;
        s_or[wave] = o;
    }
    __syncthreads();
    uint32_t diff;
    {
        uint32_t aa = 0xffffffffu, oo = 0;
#pragma unroll
        for (int w = 0; w < kWavesPerBlock; w++) {
            aa &= s_and[w];
            oo |= s_or[w];
        }
        diff = aa ^ oo;  // low key bits that vary over the segment
    }
    if (diff == 0) return;  // equal low keys: the input order is the stable order
    const int top = 31 - __builtin_clz(diff);
    const int dbits = top + 1 < kBucketBits ? top + 1 : kBucketBits;
    const int shift = top + 1 - dbits;
    const uint32_t dmask = (1u << dbits) - 1u;
    const uint32_t lowmask = (uint32_t)((1ull << shift) - 1ull);

    // 1. bucket histogram
#pragma unroll
    for (int q = 0; q < kSegItems; q++)
        if (t + q * kBlock < m) atomicAdd(&sh.fill[((uint32_t)k[q] >> shift) & dmask], 1u);
    __syncthreads();
    // 2. bucket starts (exclusive scan, 4 buckets per thread) and the fullest bucket
    uint32_t c[kBuckets / kBlock], sum = 0, mx = 0;
#pragma unroll
    for (int j = 0; j < kBuckets / kBlock; j++) {
        c[j] = sh.fill[t * (kBuckets / kBlock) + j];
        sum += c[j];
        mx = c[j] > mx ? c[j] : mx;
    }
    uint32_t dummy;
    uint32_t pre = block_exclusive_scan(sum, s_max, &dummy);  // its barriers order the reads above
#pragma unroll
    for (int s = 32; s >= 1; s >>= 1) {
        const uint32_t y = __shfl_xor(mx, s, kWave);
        mx = y > mx ? y : mx;
    }
    if (lane == 0) s_and[wave] = mx;
#pragma unroll
    for (int j = 0; j < kBuckets / kBlock; j++) {
        sh.start[t * (kBuckets / kBlock) + j] = pre;
        sh.fill[t * (kBuckets / kBlock) + j] = pre;
        pre += c[j];
    }
    __syncthreads();
    uint32_t fullest = 0;
#pragma unroll
    for (int w = 0; w < kWavesPerBlock; w++) fullest = s_and[w] > fullest ? s_and[w] : fullest;
    if (fullest > (uint32_t)kMaxBucket || shift + kIndexBits > 32) {  // crowded depths, or fields too
        // wide for 32 bits: the LSD form (block-uniform branch)
        __syncthreads();
        segment_sort_lsd(keys, vals, begin, m, diff, lds.lsd);
        return;
    }
    // 3. fill the buckets in any order
    uint32_t me[kSegItems];
    uint32_t bucket[kSegItems];
#pragma unroll
    for (int q = 0; q < kSegItems; q++) {
        const uint32_t i = t + q * kBlock;
        if (i < m) {
            bucket[q] = ((uint32_t)k[q] >> shift) & dmask;
            me[q] = (((uint32_t)k[q] & lowmask) << kIndexBits) | i;
            sh.comb[atomicAdd(&sh.fill[bucket[q]], 1u)] = me[q];
        }
    }
    __syncthreads();
    // 4. exact rank inside the bucket
    uint32_t pos[kSegItems];
#pragma unroll
    for (int q = 0; q < kSegItems; q++) {
        if (t + q * kBlock < m) {
            const uint32_t s0 = sh.start[bucket[q]], e0 = sh.fill[bucket[q]];
            uint32_t rank = 0;
            for (uint32_t j = s0; j < e0; j++) rank += sh.comb[j] < me[q] ? 1u : 0u;
            pos[q] = s0 + rank;
        }
    }
    // 5. stage (key, value) by final position in LDS, then store the segment contiguously (stores
    //    straight from registers scatter 8- and 4-byte writes over the segment: 78 -> 50 us at 8M pairs)
    __syncthreads();
    uint64_t* stage_k = reinterpret_cast<uint64_t*>(&sh);
    uint32_t* stage_v = reinterpret_cast<uint32_t*>(stage_k + kSegRun);
    const bool together = m <= (uint32_t)kSegRun;  // block-uniform
#pragma unroll
    for (int q = 0; q < kSegItems; q++) {
        if (t + q * kBlock < m) {
            stage_k[pos[q]] = k[q];
            if (together) stage_v[pos[q]] = v[q];
        }
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < kSegItems; q++) {
        const uint32_t i = t + q * kBlock;
        if (i < m) {
            keys[begin + i] = stage_k[i];
            if (together) vals[begin + i] = stage_v[i];
        }
    }
    if (together) return;
    __syncthreads();
    stage_v = reinterpret_cast<uint32_t*>(&sh);
#pragma unroll
    for (int q = 0; q < kSegItems; q++)
        if (t + q * kBlock < m) stage_v[pos[q]] = v[q];
    __syncthreads();
#pragma unroll
    for (int q = 0; q < kSegItems; q++) {
        const uint32_t i = t + q * kBlock;
        if (i < m) vals[begin + i] = stage_v[i];
    }
}

// ============================== tile ranges ====================================

// Tile ids >= num_tiles violate the caller contract; their entries are skipped rather
// than written out of bounds.
// tile = (key >> 32) & tile_mask (the public entry point passes all ones; the segmented sort
// masks to its segment bits).
// ranges[tile] = [first, last + 1) of the tile's keys (tile = (key >> 32) & tile_mask); tiles
// >= num_tiles are skipped.  Each thread checks 4 consecutive keys (two 16-byte loads) and the
// key before them; only the rare boundaries write.
constexpr int kRangeKeys = 4;
__global__ __launch_bounds__(kBlock) void identify_ranges_kernel(const uint64_t* __restrict__ keys, long long n,
                                                                 uint2* __restrict__ ranges, uint32_t num_tiles,
                                                                 uint32_t tile_mask)
{
    const long long i0 = ((long long)blockIdx.x * kBlock + threadIdx.x) * kRangeKeys;
    if (i0 >= n) return;
    uint32_t tile[kRangeKeys];
    if (i0 + kRangeKeys <= n && (reinterpret_cast<uintptr_t>(keys) & 15) == 0) {
        const ulonglong2* k2 = reinterpret_cast<const ulonglong2*>(keys + i0);
        const ulonglong2 a = k2[0], b = k2[1];
        tile[0] = (uint32_t)(a.x >> 32) & tile_mask;
        tile[1] = (uint32_t)(a.y >> 32) & tile_mask;
        tile[2] = (uint32_t)(b.x >> 32) & tile_mask;
        tile[3] = (uint32_t)(b.y >> 32) & tile_mask;
    } else {
#pragma unroll
        for (int j = 0; j < kRangeKeys; j++) tile[j] = i0 + j < n ? (uint32_t)(keys[i0 + j] >> 32) & tile_mask : 0u;
    }
    uint32_t prev = i0 == 0 ? 0u : (uint32_t)(keys[i0 - 1] >> 32) & tile_mask;
#pragma unroll
    for (int j = 0; j < kRangeKeys; j++) {
        const long long i = i0 + j;
        if (i >= n) break;
        const uint32_t cur = tile[j];
        if (i == 0) {  // the reference leaves .y of a single key's tile unset (n == 1)
            if (cur < num_tiles) ranges[cur].x = 0;
        } else {
            if (cur != prev) {
                if (prev < num_tiles) ranges[prev].y = (uint32_t)i;
                if (cur < num_tiles) ranges[cur].x = (uint32_t)i;
            }
            if (i == n - 1 && cur < num_tiles) ranges[cur].y = (uint32_t)n;
        }
        prev = cur;
    }
}

// ============================== host side ======================================

size_t scan_scratch(long long n)
{
    const int nt = ceil_div(n, kTile);
    return align_up((size_t)nt * sizeof(uint32_t)) + align_up(sizeof(uint32_t));
}

constexpr int kMaxSegmentBits = 16;        // segmented path: at most 65536 segments
constexpr long long kSegmentedMinN = 65536;  // below this the plain LSD passes are cheaper
constexpr long long kSegmentedMinAvg = 64;   // pairs per segment on average, else the plain passes: one
                                             // workgroup per ~30-pair segment (distCUDA2's 48-bit Morton
                                             // keys of 2M points) costs more than the 4 low-digit passes

template <typename K>
size_t sort_scratch(long long n)
{
    const int nt = ceil_div(n, kTile);
    size_t b = align_up((size_t)n * sizeof(K)) + align_up((size_t)n * sizeof(uint32_t)) +
               align_up((size_t)kRadix * nt * sizeof(uint32_t)) + align_up(kRadix * sizeof(uint32_t));
    if (sizeof(K) == 8)  // segmented path: the segment ranges
        b += align_up(sizeof(uint2) << kMaxSegmentBits);
    return b;
}

__global__ void identify_ranges_kernel(const uint64_t* __restrict__ keys, long long n, uint2* __restrict__ ranges,
                                       uint32_t num_tiles, uint32_t tile_mask);

// ranges_out (num_tiles entries) set: the tile ranges of the sorted keys are written too, with
// identify_tile_ranges' semantics; the caller guarantees key >> 32 < num_tiles.
template <typename K>
int sort_pairs(void* scratch, size_t scratch_bytes, const K* keys_in, K* keys_out, const uint32_t* vals_in,
               uint32_t* vals_out, long long n, int begin_bit, int end_bit, hipStream_t stream, const char* what,
               uint2* ranges_out = nullptr, int num_tiles = 0)
{
    const int kbits = (int)(8 * sizeof(K));
    if (n < 0 || begin_bit < 0 || end_bit > kbits || begin_bit > end_bit)
        return fail(HIDEGS_E_ARG, std::string(what) + ": bad size or bit range");
    if (n > 0x7fffffffLL) return fail(HIDEGS_E_ARG, std::string(what) + ": more than 2^31-1 items");
    if (n == 0)
        return ranges_out ? identify_tile_ranges(nullptr, 0, reinterpret_cast<uint32_t*>(ranges_out), num_tiles, stream)
                          : 0;
    if (!keys_in || !keys_out || !vals_in || !vals_out)
        return fail(HIDEGS_E_ARG, std::string(what) + ": NULL key/value pointer");
    if (keys_out == keys_in || vals_out == vals_in)
        return fail(HIDEGS_E_ARG, std::string(what) + ": in-place sorting is not supported");
    if (!scratch || scratch_bytes < sort_scratch<K>(n))
        return fail(HIDEGS_E_ARG, std::string(what) + ": scratch buffer too small");

    const int passes = (end_bit - begin_bit + kRadixBits - 1) / kRadixBits;
    if (passes == 0) {
        if (hipMemcpyAsync(keys_out, keys_in, n * sizeof(K), hipMemcpyDeviceToDevice, stream) != hipSuccess ||
            hipMemcpyAsync(vals_out, vals_in, n * sizeof(uint32_t), hipMemcpyDeviceToDevice, stream) != hipSuccess)
            return fail(HIDEGS_E_HIP, std::string(what) + ": copy failed");
        return ranges_out ? identify_tile_ranges(reinterpret_cast<const uint64_t*>(keys_out), n,
                                                 reinterpret_cast<uint32_t*>(ranges_out), num_tiles, stream)
                          : 0;
    }
    const int nt = ceil_div(n, kTile);
    Carver c(scratch);
    K* alt_k = c.take<K>(n);
    uint32_t* alt_v = c.take<uint32_t>(n);
    uint32_t* counts = c.take<uint32_t>((size_t)kRadix * nt);
    uint32_t* totals = c.take<uint32_t>(kRadix);

    // (tile | depth)-shaped sort: LSD over the segment bits only, then per-segment LDS sorts
    const bool segmented = sizeof(K) == 8 && begin_bit == 0 && end_bit > 32 && end_bit - 32 <= kMaxSegmentBits &&
                           n >= kSegmentedMinN && n >= (kSegmentedMinAvg << (end_bit - 32));
    const int lo_bit = segmented ? 32 : begin_bit;
    const int lsd_passes = segmented ? (end_bit - 32 + kRadixBits - 1) / kRadixBits : passes;

    const K* src_k = keys_in;
    const uint32_t* src_v = vals_in;
    // balanced digit widths (13 tile bits: 7 + 6, not 8 + 5): fewer buckets per pass mean
    // longer runs per bucket in each tile's scatter, i.e. fuller write lines
    const int span = end_bit - lo_bit;
    int shift = lo_bit;
    for (int p = 0; p < lsd_passes; p++) {
        const int bits = (span * (p + 1)) / lsd_passes - (span * p) / lsd_passes;
        const uint32_t mask = (1u << bits) - 1u;
        const bool to_out = ((lsd_passes - 1 - p) % 2) == 0;
        K* dk = to_out ? keys_out : alt_k;
        uint32_t* dv = to_out ? vals_out : alt_v;
        HIDEGS_LAUNCH((sizeof(K) == 8 ? "radix_hist_u64" : "radix_hist_u32"), radix_hist_kernel<K>, dim3(nt),
                      dim3(kBlock), 0, stream, src_k, n, shift, mask, nt, counts);
        // digits above `mask` never occur: their (stale) totals only follow the used digits in the
        // scatter's exclusive scan, and their counts are never read
        HIDEGS_LAUNCH("radix_digit_scan", radix_digit_scan_kernel, dim3(mask + 1), dim3(kBlock), 0, stream, counts,
                      nt, totals);
        HIDEGS_LAUNCH((sizeof(K) == 8 ? "radix_scatter_u64" : "radix_scatter_u32"), radix_scatter_kernel<K>,
                      dim3(nt), dim3(kSBlock), 0, stream, src_k, src_v, dk, dv, n, shift, mask, nt, counts, totals);
        src_k = dk;
        src_v = dv;
        shift += bits;
    }
    if (segmented) {
        // the segments' ranges; with ranges_out they are the caller's tile ranges (tile ids
        // < num_tiles <= 2^(end_bit-32) leave no bits above end_bit, so segment == tile)
        int nseg = 1 << (end_bit - 32);
        uint2* ranges = c.take<uint2>((size_t)1 << kMaxSegmentBits);
        uint32_t tile_mask = (uint32_t)(nseg - 1);
        if (ranges_out) {
            ranges = ranges_out;
            nseg = num_tiles;
            tile_mask = 0xffffffffu;
        }
        uint64_t* ko = reinterpret_cast<uint64_t*>(keys_out);
        if (hipMemsetAsync(ranges, 0, sizeof(uint2) * nseg, stream) != hipSuccess)
            return fail(HIDEGS_E_HIP, std::string(what) + ": memset failed");
        HIDEGS_LAUNCH("segment_ranges", identify_ranges_kernel, dim3(ceil_div(n, kBlock * kRangeKeys)), dim3(kBlock), 0, stream,
                      (const uint64_t*)ko, n, ranges, (uint32_t)nseg, tile_mask);
        HIDEGS_LAUNCH("segment_sort", segment_sort_kernel, dim3(nseg), dim3(kBlock), 0, stream, ko, vals_out, ranges,
                      reinterpret_cast<uint64_t*>(alt_k), alt_v);
    } else if (ranges_out) {
        if (int rc = check_launch(what, stream, 0)) return rc;
        return identify_tile_ranges(reinterpret_cast<const uint64_t*>(keys_out), n,
                                    reinterpret_cast<uint32_t*>(ranges_out), num_tiles, stream);
    }
    return check_launch(what, stream, 0);
}

}  // namespace

int inclusive_scan_u32(void* scratch, size_t scratch_bytes, const uint32_t* in, uint32_t* out, long long n,
                       hipStream_t stream)
{
    if (n < 0) return fail(HIDEGS_E_ARG, "inclusive_scan_u32: negative size");
    if (n == 0) return 0;
    if (!in || !out) return fail(HIDEGS_E_ARG, "inclusive_scan_u32: NULL pointer");
    if (!scratch || scratch_bytes < scan_scratch(n)) return fail(HIDEGS_E_ARG, "inclusive_scan_u32: scratch too small");
    const int nt = ceil_div(n, kTile);
    Carver c(scratch);
    uint32_t* sums = c.take<uint32_t>(nt);
    HIDEGS_LAUNCH("scan_reduce", scan_reduce_kernel, dim3(nt), dim3(kBlock), 0, stream, in, n, sums);
    const int own = nt <= kOwnOffsetTiles;
    if (!own)
        HIDEGS_LAUNCH("scan_small", scan_small_kernel, dim3(1), dim3(kBlock), 0, stream, sums, nt, (uint32_t*)nullptr);
    HIDEGS_LAUNCH("scan_downsweep", scan_downsweep_kernel, dim3(nt), dim3(kBlock), 0, stream, in, n, sums, own, out);
    return check_launch("inclusive_scan_u32", stream, 0);
}

size_t inclusive_scan_scratch(long long n) { return scan_scratch(n); }
size_t sort_u64_scratch(long long n) { return sort_scratch<uint64_t>(n); }
size_t sort_u32_scratch(long long n) { return sort_scratch<uint32_t>(n); }

int sort_pairs_u64(void* scratch, size_t bytes, const uint64_t* ki, uint64_t* ko, const uint32_t* vi, uint32_t* vo,
                   long long n, int b, int e, hipStream_t s)
{
    return sort_pairs<uint64_t>(scratch, bytes, ki, ko, vi, vo, n, b, e, s, "sort_pairs_u64");
}
int sort_pairs_u32(void* scratch, size_t bytes, const uint32_t* ki, uint32_t* ko, const uint32_t* vi, uint32_t* vo,
                   long long n, int b, int e, hipStream_t s)
{
    return sort_pairs<uint32_t>(scratch, bytes, ki, ko, vi, vo, n, b, e, s, "sort_pairs_u32");
}

int sort_tile_pairs(void* scratch, size_t bytes, const uint64_t* ki, uint64_t* ko, const uint32_t* vi, uint32_t* vo,
                    long long n, int num_tiles, uint32_t* ranges, hipStream_t s)
{
    if (num_tiles < 1) return fail(HIDEGS_E_ARG, "sort_tile_pairs: num_tiles must be >= 1");
    if (!ranges) return fail(HIDEGS_E_ARG, "sort_tile_pairs: NULL ranges");
    const int end = 32 + (int)(32u - (uint32_t)__builtin_clz((uint32_t)num_tiles | 1u));  // 32 + getHigherMsb
    if (end > 64) return fail(HIDEGS_E_ARG, "sort_tile_pairs: too many tiles");
    return sort_pairs<uint64_t>(scratch, bytes, ki, ko, vi, vo, n, 0, end, s, "sort_tile_pairs",
                                reinterpret_cast<uint2*>(ranges), num_tiles);
}

int identify_tile_ranges(const uint64_t* keys, long long n, uint32_t* ranges, int num_tiles, hipStream_t stream)
{
    if (n < 0 || num_tiles < 0) return fail(HIDEGS_E_ARG, "identify_tile_ranges: negative size");
    if (num_tiles > 0 && !ranges) return fail(HIDEGS_E_ARG, "identify_tile_ranges: NULL ranges");
    if (num_tiles > 0 && hipMemsetAsync(ranges, 0, (size_t)num_tiles * 2 * sizeof(uint32_t), stream) != hipSuccess)
        return fail(HIDEGS_E_HIP, "identify_tile_ranges: memset failed");
    if (n == 0) return check_launch("identify_tile_ranges", stream, 0);
    if (!keys) return fail(HIDEGS_E_ARG, "identify_tile_ranges: NULL keys");
    HIDEGS_LAUNCH("identify_ranges", identify_ranges_kernel, dim3(ceil_div(n, kBlock * kRangeKeys)), dim3(kBlock), 0, stream, keys, n,
                       reinterpret_cast<uint2*>(ranges), (uint32_t)num_tiles, 0xffffffffu);
    return check_launch("identify_tile_ranges", stream, 0);
}

}  // namespace hidegs

// ============================== C ABI ==========================================
extern "C" {

size_t hidegs_scan_scratch_bytes(long long n) { return n > 0 ? hidegs::inclusive_scan_scratch(n) : 0; }
int hidegs_inclusive_scan_u32(void* scratch, size_t scratch_bytes, const uint32_t* in, uint32_t* out, long long n,
                              void* stream)
{
    return hidegs::inclusive_scan_u32(scratch, scratch_bytes, in, out, n, hidegs::as_stream(stream));
}

size_t hidegs_sort_pairs_u64_scratch_bytes(long long n) { return n > 0 ? hidegs::sort_u64_scratch(n) : 0; }
int hidegs_sort_pairs_u64(void* scratch, size_t scratch_bytes, const uint64_t* keys_in, uint64_t* keys_out,
                          const uint32_t* vals_in, uint32_t* vals_out, long long n, int begin_bit, int end_bit,
                          void* stream)
{
    return hidegs::sort_pairs_u64(scratch, scratch_bytes, keys_in, keys_out, vals_in, vals_out, n, begin_bit, end_bit,
                                  hidegs::as_stream(stream));
}

size_t hidegs_sort_pairs_u32_scratch_bytes(long long n) { return n > 0 ? hidegs::sort_u32_scratch(n) : 0; }
int hidegs_sort_pairs_u32(void* scratch, size_t scratch_bytes, const uint32_t* keys_in, uint32_t* keys_out,
                          const uint32_t* vals_in, uint32_t* vals_out, long long n, int begin_bit, int end_bit,
                          void* stream)
{
    return hidegs::sort_pairs_u32(scratch, scratch_bytes, keys_in, keys_out, vals_in, vals_out, n, begin_bit, end_bit,
                                  hidegs::as_stream(stream));
}

int hidegs_sort_tile_pairs(void* scratch, size_t scratch_bytes, const uint64_t* keys_in, uint64_t* keys_out,
                           const uint32_t* vals_in, uint32_t* vals_out, long long n, int num_tiles, uint32_t* ranges,
                           void* stream)
{
    return hidegs::sort_tile_pairs(scratch, scratch_bytes, keys_in, keys_out, vals_in, vals_out, n, num_tiles, ranges,
                                   hidegs::as_stream(stream));
}

int hidegs_identify_tile_ranges(const uint64_t* sorted_keys, long long n, uint32_t* ranges, int num_tiles,
                                void* stream)
{
    return hidegs::identify_tile_ranges(sorted_keys, n, ranges, num_tiles, hidegs::as_stream(stream));
}

uint32_t hidegs_higher_msb(uint32_t n)
{
    // Number of bits needed to hold n, at least 1 -- the value getHigherMsb's
    // binary search (rasterizer_impl.cu:35-50) returns for every u32 input.
    uint32_t bits = 32u - (uint32_t)__builtin_clz(n | 1u);
    return bits;
}

}  // extern "C"
