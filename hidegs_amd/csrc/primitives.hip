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

#include <mutex>

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
#ifndef HIDEGS_SCAN_ITEMS
#define HIDEGS_SCAN_ITEMS 16  // u32 items per thread of a scan tile (experiments: tools/build_variant.py)
#endif
constexpr int kDevScanItems = HIDEGS_SCAN_ITEMS;
constexpr int kDevScanTile = kBlock * kDevScanItems;

// Loads one tile of u32 (striped 16-byte loads) and leaves it in LDS.
__device__ __forceinline__ void load_tile_u32(const uint32_t* in, long long base, long long n,
                                              uint32_t* s_tile)
{
    const int t = threadIdx.x;
    if (base + kDevScanTile <= n && ((reinterpret_cast<uintptr_t>(in) & 15) == 0)) {
        const uint4* src = reinterpret_cast<const uint4*>(in + base);
#pragma unroll
        for (int j = 0; j < kDevScanItems / 4; j++) {
            uint4 v = src[j * kBlock + t];
            reinterpret_cast<uint4*>(s_tile)[j * kBlock + t] = v;
        }
    } else {
#pragma unroll
        for (int j = 0; j < kDevScanItems; j++) {
            long long i = base + j * kBlock + t;
            s_tile[j * kBlock + t] = (i < n) ? in[i] : 0u;
        }
    }
    __syncthreads();
}

__global__ __launch_bounds__(kBlock) void scan_reduce_kernel(const uint32_t* __restrict__ in, long long n,
                                                             uint32_t* __restrict__ tile_sums)
{
    __shared__ __attribute__((aligned(16))) uint32_t s_tile[kDevScanTile];
    __shared__ uint32_t s_wave[kWavesPerBlock];
    const long long base = (long long)blockIdx.x * kDevScanTile;
    load_tile_u32(in, base, n, s_tile);
    uint32_t sum = 0;
#pragma unroll
    for (int j = 0; j < kDevScanItems; j++) sum += s_tile[threadIdx.x * kDevScanItems + j];
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
    __shared__ __attribute__((aligned(16))) uint32_t s_tile[kDevScanTile];
    __shared__ uint32_t s_wave[kWavesPerBlock];
    const long long base = (long long)blockIdx.x * kDevScanTile;
    uint32_t tile_off;
    if (sums_raw) {
        uint32_t part = 0;
        for (int i = threadIdx.x; i < (int)blockIdx.x; i += kBlock) part += tile_offsets[i];
        block_exclusive_scan(part, s_wave, &tile_off);
    } else {
        tile_off = tile_offsets[blockIdx.x];
    }
    load_tile_u32(in, base, n, s_tile);
    uint32_t v[kDevScanItems];
    uint32_t sum = 0;
#pragma unroll
    for (int j = 0; j < kDevScanItems; j++) {
        v[j] = s_tile[threadIdx.x * kDevScanItems + j];
        sum += v[j];
    }
    uint32_t total;
    uint32_t run = block_exclusive_scan(sum, s_wave, &total) + tile_off;
#pragma unroll
    for (int j = 0; j < kDevScanItems; j++) {
        run += v[j];
        s_tile[threadIdx.x * kDevScanItems + j] = run;  // inclusive
    }
    __syncthreads();
    if (base + kDevScanTile <= n && ((reinterpret_cast<uintptr_t>(out) & 15) == 0)) {
        uint4* dst = reinterpret_cast<uint4*>(out + base);
#pragma unroll
        for (int j = 0; j < kDevScanItems / 4; j++) dst[j * kBlock + threadIdx.x] = reinterpret_cast<uint4*>(s_tile)[j * kBlock + threadIdx.x];
    } else {
#pragma unroll
        for (int j = 0; j < kDevScanItems; j++) {
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
// With Based, the digit is taken of (low key half - dbase) instead (the partition queue's digits).
template <typename K, int R, bool Based = false>
__device__ __forceinline__ void wave_rank(const K (&k)[R], const bool (&ok)[R], int shift, uint32_t mask,
                                          uint32_t* cnt, uint32_t (&rank)[R], uint32_t vary, uint32_t dbase = 0u)
{
#pragma unroll
    for (int r = 0; r < R; r++) {
        const uint32_t d = Based ? ((((uint32_t)k[r]) - dbase) >> shift) & mask : digit_of(k[r], shift, mask);
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

#ifndef HIDEGS_XCD_HIST
#define HIDEGS_XCD_HIST 1  // 16.4 -> 13.5 us per pass at 8M keys (A/B builds: 0)
#endif
// counts[d * ntiles + tile] = number of keys of tile `tile` whose digit is d.
// zero_jobs: zero_count 16-byte slots cleared on the side (the hot-tile queue's job slots).
template <typename K>
__global__ __launch_bounds__(kBlock) void radix_hist_kernel(const K* __restrict__ keys, long long n, int shift,
                                                            uint32_t mask, int ntiles, uint32_t* __restrict__ counts,
                                                            uint4* __restrict__ zero_jobs, uint32_t zero_count)
{
    for (uint32_t j = blockIdx.x * kBlock + threadIdx.x; j < zero_count; j += gridDim.x * kBlock)
        zero_jobs[j] = make_uint4(0u, 0u, 0u, 0u);
    __shared__ uint32_t s_hist[kWavesPerBlock][kRadix];
    const int t = threadIdx.x;
    const int wave = t / kWave;
    for (int i = t; i < kWavesPerBlock * kRadix; i += kBlock) (&s_hist[0][0])[i] = 0;
    __syncthreads();
    // neighbouring tiles on one XCD: the counts of 32 neighbouring tiles share a 128-byte line of
    // each digit row, which then fills in one L2 instead of being written back piecewise
    const int tile = HIDEGS_XCD_HIST ? xcd_swizzle(blockIdx.x, gridDim.x) : (int)blockIdx.x;
    const long long base = (long long)tile * kTile;
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
        counts[(long long)d * ntiles + tile] = c;
    }
}

#ifndef HIDEGS_DIGIT_ITEMS
#define HIDEGS_DIGIT_ITEMS 8
#endif
constexpr int kDigitItems = HIDEGS_DIGIT_ITEMS;
// One workgroup per digit: exclusive scan of counts[d][0..ntiles) in place; totals[d] = sum.
// low_totals (nlow <= 256 digit totals of the previous pass, or NULL): workgroup 0 also writes
// their exclusive scan to low_base (the segment starts of radix_scatter_kernel<K, true>).
__global__ __launch_bounds__(kBlock) void radix_digit_scan_kernel(uint32_t* __restrict__ counts, int ntiles,
                                                                  uint32_t* __restrict__ totals,
                                                                  const uint32_t* __restrict__ low_totals, int nlow,
                                                                  uint32_t* __restrict__ low_base)
{
    if (low_totals && blockIdx.x == 0) {
        __shared__ uint32_t s_low[kWavesPerBlock];
        uint32_t dummy;
        const uint32_t b = block_exclusive_scan((int)threadIdx.x < nlow ? low_totals[threadIdx.x] : 0u, s_low, &dummy);
        if ((int)threadIdx.x < nlow) low_base[threadIdx.x] = b;
    }
    __shared__ uint32_t s_wave[kWavesPerBlock];
    uint32_t* row = counts + (long long)blockIdx.x * ntiles;
    // HIDEGS_DIGIT_ITEMS per thread: one round (one memory latency) for up to 256 x that many tiles
    uint32_t carry = 0;
    for (int base = 0; base < ntiles; base += kBlock * kDigitItems) {
        uint32_t v[kDigitItems];
        uint32_t sum = 0;
#pragma unroll
        for (int j = 0; j < kDigitItems; j++) {
            int i = base + threadIdx.x * kDigitItems + j;
            v[j] = (i < ntiles) ? row[i] : 0u;
            sum += v[j];
        }
        uint32_t total;
        uint32_t pre = block_exclusive_scan(sum, s_wave, &total) + carry;
#pragma unroll
        for (int j = 0; j < kDigitItems; j++) {
            int i = base + threadIdx.x * kDigitItems + j;
            if (i < ntiles) row[i] = pre;
            pre += v[j];
        }
        carry += total;
    }
    if (threadIdx.x == 0) totals[blockIdx.x] = carry;
}

// Stable scatter of one tile.  LDS: one staging buffer of the tile's keys (values reuse it
// afterwards), per-wave digit counters -- 43 KB at 8 waves, 3 workgroups per CU (38 KB and 4 for the
// 128-digit instances, below).
// Global offsets: tile_prefix[d][tile] (per-digit exclusive scan over tiles) + exclusive scan
// of the digit totals.  (A single-pass decoupled look-back variant measured slower on MI355X:
// the chained tile-to-tile hand-off crosses the non-coherent per-XCD L2s at every hop.)
#ifndef HIDEGS_SCATTER_WAVES
#define HIDEGS_SCATTER_WAVES 8  // wave64s per scatter workgroup (the tile stays kTile pairs); 8 waves
                                // of 8 pairs each (66 VGPRs, 6 waves/SIMD) measured 2-3% faster than 4 of 16
#endif
constexpr int kSWaves = HIDEGS_SCATTER_WAVES;
#ifndef HIDEGS_XCD_TILES
#define HIDEGS_XCD_TILES 1  // neighbouring tiles on one XCD: 46.3 -> 42.9 us per pass at 8M pairs (their
                            // shared output lines at digit-run ends merge in one L2); the same
                            // mapping for segment_sort measured 48.1 -> 49.7 us and is not used there
#endif
constexpr int kSBlock = kSWaves * kWave;
constexpr int kSItems = kTile / kSBlock;  // pairs per thread
static_assert(kSBlock >= kRadix, "one thread per digit in the digit scans");

// radix_scatter_kernel<K, true>'s segment starts (see there); every thread of the workgroup calls it.
template <typename K, int R, int D = kRadix>  // D: digit capacity (> mask, and 1 << b0 <= D)
__device__ __forceinline__ void segment_starts(const K (&k)[R], const bool (&ok)[R], const int shift, const uint32_t mask,
                                            const long long n, const int tile, const int ntiles,
                                            const long long base, const uint32_t digit_base,
                                            const uint32_t p0, const int b0, uint32_t* starts)
{
    __shared__ uint32_t s_bhist[D];
    __shared__ uint32_t s_blist[D];
    __shared__ uint32_t s_nb;
    const int t = threadIdx.x, lane = lane_id(), wave = t / kWave;
    if (t == 0) {
        s_nb = 0u;
        if (tile == 0) starts[(mask + 1u) << b0] = (uint32_t)n;
    }
    if (b0 == 0) {  // one pass: the digit bases of tile 0 are the segment starts
        if (tile == 0 && t <= (int)mask) starts[t] = digit_base;
        return;
    }
    __syncthreads();  // s_nb
    // low values whose first position p0 = base0[t] lies in this tile (position n: the last tile)
    if (t < (1 << b0) && (((long long)p0 >= base && (long long)p0 < base + kTile) ||
                          ((long long)p0 >= n && tile == ntiles - 1)))
        s_blist[atomicAdd(&s_nb, 1u)] = (uint32_t)t | (((uint32_t)((long long)p0 - base)) << 8);
    __syncthreads();
    const uint32_t nb = s_nb;  // workgroup-uniform; 0 for most tiles
    for (uint32_t b = 0; b < nb; b++) {
        const uint32_t e = s_blist[b], L = e & 0xffu, r = e >> 8;  // the tile's pairs [0, r) precede L
        if (t < D) s_bhist[t] = 0u;
        __syncthreads();
#pragma unroll
        for (int q = 0; q < R; q++) {
            const uint32_t li = (uint32_t)(wave * (R * kWave) + q * kWave + lane);
            if (ok[q] && li < r) atomicAdd(&s_bhist[digit_of(k[q], shift, mask)], 1u);
        }
        __syncthreads();
        if (t <= (int)mask) starts[((uint32_t)t << b0) | L] = digit_base + s_bhist[t];
        __syncthreads();
    }
}

// Starts (the segmented sort's last segment-bit pass): also the output position of each segment's
// first pair, starts[(H << b0) | L] for segment (H = this pass's digit, L = the b0 segment bits of
// the pass before), so that no kernel has to find the ranges in the sorted keys.  Pass 1 is stable
// and its input is ordered by L: segment (H, L) starts at this tile's global base of digit H plus
// the digit-H pairs of this tile that precede base0[L] (the first input position of L: the
// exclusive scan of pass 0's digit totals, totals0), for the tile that holds base0[L].  b0 == 0
// (one pass, the digit is the whole segment id): tile 0 writes starts[d] = base of digit d.
// starts[(mask + 1) << b0] = n closes the last segment.
// D = digit capacity: kRadix, or kNarrowRadix for passes of <= 7 bits, whose smaller LDS arrays
// (39 KB instead of 45 KB) let a fourth workgroup onto each CU: the 1080p binning sort (8.6M pairs,
// 6 + 7 bits) 189 -> 183 us.  Only up to kNarrowMaxN pairs: the 4K frame's 42.9M pairs (7 + 8 bits)
// went 880 -> 894 us with its 7-bit pass narrow -- a fourth workgroup's open digit runs cost more
// once a pass's output no longer stays in the 256 MB MALL (profiles/r04_narrow_scatter.md).
#ifndef HIDEGS_SCATTER_NARROW
#define HIDEGS_SCATTER_NARROW 1
#endif
constexpr int kNarrowRadix = 128;
#ifndef HIDEGS_SCATTER_NT_LOADS
#define HIDEGS_SCATTER_NT_LOADS 1  // the pass's input, dead after the pass, read with non-temporal loads so it
                                   // does not displace the output the next pass reads: scatter 42.8 -> 40.6 us
                                   // (1080p D2 view), 4K sort 872 -> 834 us (profiles/r04_scatter_nt.md)
#endif
#ifndef HIDEGS_NARROW_MAX_N
#define HIDEGS_NARROW_MAX_N (12ll << 20)
#endif
constexpr long long kNarrowMaxN = HIDEGS_NARROW_MAX_N;
template <typename K, bool Starts = false, int D = kRadix>
__global__ __launch_bounds__(kSBlock) __attribute__((amdgpu_waves_per_eu(D == kRadix ? 1 : 8))) void radix_scatter_kernel(const K* __restrict__ keys_in,
                                                                const uint32_t* __restrict__ vals_in,
                                                                K* __restrict__ keys_out, uint32_t* __restrict__ vals_out,
                                                                long long n, int shift, uint32_t mask, int ntiles,
                                                                const uint32_t* __restrict__ tile_prefix,
                                                                const uint32_t* __restrict__ totals,
                                                                const uint32_t* __restrict__ totals0, int b0,
                                                                uint32_t* __restrict__ starts)
{
    __shared__ __attribute__((aligned(16))) K s_stage[kTile];  // keys by tile-local rank, then values
    __shared__ uint32_t s_cnt[kSWaves][D];              // per-wave running counters
    __shared__ uint32_t s_start[D];                     // tile-local start of each digit run
    __shared__ uint32_t s_off[D];                       // global position of tile-local position 0 of digit d
    __shared__ uint32_t s_wave[kSWaves];
    uint32_t* s_vals = reinterpret_cast<uint32_t*>(s_stage);

    const int t = threadIdx.x;
    const int lane = lane_id();
    const int wave = t / kWave;
    const bool digit_thread = t < D;  // thread d owns digit d in the digit scans
    for (int i = t; i < kSWaves * D; i += kSBlock) (&s_cnt[0][0])[i] = 0;
    const int tile = HIDEGS_XCD_TILES ? xcd_swizzle(blockIdx.x, gridDim.x) : (int)blockIdx.x;
    const long long base = (long long)tile * kTile;
    const long long seg = base + (long long)wave * (kSItems * kWave);  // this wave's items
    // this tile's global digit offsets, loaded now so their latency hides behind the ranking (digits
    // above `mask` read stale counts that no item uses)
    const uint32_t digit_total = digit_thread ? totals[t] : 0u;
    const uint32_t digit_prefix = digit_thread ? tile_prefix[(long long)t * ntiles + tile] : 0u;
    const uint32_t low_base = Starts && b0 > 0 && t < (1 << b0) ? totals0[t] : 0u;  // base0[t]; b0 <= 8

    K k[kSItems];
    uint32_t v[kSItems];
    bool ok[kSItems];
#pragma unroll
    for (int r = 0; r < kSItems; r++) {
        const long long i = seg + r * kWave + lane;
        ok[r] = i < n;
#if HIDEGS_SCATTER_NT_LOADS
        k[r] = ok[r] ? __builtin_nontemporal_load(keys_in + i) : K(0);
        v[r] = ok[r] ? __builtin_nontemporal_load(vals_in + i) : 0u;
#else
        k[r] = ok[r] ? keys_in[i] : K(0);
        v[r] = ok[r] ? vals_in[i] : 0u;
#endif
    }
    // the digits' global bases, scanned while the tile's loads are in flight (workgroup barriers
    // do not wait for global loads)
    uint32_t dummy;
    const uint32_t digit_base = block_exclusive_scan<kSWaves>(digit_total, s_wave, &dummy) + digit_prefix;
    // (at the end of the kernel instead, with the keys kept live: 73 VGPRs against 61, same time)
    if (Starts) segment_starts<K, kSItems, D>(k, ok, shift, mask, n, tile, ntiles, base, digit_base, low_base, b0, starts);
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

__device__ __forceinline__ void wave_min_max(uint32_t& lo, uint32_t& hi)
{
#pragma unroll
    for (int sh = 32; sh >= 1; sh >>= 1) {
        lo = min(lo, (uint32_t)__shfl_xor(lo, sh, kWave));
        hi = max(hi, (uint32_t)__shfl_xor(hi, sh, kWave));
    }
}

// LDS of the oversized-segment forms (the one-workgroup global form, the partition jobs).
struct BigShared {
    uint32_t cnt[kWavesPerBlock][kRadix];
    uint32_t hist[kRadix];
    uint32_t run[kRadix];  // running destination of each digit
    uint32_t aux[2][kRadix];  // partition jobs: MIN / MAX of each digit's low key halves
    uint32_t wave[kWavesPerBlock];
};

// One stable step of a digit pass through global memory: the cnt <= kBigItems * kBlock items
// [base, base + cnt) of (sk, sv) are ranked by digit ((low key half - dbase) >> shift) & mask inside the step (wave w
// owns items [w * 512, w * 512 + 512) in (round, lane) order) and item i goes to
// sh.run[digit] + its rank, then sh.run advances by the step's digit counts.  sh.run must be set
// before the call (its first barrier publishes it).  Destinations outside [lo, hi) are dropped:
// never, for consistent offsets -- a guard, not a case.
constexpr int kBigItems = 8;
constexpr int kBigStep = kBigItems * kBlock;  // 2048
// A step's pairs in registers: wave w's items [w * 512, w * 512 + 512) of [base, base + cnt), in
// (round, lane) order; absent items read as 0.
__device__ __forceinline__ void step_load(const uint64_t* sk, const uint32_t* sv, const uint32_t base,
                                          const uint32_t cnt, uint64_t (&k)[kBigItems], uint32_t (&v)[kBigItems])
{
    const uint32_t w0 = (threadIdx.x / kWave) * (kBigItems * kWave);
#pragma unroll
    for (int q = 0; q < kBigItems; q++) {
        const uint32_t i = w0 + q * kWave + lane_id();
        k[q] = i < cnt ? sk[base + i] : 0ull;
        v[q] = i < cnt ? sv[base + i] : 0u;
    }
}

// Track: also fold each item's low key half into sh.aux[0][digit] (MIN) and sh.aux[1][digit] (MAX).
// (Write-through `sc1` stores here, so that the SCATTER job's release had fewer dirty lines to write
// back, measured slower: one tile 1044 -> 1188 us, D2 0.5:0.02 516 -> 547 us.)
template <bool Track = false>
__device__ __forceinline__ void step_scatter(const uint64_t (&k)[kBigItems], const uint32_t (&v)[kBigItems],
                                             const uint32_t base, const uint32_t cnt, uint64_t* dk, uint32_t* dv,
                                             const uint32_t dbase, const int shift, const uint32_t mask,
                                             const uint32_t lo, const uint32_t hi, BigShared& sh)
{
    const int t = threadIdx.x;
    const int lane = lane_id();
    const int wave = t / kWave;
    for (int i = t; i < kWavesPerBlock * kRadix; i += kBlock) (&sh.cnt[0][0])[i] = 0;
    __syncthreads();
    bool ok[kBigItems];
    uint32_t rank[kBigItems];
    const uint32_t w0 = wave * (kBigItems * kWave);
#pragma unroll
    for (int q = 0; q < kBigItems; q++) ok[q] = w0 + q * kWave + lane < cnt;
    wave_rank<uint64_t, kBigItems, true>(k, ok, shift, mask, sh.cnt[wave], rank, mask, dbase);
    __syncthreads();
    const uint32_t tot = digit_wave_prefix(sh.cnt);
    __syncthreads();
#pragma unroll
    for (int q = 0; q < kBigItems; q++) {
        if (ok[q]) {
            const uint32_t dd = (((uint32_t)k[q] - dbase) >> shift) & mask;
#ifdef HIDEGS_EXP_INORDER_SCATTER  // experiments only: input-order stores (wrong result; store-pattern A/B)
            const uint32_t dst = base + w0 + q * kWave + lane;
            (void)rank;
#else
            const uint32_t dst = sh.run[dd] + sh.cnt[wave][dd] + rank[q];
            (void)base;
#endif
            if (dst >= lo && dst < hi) {
                dk[dst] = k[q];
                dv[dst] = v[q];
            }
#ifndef HIDEGS_EXP_NO_TRACK  // experiments only: no per-digit MIN / MAX (wrong next-level digits; cost A/B)
            if (Track) {
                atomicMin(&sh.aux[0][dd], (uint32_t)k[q]);
                atomicMax(&sh.aux[1][dd], (uint32_t)k[q]);
            }
#endif
        }
    }
    __syncthreads();
    sh.run[threadIdx.x] += tot;
    __syncthreads();
}

template <bool Track = false>
__device__ __forceinline__ void scatter_step(const uint64_t* sk, const uint32_t* sv, uint64_t* dk, uint32_t* dv,
                                             const uint32_t base, const uint32_t cnt, const uint32_t dbase,
                                             const int shift, const uint32_t mask, const uint32_t lo,
                                             const uint32_t hi, BigShared& sh)
{
    uint64_t k[kBigItems];
    uint32_t v[kBigItems];
    step_load(sk, sv, base, cnt, k, v);
    step_scatter<Track>(k, v, base, cnt, dk, dv, dbase, shift, mask, lo, hi, sh);
}

// scatter_step over [base, base + cnt) in kBigStep steps, the next step's pairs loaded while the
// current one is ranked and stored (the queue's workers run one wave per SIMD: latency is hidden
// by the wave's own loads in flight or not at all; barriers do not wait for global loads).
template <bool Track = false>
__device__ __forceinline__ void scatter_steps(const uint64_t* sk, const uint32_t* sv, uint64_t* dk, uint32_t* dv,
                                              const uint32_t base, const uint32_t cnt, const uint32_t dbase,
                                              const int shift, const uint32_t mask, const uint32_t lo,
                                              const uint32_t hi, BigShared& sh)
{
    uint64_t k[kBigItems], kn[kBigItems];
    uint32_t v[kBigItems], vn[kBigItems];
    step_load(sk, sv, base, cnt < (uint32_t)kBigStep ? cnt : (uint32_t)kBigStep, k, v);
    for (uint32_t b0 = 0; b0 < cnt; b0 += kBigStep) {
        const uint32_t c = cnt - b0 < (uint32_t)kBigStep ? cnt - b0 : (uint32_t)kBigStep;
        const uint32_t b1 = b0 + kBigStep;
        if (b1 < cnt) step_load(sk, sv, base + b1, cnt - b1 < (uint32_t)kBigStep ? cnt - b1 : (uint32_t)kBigStep, kn, vn);
        step_scatter<Track>(k, v, base + b0, c, dk, dv, dbase, shift, mask, lo, hi, sh);
#pragma unroll
        for (int q = 0; q < kBigItems; q++) {
            k[q] = kn[q];
            v[q] = vn[q];
        }
    }
}

// A segment of more than kSegCap pairs sorted by ONE workgroup: 4 stable LSD passes over the low
// 32 bits through global memory (keys/vals <-> alt within the segment's range).  The last resort
// of the partition queue below (its capacity exhausted); hot tiles normally go through the queue.
__device__ __forceinline__ void segment_sort_global(uint64_t* __restrict__ keys, uint32_t* __restrict__ vals,
                                                    uint64_t* __restrict__ alt_k, uint32_t* __restrict__ alt_v,
                                                    const uint32_t begin, const uint32_t m, BigShared& sh)
{
    const int t = threadIdx.x;
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
        for (uint32_t c0 = 0; c0 < m; c0 += kBigStep)
            scatter_step(sk, sv, dk, dv, begin + c0, m - c0 < (uint32_t)kBigStep ? m - c0 : (uint32_t)kBigStep, 0u,
                         shift, kRadix - 1, begin, begin + m, sh);
    }
}

// LSD form of the per-segment sort (the fallback of segment_sort_kernel for segments whose
// depth bits crowd into a few buckets): run A (<= kSegRun) sorted in LDS, run B parked in registers
// and sorted after it, the two merged by rank; every item's high key half and value gathered by
// its index in the segment and written in place.  `diff` = the low key bits that vary.
// The segment is read from (src_k, src_v) and written to (dst_k, dst_v): the same buffers (in
// place: every read precedes the first write) or alt -> keys (a piece of a partitioned hot tile).
// InPlace: dst is ignored and written through pointers based on src (keeps __restrict__ valid).
template <bool InPlace>
__device__ __forceinline__ void segment_sort_lsd(const uint64_t* __restrict__ src_k, const uint32_t* __restrict__ src_v,
                                                 uint64_t* __restrict__ dst_k, uint32_t* __restrict__ dst_v,
                                                 const uint32_t begin, const uint32_t m, const uint32_t diff,
                                                 SegShared& sh)
{
    uint64_t* dk = InPlace ? const_cast<uint64_t*>(src_k) : dst_k;
    uint32_t* dv = InPlace ? const_cast<uint32_t*>(src_v) : dst_v;
    const int t = threadIdx.x;
    const uint32_t na = m < (uint32_t)kSegRun ? m : (uint32_t)kSegRun, nb = m - na;
    uint32_t bk[kRunItems];
#pragma unroll
    for (int q = 0; q < kRunItems; q++) {
        const uint32_t i = t + q * kBlock;
        if (i < na) {
            sh.k[0][i] = (uint32_t)src_k[begin + i];
            sh.i[0][i] = i;
        }
        bk[q] = i < nb ? (uint32_t)src_k[begin + kSegRun + i] : 0u;
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
    // unmodified until every workgroup thread has gathered), then write
    uint32_t hi[kSegItems], v[kSegItems];
#pragma unroll
    for (int q = 0; q < kSegItems; q++) {
        if (fok[q]) {
            hi[q] = (uint32_t)(src_k[begin + fi[q]] >> 32);
            v[q] = src_v[begin + fi[q]];
        }
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < kSegItems; q++) {
        if (fok[q]) {
            dk[begin + fp[q]] = ((uint64_t)hi[q] << 32) | fk[q];
            dv[begin + fp[q]] = v[q];
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

// The segment's low-key statistics for the bucket form: diff (the bits that vary: AND ^ OR) and the
// smallest low key lo, with the bucket digit over the keys' RANGE [lo, hi]: bucket = (x - lo) >> shift
// with shift = bits(hi - lo) - kBucketBits.  Float depth bits spread over many exponents (0.2 .. 100:
// bits 23..30 all vary, the top ten varying bits leave ~40 of 1024 buckets in use) fill the buckets
// evenly this way; the order is the same, x - lo being monotone over the segment.  Every thread
// passes its own partial a / o / lo / hi; s0, s1 hold kWavesPerBlock words each.
struct SegStats {
    uint32_t diff, lo;
    int shift, dbits;
};
__device__ __forceinline__ SegStats segment_stats(uint32_t a, uint32_t o, uint32_t lo, uint32_t hi, uint32_t* s0,
                                                  uint32_t* s1)
{
    const int lane = lane_id(), wave = threadIdx.x / kWave;
    wave_and_or(a, o);
    wave_min_max(lo, hi);
    if (lane == 0) {
        s0[wave] = a;
        s1[wave] = o;
    }
    __syncthreads();
    uint32_t aa = 0xffffffffu, oo = 0u;
#pragma unroll
    for (int w = 0; w < kWavesPerBlock; w++) {
        aa &= s0[w];
        oo |= s1[w];
    }
    __syncthreads();
    if (lane == 0) {
        s0[wave] = lo;
        s1[wave] = hi;
    }
    __syncthreads();
    uint32_t ll = 0xffffffffu, hh = 0u;
#pragma unroll
    for (int w = 0; w < kWavesPerBlock; w++) {
        ll = min(ll, s0[w]);
        hh = max(hh, s1[w]);
    }
    SegStats st;
    st.diff = aa ^ oo;
    st.lo = ll;
    const int nbits = hh > ll ? 32 - __builtin_clz(hh - ll) : 0;
    st.dbits = nbits < kBucketBits ? nbits : kBucketBits;
    st.shift = nbits - st.dbits;
    return st;
}


struct BucketShared {
    uint32_t comb[kSegCap];   // (key bits below the digit << kIndexBits) | index, grouped by bucket
    uint32_t start[kBuckets];
    uint32_t fill[kBuckets];  // histogram, then the running fill pointer (= bucket end after filling)
};
// after ranking, the whole struct stages the sorted segment: keys (u64) then values (u32) when
// they fit together (<= kSegRun pairs), else keys and values one after the other
static_assert(sizeof(BucketShared) >= kSegCap * sizeof(uint64_t), "staging of the keys");
static_assert(sizeof(BucketShared) >= kSegRun * (sizeof(uint64_t) + sizeof(uint32_t)), "staging of a run");
static_assert(sizeof(BucketShared) >= kSegCap * 2 * sizeof(uint32_t), "compact staging of a segment");
#ifndef HIDEGS_SEG_COMPACT_STAGE
#define HIDEGS_SEG_COMPACT_STAGE 1  // segment_sort_kernel: low halves + values staged in one pass when the
                                    // segment's high key halves are all equal (0: keys, then values)
#endif

// ---- hot tiles: the partition queue --------------------------------------------------------
//
// A segment of more than kSegCap pairs is not sorted by one workgroup (that costs ~10 ns per pair:
// a 100K-pair tile took 1 ms) but split among many.  It becomes a RECORD, partitioned stably by
// one digit -- the top <= 8 bits of (low key half - its MIN) -- in three phases of chunk jobs
// (chunk_size(m) pairs: 4K to 32K by the record's size):
//   REDUCE   MIN / MAX of the chunk's low key halves       -> the digit (last chunk decides)
//   HIST     the chunk's digit counts                      -> pool; the last chunk (of each group
//                                                             of chunks, then of the groups) scans
//                                                             them into every chunk's per-digit
//                                                             destinations
//   SCATTER  the chunk's pairs, ranked stably, to the other buffer (keys <-> alt)
// and the last SCATTER cuts the result into pieces by digit: runs of small digits merged up to
// kSegCap pairs become pieces (the bucket form of segment_sort_kernel, alt -> keys or in place,
// sorted by piece_sort_kernel after the queue; SMALL jobs only if its list is full), a digit of
// kSegCap..kWideCap pairs one WIDE job, a bigger digit a new record one digit lower.  Each level fixes the top <= 8
// varying bits, so the chain ends within 4 levels; pieces left in alt are copied back (COPY jobs).
// Every piece keeps its pairs in input order between equal digits, so the whole is the stable sort.
//
// Jobs live in a queue in scratch, zeroed each call: a producer reserves slots (fetch-add on
// `reserve`), writes them and publishes each by setting its tag; a consumer workgroup claims the next
// index (`head`, relaxed) and waits until that slot is published or every job is finished (`done` == `reserve`:
// nothing in flight, so nothing more can come).  Every wait is bounded (kMaxPolls) and flags
// Q_ERROR when exceeded.  Producers run (they reserved while resident) and publish right after
// writing, so no wait is on a workgroup that is not running.  Ordering across workgroups (and XCD
// L2s) is by agent-scope release / acquire (release_lane / acquire_lane): job payload and pair data
// before the tag, phase data before `pending` and the group countdowns.
#ifndef HIDEGS_CHUNK_STEPS
#define HIDEGS_CHUNK_STEPS 2
#endif
constexpr int kChunk = HIDEGS_CHUNK_STEPS * kBigStep;  // pairs per chunk job of a small record
// A bigger record's chunk jobs take 2, 4 or 8 kChunk pieces each: a job's hand-off (claim, acquire,
// release) costs ~10 us whatever its size, so the 2100 chunk jobs per phase of an 8.6M-pair tile
// spent most of their time in hand-offs (tools/gpu_queue_ab.sh: DESIGN.md "A known limit").
#ifndef HIDEGS_CHUNK_X2
#define HIDEGS_CHUNK_X2 32768
#endif
#ifndef HIDEGS_CHUNK_X4
#define HIDEGS_CHUNK_X4 131072
#endif
#ifndef HIDEGS_CHUNK_X8
#define HIDEGS_CHUNK_X8 1048576
#endif
static_assert((kChunk & (kChunk - 1)) == 0, "chunk sizes are kChunk << 0..3");
__device__ __forceinline__ uint32_t chunk_size(uint32_t m)
{
    return (uint32_t)kChunk << (m > HIDEGS_CHUNK_X8 ? 3 : m > HIDEGS_CHUNK_X4 ? 2 : m > HIDEGS_CHUNK_X2 ? 1 : 0);
}
#ifndef HIDEGS_QUEUE_BLOCKS
#define HIDEGS_QUEUE_BLOCKS 256  // queue workers (experiments: tools/build_variant.py)
#endif
constexpr int kQueueBlocks = HIDEGS_QUEUE_BLOCKS;
#ifndef HIDEGS_BACKOFF_MAX
#define HIDEGS_BACKOFF_MAX 16  // a waiting worker's longest sleep between polls, in s_sleep(8) units
#endif
#ifndef HIDEGS_QUEUE_MIN
#define HIDEGS_QUEUE_MIN 2048  // segments up to this many pairs: the one-workgroup global form (2048 = kSegCap:
                              // every tile over kSegCap goes to the queue; tools/skew_time.py A/B in DESIGN.md)
#endif
constexpr int kQueueMin = HIDEGS_QUEUE_MIN;
#ifndef HIDEGS_WIDE_CAP
#define HIDEGS_WIDE_CAP 12288  // segments up to this many pairs: one WIDE job (LDS sort by one worker)
#endif
constexpr int kWideCap = HIDEGS_WIDE_CAP;
#ifndef HIDEGS_PIECE_WAVES
#define HIDEGS_PIECE_WAVES 5  // waves per SIMD piece_sort_kernel's register budget is set for (6: 10 VGPRs spilled)
#endif
#ifndef HIDEGS_DEFER_PIECES
#define HIDEGS_DEFER_PIECES 1  // 0: the queue's pieces run as its own SMALL jobs (one workgroup per CU)
#endif
constexpr bool kDeferPieces = HIDEGS_DEFER_PIECES != 0;
#ifndef HIDEGS_WIDE_SCOUTS
#define HIDEGS_WIDE_SCOUTS 0  // 1: scouts hand hot tiles of <= kWideCap pairs to the queue as WIDE jobs (slower: DESIGN.md)
#endif
#ifndef HIDEGS_MAX_POLLS
#define HIDEGS_MAX_POLLS (1u << 22)  // a waiting worker gives up after this many polls (~13 s at the longest backoff)
#endif
constexpr uint32_t kMaxPolls = HIDEGS_MAX_POLLS;
enum : uint32_t { J_EXIT = 0, J_SMALL, J_COPY, J_REDUCE, J_HIST, J_SCATTER, J_GLOBAL, J_WIDE };
enum : int { Q_HEAD, Q_RESERVE, Q_DONE, Q_NREC, Q_POOL, Q_ERROR, Q_NPIECE, Q_COUNTERS = 8 };
constexpr int kCtlStride = 32;  // one 128-byte line per counter: polls of one do not queue behind another's atomics
constexpr int Q_WORDS = Q_COUNTERS * kCtlStride;
static_assert(Q_WORDS <= kBlock, "identify_ranges_kernel zeroes the counters with one workgroup");

struct BigSeg {
    uint32_t begin, m, src, chunks;  // pairs [begin, begin + m) of keys (src 0) or alt (src 1)
    uint32_t lo_bits, hi_bits;       // REDUCE: MIN / MAX of the low key halves
    uint32_t shift, bits;            // the digit: bits [shift, shift + bits) of (low key half - lo)
    uint32_t lo;                     // the digit's base: the record's smallest low key half
    uint32_t pool;                   // (chunks + 2) x 256 u32: per-chunk counts -> destinations,
                                     // then the digit starts and the digit totals
    uint32_t pending;                // jobs of the current phase not yet finished
    uint32_t csize;                  // pairs per chunk job (chunk_size(m))
};

struct BigQueue {
    uint32_t* ctl;  // Q_WORDS counters, zeroed before segment_sort_kernel
    BigSeg* rec;
    uint4* job;     // (type | src << 8, a, b, tag): tag 1 once published (zeroed each call)
    uint32_t* pool;
    uint32_t rec_cap, job_cap, pool_cap;
    uint64_t* alt_k;  // the sort's alternate buffers (the global form of a mildly hot tile)
    uint32_t* alt_v;
    uint2* piece;     // deferred pieces (begin, m | src << 31) for piece_sort_kernel
    uint32_t piece_cap;
};

#ifdef HIDEGS_QUEUE_TRACE  // experiments only: per-job timestamps (tools/queue_trace.py)
constexpr unsigned int kQTraceCap = 32768;
__device__ unsigned long long g_qtrace[kQTraceCap][4];  // (type | block << 8 | index << 32, claimed, started, ended)
__device__ unsigned int g_qtrace_n;
constexpr int kWTraceCap = 4096;
__device__ unsigned long long g_wtrace[kWTraceCap][9];  // WIDE jobs: m, then 8 phase timestamps
__device__ unsigned int g_wtrace_n;
#define WSTAMP(k) do { if (threadIdx.x == 0 && wslot < kWTraceCap) g_wtrace[wslot][1 + (k)] = wall_clock64(); } while (0)
#else
#define WSTAMP(k) do { } while (0)
#endif
__device__ __forceinline__ uint32_t q_load(uint32_t* p) { return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT); }
// polling reads: coherent but without the acquire's cache invalidation (taken once, after the wait)
__device__ __forceinline__ uint32_t q_peek(uint32_t* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ void fence_acquire() { __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent"); }
__device__ __forceinline__ void fence_release() { __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent"); }
// Cache maintenance is per CU (L1) and per XCD (L2), not per wave, and it is costly (an L2
// writeback or invalidate per fence; with fences in every wave of every job the chain of a 500K-pair
// tile ran 1.2 ms): each wave only waits for its own stores to be acknowledged, then after a barrier
// ONE thread's agent-scope release (L2 writeback) or acquire (invalidate) acts for the workgroup.
__device__ __forceinline__ void wave_stores_done() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
// ONE lane's release for its workgroup (after every storing wave's wave_stores_done and a barrier),
// before the flag, tag or count that publishes the stores.  The explicit wait after the L2 writeback
// is not redundant: ROCm 7.2 drops the compiler's own wait after `buffer_wbl2` when it thinks the
// wave has nothing outstanding, and the count then overtakes the write-back (a group countdown built
// that way let a reader on another XCD scan stale count rows: an illegal address under load).
__device__ __forceinline__ void release_lane()
{
    fence_release();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}
// ONE lane's acquire for its workgroup, after its relaxed poll matched or its countdown came last;
// the wait completes the L1 invalidate before the barrier that lets the other waves load.
__device__ __forceinline__ void acquire_lane()
{
    fence_acquire();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}
// Sticky per-device copy of every queue error (bit 1: job slots exhausted, bit 4: a worker gave up
// waiting), read and cleared by hidegs_queue_error(); the debug mode (hidegs_set_debug) checks it after
// every sort.  A set bit means the sort's output is not trustworthy.
__device__ uint32_t g_queue_error;
__device__ __forceinline__ void q_flag(const BigQueue& q, uint32_t bit)
{
    __hip_atomic_fetch_or(&q.ctl[kCtlStride * Q_ERROR], bit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_fetch_or(&g_queue_error, bit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Jobs a workgroup is about to enqueue, as runs: `count` jobs of one kind.
constexpr int kMaxRuns = kRadix + 1;
struct EmitShared {
    uint4 run[kMaxRuns];  // (type | src << 8, a, b, count)
    uint32_t off[kMaxRuns + 1];
    uint32_t nruns, base, pbase;
};

__device__ __forceinline__ void runs_begin(EmitShared& e)
{
    e.nruns = 0;
    e.off[0] = 0;
}

__device__ __forceinline__ void add_run(EmitShared& e, uint32_t type, uint32_t src, uint32_t a, uint32_t b,
                                        uint32_t count)
{
    if (count == 0) return;
    e.run[e.nruns] = make_uint4(type | (src << 8), a, b, count);
    e.off[e.nruns + 1] = e.off[e.nruns] + count;
    e.nruns++;
}

// Job j of a run: chunk j of a record, the j-th kChunk piece of a COPY range, or the one job.
__device__ __forceinline__ uint4 run_job(const uint4 r, const uint32_t j)
{
    const uint32_t type = r.x & 0xffu;
    if (type == J_COPY) {
        const uint32_t s = j * kChunk;
        return make_uint4(r.x, r.y + s, r.z - s < (uint32_t)kChunk ? r.z - s : (uint32_t)kChunk, 0u);
    }
    if (type == J_REDUCE || type == J_HIST || type == J_SCATTER) return make_uint4(r.x, r.y, j, 0u);
    return make_uint4(r.x, r.y, r.z, 0u);
}

// A record's digit over its low keys' range [lo, hi] (lo < hi): the top <= 8 bits of x - lo.  Float
// depth bits that cross exponent boundaries vary in every exponent bit; a digit of the top varying
// bits would then split by exponent only (a few crowded digits), one of the range splits the mass.
__device__ __forceinline__ void range_digit(uint32_t lo, uint32_t hi, int& shift, int& bits)
{
    const int nbits = 32 - __builtin_clz(hi - lo);
    bits = nbits < kRadixBits ? nbits : kRadixBits;
    shift = nbits - bits;
}
__device__ __forceinline__ void set_digit(BigSeg& s, uint32_t lo, uint32_t hi)
{
    int shift, bits;
    range_digit(lo, hi, shift, bits);
    s.lo = lo;
    s.shift = (uint32_t)shift;
    s.bits = (uint32_t)bits;
}
// digit of a pair of a record: bits [shift, shift + bits) of (low key half - lo)
__device__ __forceinline__ uint32_t rec_digit(uint64_t key, uint32_t lo, int shift, uint32_t mask)
{
    return (((uint32_t)key - lo) >> shift) & mask;
}

// Chunk groups of a big record.  The SCATTER phase needs, per chunk and digit, the digit's count in
// the chunks before it: one workgroup walking the digit columns of all chunks took 246 us for a
// 8.5M-pair record (2100 dependent rows).  A record of more than kGroupChunks chunks therefore
// counts its HIST phase down per group: the last chunk of a group turns the group's counts into
// prefixes within the group and its sum row, the last group plans the groups' bases (<= 256 rows).
constexpr uint32_t kGroupChunks = 32;
__device__ __forceinline__ uint32_t group_chunks(uint32_t chunks)
{
    const uint32_t g = (chunks + kRadix - 1) / kRadix;  // at most 256 groups
    return g > kGroupChunks ? g : kGroupChunks;
}
__device__ __forceinline__ uint32_t num_groups(uint32_t chunks)  // 0: an ungrouped record
{
    return chunks > kGroupChunks ? (chunks + group_chunks(chunks) - 1) / group_chunks(chunks) : 0u;
}
// Pool rows of a record: [0, chunks) per-chunk counts -> destinations (grouped: prefixes within the
// group), chunks + 0..3 the digit starts, totals, MIN and MAX, then (grouped) one row per group (its
// sums -> its bases) and one row of group countdowns.
__device__ __forceinline__ uint32_t pool_rows(uint32_t chunks)
{
    // num_groups(chunks) <= chunks / kGroupChunks + 1 (a bound without branches: the exact count
    // here cost segment_sort_kernel, where the scouts open records, 4 spilled VGPRs)
    return chunks + 4 + chunks / kGroupChunks + 2;
}
// One thread: a record's HIST countdown (chunks, or its groups with each group's own countdown);
// the stores are published by the emit_jobs that queues the HIST jobs.
__device__ __forceinline__ uint32_t hist_countdown(const BigQueue& q, const BigSeg& s)
{
    const uint32_t ng = num_groups(s.chunks);
    if (ng == 0) return s.chunks;
    const uint32_t G = group_chunks(s.chunks);
    uint32_t* down = q.pool + s.pool + (s.chunks + 4 + ng) * kRadix;
    for (uint32_t g = 0; g < ng; g++) down[g] = s.chunks - g * G < G ? s.chunks - g * G : G;
    return ng;
}

// A new record over [begin, begin + m) of buffer src, as the run of jobs that starts it: REDUCE
// chunk jobs, or -- when the low keys' range [lo, hi] is known already (from the parent's SCATTER or
// the opener; `known` false: unknown) -- HIST chunk jobs right away, or a COPY / nothing for a piece
// of equal low keys.  With the record table or the pool full: one GLOBAL job (the one-workgroup sort).
// The pool holds pool_rows(chunks) x 256 u32: per-chunk counts -> destinations, then the digit
// starts, totals, and MIN / MAX of each digit's low key halves (the next level's range), and the
// rows of the chunk groups.
template <bool Grouped = true>  // false: the caller knows m <= kGroupChunks chunks (no countdowns)
__device__ __forceinline__ uint4 record_run(const BigQueue& q, uint32_t begin, uint32_t m, uint32_t src,
                                            bool known, uint32_t lo, uint32_t hi)
{
    if (known && lo == hi)  // already in order
        return make_uint4(J_COPY | (src << 8), begin, m, src ? (m + kChunk - 1) / kChunk : 0u);
    const uint32_t csize = Grouped ? chunk_size(m) : (uint32_t)kChunk;
    const uint32_t chunks = (m + csize - 1) >> (31 - __builtin_clz(csize));
    const uint32_t need = (Grouped ? pool_rows(chunks) : chunks + 4) * kRadix;
    const uint32_t r = __hip_atomic_fetch_add(&q.ctl[kCtlStride * Q_NREC], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    uint32_t p = ~0u;
    if (r < q.rec_cap) {
        p = __hip_atomic_fetch_add(&q.ctl[kCtlStride * Q_POOL], need, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if ((uint64_t)p + need > q.pool_cap) p = ~0u;
    }
    if (p == ~0u) return make_uint4(J_GLOBAL | (src << 8), begin, m, 1u);
    BigSeg& s = q.rec[r];
    s.begin = begin;
    s.m = m;
    s.src = src;
    s.chunks = chunks;
    s.lo_bits = 0xffffffffu;
    s.hi_bits = 0u;
    s.shift = 0u;
    s.bits = 0u;
    s.lo = 0u;
    s.pool = p;
    s.pending = chunks;
    s.csize = csize;
    if (!known) return make_uint4(J_REDUCE, r, 0u, chunks);
    set_digit(s, lo, hi);
    if (Grouped) s.pending = hist_countdown(q, s);
    return make_uint4(J_HIST, r, 0u, chunks);
}

__device__ __forceinline__ void add_run(EmitShared& e, const uint4 r) { add_run(e, r.x & 0xffu, r.x >> 8, r.y, r.z, r.w); }

// All threads: enqueue the runs thread 0 put in e (its writes precede the first barrier).
__device__ __forceinline__ void emit_jobs(const BigQueue& q, EmitShared& e)
{
    const int t = threadIdx.x;
    __syncthreads();
    const uint32_t nr = e.nruns, total = e.off[nr];
    if (total == 0) return;  // block-uniform
    if (t == 0) {
        // fetch-add, not a CAS loop: 80 records of one level reserving at once retried their CAS
        // for 160 us
        uint32_t base = __hip_atomic_fetch_add(&q.ctl[kCtlStride * Q_RESERVE], total, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT);
        if ((uint64_t)base + total > q.job_cap) {  // beyond the capacity bound of sort_scratch: cannot
            q_flag(q, 1u);                          // happen; count the lost jobs done so the queue ends
            __hip_atomic_fetch_add(&q.ctl[kCtlStride * Q_DONE], total, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            base = ~0u;
        }
        e.base = base;
    }
    __syncthreads();
    const uint32_t base = e.base;
    if (base == ~0u) return;
    for (uint32_t j = t; j < total; j += kBlock) {
        // the run holding job j: off[r] <= j < off[r + 1] (a binary search -- a linear walk over a
        // split record's 256 runs cost its last SCATTER job ~60 us of dependent LDS reads)
        uint32_t r = 0, hi = nr;
        while (hi - r > 1u) {
            const uint32_t mid = (r + hi) >> 1;
            if (e.off[mid] <= j) r = mid; else hi = mid;
        }
        q.job[base + j] = run_job(e.run[r], j - e.off[r]);  // tag (.w) 0: not yet published
    }
    wave_stores_done();  // the jobs (and record / pool / pair stores) before the publish below
    __syncthreads();
    if (t == 0) release_lane();  // one L2 writeback for the workgroup (see wave_stores_done)
    __syncthreads();
    // publish: each slot's tag becomes 1 (slots publish independently -- a global publication
    // order would chain every producer behind the one that reserved before it: 80 records of one
    // level published one after another took 300 us)
    for (uint32_t j = t; j < total; j += kBlock)
        __hip_atomic_store(&q.job[base + j].w, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Thread t's result: the number of the cnt keys at sk[base..] whose digit is t (U x kChunk keys
// loaded at a time: the queue's workers, one wave per SIMD, take U = 4; open_local, inside
// segment_sort_kernel's 72-VGPR budget, 1).
constexpr int kQueueIlp = 4;
template <int U = 1>
__device__ __forceinline__ uint32_t chunk_hist(const uint64_t* sk, const uint32_t base, const uint32_t cnt,
                                               const uint32_t lo, const int shift, const uint32_t mask, BigShared& sh)
{
    const int t = threadIdx.x;
    sh.hist[t] = 0u;
    __syncthreads();
    for (uint32_t i0 = 0; i0 < cnt; i0 += U * kChunk) {
        uint32_t dg[U * kChunk / kBlock];
#pragma unroll
        for (int u = 0; u < U * kChunk / kBlock; u++) {
            const uint32_t i = i0 + t + u * kBlock;
            dg[u] = i < cnt ? rec_digit(sk[base + i], lo, shift, mask) : ~0u;
        }
#pragma unroll
        for (int u = 0; u < U * kChunk / kBlock; u++)
            if (dg[u] != ~0u) atomicAdd(&sh.hist[dg[u]], 1u);
    }
    __syncthreads();
    return sh.hist[t];
}

// Rows [r0, r0 + n) of this thread's digit column: each count becomes base + the counts before it
// (an exclusive scan down the column); returns the column's sum.
__device__ __forceinline__ uint32_t scan_column(uint32_t* col, const uint32_t r0, const uint32_t n, uint32_t base)
{
    constexpr uint32_t U = 8;  // independent loads in flight: the column is in other XCDs' writes
    for (uint32_t j0 = 0; j0 < n; j0 += U) {
        uint32_t x[U];
#pragma unroll
        for (uint32_t u = 0; u < U; u++) x[u] = j0 + u < n ? col[(r0 + j0 + u) * kRadix] : 0u;
#pragma unroll
        for (uint32_t u = 0; u < U; u++) {
            if (j0 + u < n) col[(r0 + j0 + u) * kRadix] = base;
            base += x[u];
        }
    }
    return base;
}

// After every chunk's counts are in the record's pool (col = this thread's digit column) -- for a
// grouped record, every group's sums (the chunks' rows hold prefixes within their group): every
// chunk's (group's) destination of each digit (begin + digit start + the digit's count in the chunks
// (groups) before it), the digit starts and totals, and the MIN / MAX rows the SCATTER jobs gather into.
template <bool Grouped = true>  // false: the caller knows the record is ungrouped
__device__ __forceinline__ void plan_scatter(uint32_t* col, const uint32_t chunks, const uint32_t begin, BigShared& sh)
{
    constexpr uint32_t U = 8;
    const uint32_t ng = Grouped ? num_groups(chunks) : 0u;
    const uint32_t r0 = ng ? chunks + 4 : 0u, n = ng ? ng : chunks;
    uint32_t tot = 0u;
    for (uint32_t j0 = 0; j0 < n; j0 += U) {
        uint32_t x[U];
#pragma unroll
        for (uint32_t u = 0; u < U; u++) x[u] = j0 + u < n ? col[(r0 + j0 + u) * kRadix] : 0u;
#pragma unroll
        for (uint32_t u = 0; u < U; u++) tot += x[u];
    }
    uint32_t dummy;
    const uint32_t start = block_exclusive_scan(tot, sh.wave, &dummy);
    scan_column(col, r0, n, begin + start);
    col[chunks * kRadix] = start;
    col[(chunks + 1) * kRadix] = tot;
    col[(chunks + 2) * kRadix] = 0xffffffffu;
    col[(chunks + 3) * kRadix] = 0u;
}

// The last chunk of a record's SCATTER phase (all of its pairs are in buffer dst, and col -- this
// thread's digit column of the record's pool -- holds the digit starts, totals and MIN / MAX rows):
// cut the record into the pieces the queue sorts next, as runs in e (thread 0 publishes them with
// emit_jobs).  Every thread of the workgroup calls it.
__device__ __forceinline__ void cut_pieces(const BigQueue& q, EmitShared& e, BigShared& sh, const uint32_t* col,
                                           const uint32_t chunks, const uint32_t begin, const uint32_t m,
                                           const int shift, const uint32_t dst)
{
    const int t = threadIdx.x;
    // cut the record into pieces, one thread per digit:
    //  * a digit of more than kSegCap pairs: a record of the next level (its varying
    //    bits are known: HIST jobs directly);
    //  * a digit of more than kSegRun pairs: a SMALL piece of its own;
    //  * other non-empty digits: SMALL pieces of consecutive digits whose starts share
    //    a kSegRun-aligned window (so a piece holds < 2 * kSegRun = kSegCap pairs).
    const uint32_t n_d = col[(chunks + 1) * kRadix];  // 0 above the digit mask
    const uint32_t s_d = col[chunks * kRadix];        // relative start
    const uint32_t lo_d = col[(chunks + 2) * kRadix], hi_d = col[(chunks + 3) * kRadix];  // the digit's range
    if (shift == 0) {  // every varying bit is placed: the record is sorted
        if (t == 0) {
            runs_begin(e);
            if (dst) add_run(e, J_COPY, 1u, begin, m, (m + kChunk - 1) / kChunk);  // kChunk pieces
        }
    } else {
        const bool nonempty = n_d != 0u, solo = n_d > (uint32_t)kSegRun;
        uint32_t* pv = sh.hist;  // previous non-empty digit + 1: inclusive max-scan
        uint32_t* nx = sh.run;   // start of the next piece: suffix min-scan
        pv[t] = nonempty ? (uint32_t)t + 1u : 0u;
        sh.cnt[0][t] = solo;
        sh.cnt[1][t] = s_d;
        __syncthreads();
        for (int o = 1; o < kRadix; o <<= 1) {
            const uint32_t x = t >= o ? pv[t - o] : 0u;
            __syncthreads();
            pv[t] = x > pv[t] ? x : pv[t];
            __syncthreads();
        }
        const uint32_t prev = t ? pv[t - 1] : 0u;
        const bool boundary = nonempty && (prev == 0u || solo || sh.cnt[0][prev - 1] != 0u ||
                                           (s_d / kSegRun) != (sh.cnt[1][prev - 1] / kSegRun));
        nx[t] = boundary ? s_d : m;
        __syncthreads();
        for (int o = 1; o < kRadix; o <<= 1) {
            const uint32_t x = t + o < kRadix ? nx[t + o] : m;
            __syncthreads();
            nx[t] = x < nx[t] ? x : nx[t];
            __syncthreads();
        }
        const uint32_t next = t + 1 < kRadix ? nx[t + 1] : m;
        uint4 run = make_uint4(0u, 0u, 0u, 0u);
        bool piece = false;
        if (boundary) {
            if (n_d > (uint32_t)kSegCap)
                run = n_d <= (uint32_t)kWideCap ? make_uint4(J_WIDE | (dst << 8), begin + s_d, n_d, 1u)
                                                : record_run(q, begin + s_d, n_d, dst, true, lo_d, hi_d);
            else if (next - s_d > 1u || dst) {
                if (kDeferPieces)
                    piece = true;
                else
                    run = make_uint4(J_SMALL | (dst << 8), begin + s_d, next - s_d, 1u);
            }
        }
        if (kDeferPieces) {  // pieces go to piece_sort_kernel's list (a SMALL job only if it is full)
            uint32_t npc;
            const uint32_t pi = block_exclusive_scan(piece ? 1u : 0u, sh.wave, &npc);
            if (npc) {  // workgroup-uniform
                if (t == 0)
                    e.pbase = __hip_atomic_fetch_add(&q.ctl[kCtlStride * Q_NPIECE], npc, __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_AGENT);
                __syncthreads();
                if (piece) {
                    const uint32_t k = e.pbase + pi;
                    if (k < q.piece_cap)
                        q.piece[k] = make_uint2(begin + s_d, (next - s_d) | (dst << 31));
                    else
                        run = make_uint4(J_SMALL | (dst << 8), begin + s_d, next - s_d, 1u);
                }
            }
        }
        uint32_t nruns, total;
        const uint32_t ri = block_exclusive_scan(run.w ? 1u : 0u, sh.wave, &nruns);
        const uint32_t ro = block_exclusive_scan(run.w, sh.wave, &total);
        if (run.w) {
            e.run[ri] = run;
            e.off[ri] = ro;
        }
        if (t == 0) {
            e.nruns = nruns;
            e.off[nruns] = total;
        }
    }
}

// A WIDE job: one segment of kSegCap < m <= kWideCap pairs sorted whole by ONE queue worker in LDS
// (big_segment_kernel runs at one workgroup per CU, so it can hold 152 KB): the hot tiles of a skewed
// view and the level-1 digits of a very hot one, each in one job instead of a record's chain of
// REDUCE / HIST / SCATTER hand-offs and pieces (tools/skew_time.py: DESIGN.md "Skewed views").
#ifndef HIDEGS_WIDE_ROUNDS
#define HIDEGS_WIDE_ROUNDS 4  // 64-item rounds a wave ranks at once
#endif
constexpr int kWideRounds = HIDEGS_WIDE_ROUNDS;
constexpr int kWideBatch = 8;  // global loads in flight per thread in the load and gather loops
constexpr int kWideIndexBits = 14;
#ifndef HIDEGS_WIDE_ILP
#define HIDEGS_WIDE_ILP 4
#endif
constexpr int kWideIlp = HIDEGS_WIDE_ILP;  // items per thread in flight in the bucket form's LDS phases
#ifndef HIDEGS_WIDE_MAX_BUCKET
#define HIDEGS_WIDE_MAX_BUCKET 128  // a fuller bucket sends the WIDE segment to the LSD passes
#endif
constexpr int kWideMaxBucket = HIDEGS_WIDE_MAX_BUCKET;
struct WideShared {
    uint32_t k[2][kWideCap];  // low key halves
    uint16_t i[2][kWideCap];  // index in the segment
    uint32_t cnt[kWavesPerBlock][kRadix];
    uint32_t wave[kWavesPerBlock];
    uint32_t red[2][kWavesPerBlock];
};
static_assert(kWideCap <= (1 << kWideIndexBits) && kWideCap % kBlock == 0, "WIDE segment indices are u16 / 14 bits");
static_assert(2 * kBuckets * sizeof(uint32_t) <= sizeof(uint16_t) * kWideCap, "bucket counters fit in i[0]");

// Pairs [begin, begin + m) of (src ? alt : keys) sorted stably by their low 32 key bits into
// keys / vals (m <= kWideCap).  The low halves and indices are sorted in LDS by stable 8-bit LSD
// passes over the bits that vary (per pass: per-wave digit counts, their scan, then each wave ranks
// its contiguous share in input order with wave_rank); the pairs are then gathered by index from alt
// (src 0: copied there first, so keys can be written in place).
__device__ __forceinline__ void wide_sort(uint64_t* __restrict__ keys, uint32_t* __restrict__ vals,
                                          uint64_t* __restrict__ alt_k, uint32_t* __restrict__ alt_v,
                                          const uint32_t begin, const uint32_t m, const uint32_t src, WideShared& w)
{
    const int t = threadIdx.x, lane = lane_id(), wave = t / kWave;
    const uint64_t* sk = src ? alt_k : keys;
#ifdef HIDEGS_QUEUE_TRACE
    __shared__ unsigned int s_wslot;
    if (t == 0) {
        s_wslot = atomicAdd(&g_wtrace_n, 1u);
        if (s_wslot < kWTraceCap) g_wtrace[s_wslot][0] = m;
    }
    __syncthreads();
    const unsigned int wslot = s_wslot;
#endif
    WSTAMP(0);
    uint32_t a = 0xffffffffu, o = 0u, mn = 0xffffffffu, mx = 0u;
    for (uint32_t i0 = 0; i0 < m; i0 += kBlock * kWideBatch) {  // kWideBatch loads in flight per thread
        uint64_t kk[kWideBatch];
        uint32_t vv[kWideBatch];
#pragma unroll
        for (int u = 0; u < kWideBatch; u++) {
            const uint32_t i = i0 + u * kBlock + t;
            if (i < m) {
                kk[u] = sk[begin + i];
                if (!src) vv[u] = vals[begin + i];
            }
        }
#pragma unroll
        for (int u = 0; u < kWideBatch; u++) {
            const uint32_t i = i0 + u * kBlock + t;
            if (i < m) {
                const uint32_t lo = (uint32_t)kk[u];
                w.k[0][i] = lo;
                w.i[0][i] = (uint16_t)i;
                a &= lo;
                o |= lo;
                mn = min(mn, lo);
                mx = max(mx, lo);
                if (!src) {
                    alt_k[begin + i] = kk[u];
                    alt_v[begin + i] = vv[u];
                }
            }
        }
    }
    const SegStats st = segment_stats(a, o, mn, mx, w.red[0], w.red[1]);
    const uint32_t diff = st.diff;  // block-uniform
    WSTAMP(1);
    int cur = 0;
    // Bucket form (as segment_sort's): (x - lo) >> shift over the segment's key range picks a bucket,
    // and an item's place in its bucket is its exact rank by (the bits below || index), so equal keys
    // keep their input order.  Its start / fill counters borrow the storage of i[0].
    const int bshift = st.shift;
    const uint32_t base_lo = st.lo;
    bool lsd = diff != 0u;
    if (diff && bshift + kWideIndexBits <= 32) {  // block-uniform
        const uint32_t lowmask = (uint32_t)((1ull << bshift) - 1ull);
        uint32_t* start = reinterpret_cast<uint32_t*>(&w.i[0][0]);
        uint32_t* fill = start + kBuckets;
        for (int b = t; b < kBuckets; b += kBlock) fill[b] = 0u;
        __syncthreads();
        for (uint32_t i0 = 0; i0 < m; i0 += kWideIlp * kBlock) {  // kWideIlp independent items per thread
            uint32_t x[kWideIlp];
#pragma unroll
            for (int u = 0; u < kWideIlp; u++) {
                const uint32_t i = i0 + u * kBlock + t;
                x[u] = i < m ? w.k[0][i] : 0u;
            }
#pragma unroll
            for (int u = 0; u < kWideIlp; u++)
                if (i0 + u * kBlock + t < m) atomicAdd(&fill[(x[u] - base_lo) >> bshift], 1u);
        }
        __syncthreads();
        WSTAMP(2);
        uint32_t c[kBuckets / kBlock], sum = 0, mx = 0;
#pragma unroll
        for (int j = 0; j < kBuckets / kBlock; j++) {
            c[j] = fill[t * (kBuckets / kBlock) + j];
            sum += c[j];
            mx = c[j] > mx ? c[j] : mx;
        }
        uint32_t dummy;
        uint32_t pre = block_exclusive_scan(sum, w.wave, &dummy);  // its barriers order the reads above
#pragma unroll
        for (int sft = 32; sft >= 1; sft >>= 1) {
            const uint32_t y = __shfl_xor(mx, sft, kWave);
            mx = y > mx ? y : mx;
        }
        if (lane == 0) w.red[0][wave] = mx;
#pragma unroll
        for (int j = 0; j < kBuckets / kBlock; j++) {
            start[t * (kBuckets / kBlock) + j] = pre;
            fill[t * (kBuckets / kBlock) + j] = pre;
            pre += c[j];
        }
        __syncthreads();
        uint32_t fullest = 0;
#pragma unroll
        for (int ww = 0; ww < kWavesPerBlock; ww++) fullest = w.red[0][ww] > fullest ? w.red[0][ww] : fullest;
        WSTAMP(3);
        if (fullest <= (uint32_t)kWideMaxBucket) {  // block-uniform
            uint32_t* comb = w.k[1];
            for (uint32_t i0 = 0; i0 < m; i0 += kWideIlp * kBlock) {
                uint32_t x[kWideIlp], slot[kWideIlp];
#pragma unroll
                for (int u = 0; u < kWideIlp; u++) {
                    const uint32_t i = i0 + u * kBlock + t;
                    x[u] = i < m ? w.k[0][i] : 0u;
                }
#pragma unroll
                for (int u = 0; u < kWideIlp; u++)
                    if (i0 + u * kBlock + t < m) slot[u] = atomicAdd(&fill[(x[u] - base_lo) >> bshift], 1u);
#pragma unroll
                for (int u = 0; u < kWideIlp; u++) {
                    const uint32_t i = i0 + u * kBlock + t;
                    if (i < m) comb[slot[u]] = (((x[u] - base_lo) & lowmask) << kWideIndexBits) | i;
                }
            }
            __syncthreads();
            WSTAMP(4);
            for (uint32_t i0 = 0; i0 < m; i0 += kWideIlp * kBlock) {
                uint32_t me[kWideIlp], s0[kWideIlp], e0[kWideIlp], rank[kWideIlp];
                uint32_t len = 0;
#pragma unroll
                for (int u = 0; u < kWideIlp; u++) {
                    const uint32_t i = i0 + u * kBlock + t;
                    const uint32_t x = (i < m ? w.k[0][i] : base_lo) - base_lo;
                    const uint32_t bk = x >> bshift;
                    me[u] = ((x & lowmask) << kWideIndexBits) | i;
                    s0[u] = start[bk];
                    e0[u] = i < m ? fill[bk] : s0[u];
                    rank[u] = 0u;
                    len = e0[u] - s0[u] > len ? e0[u] - s0[u] : len;
                }
                for (uint32_t j = 0; j < len; j++) {  // the kWideIlp bucket walks interleaved
#pragma unroll
                    for (int u = 0; u < kWideIlp; u++)
                        if (s0[u] + j < e0[u]) rank[u] += comb[s0[u] + j] < me[u] ? 1u : 0u;
                }
#pragma unroll
                for (int u = 0; u < kWideIlp; u++)
                    if (i0 + u * kBlock + t < m) w.i[1][s0[u] + rank[u]] = (uint16_t)(i0 + u * kBlock + t);
            }
            __syncthreads();
            WSTAMP(5);
            cur = 1;
            lsd = false;
        } else {  // crowded buckets: the LSD passes below, whose i[0] the counters overwrote
            for (uint32_t i = t; i < m; i += kBlock) w.i[0][i] = (uint16_t)i;
            __syncthreads();
        }
    }
    const uint32_t C = (m + kBlock - 1) / kBlock * kWave;  // each wave's contiguous share (64-item rounds)
    const uint32_t w0 = wave * C, w1 = w0 + C < m ? w0 + C : m;
    for (int shift = 0; shift < 32 && lsd; shift += kRadixBits) {
        const uint32_t vary = (diff >> shift) & (kRadix - 1);
        if (vary == 0) continue;  // digit constant over the segment (block-uniform)
        for (int i = t; i < kWavesPerBlock * kRadix; i += kBlock) (&w.cnt[0][0])[i] = 0u;
        __syncthreads();
        for (uint32_t i0 = w0; i0 < w1; i0 += 4 * kWave) {
            uint32_t x[4];
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const uint32_t i = i0 + u * kWave + lane;
                x[u] = i < w1 ? w.k[cur][i] : 0u;
            }
#pragma unroll
            for (int u = 0; u < 4; u++)
                if (i0 + u * kWave + lane < w1) atomicAdd(&w.cnt[wave][(x[u] >> shift) & (kRadix - 1)], 1u);
        }
        __syncthreads();
        const uint32_t tot = digit_wave_prefix(w.cnt);  // cnt[ww][d]: digit d in waves before ww
        uint32_t dummy;
        const uint32_t start = block_exclusive_scan(tot, w.wave, &dummy);  // its barriers order the above
#pragma unroll
        for (int ww = 0; ww < kWavesPerBlock; ww++) w.cnt[ww][t] += start;  // thread t owns digit t
        __syncthreads();
        for (uint32_t r0 = w0; r0 < w1; r0 += kWideRounds * kWave) {  // wave-uniform
            uint32_t kk[kWideRounds], id[kWideRounds], rank[kWideRounds];
            bool ok[kWideRounds];
#pragma unroll
            for (int q = 0; q < kWideRounds; q++) {
                const uint32_t i = r0 + q * kWave + lane;
                ok[q] = i < w1;
                kk[q] = ok[q] ? w.k[cur][i] : 0u;
                id[q] = ok[q] ? w.i[cur][i] : 0u;
            }
            // cnt starts at each digit's first position for this wave: rank = the item's position
            wave_rank<uint32_t, kWideRounds>(kk, ok, shift, kRadix - 1, w.cnt[wave], rank, vary);
#pragma unroll
            for (int q = 0; q < kWideRounds; q++) {
                if (ok[q]) {
                    w.k[cur ^ 1][rank[q]] = kk[q];
                    w.i[cur ^ 1][rank[q]] = (uint16_t)id[q];
                }
            }
        }
        __syncthreads();
        cur ^= 1;
    }
    WSTAMP(6);
    if (!diff && !src) return;  // equal low keys, in place: the input order is the stable order
    for (uint32_t j0 = 0; j0 < m; j0 += kBlock * kWideBatch) {
        uint32_t ii[kWideBatch];
        uint64_t kk[kWideBatch];
        uint32_t vv[kWideBatch];
#pragma unroll
        for (int u = 0; u < kWideBatch; u++) {
            const uint32_t j = j0 + u * kBlock + t;
            ii[u] = j < m ? w.i[cur][j] : 0u;
        }
#pragma unroll
        for (int u = 0; u < kWideBatch; u++) {
            if (j0 + u * kBlock + t < m) {
                kk[u] = alt_k[begin + ii[u]];
                vv[u] = alt_v[begin + ii[u]];
            }
        }
#pragma unroll
        for (int u = 0; u < kWideBatch; u++) {
            const uint32_t j = j0 + u * kBlock + t;
            if (j < m) {
                keys[begin + j] = kk[u];
                vals[begin + j] = vv[u];
            }
        }
    }
#ifdef HIDEGS_QUEUE_TRACE
    wave_stores_done();
    __syncthreads();
#endif
    WSTAMP(7);
}

union SegLds {
    SegShared lsd;
    BucketShared bucket;
    BigShared big;
    struct {
        BigShared big;
        EmitShared emit;
        uint32_t list[kBlock];  // segment_sort_kernel's scouts: the hot tiles of one sweep
        uint32_t nlist;
    } queue;
};

// big_segment_kernel's LDS: the queue forms, or one WIDE job's buffers (152 KB: one worker per CU)
union QueueLds {
    SegLds seg;
    WideShared wide;
};

// One segment of m <= kSegCap pairs sorted by the low 32 key bits: the bucket form, or its LSD
// fallback for crowded buckets (segment_sort_kernel carries the same code inline).  InPlace: (src_k, src_v) == (dst_k, dst_v); otherwise the pairs
// are read from alt and written to keys (a piece of a partitioned hot tile).
template <bool InPlace>
__device__ __forceinline__ void sort_segment(const uint64_t* __restrict__ src_k, const uint32_t* __restrict__ src_v,
                                             uint64_t* __restrict__ dst_k, uint32_t* __restrict__ dst_v,
                                             const uint32_t begin, const uint32_t m, SegLds& lds, uint32_t* s_and,
                                             uint32_t* s_or, uint32_t* s_max)
{
    uint64_t* dk = InPlace ? const_cast<uint64_t*>(src_k) : dst_k;
    uint32_t* dv = InPlace ? const_cast<uint32_t*>(src_v) : dst_v;
    const int t = threadIdx.x, lane = lane_id(), wave = t / kWave;
    uint64_t k[kSegItems];
    uint32_t v[kSegItems];
    uint32_t a = 0xffffffffu, o = 0, lo = 0xffffffffu, hi = 0;
    const uint32_t ref_hi = m ? (uint32_t)(src_k[begin] >> 32) : 0u;  // see segment_sort_kernel (m == 0: no read)
    uint32_t hd = 0;
#pragma unroll
    for (int q = 0; q < kSegItems; q++) {
        const uint32_t i = t + q * kBlock;
        if (i < m) {
            k[q] = src_k[begin + i];
            v[q] = src_v[begin + i];
            const uint32_t x = (uint32_t)k[q];
            a &= x;
            o |= x;
            lo = min(lo, x);
            hi = max(hi, x);
            hd |= (uint32_t)(k[q] >> 32) ^ ref_hi;
        }
    }
    BucketShared& sh = lds.bucket;
    for (int i = t; i < kBuckets; i += kBlock) sh.fill[i] = 0u;
    const SegStats st = segment_stats(a, o, lo, hi, s_and, s_or);
    const uint32_t diff = st.diff;  // low key bits that vary over the segment
    if (diff == 0) {  // equal low keys: the input order is the stable order
        if (!InPlace) {
#pragma unroll
            for (int q = 0; q < kSegItems; q++) {
                const uint32_t i = t + q * kBlock;
                if (i < m) {
                    dk[begin + i] = k[q];
                    dv[begin + i] = v[q];
                }
            }
        }
        return;
    }
    const int shift = st.shift;
    const uint32_t base_lo = st.lo;
    const uint32_t lowmask = (uint32_t)((1ull << shift) - 1ull);

    // 1. bucket histogram (bucket = (x - lo) >> shift < 2^dbits)
#pragma unroll
    for (int q = 0; q < kSegItems; q++)
        if (t + q * kBlock < m) atomicAdd(&sh.fill[((uint32_t)k[q] - base_lo) >> shift], 1u);
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
    const bool wave_hd = __ballot(hd != 0u) != 0ull;
    if (lane == 0) s_and[wave] = mx | (wave_hd ? 0x80000000u : 0u);  // mx <= kSegCap: bit 31 is free
#pragma unroll
    for (int j = 0; j < kBuckets / kBlock; j++) {
        sh.start[t * (kBuckets / kBlock) + j] = pre;
        sh.fill[t * (kBuckets / kBlock) + j] = pre;
        pre += c[j];
    }
    __syncthreads();
    uint32_t fullest = 0, mixed_hi = 0;
#pragma unroll
    for (int w = 0; w < kWavesPerBlock; w++) {
        const uint32_t f = s_and[w] & 0x7fffffffu;
        fullest = f > fullest ? f : fullest;
        mixed_hi |= s_and[w] >> 31;
    }
    if (fullest > (uint32_t)kMaxBucket || shift + kIndexBits > 32) {  // crowded depths, or fields too
        // wide for 32 bits: the LSD form (block-uniform branch)
        __syncthreads();
        segment_sort_lsd<InPlace>(src_k, src_v, dst_k, dst_v, begin, m, diff, lds.lsd);
        return;
    }
    // 3. fill the buckets in any order
    uint32_t me[kSegItems];
    uint32_t bucket[kSegItems];
#pragma unroll
    for (int q = 0; q < kSegItems; q++) {
        const uint32_t i = t + q * kBlock;
        if (i < m) {
            const uint32_t x = (uint32_t)k[q] - base_lo;
            bucket[q] = x >> shift;
            me[q] = ((x & lowmask) << kIndexBits) | i;
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
    if (HIDEGS_SEG_COMPACT_STAGE && !mixed_hi) {  // one high half: low halves + values in one pass
        uint32_t* stage_lo = reinterpret_cast<uint32_t*>(&sh);
        uint32_t* stage_vv = stage_lo + kSegCap;
#pragma unroll
        for (int q = 0; q < kSegItems; q++) {
            if (t + q * kBlock < m) {
                stage_lo[pos[q]] = (uint32_t)k[q];
                stage_vv[pos[q]] = v[q];
            }
        }
        __syncthreads();
        const uint64_t khi = (uint64_t)ref_hi << 32;
#pragma unroll
        for (int q = 0; q < kSegItems; q++) {
            const uint32_t i = t + q * kBlock;
            if (i < m) {
                dk[begin + i] = khi | stage_lo[i];
                dv[begin + i] = stage_vv[i];
            }
        }
        return;
    }
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
            dk[begin + i] = stage_k[i];
            if (together) dv[begin + i] = stage_v[i];
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
        if (i < m) dv[begin + i] = stage_v[i];
    }
}

// A record's first two phases (REDUCE, HIST) run by the workgroup that opens it, inside
// segment_sort_kernel where the other segments' sorts hide them, for a tile of up to kOpenLocal
// pairs: the queue then starts at the SCATTER jobs.
#ifndef HIDEGS_OPEN_LOCAL
#define HIDEGS_OPEN_LOCAL 24576
#endif
constexpr int kOpenLocal = HIDEGS_OPEN_LOCAL;
static_assert(kOpenLocal <= (int)kGroupChunks * kChunk, "open_local plans an ungrouped record (pending == chunks)");
#ifndef HIDEGS_SCATTER_LOCAL
#define HIDEGS_SCATTER_LOCAL 0  // ... and up to this many, its SCATTER phase too (0: never; DESIGN.md, range digits)
#endif
constexpr int kScatterLocal = HIDEGS_SCATTER_LOCAL;
#ifndef HIDEGS_SCOUTS
#define HIDEGS_SCOUTS 128  // segment_sort_kernel's first workgroups, which start the hot tiles (0: own workgroup)
#endif
constexpr int kScouts = HIDEGS_SCOUTS;
constexpr int kScoutItems = 32;  // segments per scout thread per sweep (a sweep: 8192 segments)
// a scout's share of one sweep's hot tiles fits its kBlock-entry list
static_assert(kScouts == 0 || kBlock * kScoutItems <= kScouts * kBlock, "HIDEGS_SCOUTS: at least 32 scouts (or 0)");
__device__ __forceinline__ void open_local(const uint64_t* keys, const uint32_t* vals, const BigQueue& q,
                                           const uint32_t begin,
                                           const uint32_t m, BigShared& sh, EmitShared& e, uint32_t* s_and,
                                           uint32_t* s_or)
{
    const int t = threadIdx.x, lane = lane_id(), wave = t / kWave;
    uint32_t lo = 0xffffffffu, hi = 0u;
    for (uint32_t i0 = 0; i0 < m; i0 += kChunk) {
        uint32_t x[kChunk / kBlock];
#pragma unroll
        for (int u = 0; u < kChunk / kBlock; u++) {
            const uint32_t i = i0 + u * kBlock + t;
            x[u] = (uint32_t)keys[begin + (i < m ? i : 0u)];  // a repeat changes no MIN / MAX
        }
#pragma unroll
        for (int u = 0; u < kChunk / kBlock; u++) {
            lo = min(lo, x[u]);
            hi = max(hi, x[u]);
        }
    }
    wave_min_max(lo, hi);
    if (lane == 0) {
        s_and[wave] = lo;
        s_or[wave] = hi;
    }
    __syncthreads();
    for (int w = 0; w < kWavesPerBlock; w++) {
        lo = min(lo, s_and[w]);
        hi = max(hi, s_or[w]);
    }
    if (lo == hi) return;  // equal low keys: in stable order already (block-uniform)
    if (t == 0) {
        runs_begin(e);
        const uint4 r = record_run<false>(q, begin, m, 0u, true, lo, hi);
        e.run[0] = r;
        e.base = (r.x & 0xffu) == J_HIST ? q.rec[r.y].pool : ~0u;
        if (e.base == ~0u) add_run(e, r);  // the table or pool is full: a GLOBAL job
    }
    __syncthreads();
    const uint32_t pool = e.base, rec = e.run[0].y, chunks = (m + kChunk - 1) / kChunk;
    if (pool != ~0u) {
        int shift, bits;
        range_digit(lo, hi, shift, bits);  // the record's digit (set_digit)
        const uint32_t mask = (1u << bits) - 1u;
        uint32_t* col = q.pool + pool + t;
        for (uint32_t c = 0; c < chunks; c++) {
            const uint32_t c0 = c * kChunk;
            col[c * kRadix] = chunk_hist(keys, begin + c0, m - c0 < (uint32_t)kChunk ? m - c0 : (uint32_t)kChunk,
                                         lo, shift, mask, sh);
        }
        __syncthreads();
        plan_scatter<false>(col, chunks, begin, sh);
        if (m <= (uint32_t)kScatterLocal) {
            // and the SCATTER phase too: only the pieces go to the queue
            sh.aux[0][t] = 0xffffffffu;
            sh.aux[1][t] = 0u;
            for (uint32_t c = 0; c < chunks; c++) {
                const uint32_t c0 = c * kChunk, cnt = m - c0 < (uint32_t)kChunk ? m - c0 : (uint32_t)kChunk;
                sh.run[t] = col[c * kRadix];
                for (uint32_t b = 0; b < cnt; b += kBigStep)
                    scatter_step<true>(keys, vals, q.alt_k, q.alt_v, begin + c0 + b,
                                       cnt - b < (uint32_t)kBigStep ? cnt - b : (uint32_t)kBigStep, lo, shift, mask,
                                       begin, begin + m, sh);
            }
            col[(chunks + 2) * kRadix] = sh.aux[0][t];  // this thread's own column: no barrier needed
            col[(chunks + 3) * kRadix] = sh.aux[1][t];
            __syncthreads();
            cut_pieces(q, e, sh, col, chunks, begin, m, shift, 1u);
        } else if (t == 0) {
            runs_begin(e);
            add_run(e, J_SCATTER, 0u, rec, 0u, chunks);  // pending == chunks already
        }
    }
    emit_jobs(q, e);
}

// Workgroup b sorts segment b in place by the low 32 key bits (sort_segment); a segment of more
// than kSegCap pairs becomes a record of the partition queue (big_segment_kernel runs it).
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(HIDEGS_SEG_WAVES))) void segment_sort_kernel(
    uint64_t* __restrict__ keys, uint32_t* __restrict__ vals, const uint32_t* __restrict__ starts,
    uint2* __restrict__ ranges_out, const int nseg, const BigQueue q)
{
    __shared__ __attribute__((aligned(16))) SegLds lds;
    __shared__ uint32_t s_and[kWavesPerBlock], s_or[kWavesPerBlock], s_max[kWavesPerBlock];
    if (kScouts > 0 && blockIdx.x < (unsigned)kScouts) {
        // a scout: the first workgroups dispatched find the hot tiles (over kQueueMin pairs) and start
        // them -- the local phases of open_local, or a queue record -- while the other workgroups sort
        // the ordinary tiles, instead of wherever in the grid the hot tile's own workgroup would run.
        // Every scout sweeps all segments and numbers the hot ones the same way (thread-major within a
        // sweep); scout b takes the hot tiles numbered b mod kScouts, so the hot tiles of one image
        // region -- neighbouring segment ids -- are opened side by side, not by one scout in turn
        // (71 hot tiles of a skewed view: 1.13 ms of segment_sort with 16 scouts of 256-segment stripes)
        uint32_t* list = lds.queue.list;
        uint32_t carry = 0u;  // hot tiles numbered in earlier sweeps
        for (uint32_t s0 = 0; s0 < (uint32_t)nseg; s0 += kBlock * kScoutItems) {
            if (threadIdx.x == 0) lds.queue.nlist = 0u;
            uint32_t hot = 0u;  // bit u: segment s0 + u * kBlock + threadIdx.x is hot
#pragma unroll 8
            for (int u = 0; u < kScoutItems; u++) {
                const uint32_t sg = s0 + (uint32_t)u * kBlock + threadIdx.x;
                if (sg < (uint32_t)nseg && starts[sg + 1] - starts[sg] > (uint32_t)kQueueMin) hot |= 1u << u;
            }
            uint32_t nhot;
            const uint32_t base = carry + block_exclusive_scan((uint32_t)__builtin_popcount(hot), s_max, &nhot);
            carry += nhot;  // block-uniform
            if (nhot == 0u) continue;
            uint32_t ord = base;
            for (uint32_t h = hot; h; h &= h - 1u, ord++)
                if (ord % (uint32_t)kScouts == blockIdx.x)
                    list[atomicAdd(&lds.queue.nlist, 1u)] = s0 + (uint32_t)__builtin_ctz(h) * kBlock + threadIdx.x;
            __syncthreads();
            const uint32_t nl = lds.queue.nlist;  // workgroup-uniform
            for (uint32_t j = 0; j < nl; j++) {
                const uint32_t sg2 = list[j], b = starts[sg2], mm = starts[sg2 + 1] - b;
                if (HIDEGS_WIDE_SCOUTS && mm <= (uint32_t)kWideCap) {  // one WIDE job (a queue worker sorts it in LDS)
                    if (threadIdx.x == 0) {
                        runs_begin(lds.queue.emit);
                        add_run(lds.queue.emit, J_WIDE, 0u, b, mm, 1u);
                    }
                    emit_jobs(q, lds.queue.emit);
                } else if (mm <= (uint32_t)kOpenLocal) {
                    open_local(keys, vals, q, b, mm, lds.queue.big, lds.queue.emit, s_and, s_or);
                } else {
                    if (threadIdx.x == 0) {
                        runs_begin(lds.queue.emit);
                        add_run(lds.queue.emit, record_run(q, b, mm, 0u, false, 0u, 0u));
                    }
                    emit_jobs(q, lds.queue.emit);
                }
                __syncthreads();  // the LDS is reused by the next one
            }
        }
        return;
    }
    const uint32_t seg = blockIdx.x - kScouts;
    // segment seg is [starts[seg], starts[seg + 1]); with ranges_out it is also tile seg's range,
    // (0, 0) when empty -- identifyTileRanges' result
    const uint2 r = make_uint2(starts[seg], starts[seg + 1]);
    if (ranges_out && threadIdx.x == 0) ranges_out[seg] = r.y > r.x ? r : make_uint2(0u, 0u);
    const uint32_t begin = r.x, m = r.y - r.x;
    if (r.y <= r.x + 1) return;  // absent or single pair: already in place
    if (m > (uint32_t)kSegCap) {
        if (m <= (uint32_t)kQueueMin) {  // mildly hot: this workgroup, overlapped with the others
            segment_sort_global(keys, vals, q.alt_k, q.alt_v, begin, m, lds.big);
            return;
        }
        if (kScouts > 0) return;  // hot: a scout has it
        if (m <= (uint32_t)kOpenLocal) {
            open_local(keys, vals, q, begin, m, lds.queue.big, lds.queue.emit, s_and, s_or);
            return;
        }
        if (threadIdx.x == 0) {
            runs_begin(lds.queue.emit);
            add_run(lds.queue.emit, record_run(q, begin, m, 0u, false, 0u, 0u));
        }
        emit_jobs(q, lds.queue.emit);
        return;
    }
    // sort_segment<true>'s code, written out: as an inlined call the same code spills 16 VGPRs at
    // the 72-VGPR budget of HIDEGS_SEG_WAVES (the register allocator sees it differently)
    const int t = threadIdx.x, lane = lane_id(), wave = t / kWave;
    uint64_t k[kSegItems];
    uint32_t v[kSegItems];
    uint32_t a = 0xffffffffu, o = 0, lo = 0xffffffffu, hi = 0;
    // the segment's first high key half: the segment id (tile), and with no bits above end_bit -- as
    // hidegs_sort_tile_pairs' callers guarantee -- every pair's high half; `hd` records any that differs
    const uint32_t ref_hi = (uint32_t)(keys[begin] >> 32);
    uint32_t hd = 0;
#pragma unroll
    for (int q = 0; q < kSegItems; q++) {
        const uint32_t i = t + q * kBlock;
        if (i < m) {
            k[q] = keys[begin + i];
            v[q] = vals[begin + i];
            const uint32_t x = (uint32_t)k[q];
            a &= x;
            o |= x;
            lo = min(lo, x);
            hi = max(hi, x);
            hd |= (uint32_t)(k[q] >> 32) ^ ref_hi;
        }
    }
    BucketShared& sh = lds.bucket;
    for (int i = t; i < kBuckets; i += kBlock) sh.fill[i] = 0u;
    const SegStats st = segment_stats(a, o, lo, hi, s_and, s_or);
    const uint32_t diff = st.diff;  // low key bits that vary over the segment
    if (diff == 0) return;  // equal low keys: the input order is the stable order
    const int shift = st.shift;
    const uint32_t base_lo = st.lo;
    const uint32_t lowmask = (uint32_t)((1ull << shift) - 1ull);

    // 1. bucket histogram (bucket = (x - lo) >> shift, over the segment's key range)
#pragma unroll
    for (int q = 0; q < kSegItems; q++)
        if (t + q * kBlock < m) atomicAdd(&sh.fill[((uint32_t)k[q] - base_lo) >> shift], 1u);
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
    const bool wave_hd = __ballot(hd != 0u) != 0ull;
    if (lane == 0) s_and[wave] = mx | (wave_hd ? 0x80000000u : 0u);  // mx <= kSegCap: bit 31 is free
#pragma unroll
    for (int j = 0; j < kBuckets / kBlock; j++) {
        sh.start[t * (kBuckets / kBlock) + j] = pre;
        sh.fill[t * (kBuckets / kBlock) + j] = pre;
        pre += c[j];
    }
    __syncthreads();
    uint32_t fullest = 0, mixed_hi = 0;
#pragma unroll
    for (int w = 0; w < kWavesPerBlock; w++) {
        const uint32_t f = s_and[w] & 0x7fffffffu;
        fullest = f > fullest ? f : fullest;
        mixed_hi |= s_and[w] >> 31;
    }
    if (fullest > (uint32_t)kMaxBucket || shift + kIndexBits > 32) {  // crowded depths, or fields too
        // wide for 32 bits: the LSD form (block-uniform branch)
        __syncthreads();
        segment_sort_lsd<true>(keys, vals, nullptr, nullptr, begin, m, diff, lds.lsd);
        return;
    }
    // 3. fill the buckets in any order
    uint32_t me[kSegItems];
    uint32_t bucket[kSegItems];
#pragma unroll
    for (int q = 0; q < kSegItems; q++) {
        const uint32_t i = t + q * kBlock;
        if (i < m) {
            const uint32_t x = (uint32_t)k[q] - base_lo;
            bucket[q] = x >> shift;
            me[q] = ((x & lowmask) << kIndexBits) | i;
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
    if (HIDEGS_SEG_COMPACT_STAGE && !mixed_hi) {
        // one high half for the whole segment: stage the low halves and the values, (4 + 4) B per pair,
        // so a segment of up to kSegCap pairs goes through LDS in one pass, and rebuild the keys on store
        uint32_t* stage_lo = reinterpret_cast<uint32_t*>(&sh);
        uint32_t* stage_vv = stage_lo + kSegCap;
#pragma unroll
        for (int q = 0; q < kSegItems; q++) {
            if (t + q * kBlock < m) {
                stage_lo[pos[q]] = (uint32_t)k[q];
                stage_vv[pos[q]] = v[q];
            }
        }
        __syncthreads();
        const uint64_t khi = (uint64_t)ref_hi << 32;
#pragma unroll
        for (int q = 0; q < kSegItems; q++) {
            const uint32_t i = t + q * kBlock;
            if (i < m) {
                keys[begin + i] = khi | stage_lo[i];
                vals[begin + i] = stage_vv[i];
            }
        }
        return;
    }
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


// The last workgroup to count `pending` down (a record's phase, or a chunk group of its HIST phase)
// goes on (returns true); the others return false.  The caller's global writes are published before
// the count-down.
__device__ __forceinline__ bool finish_phase(uint32_t& pending, uint32_t* s_flag)
{
    wave_stores_done();
    __syncthreads();
    if (threadIdx.x == 0) {
        release_lane();
        const bool last = __hip_atomic_fetch_add(&pending, 0xffffffffu, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 1u;
        if (last) acquire_lane();
        *s_flag = last;
    }
    __syncthreads();
    return *s_flag != 0;
}

// The partition queue's workers: kQueueBlocks workgroups take jobs until none is left or in
// flight.  With no hot tile (the common case) every workgroup reads one counter and exits.
__global__ __launch_bounds__(kBlock) void big_segment_kernel(uint64_t* __restrict__ keys, uint32_t* __restrict__ vals,
                                                             uint64_t* __restrict__ alt_k,
                                                             uint32_t* __restrict__ alt_v, const BigQueue q)
{
    __shared__ __attribute__((aligned(16))) QueueLds qlds;
    __shared__ uint32_t s_and[kWavesPerBlock], s_or[kWavesPerBlock], s_max[kWavesPerBlock];
    __shared__ uint4 s_job;
    __shared__ uint32_t s_flag;
    SegLds& lds = qlds.seg;
    const int t = threadIdx.x, lane = lane_id(), wave = t / kWave;
    BigShared& sh = lds.queue.big;
    EmitShared& e = lds.queue.emit;
    if (t == 0) s_flag = q_peek(&q.ctl[kCtlStride * Q_RESERVE]);
    __syncthreads();
    if (s_flag == 0) return;  // nothing was queued (the queue was filled by the previous launch)
#ifdef HIDEGS_QUEUE_TRACE
    unsigned long long t_claim = 0, t_got = 0;
    uint32_t t_index = 0;
#endif
    for (;;) {
        __syncthreads();  // the previous job's LDS use is over
        if (t == 0) {
            // the claim only hands out a slot index: relaxed (an acq_rel RMW here is an L2 writeback
            // and invalidate per job; the job's data is acquired after its tag is seen)
            const uint32_t i = __hip_atomic_fetch_add(&q.ctl[kCtlStride * Q_HEAD], 1u, __ATOMIC_RELAXED,
                                                      __HIP_MEMORY_SCOPE_AGENT);
#ifdef HIDEGS_QUEUE_TRACE
            t_claim = wall_clock64();
            t_index = i;
#endif
            uint4 job = make_uint4(J_EXIT, 0u, 0u, 0u);
            uint32_t polls = 0, backoff = 1;
            bool reserved = false;  // slot i is reserved: a job will be published there (reserve only grows)
            for (; polls < kMaxPolls; polls++) {
                if (i < q.job_cap && q_peek(&q.job[i].w) != 0u) {
                    acquire_lane();  // for the whole workgroup (see wave_stores_done)
                    job = q.job[i];
                    break;
                }
                // the shared counters are polled only while slot i is not reserved (reading `done` on
                // one poll in 4 only, or backing off to 64 sleeps, measured slower: DESIGN.md)
                if (!reserved) {
                    const uint32_t r0 = q_peek(&q.ctl[kCtlStride * Q_RESERVE]);
                    reserved = i < r0 && i < q.job_cap;
                    if (!reserved && q_peek(&q.ctl[kCtlStride * Q_DONE]) == r0) {
                        // confirm in order: `done` (acquire) before `reserve`
                        const uint32_t d = q_load(&q.ctl[kCtlStride * Q_DONE]);
                        const uint32_t r = q_load(&q.ctl[kCtlStride * Q_RESERVE]);
                        if (d == r && i >= r) break;  // nothing queued, nothing in flight: the end
                    }
                }
                for (uint32_t k = 0; k < backoff; k++) __builtin_amdgcn_s_sleep(8);  // ~0.2 us each
                backoff = backoff < (uint32_t)HIDEGS_BACKOFF_MAX ? 2u * backoff : (uint32_t)HIDEGS_BACKOFF_MAX;
            }
            if (polls == kMaxPolls) q_flag(q, 4u);
            s_job = job;
#ifdef HIDEGS_QUEUE_TRACE
            t_got = wall_clock64();
#endif
        }
        __syncthreads();
        const uint4 job = s_job;
        const uint32_t type = job.x & 0xffu, src = job.x >> 8;
        if (type == J_EXIT) return;

        if (type == J_WIDE) {
            wide_sort(keys, vals, alt_k, alt_v, job.y, job.z, src, qlds.wide);
        } else if (type == J_SMALL) {
            if (src)
                sort_segment<false>(alt_k, alt_v, keys, vals, job.y, job.z, lds, s_and, s_or, s_max);
            else
                sort_segment<true>(keys, vals, nullptr, nullptr, job.y, job.z, lds, s_and, s_or, s_max);
        } else if (type == J_COPY) {
            for (uint32_t i = t; i < job.z; i += kBlock) {
                keys[job.y + i] = alt_k[job.y + i];
                vals[job.y + i] = alt_v[job.y + i];
            }
        } else if (type == J_GLOBAL) {
            if (src) {
                for (uint32_t i = t; i < job.z; i += kBlock) {
                    keys[job.y + i] = alt_k[job.y + i];
                    vals[job.y + i] = alt_v[job.y + i];
                }
                __syncthreads();
            }
            segment_sort_global(keys, vals, alt_k, alt_v, job.y, job.z, sh);
        } else {  // a chunk job of record job.y
            BigSeg& s = q.rec[job.y];
            const uint32_t c = job.z, begin = s.begin, m = s.m, chunks = s.chunks, csize = s.csize;
            const uint32_t c0 = c * csize, cnt = m - c0 < csize ? m - c0 : csize;
            const uint64_t* sk = s.src ? alt_k : keys;
            uint32_t* col = q.pool + s.pool + t;  // this thread's digit column
            if (type == J_REDUCE) {
                uint32_t lo = 0xffffffffu, hi = 0u;
                for (uint32_t i0 = 0; i0 < cnt; i0 += kQueueIlp * kChunk) {
                    uint32_t x[kQueueIlp * kChunk / kBlock];
#pragma unroll
                    for (int u = 0; u < kQueueIlp * kChunk / kBlock; u++) {
                        const uint32_t i = i0 + t + u * kBlock;
                        x[u] = i < cnt ? (uint32_t)sk[begin + c0 + i] : 0xffffffffu;
                    }
#pragma unroll
                    for (int u = 0; u < kQueueIlp * kChunk / kBlock; u++) {
                        const uint32_t i = i0 + t + u * kBlock;
                        lo = min(lo, x[u]);
                        hi = i < cnt ? max(hi, x[u]) : hi;
                    }
                }
                wave_min_max(lo, hi);
                if (lane == 0) {
                    s_and[wave] = lo;
                    s_or[wave] = hi;
                }
                __syncthreads();
                if (t == 0) {
                    for (int w = 0; w < kWavesPerBlock; w++) {
                        lo = min(lo, s_and[w]);
                        hi = max(hi, s_or[w]);
                    }
                    __hip_atomic_fetch_min(&s.lo_bits, lo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    __hip_atomic_fetch_max(&s.hi_bits, hi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
                if (finish_phase(s.pending, &s_flag)) {
                    if (t == 0) {
                        runs_begin(e);
                        const uint32_t rlo = q_load(&s.lo_bits), rhi = q_load(&s.hi_bits);
                        if (rlo == rhi) {  // equal low keys: already in stable order
                            if (s.src) add_run(e, J_COPY, 1u, begin, m, (m + kChunk - 1) / kChunk);
                        } else {
                            set_digit(s, rlo, rhi);
                            s.pending = hist_countdown(q, s);
                            add_run(e, J_HIST, 0u, job.y, 0u, chunks);
                        }
                    }
                    emit_jobs(q, e);
                }
            } else if (type == J_HIST) {
                const int shift = (int)s.shift;
                const uint32_t mask = (1u << s.bits) - 1u;
                col[c * kRadix] = chunk_hist<kQueueIlp>(sk, begin + c0, cnt, s.lo, shift, mask, sh);
                const uint32_t ng = num_groups(chunks);
                bool last;
                if (ng) {  // the group's countdown first; its last chunk scans the group's rows
                    const uint32_t G = group_chunks(chunks), g = c / G, g0 = g * G;
                    last = finish_phase(q.pool[s.pool + (chunks + 4 + ng) * kRadix + g], &s_flag);
                    if (last) {
                        col[(chunks + 4 + g) * kRadix] = scan_column(col, g0, chunks - g0 < G ? chunks - g0 : G, 0u);
                        last = finish_phase(s.pending, &s_flag);
                    }
                } else {
                    last = finish_phase(s.pending, &s_flag);
                }
                if (last) {
                    plan_scatter(col, chunks, begin, sh);
                    if (t == 0) {
                        s.pending = chunks;
                        runs_begin(e);
                        add_run(e, J_SCATTER, 0u, job.y, 0u, chunks);
                    }
                    emit_jobs(q, e);
                }
            } else {  // J_SCATTER
                const int shift = (int)s.shift;
                const uint32_t mask = (1u << s.bits) - 1u;
                const uint32_t dst = s.src ^ 1u;
                const uint32_t* sv = s.src ? alt_v : vals;
                uint64_t* dk = dst ? alt_k : keys;
                uint32_t* dv = dst ? alt_v : vals;
                const uint32_t ng = num_groups(chunks);  // grouped: + the group's base
                sh.run[t] = col[c * kRadix] + (ng ? col[(chunks + 4 + c / group_chunks(chunks)) * kRadix] : 0u);
                sh.aux[0][t] = 0xffffffffu;
                sh.aux[1][t] = 0u;
                scatter_steps<true>(sk, sv, dk, dv, begin + c0, cnt, s.lo, shift, mask, begin, begin + m, sh);
                // this chunk's per-digit MIN / MAX into the record's (digits it holds only)
                if (sh.aux[0][t] != 0xffffffffu || sh.aux[1][t] != 0u) {
                    __hip_atomic_fetch_min(&col[(chunks + 2) * kRadix], sh.aux[0][t], __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
                    __hip_atomic_fetch_max(&col[(chunks + 3) * kRadix], sh.aux[1][t], __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
                }
                if (finish_phase(s.pending, &s_flag)) {
                    cut_pieces(q, e, sh, col, chunks, begin, m, shift, dst);
                    emit_jobs(q, e);
                }
            }
        }
        // `done` only ends the queue (no data hangs on it): the jobs this one queued are
        // published already, and the pairs it wrote are for kernel completion or a publish
        __syncthreads();
        if (t == 0) __hip_atomic_fetch_add(&q.ctl[kCtlStride * Q_DONE], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#ifdef HIDEGS_QUEUE_TRACE
        if (t == 0) {
            const unsigned int slot = atomicAdd(&g_qtrace_n, 1u);
            if (slot < kQTraceCap) {
                const uint32_t last = (type == J_REDUCE || type == J_HIST || type == J_SCATTER) && s_flag ? 0x80u : 0u;
                g_qtrace[slot][0] = (unsigned long long)(type | last | (blockIdx.x << 8)) | ((unsigned long long)t_index << 32);
                g_qtrace[slot][1] = t_claim;
                g_qtrace[slot][2] = t_got;
                g_qtrace[slot][3] = wall_clock64();
            }
        }
#endif
    }
}

// The queue's pieces (<= kSegCap pairs each, cut from partitioned hot tiles), sorted after the queue
// has drained, at segment_sort_kernel's occupancy instead of one queue worker per CU: 7888 pieces of
// a one-tile view took the queue ~250 us as SMALL jobs.  With no hot tile the list is empty and
// every workgroup reads one counter and exits.
constexpr int kPieceBlocks = 256 * HIDEGS_PIECE_WAVES;  // one workgroup per resident slot
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(HIDEGS_PIECE_WAVES))) void piece_sort_kernel(
    uint64_t* __restrict__ keys, uint32_t* __restrict__ vals, const uint64_t* __restrict__ alt_k,
    const uint32_t* __restrict__ alt_v, const BigQueue q, uint32_t* async_err)
{
    __shared__ __attribute__((aligned(16))) SegLds lds;
    __shared__ uint32_t s_and[kWavesPerBlock], s_or[kWavesPerBlock], s_max[kWavesPerBlock];
    // the queue has drained (stream order): its error word is final.  A set word is ORed into the
    // stream's mapped host word (vector load and store at system scope), which an entry-point call on
    // this stream takes as HIDEGS_E_ASYNC.  Not an atomic OR (system-scope atomics on host memory are
    // not relied on): earlier sorts on the stream have finished, so only the host's take can fall
    // between the load and the store, and then those bits are reported twice -- never lost.
    if (async_err && blockIdx.x == 0 && threadIdx.x == 0) {
        const uint32_t err = q_peek(&q.ctl[kCtlStride * Q_ERROR]);
        if (err) {
            const uint32_t old = __hip_atomic_load(async_err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(async_err, old | err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
    const uint32_t np = min(q.ctl[kCtlStride * Q_NPIECE], q.piece_cap);
    for (uint32_t p = blockIdx.x; p < np; p += gridDim.x) {
        const uint2 e = q.piece[p];
        const uint32_t m = e.y & 0x7fffffffu;
        if (e.y >> 31)
            sort_segment<false>(alt_k, alt_v, keys, vals, e.x, m, lds, s_and, s_or, s_max);
        else
            sort_segment<true>(keys, vals, nullptr, nullptr, e.x, m, lds, s_and, s_or, s_max);
        __syncthreads();  // the LDS is reused by the next piece
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
// zero (or NULL): the partition queue, reset for the segment_sort_kernel that follows -- its
// Q_WORDS counters and its job_cap slots (slot tags read 0 until published).
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
    const int nt = ceil_div(n, kDevScanTile);
    return align_up((size_t)nt * sizeof(uint32_t)) + align_up(sizeof(uint32_t));
}

constexpr int kMaxSegmentBits = 16;        // segmented path: at most 65536 segments
constexpr long long kSegmentedMinN = 65536;  // below this the plain LSD passes are cheaper
constexpr long long kSegmentedMinAvg = 64;   // pairs per segment on average, else the plain passes: one
                                             // workgroup per ~30-pair segment (distCUDA2's 48-bit Morton
                                             // keys of 2M points) costs more than the 4 low-digit passes
#ifndef HIDEGS_TILE_SEG_MIN_AVG
#define HIDEGS_TILE_SEG_MIN_AVG 8  // the same for hidegs_sort_tile_pairs, per tile of the caller's grid: small
                                   // views (config 2, 100k Gaussians) took 6 plain passes, 105-115 us, against
                                   // 68-70 us segmented (64 / 32 / 16 / 8 / 1 A/B in DESIGN.md, "Small views")
#endif
constexpr long long kTileSegmentedMinAvg = HIDEGS_TILE_SEG_MIN_AVG;

// Capacities of the partition queue for n pairs.  Every record holds > kSegCap pairs and the
// records of one level are disjoint: <= n / 2049 per level, 5 levels (4 digits + the copy).  A
// record queues <= 3 jobs per chunk of >= 4096 pairs and <= 2 pieces per kSegRun pairs (a piece lies in
// one kSegRun window or is a digit of its own) -- under n / 39 jobs in all, so job_cap (n / 24,
// zeroed every call: n / 1.5 bytes) cannot overflow.  The pool (pool_rows(chunks) x 256 u32 per record)
// is sized for a few hot tiles' worth; a record that finds it (or the record table) full is sorted
// by one workgroup instead (a GLOBAL job) -- slower, same result.
BigQueue queue_caps(long long n)
{
    BigQueue q{};
    q.rec_cap = (uint32_t)(5 * (n / (kSegCap + 1)) + 8);
#ifdef HIDEGS_JOB_CAP  // tests only: a tiny job capacity forces the overflow path (tests/test_binning_gpu.py)
    q.job_cap = (uint32_t)HIDEGS_JOB_CAP;
#else
    q.job_cap = (uint32_t)(n / 24 + 1024);
#endif
    q.pool_cap = (uint32_t)(n / 2 + 16 * kRadix);
#ifdef HIDEGS_PIECE_CAP  // tests only: a tiny piece list sends the pieces beyond it to SMALL jobs
    q.piece_cap = (uint32_t)HIDEGS_PIECE_CAP;
#else
    q.piece_cap = (uint32_t)(n / 512 + 1024);  // <= 2 pieces per kSegRun pairs; beyond: SMALL jobs
#endif
    return q;
}

template <typename K>
size_t sort_scratch(long long n)
{
    const int nt = ceil_div(n, kTile);
    size_t b = align_up((size_t)n * sizeof(K)) + align_up((size_t)n * sizeof(uint32_t)) +
               align_up((size_t)kRadix * nt * sizeof(uint32_t)) + 2 * align_up(kRadix * sizeof(uint32_t));
    if (sizeof(K) == 8) {  // segmented path: the segment ranges and the partition queue
        const BigQueue q = queue_caps(n);
        b += align_up(sizeof(uint32_t) * (((size_t)1 << kMaxSegmentBits) + 1)) + align_up(kRadix * sizeof(uint32_t)) +
             align_up(Q_WORDS * sizeof(uint32_t)) +
             align_up((size_t)q.rec_cap * sizeof(BigSeg)) + align_up((size_t)q.job_cap * sizeof(uint4)) +
             align_up((size_t)q.pool_cap * sizeof(uint32_t)) + align_up((size_t)q.piece_cap * sizeof(uint2));
    }
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
    uint32_t* totals_pass[2] = {c.take<uint32_t>(kRadix), c.take<uint32_t>(kRadix)};  // alternate passes

    // (tile | depth)-shaped sort: LSD over the segment bits only, then per-segment LDS sorts
    // average pairs per segment: per tile of the caller's grid with ranges_out, else per segment-bit value
    const bool avg_ok = ranges_out ? n >= kTileSegmentedMinAvg * (long long)num_tiles
                                   : n >= (kSegmentedMinAvg << (end_bit - 32));
    const bool segmented = sizeof(K) == 8 && begin_bit == 0 && end_bit > 32 && end_bit - 32 <= kMaxSegmentBits &&
                           n >= kSegmentedMinN && avg_ok;
    const int lo_bit = segmented ? 32 : begin_bit;
    const int lsd_passes = segmented ? (end_bit - 32 + kRadixBits - 1) / kRadixBits : passes;

    // segmented path: the segment ranges (the caller's tile ranges with ranges_out: tile ids
    // < num_tiles <= 2^(end_bit-32) leave no bits above end_bit, so segment == tile) and the
    // hot-tile queue (its job slots are cleared by the last histogram pass)
    int nseg = 0;
    uint32_t* seg_starts = nullptr;
    uint32_t* low_base = nullptr;
    BigQueue q{};
    if (segmented) {
        nseg = ranges_out ? num_tiles : 1 << (end_bit - 32);
        seg_starts = c.take<uint32_t>(((size_t)1 << kMaxSegmentBits) + 1);
        low_base = c.take<uint32_t>(kRadix);
        q = queue_caps(n);
        q.ctl = c.take<uint32_t>(Q_WORDS);  // the counters and the job slots are contiguous (1 KB + ...):
        q.job = c.take<uint4>(q.job_cap);   // the last histogram pass clears them as one range
        q.rec = c.take<BigSeg>(q.rec_cap);
        q.pool = c.take<uint32_t>(q.pool_cap);
        q.alt_k = reinterpret_cast<uint64_t*>(alt_k);
        q.alt_v = alt_v;
        q.piece = c.take<uint2>(q.piece_cap);
    }

    const K* src_k = keys_in;
    const uint32_t* src_v = vals_in;
    // balanced digit widths (13 tile bits: 7 + 6, not 8 + 5): fewer buckets per pass mean
    // longer runs per bucket in each tile's scatter, i.e. fuller write lines
    const int span = end_bit - lo_bit;
    int shift = lo_bit;
    int pass_bits[2] = {0, 0};
    for (int p = 0; p < lsd_passes; p++) {
        const int bits = (span * (p + 1)) / lsd_passes - (span * p) / lsd_passes;
        const uint32_t mask = (1u << bits) - 1u;
        const bool to_out = ((lsd_passes - 1 - p) % 2) == 0;
        K* dk = to_out ? keys_out : alt_k;
        uint32_t* dv = to_out ? vals_out : alt_v;
        uint32_t* totals = totals_pass[p & 1];
        const bool last = p == lsd_passes - 1;
        uint4* zero_jobs = segmented && last ? reinterpret_cast<uint4*>(q.ctl) : nullptr;
        static_assert(Q_WORDS * sizeof(uint32_t) % kAlign == 0, "ctl and job slots contiguous");
        HIDEGS_LAUNCH((sizeof(K) == 8 ? "radix_hist_u64" : "radix_hist_u32"), radix_hist_kernel<K>, dim3(nt),
                      dim3(kBlock), 0, stream, src_k, n, shift, mask, nt, counts, zero_jobs,
                      zero_jobs ? q.job_cap + Q_WORDS / 4 : 0u);
        // digits above `mask` never occur: their (stale) totals only follow the used digits in the
        // scatter's exclusive scan, and their counts are never read
        const bool low = segmented && last && lsd_passes == 2;  // the previous pass's digit bases, for the starts
        HIDEGS_LAUNCH("radix_digit_scan", radix_digit_scan_kernel, dim3(mask + 1), dim3(kBlock), 0, stream, counts,
                      nt, totals, low ? totals_pass[0] : nullptr, low ? 1 << pass_bits[0] : 0, low_base);
        if (p < 2) pass_bits[p] = bits;
        // narrow digits (and, for the starts, a narrower previous pass: the passes are balanced, so
        // pass_bits[0] <= bits) take the smaller-LDS instance
        const bool narrow = HIDEGS_SCATTER_NARROW && (int)mask < kNarrowRadix && n <= kNarrowMaxN;
        if (segmented && last) {  // also the segments' first positions (no pass over the sorted keys)
            const int b0 = lsd_passes == 2 ? pass_bits[0] : 0;
            if (narrow && (1 << b0) <= kNarrowRadix)
                HIDEGS_LAUNCH("radix_scatter_u64", (radix_scatter_kernel<K, true, kNarrowRadix>), dim3(nt), dim3(kSBlock),
                              0, stream, src_k, src_v, dk, dv, n, shift, mask, nt, counts, totals, low_base, b0, seg_starts);
            else
                HIDEGS_LAUNCH("radix_scatter_u64", (radix_scatter_kernel<K, true>), dim3(nt), dim3(kSBlock), 0, stream,
                              src_k, src_v, dk, dv, n, shift, mask, nt, counts, totals, low_base, b0, seg_starts);
        } else if (narrow) {
            HIDEGS_LAUNCH((sizeof(K) == 8 ? "radix_scatter_u64" : "radix_scatter_u32"),
                          (radix_scatter_kernel<K, false, kNarrowRadix>), dim3(nt), dim3(kSBlock), 0, stream, src_k, src_v,
                          dk, dv, n, shift, mask, nt, counts, totals, nullptr, 0, nullptr);
        } else {
            HIDEGS_LAUNCH((sizeof(K) == 8 ? "radix_scatter_u64" : "radix_scatter_u32"), (radix_scatter_kernel<K, false>),
                          dim3(nt), dim3(kSBlock), 0, stream, src_k, src_v, dk, dv, n, shift, mask, nt, counts, totals,
                          nullptr, 0, nullptr);
        }
        src_k = dk;
        src_v = dv;
        shift += bits;
    }
    if (segmented) {
        uint64_t* ko = reinterpret_cast<uint64_t*>(keys_out);
        HIDEGS_LAUNCH("segment_sort", segment_sort_kernel, dim3(nseg + kScouts), dim3(kBlock), 0, stream, ko,
                      vals_out, seg_starts, ranges_out, nseg, q);
        HIDEGS_LAUNCH("big_segments", big_segment_kernel, dim3(kQueueBlocks), dim3(kBlock), 0, stream, ko, vals_out,
                      reinterpret_cast<uint64_t*>(alt_k), alt_v, q);
        // debug mode checks this call's queue itself (below); otherwise the last kernel hands a queue
        // error to the mapped host word, which fails the next entry-point call
        const bool debug = debug_enabled();
        uint32_t* async_err = debug ? nullptr : async_error_slot(stream);
        static_assert(kDeferPieces, "piece_sort_kernel is the sort's last kernel: it reports the queue's error");
        HIDEGS_LAUNCH("piece_sort", piece_sort_kernel, dim3(kPieceBlocks), dim3(kBlock), 0, stream, ko, vals_out,
                      reinterpret_cast<const uint64_t*>(alt_k), alt_v, q, async_err);
        if (debug) {  // debug mode: this call's own queue error word (in its scratch), after the grid has drained
            if (int rc = check_launch(what, stream, 1)) return rc;
            uint32_t err = 0;
            if (hipMemcpyAsync(&err, q.ctl + kCtlStride * Q_ERROR, sizeof(err), hipMemcpyDeviceToHost, stream) !=
                    hipSuccess ||
                hipStreamSynchronize(stream) != hipSuccess)
                return fail(HIDEGS_E_HIP, std::string(what) + ": queue error readback failed");
            if (err)
                return fail(HIDEGS_E_HIP, std::string(what) + ": hot-tile partition queue error " + std::to_string(err) +
                                              ((err & 1u) ? " (job slots exhausted)" : "") +
                                              ((err & 4u) ? " (a worker gave up waiting)" : "") +
                                              ": the output is not sorted");
        }
    } else if (ranges_out) {
        if (int rc = check_launch(what, stream, 0)) return rc;
        return identify_tile_ranges(reinterpret_cast<const uint64_t*>(keys_out), n,
                                    reinterpret_cast<uint32_t*>(ranges_out), num_tiles, stream);
    }
    return check_launch(what, stream, 0);
}

}  // namespace

// Reads (clear: exchanges with 0) the sticky word in one device-side atomic, so an error raised
// between a read and a separate clear cannot be lost.
__device__ uint32_t g_queue_error_read;
__global__ void queue_error_take_kernel(int clear)
{
    g_queue_error_read = clear ? __hip_atomic_exchange(&g_queue_error, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                               : __hip_atomic_load(&g_queue_error, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

int queue_error(hipStream_t stream, int clear, uint32_t* flags)
{
    // one reader at a time: g_queue_error_read is a single word per device
    static std::mutex m;
    std::lock_guard<std::mutex> lock(m);
    uint32_t v = 0;
    hipLaunchKernelGGL(queue_error_take_kernel, dim3(1), dim3(1), 0, stream, clear);
    if (hipGetLastError() != hipSuccess ||
        hipMemcpyFromSymbolAsync(&v, HIP_SYMBOL(g_queue_error_read), sizeof(v), 0, hipMemcpyDeviceToHost, stream) !=
            hipSuccess ||
        hipStreamSynchronize(stream) != hipSuccess)
        return fail(HIDEGS_E_HIP, "queue_error: readback failed");
    // the asynchronous copy of the same failures on this stream: reported here and taken with the clear
    if (clear) v |= take_async_bits(stream);
    *flags = v;
    return 0;
}

int inclusive_scan_u32(void* scratch, size_t scratch_bytes, const uint32_t* in, uint32_t* out, long long n,
                       hipStream_t stream)
{
    if (n < 0) return fail(HIDEGS_E_ARG, "inclusive_scan_u32: negative size");
    if (n == 0) return 0;
    if (!in || !out) return fail(HIDEGS_E_ARG, "inclusive_scan_u32: NULL pointer");
    if (!scratch || scratch_bytes < scan_scratch(n)) return fail(HIDEGS_E_ARG, "inclusive_scan_u32: scratch too small");
    const int nt = ceil_div(n, kDevScanTile);
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
    if (int rc = hidegs::take_async_error("hidegs_inclusive_scan_u32", hidegs::as_stream(stream))) return rc;
    return hidegs::inclusive_scan_u32(scratch, scratch_bytes, in, out, n, hidegs::as_stream(stream));
}

size_t hidegs_sort_pairs_u64_scratch_bytes(long long n) { return n > 0 ? hidegs::sort_u64_scratch(n) : 0; }
int hidegs_sort_pairs_u64(void* scratch, size_t scratch_bytes, const uint64_t* keys_in, uint64_t* keys_out,
                          const uint32_t* vals_in, uint32_t* vals_out, long long n, int begin_bit, int end_bit,
                          void* stream)
{
    if (int rc = hidegs::take_async_error("hidegs_sort_pairs_u64", hidegs::as_stream(stream))) return rc;
    return hidegs::sort_pairs_u64(scratch, scratch_bytes, keys_in, keys_out, vals_in, vals_out, n, begin_bit, end_bit,
                                  hidegs::as_stream(stream));
}

size_t hidegs_sort_pairs_u32_scratch_bytes(long long n) { return n > 0 ? hidegs::sort_u32_scratch(n) : 0; }
int hidegs_sort_pairs_u32(void* scratch, size_t scratch_bytes, const uint32_t* keys_in, uint32_t* keys_out,
                          const uint32_t* vals_in, uint32_t* vals_out, long long n, int begin_bit, int end_bit,
                          void* stream)
{
    if (int rc = hidegs::take_async_error("hidegs_sort_pairs_u32", hidegs::as_stream(stream))) return rc;
    return hidegs::sort_pairs_u32(scratch, scratch_bytes, keys_in, keys_out, vals_in, vals_out, n, begin_bit, end_bit,
                                  hidegs::as_stream(stream));
}

int hidegs_sort_tile_pairs(void* scratch, size_t scratch_bytes, const uint64_t* keys_in, uint64_t* keys_out,
                           const uint32_t* vals_in, uint32_t* vals_out, long long n, int num_tiles, uint32_t* ranges,
                           void* stream)
{
    if (int rc = hidegs::take_async_error("hidegs_sort_tile_pairs", hidegs::as_stream(stream))) return rc;
    return hidegs::sort_tile_pairs(scratch, scratch_bytes, keys_in, keys_out, vals_in, vals_out, n, num_tiles, ranges,
                                   hidegs::as_stream(stream));
}

int hidegs_identify_tile_ranges(const uint64_t* sorted_keys, long long n, uint32_t* ranges, int num_tiles,
                                void* stream)
{
    if (int rc = hidegs::take_async_error("hidegs_identify_tile_ranges", hidegs::as_stream(stream))) return rc;
    return hidegs::identify_tile_ranges(sorted_keys, n, ranges, num_tiles, hidegs::as_stream(stream));
}

int hidegs_queue_error(void* stream, int clear, uint32_t* flags)
{
    if (!flags) return hidegs::fail(HIDEGS_E_ARG, "hidegs_queue_error: NULL flags");
    return hidegs::queue_error(hidegs::as_stream(stream), clear, flags);
}

uint32_t hidegs_higher_msb(uint32_t n)
{
    // Number of bits needed to hold n, at least 1 -- the value getHigherMsb's
    // binary search (rasterizer_impl.cu:35-50) returns for every u32 input.
    uint32_t bits = 32u - (uint32_t)__builtin_clz(n | 1u);
    return bits;
}

#ifdef HIDEGS_QUEUE_TRACE
// experiments only: copy out (and reset) the partition queue's job trace; returns the job count
int hidegs_debug_wide_trace(unsigned long long* host, int max_jobs)
{
    unsigned int n = 0;
    if (hipDeviceSynchronize() != hipSuccess || hipMemcpyFromSymbol(&n, HIP_SYMBOL(hidegs::g_wtrace_n), sizeof(n)) != hipSuccess)
        return -1;
    const int m = (int)(n < (unsigned)max_jobs ? n : (unsigned)max_jobs);
    if (m > 0 && hipMemcpyFromSymbol(host, HIP_SYMBOL(hidegs::g_wtrace), (size_t)m * 9 * sizeof(unsigned long long)) != hipSuccess)
        return -1;
    n = 0;
    if (hipMemcpyToSymbol(HIP_SYMBOL(hidegs::g_wtrace_n), &n, sizeof(n)) != hipSuccess) return -1;
    return m;
}

int hidegs_debug_queue_trace(unsigned long long* host, int max_jobs)
{
    unsigned int n = 0;
    if (hipDeviceSynchronize() != hipSuccess || hipMemcpyFromSymbol(&n, HIP_SYMBOL(hidegs::g_qtrace_n), sizeof(n)) != hipSuccess)
        return -1;
    const int m = (int)(n < (unsigned)max_jobs ? n : (unsigned)max_jobs);
    if (m > 0 && hipMemcpyFromSymbol(host, HIP_SYMBOL(hidegs::g_qtrace), (size_t)m * 4 * sizeof(unsigned long long)) != hipSuccess)
        return -1;
    n = 0;
    if (hipMemcpyToSymbol(HIP_SYMBOL(hidegs::g_qtrace_n), &n, sizeof(n)) != hipSuccess) return -1;
    return m;
}
#endif
}  // extern "C"
