// wire.hip -- the local steps of the view-DP exchange around its collectives (SURVEY §8(e) E2;
// hidegs_amd/view_dp.py): the visibility masks' bit packing and union / view count, and the bf16
// wire format ("optionally bf16 transport, behind a parity flag": transport="bf16").
//
// One bucket of fp32 gradients travels as bf16: packed (round to nearest even), split into one
// chunk per rank and handed to its owner by an all-to-all, summed there in fp32 in rank order and
// rounded once more, then all-gathered and widened back to fp32 in place.  The three local steps
// are one HBM pass each here (6, 2w + 2 and 6 bytes per element) instead of the chain of torch
// conversions, fills and adds they were (measured: a one-rank forced exchange of 472 MB of
// gradients, 1.40 ms).  Their results are the torch definitions bit for bit:
//   pack     x.to(torch.bfloat16), zero padding      c10's round_to_nearest_even: NaN -> 0x7FC0,
//                                                    else (u + 0x7FFF + ((u >> 16) & 1)) >> 16
//   sum      acc = parts[0].float(); acc += parts[r].float() for r = 1 .. w-1; acc.to(bfloat16)
//   unpack   x.float()                               exact (the bf16 bits are the high half)
#include <stdint.h>

#include <string>

#include "common.h"

namespace hidegs {
namespace {

constexpr int kBlock = 256;
constexpr int kVec = 8;  // elements per thread per step: 32 B of fp32 in, 16 B of bf16 out

__device__ __forceinline__ uint16_t bf16_rne(float x)
{
    const uint32_t u = __float_as_uint(x);
    if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)0x7FC0;  // NaN
    return (uint16_t)((u + 0x7FFFu + ((u >> 16) & 1u)) >> 16);
}

__device__ __forceinline__ float bf16_float(uint16_t h) { return __uint_as_float((uint32_t)h << 16); }

typedef float f4 __attribute__((ext_vector_type(4)));

// dst[i] = bf16(src[i]) for i < n, 0 for n <= i < n_pad.
__global__ __launch_bounds__(kBlock) void bf16_pack_kernel(const float* __restrict__ src, uint16_t* __restrict__ dst,
                                                           long long n, long long n_pad, int vec)
{
    const long long i0 = ((long long)blockIdx.x * kBlock + threadIdx.x) * kVec;
    if (i0 >= n_pad) return;
    if (vec && i0 + kVec <= n) {
        const f4 a = *reinterpret_cast<const f4*>(src + i0);
        const f4 b = *reinterpret_cast<const f4*>(src + i0 + 4);
        uint4 o;
        o.x = (uint32_t)bf16_rne(a[0]) | ((uint32_t)bf16_rne(a[1]) << 16);
        o.y = (uint32_t)bf16_rne(a[2]) | ((uint32_t)bf16_rne(a[3]) << 16);
        o.z = (uint32_t)bf16_rne(b[0]) | ((uint32_t)bf16_rne(b[1]) << 16);
        o.w = (uint32_t)bf16_rne(b[2]) | ((uint32_t)bf16_rne(b[3]) << 16);
        *reinterpret_cast<uint4*>(dst + i0) = o;
        return;
    }
    for (int j = 0; j < kVec; j++) {
        const long long i = i0 + j;
        if (i < n_pad) dst[i] = i < n ? bf16_rne(src[i]) : (uint16_t)0;
    }
}

// out[j] = bf16(((float)parts[0][j] + (float)parts[1][j]) + ...), the w rows of `chunk` elements in rank order.
__global__ __launch_bounds__(kBlock) void bf16_sum_ranks_kernel(const uint16_t* __restrict__ parts, int w,
                                                                long long chunk, uint16_t* __restrict__ out, int vec)
{
    const long long j0 = ((long long)blockIdx.x * kBlock + threadIdx.x) * kVec;
    if (j0 >= chunk) return;
    if (vec && j0 + kVec <= chunk) {
        float acc[kVec];
        uint4 h = *reinterpret_cast<const uint4*>(parts + j0);
        const uint32_t* hw = reinterpret_cast<const uint32_t*>(&h);
#pragma unroll
        for (int e = 0; e < kVec; e++) acc[e] = bf16_float((uint16_t)(hw[e / 2] >> (16 * (e & 1))));
        for (int r = 1; r < w; r++) {
            h = *reinterpret_cast<const uint4*>(parts + (long long)r * chunk + j0);
#pragma unroll
            for (int e = 0; e < kVec; e++) acc[e] += bf16_float((uint16_t)(hw[e / 2] >> (16 * (e & 1))));
        }
        uint4 o;
        uint32_t* ow = reinterpret_cast<uint32_t*>(&o);
#pragma unroll
        for (int e = 0; e < kVec / 2; e++)
            ow[e] = (uint32_t)bf16_rne(acc[2 * e]) | ((uint32_t)bf16_rne(acc[2 * e + 1]) << 16);
        *reinterpret_cast<uint4*>(out + j0) = o;
        return;
    }
    for (int e = 0; e < kVec; e++) {
        const long long j = j0 + e;
        if (j >= chunk) break;
        float acc = bf16_float(parts[j]);
        for (int r = 1; r < w; r++) acc += bf16_float(parts[(long long)r * chunk + j]);
        out[j] = bf16_rne(acc);
    }
}

// dst[i] = float(src[i]) for i < n.
__global__ __launch_bounds__(kBlock) void bf16_unpack_kernel(const uint16_t* __restrict__ src, float* __restrict__ dst,
                                                             long long n, int vec)
{
    const long long i0 = ((long long)blockIdx.x * kBlock + threadIdx.x) * kVec;
    if (i0 >= n) return;
    if (vec && i0 + kVec <= n) {
        const uint4 h = *reinterpret_cast<const uint4*>(src + i0);
        const f4 a = {__uint_as_float(h.x << 16), __uint_as_float(h.x & 0xffff0000u), __uint_as_float(h.y << 16),
                      __uint_as_float(h.y & 0xffff0000u)};
        const f4 b = {__uint_as_float(h.z << 16), __uint_as_float(h.z & 0xffff0000u), __uint_as_float(h.w << 16),
                      __uint_as_float(h.w & 0xffff0000u)};
        *reinterpret_cast<f4*>(dst + i0) = a;
        *reinterpret_cast<f4*>(dst + i0 + 4) = b;
        return;
    }
    for (int j = 0; j < kVec; j++) {
        const long long i = i0 + j;
        if (i < n) dst[i] = bf16_float(src[i]);
    }
}

// Visibility masks (the exchange's first collective): bits[j] = sum_i (mask[8j + i] != 0) << i.
__global__ __launch_bounds__(kBlock) void mask_pack_kernel(const uint8_t* __restrict__ mask, long long n,
                                                           uint8_t* __restrict__ bits)
{
    const long long j = (long long)blockIdx.x * kBlock + threadIdx.x;
    const long long i0 = 8 * j;
    if (i0 >= n) return;
    uint32_t b = 0;
    for (int i = 0; i < 8; i++)
        if (i0 + i < n && mask[i0 + i]) b |= 1u << i;
    bits[j] = (uint8_t)b;
}

// After the all-gather of `ranks` packed masks (rows of nbytes): every Gaussian's view count over the
// ranks and its union bit -- unpack_mask + sum + compare of the torch definition, in one pass.
__global__ __launch_bounds__(kBlock) void mask_union_count_kernel(const uint8_t* __restrict__ bits, int ranks,
                                                                  long long nbytes, long long n,
                                                                  uint8_t* __restrict__ any, float* __restrict__ count)
{
    const long long i = (long long)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    uint32_t c = 0;
    for (int r = 0; r < ranks; r++) c += (bits[(long long)r * nbytes + (i >> 3)] >> (i & 7)) & 1u;
    any[i] = c != 0;
    count[i] = (float)c;
}

bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

unsigned grid_for(long long n)
{
    return (unsigned)((n + (long long)kBlock * kVec - 1) / ((long long)kBlock * kVec));
}

constexpr long long kMaxWire = (long long)kBlock * kVec * 0x7fffffffLL;

}  // namespace
}  // namespace hidegs

extern "C" int hidegs_bf16_pack(const float* src, uint16_t* dst, long long n, long long n_padded, void* stream)
{
    using namespace hidegs;
    if (int rc = take_async_error("hidegs_bf16_pack", hidegs::as_stream(stream))) return rc;
    if (n < 0 || n_padded < n || n_padded > kMaxWire) return fail(HIDEGS_E_ARG, "bf16_pack: bad sizes");
    if (n_padded == 0) return 0;
    if (!dst || (n > 0 && !src)) return fail(HIDEGS_E_ARG, "bf16_pack: NULL pointer");
    const int vec = aligned16(src) && aligned16(dst);
    HIDEGS_LAUNCH("bf16_pack", bf16_pack_kernel, dim3(grid_for(n_padded)), dim3(kBlock), 0, as_stream(stream), src, dst,
                  n, n_padded, vec);
    return check_launch("bf16_pack", as_stream(stream), 0);
}

extern "C" int hidegs_bf16_sum_ranks(const uint16_t* parts, int world, long long chunk, uint16_t* out, void* stream)
{
    using namespace hidegs;
    if (int rc = take_async_error("hidegs_bf16_sum_ranks", hidegs::as_stream(stream))) return rc;
    if (world < 1 || chunk < 0 || chunk > kMaxWire) return fail(HIDEGS_E_ARG, "bf16_sum_ranks: bad sizes");
    if (chunk == 0) return 0;
    if (!parts || !out) return fail(HIDEGS_E_ARG, "bf16_sum_ranks: NULL pointer");
    // rows of `chunk` elements start 16-byte aligned only if chunk is a multiple of 8
    const int vec = aligned16(parts) && aligned16(out) && (chunk % 8) == 0;
    HIDEGS_LAUNCH("bf16_sum_ranks", bf16_sum_ranks_kernel, dim3(grid_for(chunk)), dim3(kBlock), 0, as_stream(stream),
                  parts, world, chunk, out, vec);
    return check_launch("bf16_sum_ranks", as_stream(stream), 0);
}

extern "C" int hidegs_bf16_unpack(const uint16_t* src, float* dst, long long n, void* stream)
{
    using namespace hidegs;
    if (int rc = take_async_error("hidegs_bf16_unpack", hidegs::as_stream(stream))) return rc;
    if (n < 0 || n > kMaxWire) return fail(HIDEGS_E_ARG, "bf16_unpack: bad size");
    if (n == 0) return 0;
    if (!src || !dst) return fail(HIDEGS_E_ARG, "bf16_unpack: NULL pointer");
    const int vec = aligned16(src) && aligned16(dst);
    HIDEGS_LAUNCH("bf16_unpack", bf16_unpack_kernel, dim3(grid_for(n)), dim3(kBlock), 0, as_stream(stream), src, dst, n,
                  vec);
    return check_launch("bf16_unpack", as_stream(stream), 0);
}

extern "C" int hidegs_mask_pack(const unsigned char* mask, long long n, unsigned char* bits, void* stream)
{
    using namespace hidegs;
    if (int rc = take_async_error("hidegs_mask_pack", hidegs::as_stream(stream))) return rc;
    if (n < 0 || n > (long long)kBlock * 8 * 0x7fffffffLL) return fail(HIDEGS_E_ARG, "mask_pack: bad size");
    if (n == 0) return 0;
    if (!mask || !bits) return fail(HIDEGS_E_ARG, "mask_pack: NULL pointer");
    const long long nb = (n + 7) / 8;
    HIDEGS_LAUNCH("mask_pack", mask_pack_kernel, dim3((unsigned)((nb + kBlock - 1) / kBlock)), dim3(kBlock), 0,
                  as_stream(stream), mask, n, bits);
    return check_launch("mask_pack", as_stream(stream), 0);
}

extern "C" int hidegs_mask_union_count(const unsigned char* bits, int ranks, long long n, unsigned char* any,
                                       float* count, void* stream)
{
    using namespace hidegs;
    if (int rc = take_async_error("hidegs_mask_union_count", hidegs::as_stream(stream))) return rc;
    if (ranks < 1 || n < 0 || n > (long long)kBlock * 0x7fffffffLL) return fail(HIDEGS_E_ARG, "mask_union_count: bad sizes");
    if (n == 0) return 0;
    if (!bits || !any || !count) return fail(HIDEGS_E_ARG, "mask_union_count: NULL pointer");
    HIDEGS_LAUNCH("mask_union_count", mask_union_count_kernel, dim3((unsigned)((n + kBlock - 1) / kBlock)),
                  dim3(kBlock), 0, as_stream(stream), bits, ranks, (n + 7) / 8, n, any, count);
    return check_launch("mask_union_count", as_stream(stream), 0);
}
