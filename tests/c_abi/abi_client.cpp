// abi_client.cpp -- a C++ caller of include/hidegs.h with no Python and no torch: what the reference's own
// C++ glue (HR/rasterize_points.cu, SK/spatial.cu) would do over this ABI.  Test infrastructure: built by
// hidegs_amd/build.py, run on the MI355X by tests/test_c_abi_gpu.py.
//
//   1. the binning sequence of Rasterizer::forward (rasterizer_impl.cu:321-371) on a Gaussian-major pair
//      list: hidegs_inclusive_scan_u32 of tiles_touched, then hidegs_sort_tile_pairs -- checked against
//      std::stable_sort of the same pairs and the tile ranges derived from it (bit for bit);
//   2. distCUDA2 (SK/spatial.cu:15-25) through hidegs_dist_cuda2 with a resize-functional style allocation
//      callback -- checked bit for bit against a brute force of its definition;
//   3. the error channel: a bad argument returns HIDEGS_E_ARG with a message.
// Prints ABI_CLIENT_OK and returns 0 when every check holds.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

#include "../../include/hidegs.h"

#define CHECK_HIP(x)                                                                   \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            std::fprintf(stderr, "%s:%d: %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            return 2;                                                                  \
        }                                                                              \
    } while (0)
#define CHECK(c, ...)                          \
    do {                                               \
        if (!(c)) {                                    \
            std::fprintf(stderr, "FAILED: " __VA_ARGS__); \
            std::fprintf(stderr, "\n");                \
            return 1;                                  \
        }                                              \
    } while (0)

namespace {

// growable device scratch: the C form of the reference's resizeFunctional (rasterize_points.cu:27-33)
struct DeviceBuffer {
    void* ptr = nullptr;
    size_t size = 0;
};
char* grow(void* user, size_t nbytes)
{
    auto* b = static_cast<DeviceBuffer*>(user);
    if (nbytes > b->size) {
        if (b->ptr) (void)hipFree(b->ptr);
        b->ptr = nullptr;
        b->size = 0;
        if (hipMalloc(&b->ptr, nbytes) != hipSuccess) return nullptr;
        b->size = nbytes;
    }
    return static_cast<char*>(b->ptr);
}

float sqdist(const float* q, const float* c)
{
    const float dx = c[0] - q[0], dy = c[1] - q[1], dz = c[2] - q[2];
    return std::fma(dz, dz, std::fma(dx, dx, dy * dy));
}

int binning(hipStream_t stream)
{
    // 20,000 Gaussians on a 1080p tile grid (120 x 68 tiles), each touching a w x h rect, emitted
    // Gaussian-major with value = Gaussian index (duplicateWithKeys, rasterizer_impl.cu:89-113)
    const int gx = 120, gy = 68, T = gx * gy, G = 20000;
    std::mt19937 rng(7);
    std::uniform_int_distribution<int> wh(1, 4), px(0, gx - 1), py(0, gy - 1);
    std::uniform_real_distribution<float> z(2.0f, 20.0f);
    std::vector<uint32_t> touched(G);
    std::vector<uint64_t> keys;
    std::vector<uint32_t> vals;
    for (int g = 0; g < G; g++) {
        const int x0 = px(rng), y0 = py(rng), w = wh(rng), h = wh(rng);
        float depth = z(rng);
        if (g % 7 == 0) depth = 5.0f;  // repeated depths: the order of equal keys shows
        uint32_t bits;
        std::memcpy(&bits, &depth, 4);
        uint32_t n = 0;
        for (int y = y0; y < std::min(gy, y0 + h); y++)
            for (int x = x0; x < std::min(gx, x0 + w); x++, n++) {
                keys.push_back(((uint64_t)(y * gx + x) << 32) | bits);
                vals.push_back((uint32_t)g);
            }
        touched[g] = n;
    }
    const long long K = (long long)keys.size();

    uint32_t *d_touched, *d_offsets, *d_vin, *d_vout, *d_ranges;
    uint64_t *d_kin, *d_kout;
    CHECK_HIP(hipMalloc(&d_touched, G * 4));
    CHECK_HIP(hipMalloc(&d_offsets, G * 4));
    CHECK_HIP(hipMalloc(&d_kin, K * 8));
    CHECK_HIP(hipMalloc(&d_kout, K * 8));
    CHECK_HIP(hipMalloc(&d_vin, K * 4));
    CHECK_HIP(hipMalloc(&d_vout, K * 4));
    CHECK_HIP(hipMalloc(&d_ranges, (size_t)T * 8));
    CHECK_HIP(hipMemcpy(d_touched, touched.data(), G * 4, hipMemcpyHostToDevice));
    CHECK_HIP(hipMemcpy(d_kin, keys.data(), K * 8, hipMemcpyHostToDevice));
    CHECK_HIP(hipMemcpy(d_vin, vals.data(), K * 4, hipMemcpyHostToDevice));

    DeviceBuffer scan_tmp, sort_tmp;
    char* st = grow(&scan_tmp, hidegs_scan_scratch_bytes(G));
    CHECK(st, "scan scratch");
    int rc = hidegs_inclusive_scan_u32(st, scan_tmp.size, d_touched, d_offsets, G, stream);
    CHECK(rc == 0, "hidegs_inclusive_scan_u32: %s", hidegs_last_error());
    char* so = grow(&sort_tmp, hidegs_sort_pairs_u64_scratch_bytes(K));
    CHECK(so, "sort scratch");
    rc = hidegs_sort_tile_pairs(so, sort_tmp.size, d_kin, d_kout, d_vin, d_vout, K, T, d_ranges, stream);
    CHECK(rc == 0, "hidegs_sort_tile_pairs: %s", hidegs_last_error());
    CHECK_HIP(hipStreamSynchronize(stream));
    uint32_t qerr = 0;
    CHECK(hidegs_queue_error(stream, 1, &qerr) == 0 && qerr == 0, "partition queue error %u", qerr);

    std::vector<uint32_t> offsets(G), got_v(K), got_r(2 * (size_t)T);
    std::vector<uint64_t> got_k(K);
    CHECK_HIP(hipMemcpy(offsets.data(), d_offsets, G * 4, hipMemcpyDeviceToHost));
    CHECK_HIP(hipMemcpy(got_k.data(), d_kout, K * 8, hipMemcpyDeviceToHost));
    CHECK_HIP(hipMemcpy(got_v.data(), d_vout, K * 4, hipMemcpyDeviceToHost));
    CHECK_HIP(hipMemcpy(got_r.data(), d_ranges, (size_t)T * 8, hipMemcpyDeviceToHost));

    uint32_t run = 0;
    for (int g = 0; g < G; g++) {
        run += touched[g];
        CHECK(offsets[g] == run, "scan at %d", g);
    }
    // the reference's order: stable by the key bits [0, 32 + getHigherMsb(T))
    const int end = 32 + (int)hidegs_higher_msb((uint32_t)T);
    const uint64_t mask = end >= 64 ? ~0ull : ((1ull << end) - 1ull);
    std::vector<uint32_t> perm(K);
    for (long long i = 0; i < K; i++) perm[i] = (uint32_t)i;
    std::stable_sort(perm.begin(), perm.end(), [&](uint32_t a, uint32_t b) { return (keys[a] & mask) < (keys[b] & mask); });
    std::vector<uint32_t> exp_r(2 * (size_t)T, 0u);
    for (long long i = 0; i < K; i++) {
        CHECK(got_k[i] == keys[perm[i]] && got_v[i] == vals[perm[i]], "sorted pair %lld", i);
        const uint32_t t = (uint32_t)(keys[perm[i]] >> 32);
        if (i == 0 || (uint32_t)(keys[perm[i - 1]] >> 32) != t) exp_r[2 * t] = (uint32_t)i;
        exp_r[2 * t + 1] = (uint32_t)(i + 1);
    }
    for (int t = 0; t < T; t++)
        CHECK(got_r[2 * t] == exp_r[2 * t] && got_r[2 * t + 1] == exp_r[2 * t + 1], "range of tile %d", t);
    std::printf("binning: %lld pairs of %d Gaussians over %d tiles: scan, sort and ranges bit-identical\n", K, G, T);

    (void)hipFree(scan_tmp.ptr);
    (void)hipFree(sort_tmp.ptr);
    for (void* p : {(void*)d_touched, (void*)d_offsets, (void*)d_kin, (void*)d_kout, (void*)d_vin, (void*)d_vout,
                    (void*)d_ranges})
        (void)hipFree(p);
    return 0;
}

int knn(hipStream_t stream)
{
    const int P = 3000;
    std::mt19937 rng(11);
    std::normal_distribution<float> nd(0.0f, 1.0f);
    std::vector<float> pts(3 * (size_t)P);
    for (auto& v : pts) v = nd(rng);
    for (int i = 0; i < 30; i++)  // duplicates: distance 0 to another index
        std::memcpy(&pts[3 * (size_t)(P - 1 - i)], &pts[3 * (size_t)i], 12);
    float *d_pts, *d_out;
    CHECK_HIP(hipMalloc(&d_pts, pts.size() * 4));
    CHECK_HIP(hipMalloc(&d_out, (size_t)P * 4));
    CHECK_HIP(hipMemcpy(d_pts, pts.data(), pts.size() * 4, hipMemcpyHostToDevice));
    DeviceBuffer scratch;
    int rc = hidegs_dist_cuda2(grow, &scratch, P, d_pts, d_out, stream);
    CHECK(rc == 0, "hidegs_dist_cuda2: %s", hidegs_last_error());
    CHECK(scratch.size == hidegs_knn_scratch_bytes(P), "scratch request %zu", scratch.size);
    std::vector<float> got(P);
    CHECK_HIP(hipMemcpyAsync(got.data(), d_out, (size_t)P * 4, hipMemcpyDeviceToHost, stream));
    CHECK_HIP(hipStreamSynchronize(stream));
    for (int i = 0; i < P; i++) {
        float best[3] = {FLT_MAX, FLT_MAX, FLT_MAX};
        for (int j = 0; j < P; j++) {
            if (j == i) continue;
            float d = sqdist(&pts[3 * (size_t)i], &pts[3 * (size_t)j]);
            for (int k = 0; k < 3; k++)
                if (best[k] > d) std::swap(best[k], d);
        }
        const float exp = ((best[0] + best[1]) + best[2]) / 3.0f;
        CHECK(std::memcmp(&exp, &got[i], 4) == 0, "distCUDA2 point %d: %.9g vs %.9g", i, got[i], exp);
    }
    std::printf("distCUDA2: %d points bit-identical to the brute force of its definition\n", P);
    (void)hipFree(scratch.ptr);
    (void)hipFree(d_pts);
    (void)hipFree(d_out);
    return 0;
}

}  // namespace

int main()
{
    hipStream_t stream;
    CHECK_HIP(hipStreamCreate(&stream));
    if (int rc = binning(stream)) return rc;
    if (int rc = knn(stream)) return rc;
    // the error channel: a bad bit range, reported without touching the device
    const int rc = hidegs_sort_pairs_u64(nullptr, 0, nullptr, nullptr, nullptr, nullptr, 10, 0, 65, stream);
    CHECK(rc == HIDEGS_E_ARG && std::strlen(hidegs_last_error()) > 0, "error channel");
    std::printf("error channel: HIDEGS_E_ARG with \"%s\"\n", hidegs_last_error());
    CHECK_HIP(hipStreamDestroy(stream));
    std::printf("ABI_CLIENT_OK\n");
    return 0;
}
