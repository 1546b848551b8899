// Streaming-bandwidth probe (measurement tool, not product code): a kernel that reads R and writes
// W float4 streams of n elements, to price the masked Adam's 4-read / 3-write mix against a copy.
#include <hip/hip_runtime.h>

typedef float f4 __attribute__((ext_vector_type(4)));

template <int R, int W>
__global__ __launch_bounds__(256) void mix(const f4* const* in, f4* const* out, long long n4)
{
    for (long long i = (long long)blockIdx.x * 512 + threadIdx.x; i < n4; i += (long long)gridDim.x * 512) {
        f4 a[2];
#pragma unroll
        for (int u = 0; u < 2; u++) {
            a[u] = 0.f;
            if (i + u * 256 < n4)
#pragma unroll
                for (int r = 0; r < R; r++) a[u] += __builtin_nontemporal_load(in[r] + i + u * 256);
        }
#pragma unroll
        for (int u = 0; u < 2; u++)
            if (i + u * 256 < n4)
#pragma unroll
                for (int w = 0; w < W; w++) __builtin_nontemporal_store(a[u] + (float)w, out[w] + i + u * 256);
    }
}

extern "C" int stream_mix(int R, int W, const void* const* in, void* const* out, long long n, int grid, void* stream)
{
    const f4* const* i = reinterpret_cast<const f4* const*>(in);
    f4* const* o = reinterpret_cast<f4* const*>(out);
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const long long n4 = n / 4;
    if (R == 1 && W == 1) hipLaunchKernelGGL((mix<1, 1>), dim3(grid), dim3(256), 0, s, i, o, n4);
    else if (R == 4 && W == 3) hipLaunchKernelGGL((mix<4, 3>), dim3(grid), dim3(256), 0, s, i, o, n4);
    else if (R == 2 && W == 1) hipLaunchKernelGGL((mix<2, 1>), dim3(grid), dim3(256), 0, s, i, o, n4);
    else return -1;
    return hipGetLastError() == hipSuccess ? 0 : -2;
}
