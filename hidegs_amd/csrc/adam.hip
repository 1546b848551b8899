// adam.hip -- fused row-masked Adam step for one parameter tensor.
//
// Replaces the per-parameter loop of the reference optimizer scene/OurAdam.py: the masked path
// _single_tensor_adam (:249-337) gathers grad / exp_avg / exp_avg_sq / param rows with a
// boolean index, runs eight elementwise torch ops on the copies and scatters them back; the
// empty-mask path _single_tensor_adam2 (:340-420) runs the same ops on whole tensors.  Here one
// kernel reads each relevant element's param, grad and both moments once and writes param and
// moments once (28 B/element), and rows outside `relevant` are neither read nor written.
//
// The per-element arithmetic reproduces the rounding of those torch ops as PyTorch's ROCm build
// executes them (probed on MI355X, tools/probe_torch_contraction.py):
//   exp_avg.mul_(b1)                  m = m * b1
//   .add_(grad, alpha=1-b1)           m = fma(1-b1, g, m)          (add with alpha contracts)
//   exp_avg_sq.mul_(b2)               v = v * b2
//   .addcmul_(g, g, value=1-b2)       v = fma(1-b2, g * g, v)        (alpha * (t1 * t2))
//   exp_avg_sq.sqrt()                 s = sqrt(v)                  (correctly rounded)
//   / bias_correction2_sqrt           s = s * (float)(1.0 / bc2)   (division by a CPU scalar is a
//                                                                   multiply by its double reciprocal
//                                                                   rounded to float)
//   .add_(eps)                        d = s + eps
//   param.addcdiv_(m, d, value=-ss)   p = fma(-ss, m / d, p)
//   weight decay (grad.add(param, alpha=wd))  g = fma(wd, p, g)
// Every scalar is the float the reference passes (Python doubles cast once), computed on the
// host as the reference computes them from step_t.item().
#include <math.h>

#include "common.h"

namespace hidegs {
namespace {

constexpr int kBlock = 256;

struct AdamScalars {
    float b1, a1, b2, a2, inv_bc2, eps, neg_step_size, wd;
};

__device__ __forceinline__ void adam_element(float& p, float g, float& m, float& v, const AdamScalars& s)
{
    if (s.wd != 0.f) g = fmaf(s.wd, p, g);
    m = m * s.b1;
    m = fmaf(s.a1, g, m);
    v = v * s.b2;
    v = fmaf(s.a2, g * g, v);
    float d = sqrtf(v);
    d = d * s.inv_bc2;
    d = d + s.eps;
    p = fmaf(s.neg_step_size, m / d, p);
}

// Row index of element e for a row width w (e < 2^52): double estimate, exact after correction.
__device__ __forceinline__ long long row_of(long long e, int w, double inv_w)
{
    long long r = (long long)((double)e * inv_w);
    if (r * w > e) r--;
    if ((r + 1) * w <= e) r++;
    return r;
}

// Each thread owns 4 consecutive elements (one 16-byte vector when the tensors allow it).
__global__ __launch_bounds__(kBlock) void masked_adam_kernel(float* __restrict__ param, const float* __restrict__ grad,
                                                             float* __restrict__ exp_avg,
                                                             float* __restrict__ exp_avg_sq,
                                                             const unsigned char* __restrict__ relevant,
                                                             long long n, int width, double inv_w, AdamScalars s,
                                                             int vec4)
{
    const long long stride = (long long)gridDim.x * kBlock;
    for (long long q = (long long)blockIdx.x * kBlock + threadIdx.x; 4 * q < n; q += stride) {
        const long long e0 = 4 * q;
        bool rel[4];
        bool any = false;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const long long e = e0 + j;
            rel[j] = e < n && (relevant == nullptr || relevant[row_of(e, width, inv_w)] != 0);
            any |= rel[j];
        }
        if (!any) continue;  // rows outside the mask: no traffic
        if (vec4 && e0 + 4 <= n) {
            float4 p = reinterpret_cast<float4*>(param)[q];
            const float4 g = reinterpret_cast<const float4*>(grad)[q];
            float4 m = reinterpret_cast<float4*>(exp_avg)[q];
            float4 v = reinterpret_cast<float4*>(exp_avg_sq)[q];
            float pp[4] = {p.x, p.y, p.z, p.w}, gg[4] = {g.x, g.y, g.z, g.w};
            float mm[4] = {m.x, m.y, m.z, m.w}, vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int j = 0; j < 4; j++)
                if (rel[j]) adam_element(pp[j], gg[j], mm[j], vv[j], s);
            reinterpret_cast<float4*>(param)[q] = make_float4(pp[0], pp[1], pp[2], pp[3]);
            reinterpret_cast<float4*>(exp_avg)[q] = make_float4(mm[0], mm[1], mm[2], mm[3]);
            reinterpret_cast<float4*>(exp_avg_sq)[q] = make_float4(vv[0], vv[1], vv[2], vv[3]);
        } else {
#pragma unroll
            for (int j = 0; j < 4; j++) {
                if (!rel[j]) continue;
                const long long e = e0 + j;
                float p = param[e], m = exp_avg[e], v = exp_avg_sq[e];
                adam_element(p, grad[e], m, v, s);
                param[e] = p;
                exp_avg[e] = m;
                exp_avg_sq[e] = v;
            }
        }
    }
}

}  // namespace

int masked_adam(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, const unsigned char* relevant,
                long long rows, int width, double lr, double beta1, double beta2, double eps, double weight_decay,
                long long step, hipStream_t stream)
{
    if (rows < 0 || width <= 0) return fail(HIDEGS_E_ARG, "masked_adam: bad shape");
    if (step < 1) return fail(HIDEGS_E_ARG, "masked_adam: step counts from 1 (after the increment)");
    const long long n = rows * (long long)width;
    if (n == 0) return 0;
    if (!param || !grad || !exp_avg || !exp_avg_sq) return fail(HIDEGS_E_ARG, "masked_adam: NULL tensor");
    // scalars exactly as the reference forms them (OurAdam.py:305-325), in double, cast once
    const double bias_correction1 = 1.0 - pow(beta1, (double)step);
    const double bias_correction2 = 1.0 - pow(beta2, (double)step);
    const double step_size = lr / bias_correction1;
    const double bc2_sqrt = sqrt(bias_correction2);
    AdamScalars s;
    s.b1 = (float)beta1;
    s.a1 = (float)(1.0 - beta1);
    s.b2 = (float)beta2;
    s.a2 = (float)(1.0 - beta2);
    s.inv_bc2 = (float)(1.0 / bc2_sqrt);  // reciprocal in double, rounded once (torch probe)
    s.eps = (float)eps;
    s.neg_step_size = (float)(-step_size);
    s.wd = (float)weight_decay;
    const bool aligned = ((reinterpret_cast<uintptr_t>(param) | reinterpret_cast<uintptr_t>(grad) |
                           reinterpret_cast<uintptr_t>(exp_avg) | reinterpret_cast<uintptr_t>(exp_avg_sq)) & 15) == 0;
    const long long quads = (n + 3) / 4;
    const long long want = (quads + kBlock - 1) / kBlock;
    const int grid = (int)(want < 8192 ? want : 8192);
    HIDEGS_LAUNCH("masked_adam", masked_adam_kernel, dim3(grid), dim3(kBlock), 0, stream, param, grad, exp_avg,
                  exp_avg_sq, relevant, n, width, 1.0 / (double)width, s, aligned ? 1 : 0);
    return check_launch("masked_adam", stream, 0);
}

}  // namespace hidegs

extern "C" int hidegs_masked_adam(float* param, const float* grad, float* exp_avg, float* exp_avg_sq,
                                  const unsigned char* relevant, long long rows, int width, double lr, double beta1,
                                  double beta2, double eps, double weight_decay, long long step, void* stream)
{
    return hidegs::masked_adam(param, grad, exp_avg, exp_avg_sq, relevant, rows, width, lr, beta1, beta2, eps,
                               weight_decay, step, hidegs::as_stream(stream));
}
