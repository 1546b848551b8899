// adam.hip -- fused row-masked Adam step for a list of parameter tensors.
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

#include <string>

#include "common.h"

namespace hidegs {
namespace {

constexpr int kBlock = 256;
#ifndef HIDEGS_ADAM_QUADS
#define HIDEGS_ADAM_QUADS 2
#endif
constexpr int kQuadsPerThread = HIDEGS_ADAM_QUADS;      // 16-byte vectors per tensor in flight
constexpr int kQuadsPerBlock = kBlock * kQuadsPerThread;  // 2048 elements per workgroup
constexpr int kMaxTensors = 8;                          // tensors per launch

typedef float f4 __attribute__((ext_vector_type(4)));

struct AdamScalars {
    float b1, a1, b2, a2, inv_bc2, eps, neg_step_size, wd;
};

struct AdamTensor {
    float* param;
    const float* grad;
    float* exp_avg;
    float* exp_avg_sq;
    const unsigned char* relevant;
    long long n;       // elements
    int width;         // elements per row
    int vec4;          // all four tensors 16-byte aligned
    double inv_w;
    AdamScalars s;
};

// One launch updates up to kMaxTensors parameters: workgroups [first[t], first[t+1]) own tensor t.
struct AdamBatch {
    int count;
    int first[kMaxTensors + 1];
    AdamTensor t[kMaxTensors];
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

// Which of the 4 elements from e0 lie in relevant rows (bit j = element e0 + j, e0 + j < n).
__device__ __forceinline__ uint32_t relevant_bits(const AdamTensor& T, long long e0)
{
    uint32_t bits = 0;
    if (T.relevant == nullptr) {
#pragma unroll
        for (int j = 0; j < 4; j++) bits |= (e0 + j < T.n ? 1u : 0u) << j;
        return bits;
    }
    long long r = row_of(e0, T.width, T.inv_w);
    long long c = e0 - r * T.width;
    bool rel = T.relevant[r] != 0;
#pragma unroll
    for (int j = 0; j < 4; j++) {
        if (j > 0 && ++c == T.width) {  // next row (width 1..3 can cross several rows in a quad)
            c = 0;
            r++;
            if (e0 + j < T.n) rel = T.relevant[r] != 0;
        }
        bits |= (e0 + j < T.n && rel ? 1u : 0u) << j;
    }
    return bits;
}

__device__ __forceinline__ f4 ld(const float* p, long long q) { return __builtin_nontemporal_load(reinterpret_cast<const f4*>(p) + q); }
__device__ __forceinline__ void st(float* p, long long q, f4 v) { __builtin_nontemporal_store(v, reinterpret_cast<f4*>(p) + q); }

__global__ __launch_bounds__(kBlock) void masked_adam_kernel(const AdamBatch batch)
{
    int ti = 0;
    while (ti + 1 < batch.count && (int)blockIdx.x >= batch.first[ti + 1]) ti++;  // workgroup-uniform
    const AdamTensor& T = batch.t[ti];
    const long long q0 = (long long)(blockIdx.x - batch.first[ti]) * kQuadsPerBlock + threadIdx.x;
    uint32_t bits[kQuadsPerThread];
#pragma unroll
    for (int u = 0; u < kQuadsPerThread; u++) {
        const long long q = q0 + u * kBlock;
        bits[u] = 4 * q < T.n ? relevant_bits(T, 4 * q) : 0u;
    }
    if (T.vec4) {
        f4 p[kQuadsPerThread], g[kQuadsPerThread], m[kQuadsPerThread], v[kQuadsPerThread];
#pragma unroll
        for (int u = 0; u < kQuadsPerThread; u++) {  // every load issued before any is used
            const long long q = q0 + u * kBlock;
            if (bits[u] && 4 * q + 4 <= T.n) {
                p[u] = ld(T.param, q);
                g[u] = ld(T.grad, q);
                m[u] = ld(T.exp_avg, q);
                v[u] = ld(T.exp_avg_sq, q);
            }
        }
#pragma unroll
        for (int u = 0; u < kQuadsPerThread; u++) {
            const long long q = q0 + u * kBlock;
            if (bits[u] == 0) continue;  // rows outside the mask: no traffic
            if (4 * q + 4 <= T.n) {
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    if (!(bits[u] >> j & 1u)) continue;
                    float pp = p[u][j], mm = m[u][j], vv = v[u][j];
                    adam_element(pp, g[u][j], mm, vv, T.s);
                    p[u][j] = pp;
                    m[u][j] = mm;
                    v[u][j] = vv;
                }
                st(T.param, q, p[u]);
                st(T.exp_avg, q, m[u]);
                st(T.exp_avg_sq, q, v[u]);
            } else {  // ragged end of the tensor
                for (int j = 0; j < 4; j++) {
                    if (!(bits[u] >> j & 1u)) continue;
                    const long long e = 4 * q + j;
                    float pp = T.param[e], mm = T.exp_avg[e], vv = T.exp_avg_sq[e];
                    adam_element(pp, T.grad[e], mm, vv, T.s);
                    T.param[e] = pp;
                    T.exp_avg[e] = mm;
                    T.exp_avg_sq[e] = vv;
                }
            }
        }
    } else {
#pragma unroll
        for (int u = 0; u < kQuadsPerThread; u++) {
            const long long q = q0 + u * kBlock;
            for (int j = 0; j < 4; j++) {
                if (!(bits[u] >> j & 1u)) continue;
                const long long e = 4 * q + j;
                float pp = T.param[e], mm = T.exp_avg[e], vv = T.exp_avg_sq[e];
                adam_element(pp, T.grad[e], mm, vv, T.s);
                T.param[e] = pp;
                T.exp_avg[e] = mm;
                T.exp_avg_sq[e] = vv;
            }
        }
    }
}

int check_tensor(const hidegs_adam_tensor& a, int i)
{
    const std::string who = "masked_adam: tensor " + std::to_string(i);
    if (a.rows < 0 || a.width <= 0) return fail(HIDEGS_E_ARG, who + ": bad shape");
    if (a.step < 1) return fail(HIDEGS_E_ARG, who + ": step counts from 1 (after the increment)");
    if (a.rows * (long long)a.width > 0 && (!a.param || !a.grad || !a.exp_avg || !a.exp_avg_sq))
        return fail(HIDEGS_E_ARG, who + ": NULL tensor");
    return 0;
}

AdamTensor describe(const hidegs_adam_tensor& a)
{
    AdamTensor T;
    T.param = a.param;
    T.grad = a.grad;
    T.exp_avg = a.exp_avg;
    T.exp_avg_sq = a.exp_avg_sq;
    T.relevant = a.relevant;
    T.n = a.rows * (long long)a.width;
    T.width = a.width;
    T.inv_w = 1.0 / (double)a.width;
    T.vec4 = ((reinterpret_cast<uintptr_t>(a.param) | reinterpret_cast<uintptr_t>(a.grad) |
               reinterpret_cast<uintptr_t>(a.exp_avg) | reinterpret_cast<uintptr_t>(a.exp_avg_sq)) & 15) == 0;
    // scalars exactly as the reference forms them (OurAdam.py:305-325), in double, cast once
    const double bias_correction1 = 1.0 - pow(a.beta1, (double)a.step);
    const double bias_correction2 = 1.0 - pow(a.beta2, (double)a.step);
    const double step_size = a.lr / bias_correction1;
    const double bc2_sqrt = sqrt(bias_correction2);
    T.s.b1 = (float)a.beta1;
    T.s.a1 = (float)(1.0 - a.beta1);
    T.s.b2 = (float)a.beta2;
    T.s.a2 = (float)(1.0 - a.beta2);
    T.s.inv_bc2 = (float)(1.0 / bc2_sqrt);  // reciprocal in double, rounded once (torch probe)
    T.s.eps = (float)a.eps;
    T.s.neg_step_size = (float)(-step_size);
    T.s.wd = (float)a.weight_decay;
    return T;
}

}  // namespace

int masked_adam_multi(const hidegs_adam_tensor* tensors, int count, hipStream_t stream)
{
    if (count < 0 || (count > 0 && !tensors)) return fail(HIDEGS_E_ARG, "masked_adam: bad tensor list");
    for (int i = 0; i < count; i++)
        if (int rc = check_tensor(tensors[i], i)) return rc;
    for (int i0 = 0; i0 < count; i0 += kMaxTensors) {  // kMaxTensors per launch
        AdamBatch batch;
        batch.count = 0;
        long long blocks = 0;
        for (int i = i0; i < count && i < i0 + kMaxTensors; i++) {
            const AdamTensor T = describe(tensors[i]);
            if (T.n == 0) continue;
            const long long quads = (T.n + 3) / 4;
            batch.first[batch.count] = (int)blocks;
            batch.t[batch.count++] = T;
            blocks += (quads + kQuadsPerBlock - 1) / kQuadsPerBlock;
            if (blocks > 0x7fffffffLL) return fail(HIDEGS_E_ARG, "masked_adam: tensors too large for one launch");
        }
        if (batch.count == 0) continue;
        batch.first[batch.count] = (int)blocks;
        HIDEGS_LAUNCH("masked_adam", masked_adam_kernel, dim3((unsigned)blocks), dim3(kBlock), 0, stream, batch);
    }
    return check_launch("masked_adam", stream, 0);
}

}  // namespace hidegs

extern "C" int hidegs_masked_adam_multi(const hidegs_adam_tensor* tensors, int count, void* stream)
{
    if (int rc = hidegs::take_async_error("hidegs_masked_adam_multi", hidegs::as_stream(stream))) return rc;
    return hidegs::masked_adam_multi(tensors, count, hidegs::as_stream(stream));
}

extern "C" int hidegs_masked_adam(float* param, const float* grad, float* exp_avg, float* exp_avg_sq,
                                  const unsigned char* relevant, long long rows, int width, double lr, double beta1,
                                  double beta2, double eps, double weight_decay, long long step, void* stream)
{
    if (int rc = hidegs::take_async_error("hidegs_masked_adam", hidegs::as_stream(stream))) return rc;
    hidegs_adam_tensor t;
    t.param = param;
    t.grad = grad;
    t.exp_avg = exp_avg;
    t.exp_avg_sq = exp_avg_sq;
    t.relevant = relevant;
    t.rows = rows;
    t.width = width;
    t.lr = lr;
    t.beta1 = beta1;
    t.beta2 = beta2;
    t.eps = eps;
    t.weight_decay = weight_decay;
    t.step = step;
    return hidegs::masked_adam_multi(&t, 1, hidegs::as_stream(stream));
}
