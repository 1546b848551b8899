/*
 * adam_ref.c -- TEST INFRASTRUCTURE ONLY.  CPU oracle for the fused masked Adam step.
 *
 * Restates, from the text of the reference optimizer scene/OurAdam.py, the value one step
 * produces for each element of a parameter tensor: the masked path _single_tensor_adam
 * (:249-337; rows where `relevant` is set) and the empty-mask path _single_tensor_adam2
 * (:340-420; every row).  The op-by-op rounding is that of the torch ops the reference calls
 * as PyTorch's ROCm build executes them on the GPU (tools/probe_torch_contraction.py):
 * add-with-alpha, addcmul and addcdiv contract into one fma, division by a Python scalar is a
 * multiply by its reciprocal formed in double and rounded to float, sqrt and division are
 * correctly rounded.  Scalars are formed in double as
 * the reference forms them from step_t.item() and cast to float once.
 * The reference itself may not be run here (DESIGN.md, round-3 decision), so this restatement
 * is unpinned against its outputs.
 *
 * Build: oracle/Makefile (-ffp-contract=off: only the explicit fmaf calls fuse).
 */
#include <math.h>
#include <stdint.h>

void oracle_masked_adam(float* param, const float* grad, float* exp_avg, float* exp_avg_sq,
                        const unsigned char* relevant, long long rows, int width, double lr, double beta1,
                        double beta2, double eps, double weight_decay, long long step)
{
    const double bias_correction1 = 1.0 - pow(beta1, (double)step);
    const double bias_correction2 = 1.0 - pow(beta2, (double)step);
    const double step_size = lr / bias_correction1;
    const double bc2_sqrt = sqrt(bias_correction2);
    const float b1 = (float)beta1, a1 = (float)(1.0 - beta1), b2 = (float)beta2, a2 = (float)(1.0 - beta2);
    const float inv_bc2 = (float)(1.0 / bc2_sqrt), epsf = (float)eps, neg_ss = (float)(-step_size);
    const float wd = (float)weight_decay;
    /* rows are independent: any thread split gives the same bits */
#pragma omp parallel for schedule(static)
    for (long long r = 0; r < rows; r++) {
        if (relevant && !relevant[r]) continue;
        for (int j = 0; j < width; j++) {
            const long long e = r * width + j;
            float g = grad[e], p = param[e], m = exp_avg[e], v = exp_avg_sq[e];
            if (wd != 0.f) g = fmaf(wd, p, g);   /* grad.add(param, alpha=weight_decay) */
            m = m * b1;                          /* exp_avg.mul_(beta1) */
            m = fmaf(a1, g, m);                  /* .add_(grad, alpha=1 - beta1) */
            v = v * b2;                          /* exp_avg_sq.mul_(beta2) */
            v = fmaf(a2, g * g, v);              /* .addcmul_(grad, grad, value=1 - beta2) */
            float d = sqrtf(v);                  /* exp_avg_sq.sqrt() */
            d = d * inv_bc2;                     /* / bias_correction2_sqrt */
            d = d + epsf;                        /* .add_(eps) */
            p = fmaf(neg_ss, m / d, p);          /* param.addcdiv_(exp_avg, denom, value=-step_size) */
            param[e] = p;
            exp_avg[e] = m;
            exp_avg_sq[e] = v;
        }
    }
}
