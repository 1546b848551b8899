/*
 * sort_ref.c -- TEST INFRASTRUCTURE ONLY (checker and the timed CPU baseline of the binning sort).
 *
 * Stable sort of (u64 key, u32 value) pairs by key bits [begin_bit, end_bit): the contract of
 * cub::DeviceRadixSort::SortPairs as the reference's forward calls it (rasterizer_impl.cu:354-362).
 * A generic multi-threaded LSD radix sort: 8-bit digits; each pass splits the input into one
 * contiguous chunk per thread, counts digits per chunk, and every thread scatters its chunk in
 * order to offsets = (pairs of smaller digits) + (pairs of its digit in earlier chunks), so each
 * pass is stable and so is the whole.  Checked against oracle/binning.py's numpy definition
 * (tests/test_oracle.py).
 *
 * Build: oracle/Makefile.
 */
#include <omp.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

int oracle_sort_pairs_u64(const uint64_t* keys_in, const uint32_t* vals_in, uint64_t* keys_out, uint32_t* vals_out,
                          long long n, int begin_bit, int end_bit, int threads)
{
    if (n <= 0) return 0;
    if (threads <= 0) threads = omp_get_max_threads();
    const int passes = (end_bit - begin_bit + 7) / 8;
    if (passes <= 0) {
        memcpy(keys_out, keys_in, (size_t)n * sizeof(uint64_t));
        memcpy(vals_out, vals_in, (size_t)n * sizeof(uint32_t));
        return 0;
    }
    uint64_t* tk = (uint64_t*)malloc((size_t)n * sizeof(uint64_t));
    uint32_t* tv = (uint32_t*)malloc((size_t)n * sizeof(uint32_t));
    long long* hist = (long long*)calloc((size_t)threads * 256, sizeof(long long));
    if (!tk || !tv || !hist) {
        free(tk);
        free(tv);
        free(hist);
        return -1;
    }
    /* the last pass writes the output: an odd pass count starts there */
    const uint64_t* sk = keys_in;
    const uint32_t* sv = vals_in;
    for (int p = 0; p < passes; p++) {
        const int shift = begin_bit + 8 * p;
        const int bits = end_bit - shift < 8 ? end_bit - shift : 8;
        const uint64_t mask = ((uint64_t)1 << bits) - 1;
        const int to_out = ((passes - 1 - p) % 2) == 0;
        uint64_t* dk = to_out ? keys_out : tk;
        uint32_t* dv = to_out ? vals_out : tv;
        memset(hist, 0, (size_t)threads * 256 * sizeof(long long));
#pragma omp parallel num_threads(threads)
        {
            const int t = omp_get_thread_num(), nt = omp_get_num_threads();
            const long long lo = n * t / nt, hi = n * (t + 1) / nt;
            long long* h = hist + (size_t)t * 256;
            for (long long i = lo; i < hi; i++) h[(sk[i] >> shift) & mask]++;
#pragma omp barrier
#pragma omp single
            {
                long long run = 0;
                for (int d = 0; d < 256; d++)
                    for (int u = 0; u < nt; u++) {
                        const long long c = hist[(size_t)u * 256 + d];
                        hist[(size_t)u * 256 + d] = run;
                        run += c;
                    }
            }
            for (long long i = lo; i < hi; i++) {
                const long long o = h[(sk[i] >> shift) & mask]++;
                dk[o] = sk[i];
                dv[o] = sv[i];
            }
        }
        sk = dk;
        sv = dv;
    }
    free(tk);
    free(tv);
    free(hist);
    return 0;
}

/* Thread count of later OpenMP regions (the oracle's CPU baselines use every core they are given). */
void oracle_set_threads(int threads)
{
    if (threads > 0) omp_set_num_threads(threads);
}

int oracle_max_threads(void) { return omp_get_max_threads(); }
