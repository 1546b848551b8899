/*
 * knn_ref.c -- TEST INFRASTRUCTURE ONLY.  CPU oracle for distCUDA2.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg load this
 * library, and only as the checker / the timed CPU baseline; the product path
 * (simple_knn._C.distCUDA2 -> hidegs_dist_cuda2) never touches it.
 *
 * What it restates: the VALUE distCUDA2 returns (submodules/simple-knn/spatial.cu:15-25,
 * simple_knn.cu:148-184), written from its definition, not from its search:
 *   - for each query i, the three smallest squared distances to points j != i (by index,
 *     so duplicates contribute 0; simple_knn.cu:159,178), kept as updateKBest<3> keeps them
 *     (strict '>' insertion into a list initialised to FLT_MAX, :133-146,155);
 *   - squared distance of d = candidate - query (:135-136), d.x*d.x + d.y*d.y + d.z*d.z,
 *     evaluated here and on the device as fmaf(dz, dz, fmaf(dx, dx, dy * dy)): the
 *     contraction clang and gcc give that very expression under FMA contraction (the left
 *     product of a*b + c*d fused; tools/probe_contraction.c), which an LLVM-based nvcc shares
 *     (nvcc itself cannot run here; see DESIGN.md, "Parity");
 *   - result ((b0 + b1) + b2) / 3.0f (:183).
 * The reference's search (Morton boxes, :186-221) is exact, so it returns this value.
 * Brute force, O(P^2): used at P <= ~1e5 and on sampled queries at larger P.
 *
 * Build: gcc -O2 -mfma -fopenmp -ffp-contract=off -shared -fPIC (oracle/Makefile); with -ffp-contract=off
 * only the explicit fmaf calls fuse (correctly rounded with or without -mfma).
 */
#include <float.h>
#include <math.h>
#include <stdint.h>

static inline float sqdist(const float* q, const float* c)
{
    const float dx = c[0] - q[0], dy = c[1] - q[1], dz = c[2] - q[2];
    return fmaf(dz, dz, fmaf(dx, dx, dy * dy));
}

static inline void update_kbest3(float dist, float* knn)
{
    for (int j = 0; j < 3; j++) {
        if (knn[j] > dist) {
            const float t = knn[j];
            knn[j] = dist;
            dist = t;
        }
    }
}

static float mean3_of(const float* pts, long long P, long long i)
{
    float best[3] = {FLT_MAX, FLT_MAX, FLT_MAX};
    const float* q = pts + 3 * i;
    for (long long j = 0; j < P; j++) {
        if (j == i) continue;
        update_kbest3(sqdist(q, pts + 3 * j), best);
    }
    return (best[0] + best[1] + best[2]) / 3.0f;
}

/* out[i] for every i in [0, P). */
void oracle_knn_mean3(const float* pts, long long P, float* out)
{
#pragma omp parallel for schedule(dynamic, 64)
    for (long long i = 0; i < P; i++) out[i] = mean3_of(pts, P, i);
}

/* out[k] = value for query index idx[k] (sampled check at large P). */
void oracle_knn_mean3_subset(const float* pts, long long P, const int64_t* idx, long long nq, float* out)
{
#pragma omp parallel for schedule(dynamic, 1)
    for (long long k = 0; k < nq; k++) out[k] = mean3_of(pts, P, idx[k]);
}
