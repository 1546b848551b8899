/*
 * hidegs.h -- C ABI of the MI355X-native (gfx950) differentiable Gaussian
 * rasterizer and distCUDA2.  Plain pointers and sizes only: every pointer below
 * is a device pointer unless marked [host].  Every entry point is stream-ordered
 * on the hipStream_t passed as `stream` (NULL = legacy default stream) and
 * returns 0 on success or a negative HIDEGS_E_* code; hidegs_last_error() then
 * holds a message.
 *
 * The entry points replace the interfaces the reference's Python binding calls
 * (liuxinren456852/HiDeGS, paths relative to submodules/hierarchy-rasterizer):
 *   hidegs_rasterize_forward   <- CudaRasterizer::Rasterizer::forward
 *                                 (cuda_rasterizer/rasterizer.h:33-77), driven by
 *                                 RasterizeGaussiansCUDA (rasterize_points.cu:35-147)
 *   hidegs_rasterize_backward  <- CudaRasterizer::Rasterizer::backward
 *                                 (cuda_rasterizer/rasterizer.h:79-118), driven by
 *                                 RasterizeGaussiansBackwardCUDA (rasterize_points.cu:149-279)
 *   hidegs_mark_visible        <- CudaRasterizer::Rasterizer::markVisible
 *                                 (cuda_rasterizer/rasterizer.h:24-29; never bound in ext.cpp:15-17)
 *   hidegs_dist_cuda2          <- distCUDA2 / SimpleKNN::knn
 *                                 (submodules/simple-knn/spatial.cu:15-25, simple_knn.cu:186-221)
 * INTEGRATION.md shows the Python-side binding (diff_gaussian_rasterization._C).
 */
#ifndef HIDEGS_H_INCLUDED
#define HIDEGS_H_INCLUDED

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HIDEGS_E_ARG (-1)        /* bad argument (reference: AT_ERROR / runtime_error) */
#define HIDEGS_E_HIP (-2)        /* HIP runtime or kernel error */
#define HIDEGS_E_ALLOC (-3)      /* a buffer callback returned NULL */
#define HIDEGS_E_UNSUPPORTED (-4) /* feature outside the implemented path */

/*
 * Scratch allocator callback, the C form of the reference's
 * std::function<char*(size_t)> resize functionals (rasterize_points.cu:27-33).
 * Must return a device buffer of at least `nbytes` bytes (128-byte aligned),
 * valid until the caller frees it, or NULL on failure.
 */
typedef char* (*hidegs_alloc_fn)(void* user, size_t nbytes);

/*
 * Forward rasterization.  P Gaussians, SH degree D, M SH coefficients per
 * Gaussian (0 when colors_precomp is given).  The hierarchy inputs (indices,
 * parent_indices, ts, kids) must be NULL in this release (HIDEGS_E_UNSUPPORTED
 * otherwise).  Exactly one of shs/colors_precomp and one of (scales,
 * rotations)/cov3D_precomp must be non-NULL.  all_map (P,5) may be NULL when
 * render_geo == 0.  out_invdepth may be NULL (do_depth == False).  All outputs
 * are fully written (no pre-zeroing needed).  *num_rendered [host] receives the
 * number of Gaussian/tile pairs; the geometry / binning / image buffers are
 * opaque and must be handed back unchanged to hidegs_rasterize_backward.
 */
int hidegs_rasterize_forward(
    hidegs_alloc_fn geometry_buffer, hidegs_alloc_fn binning_buffer, hidegs_alloc_fn image_buffer, void* alloc_user,
    int P, int D, int M,
    const float* background, int width, int height,
    const int* indices, const int* parent_indices, const float* ts, const int* kids,
    const float* means3D, const float* shs, const float* colors_precomp, const float* all_map,
    const float* opacities, const float* scales, float scale_modifier, const float* rotations,
    const float* cov3D_precomp, const float* viewmatrix, const float* projmatrix, const float* cam_pos,
    float tan_fovx, float tan_fovy, int prefiltered,
    float* out_color, float* out_invdepth, int* out_observe, float* out_all_map, float* out_plane_depth,
    int render_geo, int* radii, int debug, void* stream, int* num_rendered);

/* Byte sizes of the opaque buffers for given P, K (= num_rendered), W, H. */
size_t hidegs_geometry_bytes(int P);
size_t hidegs_binning_bytes(int K);
size_t hidegs_image_bytes(int width, int height);

/*
 * Backward pass.  R = num_rendered returned by the forward.  all_map_pixels is
 * the forward's out_all_map (5,H,W).  dL_dinvdepth may be NULL.  Every gradient
 * output is (P, ...) and fully written (rows of invisible Gaussians are zeros).
 * dL_dcolor / dL_dcov3D may be NULL when the caller does not need them.
 * scratch_buffer receives one request of 64*R bytes (per-pair partial rows).
 */
int hidegs_rasterize_backward(
    hidegs_alloc_fn scratch_buffer, void* alloc_user,
    int P, int D, int M, int R,
    const float* background, const float* all_map_pixels, int width, int height,
    const int* indices, const int* parent_indices, const float* ts, const int* kids,
    const float* means3D, const float* shs, const float* colors_precomp, const float* all_maps,
    const float* scales, const float* opacities, const float* rotations, float scale_modifier,
    const float* cov3D_precomp, const float* viewmatrix, const float* projmatrix, const float* campos,
    float tan_fovx, float tan_fovy, const int* radii,
    char* geom_buffer, char* binning_buffer, char* image_buffer,
    const float* dL_dpix, const float* dL_dout_all_map, const float* dL_dout_plane_depth, const float* dL_dinvdepth,
    float* dL_dmean2D, float* dL_dopacity, float* dL_dcolor, float* dL_dmean3D, float* dL_dcov3D,
    float* dL_dsh, float* dL_dscale, float* dL_drot, float* dL_dall_map,
    int render_geo, int debug, void* stream);

/* Near-plane visibility (p_view.z > 0.2), one byte per Gaussian. */
int hidegs_mark_visible(int P, const float* means3D, const float* viewmatrix, const float* projmatrix,
                        unsigned char* present, void* stream);

/*
 * Mean squared distance to the 3 nearest other points, (P,3) -> (P).
 * scratch_buffer receives one request of hidegs_knn_scratch_bytes(P) bytes.
 */
int hidegs_dist_cuda2(hidegs_alloc_fn scratch_buffer, void* alloc_user, int P, const float* points,
                      float* mean_dists, void* stream);
size_t hidegs_knn_scratch_bytes(int P);

/*
 * Anti-aliasing kernel variance used by the backward's covariance step.  The
 * reference uses 0.3 there (backward.cu:211) against 0.1 in the forward
 * (forward.cu:356); 0.3 is the default (parity).  0.1 gives the exact gradient
 * of the forward ("consistent" mode, used by finite-difference tests).
 */
void hidegs_set_backward_hvar(float h_var);
float hidegs_get_backward_hvar(void);

/*
 * Per-stage device timing, measured with hipEvents on the launch stream.
 * When enabled, every forward/backward records events around its stages;
 * hidegs_stage_times copies the accumulated milliseconds and launch counts
 * ([host] arrays of HIDEGS_NUM_STAGES) and hidegs_reset_stage_times clears them.
 */
#define HIDEGS_NUM_STAGES 12
void hidegs_enable_stage_timing(int enable);
void hidegs_reset_stage_times(void);
int hidegs_stage_times(double* ms, long long* launches);
const char* hidegs_stage_name(int stage);

const char* hidegs_last_error(void);
const char* hidegs_version(void);

#ifdef __cplusplus
}
#endif
#endif /* HIDEGS_H_INCLUDED */
