/*
 * hidegs.h -- C ABI of the MI355X-native (gfx950) Gaussian-rasterizer hot path.
 *
 * Plain pointers and sizes only: every pointer is a device pointer unless marked
 * [host].  Every entry point is stream-ordered on `stream`, which must be the
 * caller's hipStream_t (PyTorch's current stream for the tensors' device; NULL
 * selects the legacy null stream and serialises with everything on the device).
 * Entry points return 0 on success or a negative HIDEGS_E_* code; the calling
 * thread's hidegs_last_error() then holds a message.  No entry point synchronises
 * the host except where noted (the forward's num_rendered readback).
 *
 * Interfaces replaced (liuxinren456852/HiDeGS; HR = submodules/hierarchy-rasterizer,
 * SK = submodules/simple-knn):
 *   hidegs_rasterize_forward    <- CudaRasterizer::Rasterizer::forward (HR/cuda_rasterizer/rasterizer.h:33-77),
 *                                  driven by RasterizeGaussiansCUDA (HR/rasterize_points.cu:35-147)
 *   hidegs_rasterize_backward   <- CudaRasterizer::Rasterizer::backward (HR/cuda_rasterizer/rasterizer.h:79-118),
 *                                  driven by RasterizeGaussiansBackwardCUDA (HR/rasterize_points.cu:149-279)
 *   hidegs_mark_visible         <- CudaRasterizer::Rasterizer::markVisible (HR/cuda_rasterizer/rasterizer.h:24-29)
 *   hidegs_dist_cuda2           <- distCUDA2 / SimpleKNN::knn (SK/spatial.cu:15-25, SK/simple_knn.cu:186-221)
 *   hidegs_inclusive_scan_u32   <- cub::DeviceScan::InclusiveSum (HR/cuda_rasterizer/rasterizer_impl.cu:171,321)
 *   hidegs_sort_pairs_u64/_u32  <- cub::DeviceRadixSort::SortPairs (HR/cuda_rasterizer/rasterizer_impl.cu:193-196,354-362;
 *                                  SK/simple_knn.cu:211-214)
 *   hidegs_identify_tile_ranges <- cudaMemsetAsync(ranges) + identifyTileRanges (HR/cuda_rasterizer/rasterizer_impl.cu:364-371,120-142)
 *   hidegs_sort_tile_pairs      <- SortPairs + memset + identifyTileRanges as one call (rasterizer_impl.cu:354-371)
 *   hidegs_higher_msb           <- getHigherMsb (HR/cuda_rasterizer/rasterizer_impl.cu:35-50)
 *   hidegs_masked_adam          <- the per-parameter update of scene/OurAdam.py (_single_tensor_adam :249-337,
 *                                  _single_tensor_adam2 :340-420)
 *   hidegs_masked_adam_multi    <- the loop over parameters of Adam.step(relevant) (scene/OurAdam.py:106-175)
 *   hidegs_bf16_pack / _sum_ranks / _unpack, hidegs_mask_pack / _union_count
 *                               <- no reference counterpart: local steps of the view-DP exchange
 *                                  (the reference trains on one GPU)
 * INTEGRATION.md shows the Python-side bindings.
 */
#ifndef HIDEGS_H_INCLUDED
#define HIDEGS_H_INCLUDED

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HIDEGS_E_ARG (-1)         /* bad argument (reference: AT_ERROR / runtime_error) */
#define HIDEGS_E_HIP (-2)         /* HIP runtime or kernel error */
#define HIDEGS_E_ALLOC (-3)       /* a buffer callback returned NULL for a non-zero request */
#define HIDEGS_E_UNSUPPORTED (-4) /* entry point not built in this release */
#define HIDEGS_E_ASYNC (-5)       /* not run: an earlier sort on the same stream (or one replayed from a graph)
                                     failed asynchronously in its partition queue; see hidegs_queue_error for
                                     when this is reported */

/*
 * Scratch allocator callback, the C form of the reference's std::function<char*(size_t)>
 * resize functionals (HR/rasterize_points.cu:27-33).  Returns a device buffer of at
 * least `nbytes` bytes, 256-byte aligned, valid until the caller releases it.  A NULL
 * return for nbytes > 0 is an allocation failure (HIDEGS_E_ALLOC); for nbytes == 0 the
 * callback is never invoked.
 */
typedef char* (*hidegs_alloc_fn)(void* user, size_t nbytes);

/*
 * ABI deltas.  The three rasterizer entry points below keep the parameters of the interfaces they
 * replace (HR/cuda_rasterizer/rasterizer.h:24-118), in the same order and under the same names, except
 * for the parameters listed here.  A dropped parameter is one the reference glue (HR/rasterize_points.cu)
 * always passes with the same value; the value given is the one this ABI assumes.  An added parameter
 * has no reference counterpart.  tests/test_abi.py parses these lines and checks them against the
 * reference signatures and the prototypes below.
 * Line format:  DELTA <entry point> <dropped|added|renamed|retyped> <reference name>[ -> <name here>] : <meaning>
 *
 * DELTA hidegs_rasterize_forward dropped rects : non-null in the glue (rasterize_points.cu:94,141), so the rect-bounded tile path (forward.cu:390-395) is always taken; the rects are per-call scratch (the glue never returns them)
 * DELTA hidegs_rasterize_forward dropped boxmin : NULL in the glue (rasterize_points.cu:142): no bounding-box cull
 * DELTA hidegs_rasterize_forward dropped boxmax : NULL in the glue (rasterize_points.cu:143): no bounding-box cull
 * DELTA hidegs_rasterize_forward dropped skyboxnum : the default 0 (rasterizer.h:69; the glue passes nothing after debug)
 * DELTA hidegs_rasterize_forward dropped biglimit : the default INFINITY (rasterizer.h:72): no cull of large Gaussians
 * DELTA hidegs_rasterize_forward dropped on_cpu : the default false (rasterizer.h:73): device buffers only
 * DELTA hidegs_rasterize_forward added alloc_user : the user argument handed to the three hidegs_alloc_fn callbacks (the C form of a capturing std::function)
 * DELTA hidegs_rasterize_forward renamed depth -> out_invdepth : the inverse-depth image, NULL when do_depth is false (rasterize_points.cu:76-82,135)
 * DELTA hidegs_rasterize_forward retyped geometryBuffer : std::function<char*(size_t)> -> hidegs_alloc_fn (binningBuffer and imageBuffer likewise)
 * DELTA hidegs_rasterize_forward retyped prefiltered : bool -> int (render_geo and debug likewise)
 * DELTA hidegs_rasterize_forward retyped stream : the glue passes nothing, i.e. the legacy default stream (rasterizer.h:70) -> the caller's current stream
 * DELTA hidegs_rasterize_forward retyped num_rendered : the glue passes nothing (nullptr) and takes the pair count from the return value (rasterize_points.cu:108) -> [host] out-pointer written with the count; the return value is the status
 * DELTA hidegs_rasterize_backward dropped dL_dconic : (fullP, 2, 2) zeros the glue allocates and discards (rasterize_points.cu:200,264); here an internal intermediate
 * DELTA hidegs_rasterize_backward dropped dL_dinvdepth : per-Gaussian (fullP, 1) zeros the glue allocates when dL_invdepths is given and discards (rasterize_points.cu:206-216,267); here an internal intermediate
 * DELTA hidegs_rasterize_backward added h_var_bwd : anti-aliasing variance of the covariance backward, a constant 0.3 in the reference (backward.cu:211; the forward uses 0.1, forward.cu:356); the binding passes _C.H_VAR_BWD (0.3)
 * DELTA hidegs_rasterize_backward added stream : the caller's current stream (the reference launches on the legacy default stream)
 * DELTA hidegs_rasterize_backward retyped render_geo : bool -> int (debug likewise)
 * DELTA hidegs_mark_visible added stream : the caller's current stream (the reference launches on the legacy default stream)
 * DELTA hidegs_mark_visible retyped present : bool* -> unsigned char*, one byte per Gaussian, 0 or 1
 */

/*
 * Forward rasterization (P Gaussians, SH degree D, M SH coefficients per Gaussian).
 * Argument meaning as RasterizeGaussiansCUDA; hierarchy inputs (indices, parent_indices,
 * ts, kids) may be NULL.  *num_rendered [host] receives the Gaussian/tile pair count
 * (one host readback).  Not built in this release: returns HIDEGS_E_UNSUPPORTED.
 */
int hidegs_rasterize_forward(
    hidegs_alloc_fn geometryBuffer, hidegs_alloc_fn binningBuffer, hidegs_alloc_fn imageBuffer, void* alloc_user,
    int P, int D, int M,
    const float* background, int width, int height,
    const int* indices, const int* parent_indices, const float* ts, const int* kids,
    const float* means3D, const float* shs, const float* colors_precomp, const float* all_map,
    const float* opacities, const float* scales, float scale_modifier, const float* rotations,
    const float* cov3D_precomp, const float* viewmatrix, const float* projmatrix, const float* cam_pos,
    float tan_fovx, float tan_fovy, int prefiltered,
    float* out_color, float* out_invdepth, int* out_observe, float* out_all_map, float* out_plane_depth,
    int render_geo, int* radii, int debug, void* stream, int* num_rendered);

/*
 * Backward pass.  R = num_rendered of the forward.  h_var_bwd is the anti-aliasing
 * filter variance of the covariance backward (the reference uses 0.3 there against 0.1
 * in its forward, HR/cuda_rasterizer/backward.cu:211 vs forward.cu:356); it is a per-call
 * argument so autograd's device thread sees the caller's value.  Gradient outputs are
 * (P, ...) and fully written; no per-pair scratch is requested.
 * Not built in this release: returns HIDEGS_E_UNSUPPORTED.
 */
int hidegs_rasterize_backward(
    int P, int D, int M, int R,
    const float* background, const float* all_map_pixels, int width, int height,
    const int* indices, const int* parent_indices, const float* ts, const int* kids,
    const float* means3D, const float* shs, const float* colors_precomp, const float* all_maps,
    const float* scales, const float* opacities, const float* rotations, float scale_modifier,
    const float* cov3D_precomp, const float* viewmatrix, const float* projmatrix, const float* campos,
    float tan_fovx, float tan_fovy, const int* radii, float h_var_bwd,
    char* geom_buffer, char* binning_buffer, char* image_buffer,
    const float* dL_dpix, const float* dL_dout_all_map, const float* dL_dout_plane_depth, const float* dL_invdepths,
    float* dL_dmean2D, float* dL_dopacity, float* dL_dcolor, float* dL_dmean3D, float* dL_dcov3D,
    float* dL_dsh, float* dL_dscale, float* dL_drot, float* dL_dall_map,
    int render_geo, int debug, void* stream);

/* Near-plane visibility, one byte per Gaussian.  Not built in this release (HIDEGS_E_UNSUPPORTED). */
int hidegs_mark_visible(int P, const float* means3D, const float* viewmatrix, const float* projmatrix,
                        unsigned char* present, void* stream);

/*
 * distCUDA2: for each of P points (P,3) fp32, the mean of the squared distances to its
 * 3 nearest other points, written to mean_dists (P).  Exact 3-NN:
 * squared distance fmaf(dz,dz,fmaf(dx,dx,dy*dy)) of (candidate - query), three best
 * initialised to FLT_MAX (P <= 3 keeps FLT_MAX terms: P = 1, 2 give inf, P = 3 gives
 * FLT_MAX/3), a point never matches itself (duplicates give 0), result
 * ((b0 + b1) + b2) / 3.0f.  scratch_buffer receives exactly one request of
 * hidegs_knn_scratch_bytes(P) bytes when P > 0.  No host synchronisation.
 */
int hidegs_dist_cuda2(hidegs_alloc_fn scratch_buffer, void* alloc_user, int P, const float* points,
                      float* mean_dists, void* stream);
size_t hidegs_knn_scratch_bytes(int P);

/*
 * Inclusive prefix sum of n uint32 values (wrapping mod 2^32).  scratch holds at least
 * hidegs_scan_scratch_bytes(n) bytes.  in == out is allowed.
 */
size_t hidegs_scan_scratch_bytes(long long n);
int hidegs_inclusive_scan_u32(void* scratch, size_t scratch_bytes, const uint32_t* in, uint32_t* out, long long n,
                              void* stream);

/*
 * Stable LSD radix sort of n (key, value) pairs by key bits [begin_bit, end_bit)
 * (bits outside the range do not take part in the order, as in cub::DeviceRadixSort).
 * keys_in/vals_in are not modified; outputs must not alias inputs.  n < 2^31.
 */
size_t hidegs_sort_pairs_u64_scratch_bytes(long long n);
int hidegs_sort_pairs_u64(void* scratch, size_t scratch_bytes, const uint64_t* keys_in, uint64_t* keys_out,
                          const uint32_t* vals_in, uint32_t* vals_out, long long n, int begin_bit, int end_bit,
                          void* stream);
size_t hidegs_sort_pairs_u32_scratch_bytes(long long n);
int hidegs_sort_pairs_u32(void* scratch, size_t scratch_bytes, const uint32_t* keys_in, uint32_t* keys_out,
                          const uint32_t* vals_in, uint32_t* vals_out, long long n, int begin_bit, int end_bit,
                          void* stream);

/*
 * Tile ranges over n sorted keys (tile id = key >> 32): ranges (uint2 per tile, num_tiles
 * entries) is zeroed, then ranges[t] = [first, last + 1) for every tile present.  As in
 * the reference, n == 1 leaves ranges[t] = {0, 0} (identifyTileRanges sets the end of the
 * last range only for idx > 0, rasterizer_impl.cu:130-141).  Tile ids must be < num_tiles.
 */
int hidegs_identify_tile_ranges(const uint64_t* sorted_keys, long long n, uint32_t* ranges, int num_tiles,
                                void* stream);

/*
 * The binning sort as the reference's forward runs it -- SortPairs over [0, 32 + getHigherMsb(num_tiles)),
 * the memset of the ranges and identifyTileRanges (HR/cuda_rasterizer/rasterizer_impl.cu:354-371) --
 * in one call: the same keys_out, vals_out and ranges (num_tiles uint2) as hidegs_sort_pairs_u64
 * followed by hidegs_identify_tile_ranges.  Keys are (tile << 32) | depth bits with tile < num_tiles.
 * The sort partitions the pairs by tile anyway; the partition's ranges are the output, so the
 * separate range pass is saved.  scratch: hidegs_sort_pairs_u64_scratch_bytes(n).
 */
int hidegs_sort_tile_pairs(void* scratch, size_t scratch_bytes, const uint64_t* keys_in, uint64_t* keys_out,
                           const uint32_t* vals_in, uint32_t* vals_out, long long n, int num_tiles, uint32_t* ranges,
                           void* stream);

/*
 * [host] Error word of the hot-tile partition queue inside hidegs_sort_pairs_u64 /
 * hidegs_sort_tile_pairs, sticky per device since it was last cleared: bit 1 = job slots
 * exhausted, bit 4 = a queue worker gave up waiting.  Non-zero means some sort since the last
 * clear returned pairs that are not fully sorted.  Synchronises `stream`; clear != 0 resets it (one
 * device-side exchange, so no error raised meanwhile is lost) and also takes `stream`'s asynchronous
 * word and the graph word below.
 * Asynchronous report (no host synchronisation per sort): outside debug mode a failing sort's last
 * kernel ORs the failure into a word of mapped host memory that belongs to the sort's stream.  A later
 * compute entry-point call on that stream, made once that kernel has run, finds the word set, takes it
 * and returns HIDEGS_E_ASYNC without running.  The sort returns before its kernels run, so the call right
 * after it normally does NOT see the failure yet; a call that already consumed the unsorted pairs (on
 * the GPU) cannot be stopped by this report.  Calls on other streams never see it.  A caller that
 * needs the failure before consuming the output must either run in debug mode (hidegs_set_debug:
 * every sort synchronises, checks its own queue and returns HIDEGS_E_HIP itself) or call
 * hidegs_queue_error at a synchronisation point it already has.  A sort captured into a graph cannot
 * know the stream it will be replayed on: it reports to a graph word that the next compute call on ANY
 * stream takes.  The words are allocated by the first entry-point call that is not made while its
 * stream is captured into a graph; sorts captured before any such call report through debug mode and
 * hidegs_queue_error only.
 */
int hidegs_queue_error(void* stream, int clear, uint32_t* flags);

/*
 * [host] Library-wide debug mode, the reference's per-call `debug` flag (auxiliary.h:23-30) for
 * the entry points that have none: every launch check synchronises its stream and reports an
 * asynchronous fault at its stage, and sorts verify the partition queue's error word.
 */
void hidegs_set_debug(int enable);

/* [host] getHigherMsb: bits needed to hold n, at least 1; the sort end bit is 32 + this of the tile count. */
uint32_t hidegs_higher_msb(uint32_t n);

/*
 * Fused row-masked Adam step on one fp32 parameter of rows x width values (row-major).  Rows
 * with relevant[r] != 0 -- every row when relevant is NULL (the reference's empty-mask path) --
 * are updated exactly as OurAdam's torch ops update them on this GPU (op order and rounding in
 * hidegs_amd/csrc/adam.hip); other rows keep their bits (a 16-byte vector that straddles a relevant
 * row is rewritten unchanged; rows without a relevant element are not accessed).  `step` is the
 * parameter's step count after this call's increment (>= 1); lr, betas, eps, weight_decay are
 * the Python doubles the reference passes.  param, exp_avg, exp_avg_sq are updated in place.
 */
int hidegs_masked_adam(float* param, const float* grad, float* exp_avg, float* exp_avg_sq,
                       const unsigned char* relevant, long long rows, int width, double lr, double beta1,
                       double beta2, double eps, double weight_decay, long long step, void* stream);

/* One parameter of a multi-tensor masked Adam step (the fields of hidegs_masked_adam). */
typedef struct hidegs_adam_tensor {
    float* param;
    const float* grad;
    float* exp_avg;
    float* exp_avg_sq;
    const unsigned char* relevant; /* rows bytes; NULL = every row */
    long long rows;
    int width;
    double lr, beta1, beta2, eps, weight_decay;
    long long step;
} hidegs_adam_tensor;

/*
 * The whole optimizer step of OurAdam.step(relevant) (scene/OurAdam.py:106-175): every listed
 * parameter updated as hidegs_masked_adam would, with its own hyper-parameters and step count,
 * in one launch per 8 tensors.  `tensors` is a host array of `count` descriptors.
 */
int hidegs_masked_adam_multi(const hidegs_adam_tensor* tensors, int count, void* stream);

/*
 * bf16 wire format of the view-DP gradient exchange (hidegs_amd/view_dp.py, transport "bf16"), bit for
 * bit the torch definitions of hidegs_amd/csrc/wire.hip.  bf16 values are uint16_t bit patterns.
 *   hidegs_bf16_pack:      dst[i] = bf16(src[i]) (round to nearest even, NaN -> 0x7FC0) for i < n,
 *                          0 for n <= i < n_padded.
 *   hidegs_bf16_sum_ranks: out[j] = bf16(fp32 sum of parts[r * chunk + j] for r = 0 .. world-1, added in
 *                          rank order), j < chunk.
 *   hidegs_bf16_unpack:    dst[i] = float(src[i]) (exact), i < n.
 */
int hidegs_bf16_pack(const float* src, uint16_t* dst, long long n, long long n_padded, void* stream);
int hidegs_bf16_sum_ranks(const uint16_t* parts, int world, long long chunk, uint16_t* out, void* stream);
int hidegs_bf16_unpack(const uint16_t* src, float* dst, long long n, void* stream);

/*
 * Visibility masks of the view-DP exchange (hidegs_amd/view_dp.py gather_visibility), bit for bit its
 * torch definitions pack_mask / unpack_mask:
 *   hidegs_mask_pack:        bits[j] = sum over i < 8 of (mask[8j + i] != 0) << i, ceil(n / 8) bytes.
 *   hidegs_mask_union_count: bits holds `ranks` packed masks of ceil(n / 8) bytes each; for i < n,
 *                            count[i] = number of ranks with bit i set (float), any[i] = count[i] > 0.
 */
int hidegs_mask_pack(const unsigned char* mask, long long n, unsigned char* bits, void* stream);
int hidegs_mask_union_count(const unsigned char* bits, int ranks, long long n, unsigned char* any, float* count,
                            void* stream);

/*
 * [host] Per-kernel device timing.  While enabled, every kernel this library launches is
 * bracketed by two hipEvents on its stream (a few microseconds of overhead per launch);
 * hidegs_kernel_time resolves them and returns the accumulated milliseconds and launch
 * count for one kernel name (e.g. "radix_scatter_u64", "knn_leaf"), -1 if it never ran.
 */
void hidegs_kernel_timing(int enable);
void hidegs_kernel_timing_reset(void);
int hidegs_kernel_time(const char* name, double* total_ms, long long* launches);

const char* hidegs_last_error(void);
const char* hidegs_version(void);

#ifdef __cplusplus
}
#endif
#endif /* HIDEGS_H_INCLUDED */
