/*
 * gs4d.h -- C ABI of libgs4d, the MI355X (gfx950) differentiable Gaussian rasterizer.
 *
 * Drop-in boundary for the reference's native layer
 *   submodules/depth-diff-gaussian-rasterization/cuda_rasterizer/rasterizer.h:20-85
 *   (CudaRasterizer::Rasterizer::{markVisible, forward, backward})
 * which the reference's torch glue (rasterize_points.cu:36-219) binds through pybind (ext.cpp:15-18).
 * Signatures keep the reference's argument order and meaning; the differences are the ones a C ABI
 * needs: std::function allocators become (function pointer, context) pairs, the stream is explicit,
 * errors are returned as a status code instead of C++ exceptions/__trap, and outputs of the
 * reference's return value (num_rendered) come back through an out-pointer.
 *
 * Conventions (identical to the reference):
 *   - all float arrays are fp32, C-contiguous, device pointers (hipMalloc'd / torch HIP tensors);
 *   - "not provided" optional inputs are NULL (the reference passes empty tensors -> nullptr,
 *     rasterize_points.cu:95-106; branches at forward.cu:205,241 and backward.cu:390,394);
 *   - matrices are 4x4 column-major flat (viewmatrix = world_view_transform, projmatrix =
 *     full_proj_transform of scene/cameras.py:61-66);
 *   - color/depth outputs are planar CHW: out_color[ch*H*W + y*W + x] (forward.cu:376-377);
 *   - every launch is enqueued on `stream`; the forward performs exactly one device->host copy of
 *     num_rendered on that stream (rasterizer_impl.cu:282), nothing else synchronises.
 * Scratch buffers are requested through the allocator callbacks; their contents are opaque and only
 * meaningful to the matching gs4d_backward call (GeometryState/BinningState/ImageState analogue,
 * rasterizer_impl.h:31-67).  The internal layout is this library's own, not the reference's.
 */
#ifndef GS4D_H_INCLUDED
#define GS4D_H_INCLUDED

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Status codes */
#define GS4D_OK 0
#define GS4D_ERR_ARG 1          /* invalid argument (shape, degree, NULL where required) */
#define GS4D_ERR_ALLOC 2        /* allocator callback returned NULL */
#define GS4D_ERR_HIP 3          /* a HIP runtime call or kernel launch failed */
#define GS4D_ERR_PREFILTERED 4  /* prefiltered=1 but a point fails the near-plane test (auxiliary.h:156-160) */

/* Scratch allocator: returns a device pointer to at least `nbytes` bytes (16-byte aligned) that stays
 * valid until the matching backward has run, or NULL on failure.  Replaces the reference's
 * std::function<char*(size_t)> resize functors (rasterize_points.cu:27-33). */
typedef char *(*gs4d_alloc_fn)(void *ctx, size_t nbytes);

/* Replaces CudaRasterizer::Rasterizer::markVisible (rasterizer.h:24-29, rasterizer_impl.cu:141-153).
 * present[i] = 1 iff point i passes the near-plane test (auxiliary.h:139-164). */
int gs4d_mark_visible(int P, const float *means3D, const float *viewmatrix, const float *projmatrix,
                      uint8_t *present, void *stream);

/* Replaces CudaRasterizer::Rasterizer::forward (rasterizer.h:31-57, rasterizer_impl.cu:198-339).
 * radii may be NULL (internal radii are then used).  *num_rendered receives the number of
 * (tile, Gaussian) instances L.  Limits (GS4D_ERR_ARG beyond them): P < 2^30, L < 2^30, fewer than
 * 2^30 16x16 tiles. */
int gs4d_forward(gs4d_alloc_fn geometry_alloc, void *geometry_ctx, gs4d_alloc_fn binning_alloc, void *binning_ctx,
                 gs4d_alloc_fn image_alloc, void *image_ctx, int P, int D, int M, const float *background, int width,
                 int height, const float *means3D, const float *shs, const float *colors_precomp,
                 const float *opacities, const float *scales, float scale_modifier, const float *rotations,
                 const float *cov3D_precomp, const float *viewmatrix, const float *projmatrix, const float *cam_pos,
                 float tan_fovx, float tan_fovy, int prefiltered, float *out_color, float *out_depth, int *radii,
                 int debug, void *stream, int *num_rendered);

/* Replaces CudaRasterizer::Rasterizer::backward (rasterizer.h:59-85, rasterizer_impl.cu:343-437).
 * R = num_rendered of the matching forward; geom/binning/image are the buffers it allocated.
 * scratch_alloc provides the backward's own temporary (per-instance gradient terms).
 * Unlike the reference (which requires zero-filled gradient buffers, rasterize_points.cu:153-161),
 * every element of every gradient output is written, so the buffers may be uninitialised.
 * dL_dconic may be NULL (the reference allocates it but never returns it). */
int gs4d_backward(int P, int D, int M, int R, const float *background, int width, int height, const float *means3D,
                  const float *shs, const float *colors_precomp, const float *scales, float scale_modifier,
                  const float *rotations, const float *cov3D_precomp, const float *viewmatrix,
                  const float *projmatrix, const float *campos, float tan_fovx, float tan_fovy, const int *radii,
                  char *geom_buffer, char *binning_buffer, char *image_buffer, const float *dL_dpix,
                  float *dL_dmean2D, float *dL_dconic, float *dL_dopacity, float *dL_dcolor, float *dL_dmean3D,
                  float *dL_dcov3D, float *dL_dsh, float *dL_dscale, float *dL_drot, gs4d_alloc_fn scratch_alloc,
                  void *scratch_ctx, int debug, void *stream);

/* The same three entry points for a view matrix handed over transposed (view_transposed = 1: the 16
 * floats hold the transpose of the column-major matrix, i.e. a (1, 4)-strided 4x4 view such as the
 * reference callers' world_view_transform.cuda(), gaussian_renderer/__init__.py:45).  Reading it in
 * place saves the caller a copy per call; view_transposed = 0 is the plain entry point.  projmatrix
 * is always the column-major flat layout. */
int gs4d_mark_visible_ex(int P, const float *means3D, const float *viewmatrix, const float *projmatrix,
                         uint8_t *present, void *stream, int view_transposed);
int gs4d_forward_ex(gs4d_alloc_fn geometry_alloc, void *geometry_ctx, gs4d_alloc_fn binning_alloc, void *binning_ctx,
                    gs4d_alloc_fn image_alloc, void *image_ctx, int P, int D, int M, const float *background,
                    int width, int height, const float *means3D, const float *shs, const float *colors_precomp,
                    const float *opacities, const float *scales, float scale_modifier, const float *rotations,
                    const float *cov3D_precomp, const float *viewmatrix, const float *projmatrix,
                    const float *cam_pos, float tan_fovx, float tan_fovy, int prefiltered, float *out_color,
                    float *out_depth, int *radii, int debug, void *stream, int *num_rendered, int view_transposed);
int gs4d_backward_ex(int P, int D, int M, int R, const float *background, int width, int height,
                     const float *means3D, const float *shs, const float *colors_precomp, const float *scales,
                     float scale_modifier, const float *rotations, const float *cov3D_precomp,
                     const float *viewmatrix, const float *projmatrix, const float *campos, float tan_fovx,
                     float tan_fovy, const int *radii, char *geom_buffer, char *binning_buffer, char *image_buffer,
                     const float *dL_dpix, float *dL_dmean2D, float *dL_dconic, float *dL_dopacity,
                     float *dL_dcolor, float *dL_dmean3D, float *dL_dcov3D, float *dL_dsh, float *dL_dscale,
                     float *dL_drot, gs4d_alloc_fn scratch_alloc, void *scratch_ctx, int debug, void *stream,
                     int view_transposed);

/* Replaces SimpleKNN::knn (submodules/simple-knn/simple_knn.h:14-20, simple_knn.cu:187-223), the
 * native layer behind simple_knn._C.distCUDA2 (spatial.cu:15-25, ext.cpp:15-16), which
 * scene/gaussian_model.py:148-149 uses to initialise the Gaussian scales.
 * points: P x 3 fp32 (device, contiguous).  mean_dists[i] = mean of the squared distances from point i
 * to its 3 nearest other points (the reference's Morton-box search, which prunes but never changes the
 * result).  The scratch buffer comes from scratch_alloc and must stay valid until the stream has run
 * the launches.  P == 0 is a no-op. */
int gs4d_knn_mean_dist(int P, const float *points, float *mean_dists, gs4d_alloc_fn scratch_alloc, void *scratch_ctx,
                       void *stream);

/* Diagnostic for the parity tests (no reference counterpart): for n (Gaussian, pixel) pairs, o G (the
 * blend's alpha before the 0.99 cap) and the base-2 exponent log2(G), evaluated by the exact arithmetic
 * of the blend kernels from the packed splat records a gs4d_forward left in geometry_buffer (P Gaussians,
 * a width x height image).  gid/px/py: n int32 device arrays; og/pw: n fp32 device outputs. */
int gs4d_debug_pair_alpha(int P, int width, int height, const char *geometry_buffer, int n, const int *gid,
                          const int *px, const int *py, float *og, float *pw, void *stream);

/* Human-readable message for the last error on this thread (never NULL). */
const char *gs4d_last_error(void);

/* Library version string, e.g. "gs4d 0.1.0 gfx950". */
const char *gs4d_version(void);

/* Per-kernel timing of the most recent gs4d_forward / gs4d_backward on this thread, recorded with
 * hipEvents on the launch stream when profiling is enabled (bench.py).  names[i] / ms[i] for
 * i < *count; returns the number of entries.  enabled >= 2 launches the two blend kernels (render,
 * render_backward) that many times back to back and reports their per-launch average (an entry
 * "<name>_pre" then holds the time up to that stage). */
void gs4d_set_profiling(int enabled);
int gs4d_last_timings(const char **names, float *ms, int max_entries);

#ifdef __cplusplus
}
#endif

#endif /* GS4D_H_INCLUDED */
