// gs4d_internal.h -- scratch layouts and kernel launchers shared by the libgs4d translation units.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "gs4d_math.h"

namespace gs4d {

constexpr int kTilePixels = kBlockX * kBlockY;   // 256 pixels per 16x16 tile
constexpr int kPreprocessBlock = 256;            // Gaussians per preprocess / duplicate workgroup
constexpr int kSortBlockItems = 4096;            // keys per radix-sort workgroup (256 threads x 16)
constexpr int kContribStride = 9;                // per-instance gradient terms: m2x m2y ca cb cc op r g b

// ---- scratch layouts -------------------------------------------------------------------------
// Each state is carved from one caller-allocated byte buffer with 256-byte aligned sub-arrays.
// They play the role of GeometryState / BinningState / ImageState (rasterizer_impl.h:31-67) but
// the layout is this library's own (SoA, float4-packed render attributes).
struct GeomState {
    float *depths;            // P   view-space z (forward.cu:250)
    int *radii;               // P   internal radii (used when the caller passes none)
    float2 *xy;               // P   pixel-space centre (forward.cu:233)
    float4 *conic_opacity;    // P   (conic.a, conic.b, conic.c, opacity) (forward.cu:254)
    float4 *rgbd;             // P   (r, g, b, depth) render attributes
    float *cov3D;             // 6P  world covariance (forward.cu:211)
    uint8_t *clamped;         // P   bit c set when channel c was clamped (forward.cu:67-69)
    uint32_t *tiles_touched;  // P
    uint32_t *point_offsets;  // P   exclusive offsets of each Gaussian's instances
    uint32_t *block_sums;     // nblk_pre + 1 (last entry: total L)
    static size_t required(int P);
    static GeomState carve(char *base, int P);
};

struct ImageState {
    float *final_T;      // W*H
    uint32_t *n_contrib; // W*H
    uint2 *ranges;       // T tiles
    static size_t required(int W, int H);
    static ImageState carve(char *base, int W, int H);
};

struct BinningState {
    uint64_t *keys[2];     // L each (radix ping-pong)
    uint32_t *vals[2];     // L each: unsorted instance positions
    uint32_t *gid_by_upos; // L   Gaussian id of each unsorted instance
    uint32_t *point_list;  // L   Gaussian id of each sorted instance (render order)
    uint32_t *sorted_upos; // L   unsorted position of each sorted instance
    uint32_t *hist;        // 256 * nblk_sort
    static size_t required(int L);
    static BinningState carve(char *base, int L);
};

// Camera constants stay in device memory (the caller's tensors) and are read by each kernel with
// scalar loads: no host round trip is needed to launch.
struct Args {
    int P, D, M, W, H, gx, gy;
    float scale_modifier, tan_fovx, tan_fovy, focal_x, focal_y;
    const float *viewmatrix, *projmatrix, *campos, *bg;
    int prefiltered;
};
__device__ __forceinline__ Mat4 load_mat4(const float *__restrict__ p) {
    Mat4 m;
#pragma unroll
    for (int i = 0; i < 16; i++) m.m[i] = p[i];
    return m;
}
__device__ __forceinline__ V3 load_v3(const float *__restrict__ p) { return v3(p[0], p[1], p[2]); }

// ---- launchers (each enqueues on `stream`, returns hipError_t of the launch) ------------------
hipError_t launch_preprocess(const Args &a, const float *means3D, const float *scales, const float *rotations,
                             const float *opacities, const float *shs, const float *cov3D_precomp,
                             const float *colors_precomp, int *radii, GeomState g, int *err_flag, hipStream_t s);
hipError_t launch_mark_visible(int P, const float *means3D, const float *viewmatrix, uint8_t *present, hipStream_t s);
hipError_t launch_scan_blocks(int P, GeomState g, hipStream_t s);
hipError_t launch_duplicate(const Args &a, GeomState g, const int *radii, BinningState b, hipStream_t s);
// sorts (keys[0], vals[0]) on bits [0, nbits); returns the index (0/1) of the buffers holding the result
hipError_t launch_radix_sort(BinningState b, int L, int nbits, int *result_buf, hipStream_t s);
hipError_t launch_tile_ranges(BinningState b, int L, int buf, ImageState img, int T, hipStream_t s);
hipError_t launch_render_forward(const Args &a, GeomState g, BinningState b, ImageState img, float *out_color,
                                 float *out_depth, hipStream_t s);
hipError_t launch_render_backward(const Args &a, GeomState g, const uint32_t *point_list, const uint32_t *sorted_upos,
                                  ImageState img, const float *colors, const float *dL_dpix, float *contrib,
                                  hipStream_t s);
hipError_t launch_preprocess_backward(const Args &a, GeomState g, const int *radii, const float *contrib,
                                      const float *means3D, const float *shs, const float *scales,
                                      const float *rotations, const float *cov3D, float *dL_dmean2D,
                                      float *dL_dconic, float *dL_dopacity, float *dL_dcolor, float *dL_dmean3D,
                                      float *dL_dcov3D, float *dL_dsh, float *dL_dscale, float *dL_drot,
                                      hipStream_t s);

inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

}  // namespace gs4d
