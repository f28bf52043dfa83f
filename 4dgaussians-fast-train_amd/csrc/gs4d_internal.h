// gs4d_internal.h -- scratch layouts and kernel launchers shared by the libgs4d translation units.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "gs4d_math.h"

namespace gs4d {

constexpr int kTilePixels = kBlockX * kBlockY;  // 256 pixels per 16x16 tile
constexpr int kPreprocessBlock = 256;           // Gaussians per preprocess / duplicate workgroup
constexpr int kSortBlockItems = 4096;           // keys per radix-sort workgroup (256 threads x 16)
// Per-instance gradient record written by the render backward at the instance's sorted position:
// m2x m2y conic_a conic_b conic_c opacity r g b + 3 pad (48 bytes = three 16-byte stores)
constexpr int kContribStride = 12;

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
    uint32_t *dkeys[2];       // P   depth-sort keys (ping-pong)
    uint32_t *dvals[2];       // P   depth-sort ids; dvals[0] = Gaussian id by depth rank after the sort
    uint32_t *rank;           // P   depth rank of each Gaussian
    uint32_t *sort_scratch;   // radix_scratch_words(P)
    static size_t required(int P);
    static GeomState carve(char *base, int P);
};

struct ImageState {
    float *final_T;       // W*H
    uint32_t *n_contrib;  // W*H
    uint2 *ranges;        // T tiles
    static size_t required(int W, int H);
    static ImageState carve(char *base, int W, int H);
};

struct BinningState {
    void *keys[2];          // L each: u32 or u64 instance keys (tile << rank_bits | depth rank)
    uint32_t *point_list;   // L   Gaussian id of each sorted instance (render order)
    uint32_t *upos;         // L   unsorted position (point_offsets[g] + k) of each sorted instance
    uint32_t *scratch;      // radix_scratch_words(L)
    int rank_bits, key_bits;
    bool wide;              // u64 keys
    static void geometry(int P, int T, int &rank_bits, int &key_bits, bool &wide);
    static size_t required(int L, int P, int T);
    static BinningState carve(char *base, int L, int P, int T);
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

size_t radix_scratch_words(int n);

// ---- launchers (each enqueues on `stream`, returns hipError_t of the launch) ------------------
hipError_t launch_preprocess(const Args &a, const float *means3D, const float *scales, const float *rotations,
                             const float *opacities, const float *shs, const float *cov3D_precomp,
                             const float *colors_precomp, int *radii, GeomState g, int *err_flag, hipStream_t s);
hipError_t launch_mark_visible(int P, const float *means3D, const float *viewmatrix, uint8_t *present, hipStream_t s);
hipError_t launch_scan_blocks(int P, GeomState g, hipStream_t s);
hipError_t launch_depth_order(const Args &a, GeomState g, hipStream_t s);
hipError_t launch_binning(const Args &a, GeomState g, const int *radii, BinningState b, int L, ImageState img,
                          hipStream_t s);
hipError_t launch_render_forward(const Args &a, GeomState g, BinningState b, ImageState img, float *out_color,
                                 float *out_depth, hipStream_t s);
hipError_t launch_render_backward(const Args &a, GeomState g, const uint32_t *point_list, const uint32_t *upos, ImageState img,
                                  const float *colors, const float *dL_dpix, float *contrib, hipStream_t s);
hipError_t launch_contrib_reduce(const Args &a, GeomState g, const float *contrib, float *dL_dmean2D,
                                 float4 *dL_dconic, float *dL_dopacity, float *dL_dcolor, hipStream_t s);
hipError_t launch_gaussian_backward(const Args &a, GeomState g, const int *radii, const float *means3D,
                                    const float *shs, const float *scales, const float *rotations, const float *cov3D,
                                    const float *dL_dmean2D, const float4 *dL_dconic, const float *dL_dcolor,
                                    float *dL_dmean3D, float *dL_dcov3D, float *dL_dsh, float *dL_dscale,
                                    float *dL_drot, hipStream_t s);

inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

}  // namespace gs4d
