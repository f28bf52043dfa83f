// gs4d_internal.h -- scratch layouts and kernel launchers shared by the libgs4d translation units.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "gs4d_math.h"

namespace gs4d {

constexpr int kTilePixels = kBlockX * kBlockY;  // 256 pixels per 16x16 tile
constexpr float kLog2e = 1.4426950408889634f;    // the blend kernels evaluate the falloff in base 2
constexpr int kPreprocessBlock = 256;           // Gaussians per preprocess / duplicate workgroup
constexpr int kMaxDevices = 64;                 // per-device host state (the forward's readback word)
// Per-instance gradient record written by the render backward at the instance's emission slot:
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
    float4 *splat;            // 3P  packed blend record per Gaussian (render.hip): (x, y, -a/2 log2e, -b log2e),
                              //     (-c/2 log2e, m, 1/opacity, depth), (r, g, b, lo): m = 1 and lo = log2 opacity
                              //     for a positive-definite conic (o G = 2^(power2 + lo)), else m = opacity, lo = 0
    float *cov3D;             // 6P  world covariance (forward.cu:211)
    uint8_t *clamped;         // P   bit c set when channel c was clamped (forward.cu:67-69)
    uint32_t *tiles_touched;  // P   3-sigma rect area (the reference's tiles_touched, forward.cu:255)
    uint32_t *n_inst;         // P   tiles of the rect actually reached (half_reach), <= tiles_touched
    uint32_t *vis_gid;        // P   id of the v-th visible Gaussian (tiles_touched > 0), id order
    uint32_t *cand_off;       // P+1 exclusive scan of tiles_touched over the visible Gaussians: first
                              //     candidate instance of each (cand_off[V] = num_rendered)
    uint32_t *first_vis;      // nchunk_max: visible index owning candidate j * kEmitChunk
    uint32_t *emit_chain;     // nchunk_max + 64: the emission's chunk-prefix chain (+ err word), cleared
                              //     for this call's chunks by visible_scan (no memset)
    uint32_t *zero;           // geom_zero_words(P): counters, histograms, look-back words (one memset)
    static size_t required(int P, int T);
    static GeomState carve(char *base, int P, int T);
};
// Zero regions (u32 words) of the geometry and binning states: [0..63] counters, then the per-state
// regions of binning.hip (chunk-prefix chains, digit histograms, look-back words).
// geometry (one memset per forward): [0] prefiltered flag, [8..23] 8 u64 shards of num_rendered,
// [24] V (visible Gaussians); binning (cleared by the kernels themselves): [0] = L'.  Radix-sort users (knn.hip) keep digit histograms [kHistShards][kMaxPasses][256]
// of their own: producers add with atomics sharded by workgroup.
constexpr int kZeroFlag = 0, kZeroL = 8, kZeroV = 24, kZeroHist = 64;
constexpr int kHistShards = 8, kMaxPasses = 4;
constexpr int kHistWords = kHistShards * kMaxPasses * 256;

struct ImageState {
    float *final_T;       // W*H
    uint32_t *n_contrib;  // W*H
    uint2 *ranges;        // T tiles
    uint32_t *order;      // T tiles, longest run first: the blend kernels' workgroup -> tile map
    static size_t required(int W, int H);
    static ImageState carve(char *base, int W, int H);
};

// Sized for L = num_rendered instances; only the L' <= L reached ones are used (L' lives on the device).
constexpr int kEmitChunk = 2048;  // candidate instances per emission workgroup
size_t max_emit_chunks(int P, int T);

struct BinningState {
    uint32_t *keys[2];      // L each: tile id of each instance (ping-pong radix sort)
    uint32_t *vals[2];      // L each: emission slot of each instance (ping-pong)
    uint32_t *gid_by_e;     // L   Gaussian id | half-reach bits of each emission slot
    uint32_t *upos;         // = the vals buffer holding the sorted result: emission slot of each instance in
                            //     render order (tile, depth, id); its Gaussian is gid_by_e[upos[i]], its
                            //     gradient record goes to slot upos[i]
    uint32_t *sorted_keys;  // = the keys buffer holding the sorted tile ids
    uint32_t *tmp_hi, *tmp_lo;  // = the other ping-pong pair: long-tile sort keys
    uint32_t *tile_hist;    // counting binning: chunks x T per-chunk tile counts, then their (tile, chunk)
                            //     exclusive offsets (binning.hip); nullptr when the radix sort bins
    uint32_t *scratch;      // binning_zero_words(L, T), zeroed by one memset; word 0 = L' (emitted instances)
    int key_bits;           // msb(T) (rasterizer_impl.cu:301)
    int count_items;        // keys per lane of the counting binning (4, 8 or 16), 0 = radix-sort binning
    static size_t required(int L, int T);
    static BinningState carve(char *base, int L, int T);
};

// Camera constants stay in device memory (the caller's tensors) and are read by each kernel with
// scalar loads: no host round trip is needed to launch.
struct Args {
    int P, D, M, W, H, gx, gy;
    float scale_modifier, tan_fovx, tan_fovy, focal_x, focal_y;
    const float *viewmatrix, *projmatrix, *campos, *bg;
    int prefiltered;
    int view_transposed;  // the 16 view-matrix floats are stored transposed (a (1, 4)-strided 4x4 view)
    int exact_div;        // grids of 2^20 tiles or more: the emission's rect position by integer div/mod
};
// The 4x4 column-major flat matrix m[0..15]; `transposed`: p holds its transpose (p[4 r + c] = m[4 c + r]),
// which is how the reference's callers hand over world_view_transform (a transposed torch view).
__device__ __forceinline__ Mat4 load_mat4(const float *__restrict__ p, bool transposed = false) {
    Mat4 m;
#pragma unroll
    for (int i = 0; i < 16; i++) m.m[i] = transposed ? p[(i & 3) * 4 + (i >> 2)] : p[i];
    return m;
}
__device__ __forceinline__ V3 load_v3(const float *__restrict__ p) { return v3(p[0], p[1], p[2]); }

size_t geom_zero_words(int P);
size_t binning_zero_words(int L, int T);
int count_items(int L, int T);          // binning.hip: the counting binning's keys per lane, 0 = radix sort
size_t tile_hist_words(int L, int T);   // binning.hip: chunks x T (counting binning)

// ---- exact tile culling ------------------------------------------------------------------------
// The reference bins a splat into every tile of its 3-sigma rectangle (forward.cu:232-237), but a
// pixel only blends a splat when alpha = min(0.99, o * exp(power)) >= 1/255 (forward.cu:346-348).
// A half tile is reached when SOME pixel centre of its rectangle [x0,x1] x [y0,y1] can reach the
// threshold: the minimum of the quadratic form q = a dx^2 + 2b dx dy + c dy^2 (power = -q/2) over the
// rectangle (d = mean - pixel centre) is taken in closed form -- 0 when the mean lies inside, else the
// least of the four edges' minima (convex q: the edge's stationary point, clamped to the edge) -- and
// compared with q_thr = 2 ln(255 * 1.001 o), i.e. o exp(-q/2) >= (1/255) / 1.001: a 0.1% margin that
// dwarfs the rounding of this evaluation (fast reciprocals and log, fused multiply-adds).  Dropping
// an unreached (tile, splat) pair -- or half tile in the blend kernels -- changes no output bit: the
// reference skips every one of their pixel evaluations.  A conic that is not positive definite is
// never culled.
__device__ __forceinline__ float edge_q(float a, float b2, float c, float X, float y) {
    return __builtin_fmaf(X, __builtin_fmaf(b2, y, a * X), c * y * y);  // a X^2 + 2b X y + c y^2
}
__device__ __forceinline__ float clampf(float v, float lo, float hi) { return fminf(fmaxf(v, lo), hi); }
// Rows [8h, 8h+7] of a tile are blended by the pixel pair h of every lane (render.hip), so the
// emission records, per instance, which half tiles the splat reaches (bit h; pixel centres inside the
// image) and the blend kernels skip a half it cannot reach.  An instance reaching neither half is
// not emitted.
__device__ __forceinline__ uint32_t half_reach(float mx, float my, float4 co, int tx, int ty, int W, int H) {
    const float a = co.x, b = co.y, c = co.z, o = co.w;
    const int px0 = tx * kBlockX, px1 = min(px0 + kBlockX - 1, W - 1);
    const int y00 = ty * kBlockY, y01 = min(y00 + 7, H - 1), y10 = y00 + 8, y11 = min(y00 + 15, H - 1);
    const uint32_t exists = 1u | (y10 <= y11 ? 2u : 0u);
    if (!(a > 0.f && c > 0.f && a * c - b * b > 0.f)) return exists;
    const float thr = (2.f * 0.693147181f) * __log2f(o * (255.f * 1.001f));  // -inf / NaN: never reached
    const float b2 = 2.f * b, ia = __builtin_amdgcn_rcpf(a), ic = __builtin_amdgcn_rcpf(c);
    const float X0 = mx - (float)px1, X1 = mx - (float)px0;
    const float ys0 = -b * X0 * ic, ys1 = -b * X1 * ic;  // stationary y of the x edges (unclamped)
    const bool xin = X0 <= 0.f && X1 >= 0.f;
    uint32_t r = 0;
#pragma unroll
    for (int h = 0; h < 2; h++) {
        const float Y0 = my - (float)(h ? y11 : y01), Y1 = my - (float)(h ? y10 : y00);
        const float q0 = edge_q(a, b2, c, X0, clampf(ys0, Y0, Y1));
        const float q1 = edge_q(a, b2, c, X1, clampf(ys1, Y0, Y1));
        const float q2 = edge_q(c, b2, a, Y0, clampf(-b * Y0 * ia, X0, X1));  // q symmetric in (x, a) <-> (y, c)
        const float q3 = edge_q(c, b2, a, Y1, clampf(-b * Y1 * ia, X0, X1));
        const float qmin = (xin && Y0 <= 0.f && Y1 >= 0.f) ? 0.f : fminf(fminf(q0, q1), fminf(q2, q3));
        if (qmin <= thr) r |= 1u << h;
    }
    return r & exists;
}
// Tile runs of up to kWaveSortMax instances are depth-sorted by the render forward (render.hip), longer
// ones by tile_sort_kernel (binning.hip) before it.
constexpr int kWaveSortMax = 256;
// gid_by_e[e] = Gaussian id | half-reach bits << kReachShift (P < 2^30)
constexpr int kReachShift = 30;
constexpr uint32_t kGidMask = (1u << kReachShift) - 1u;

// v from lane (lane ^ lx) of the wave, for the bitonic networks' lane masks (lx is a constant once
// their loops are unrolled): one DPP move where a row pattern matches (quad permutes, row mirrors,
// row rotate by 8), ds_swizzle inside 32-lane halves, v_permlane32_swap across them, ds_bpermute for
// the rest.
__device__ __forceinline__ uint32_t xor_lane(uint32_t v, int lx) {
    switch (lx) {
    case 1: return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);   // quad_perm [1,0,3,2]
    case 2: return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, false);   // quad_perm [2,3,0,1]
    case 3: return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x1B, 0xF, 0xF, false);   // quad_perm [3,2,1,0]
    case 7: return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x141, 0xF, 0xF, false);  // row_half_mirror
    case 8: return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x128, 0xF, 0xF, false);  // row_ror:8
    case 15: return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x140, 0xF, 0xF, false); // row_mirror
    case 4: return (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, 0x1F | (4 << 10));
    case 16: return (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, 0x1F | (16 << 10));
    case 31: return (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, 0x1F | (31 << 10));
    case 32: {
        const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
        return (threadIdx.x & 32) ? r[0] : r[1];
    }
    case 63: {  // lane ^ 63 = (lane ^ 32) ^ 31
        const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
        const uint32_t h = (threadIdx.x & 32) ? r[0] : r[1];
        return (uint32_t)__builtin_amdgcn_ds_swizzle((int)h, 0x1F | (31 << 10));
    }
    default: return (uint32_t)__shfl_xor((int)v, lx);
    }
}

// ---- launchers (each enqueues on `stream`, returns hipError_t of the launch) ------------------
hipError_t launch_preprocess(const Args &a, const float *means3D, const float *scales, const float *rotations,
                             const float *opacities, const float *shs, const float *cov3D_precomp,
                             const float *colors_precomp, int *radii, GeomState g, int *err_flag, hipStream_t s);
hipError_t launch_mark_visible(int P, const float *means3D, const float *viewmatrix, int view_transposed,
                               uint8_t *present, hipStream_t s);
hipError_t launch_visible_scan(const Args &a, GeomState g, hipStream_t s);
hipError_t launch_binning(const Args &a, GeomState g, const int *radii, BinningState b, int L, ImageState img,
                          hipStream_t s);
hipError_t launch_render_forward(const Args &a, GeomState g, BinningState b, ImageState img, float *out_color,
                                 float *out_depth, hipStream_t s);  // also sorts runs <= kWaveSortMax
hipError_t launch_pair_alpha(GeomState g, int n, const int *gid, const int *px, const int *py, float *og, float *pw,
                             hipStream_t s);
hipError_t launch_render_backward(const Args &a, GeomState g, const uint32_t *gid_by_e, const uint32_t *upos, ImageState img,
                                  const float *colors, const float *dL_dpix, float *contrib, hipStream_t s);
size_t contrib_scratch_bytes(int R, int P);
hipError_t launch_contrib_reduce(const Args &a, GeomState g, BinningState b, int R, const float *contrib,
                                 char *scratch, float *dL_dmean2D, float4 *dL_dconic, float *dL_dopacity,
                                 float *dL_dcolor, hipStream_t s);
// also finishes the contrib_reduce sums of Gaussians spanning waves (same scratch) and zero-fills the
// render-level gradients of Gaussians without instances
hipError_t launch_gaussian_backward(const Args &a, GeomState g, int R, char *scratch, const int *radii,
                                    const float *means3D, const float *shs, const float *scales, const float *rotations,
                                    const float *cov3D, float *dL_dmean2D, float4 *dL_dconic, float *dL_dopacity,
                                    float *dL_dcolor, float *dL_dmean3D, float *dL_dcov3D, float *dL_dsh,
                                    float *dL_dscale, float *dL_drot, hipStream_t s);

size_t knn_scratch_bytes(int P);
hipError_t launch_knn(int P, const float *pts, float *mean_dists, char *scratch, hipStream_t s);

inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

}  // namespace gs4d
