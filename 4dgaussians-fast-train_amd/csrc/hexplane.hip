// hexplane.hip -- the HexPlane field of the deformation network, fused.
//
// Reference: scene/hexplane.py:75-110 (interpolate_ms_features, concat_features=True) over the
// grids of init_grid_param (:50-72): for every point (x, y, z, t) in normalised coordinates and every
// resolution level, the product over the 6 coordinate pairs (0,1) (0,2) (0,3) (1,2) (1,3) (2,3) of a
// bilinear F.grid_sample (align_corners=True, padding_mode="border", :22-48) of the pair's plane
// (1, F, reso[c1], reso[c0]); the levels are concatenated.  The backward is the one torch's autograd
// derives from that graph: grid_sampler_2d_backward's tap weights and coordinate gradients
// (border-clipped coordinates, borders included, get zero coordinate gradient) chained through the
// left-to-right product.
//
// The reference runs 2 x 6 grid_sample launches + gathers + 10 products forward and the same again
// backward (~10 ms of the 100k-Gaussian train step, dominated by grid_sampler_2d_backward's atomics
// and the gather backward).  Here: one forward and one backward launch.  MI355X mapping:
//   - planes are repacked channels-last, (H, W, F) per plane, in one buffer: a bilinear tap is F
//     contiguous floats, so a thread serving 4 features reads one float4 per tap;
//   - a point is served by F/4 consecutive lanes; plane values stay in registers, so the backward
//     recomputes them instead of storing the 6 x levels intermediate tensors the reference keeps;
//   - coordinate gradients are reduced over the point's lanes with shuffles (no atomics);
//   - points are visited in a 3-D Morton order (gs4d_hexplane_order: 24-bit codes of the normalised
//     coordinates, the library's onesweep sort), so the ~128 points of a backward workgroup cover a
//     small box of the field and each plane sees only a small window of cells;
//   - grid gradients are gathered, not scattered: the workgroup's points are bucketed by bilinear
//     anchor cell in LDS and each touched (cell, feature) sums its neighbouring buckets with plain LDS
//     reads, then goes to HBM with one no-return atomic per workgroup; a plane whose anchor box is too
//     large falls back to direct atomics.  The channels-last gradient buffer is repacked to the
//     (1, F, H, W) parameter layout by one launch;
//   - deterministic mode (opt-in; the default sums with float atomics like the reference's
//     grid_sampler backward, and is faster): inside a workgroup a cell's taps are summed in a fixed rank order
//     (tap slot, wave, lane: ballot-matched peers, no LDS atomics), and each workgroup's sum is
//     converted to a 64-bit fixed-point integer (round to nearest, a power-of-two scale) and added
//     across workgroups by integer atomics -- exact, so no schedule changes a bit.  The scale
//     (hex_scale_of) bounds every cell's sum by 2^61: |dv| <= max|dfeat| max|param|^5 (a product of
//     5 bilinear samples, each a convex combination of parameters) and a cell takes at most one tap per
//     point, so |sum| <= N max|dfeat| max|param|^5; the resolution is that bound times 2^-61 (~1e-13
//     of the largest possible sum at 10^5 points, below fp32 rounding of any sum it can affect).
#include <algorithm>
#include <climits>

#include "../../include/gs4d_train.h"
#include "gs4d_internal.h"
#include "radix_sort.h"

namespace gs4d {

constexpr int kHexThreads = 256;
__constant__ int kPairC0[6] = {0, 0, 0, 1, 1, 2};
__constant__ int kPairC1[6] = {1, 2, 3, 2, 3, 3};

struct Tap {
    int i00, i10, i01, i11;  // cell indices (row-major H x W) of nw, ne, sw, se; -1 when outside
    float w00, w10, w01, w11;
    float ix, iy, gxm, gym;  // unnormalised coordinates and their chain factors (0 when clipped)
    int x0, y0;
};

// grid_sampler_unnormalize (align_corners) + clip_coordinates(_set_grad) for border padding
__device__ __forceinline__ float unnorm_clip(float c, int size, float &gmul) {
    float v = ((c + 1.f) / 2.f) * (float)(size - 1);
    const float lim = (float)(size - 1);
    if (v <= 0.f) {
        gmul = 0.f;
        return 0.f;
    }
    if (v >= lim) {
        gmul = 0.f;
        return lim;
    }
    gmul = (float)(size - 1) / 2.f;
    return v;
}

__device__ __forceinline__ Tap make_tap(float x, float y, int W, int H) {
    Tap t;
    t.ix = unnorm_clip(x, W, t.gxm);
    t.iy = unnorm_clip(y, H, t.gym);
    t.x0 = (int)floorf(t.ix);
    t.y0 = (int)floorf(t.iy);
    const int x1 = t.x0 + 1, y1 = t.y0 + 1;
    t.w00 = ((float)x1 - t.ix) * ((float)y1 - t.iy);
    t.w10 = (t.ix - (float)t.x0) * ((float)y1 - t.iy);
    t.w01 = ((float)x1 - t.ix) * (t.iy - (float)t.y0);
    t.w11 = (t.ix - (float)t.x0) * (t.iy - (float)t.y0);
    const bool in_x0 = t.x0 >= 0 && t.x0 < W, in_x1 = x1 >= 0 && x1 < W;
    const bool in_y0 = t.y0 >= 0 && t.y0 < H, in_y1 = y1 >= 0 && y1 < H;
    t.i00 = (in_x0 && in_y0) ? t.y0 * W + t.x0 : -1;
    t.i10 = (in_x1 && in_y0) ? t.y0 * W + x1 : -1;
    t.i01 = (in_x0 && in_y1) ? y1 * W + t.x0 : -1;
    t.i11 = (in_x1 && in_y1) ? y1 * W + x1 : -1;
    return t;
}

__device__ __forceinline__ float4 ld4(const float *base, int cell, int F, int q) {
    return cell >= 0 ? *reinterpret_cast<const float4 *>(base + (size_t)cell * F + 4 * q)
                     : make_float4(0.f, 0.f, 0.f, 0.f);
}
__device__ __forceinline__ float sel(const float4 &v, int k) { return k == 0 ? v.x : k == 1 ? v.y : k == 2 ? v.z : v.w; }

// the 4 taps of one plane for features [4q, 4q+4): value (grid_sampler_2d accumulation order)
struct TapVals {
    float4 v00, v10, v01, v11;
};
__device__ __forceinline__ TapVals load_taps(const float *plane, const Tap &t, int F, int q) {
    TapVals r;
    r.v00 = ld4(plane, t.i00, F, q);
    r.v10 = ld4(plane, t.i10, F, q);
    r.v01 = ld4(plane, t.i01, F, q);
    r.v11 = ld4(plane, t.i11, F, q);
    return r;
}
__device__ __forceinline__ float interp(const TapVals &r, const Tap &t, int k) {
    float v = 0.f;
    v = fmaf(sel(r.v00, k), t.w00, v);
    v = fmaf(sel(r.v10, k), t.w10, v);
    v = fmaf(sel(r.v01, k), t.w01, v);
    v = fmaf(sel(r.v11, k), t.w11, v);
    return v;
}

__global__ __launch_bounds__(kHexThreads) void hexplane_forward_kernel(int N, const float *__restrict__ pts,
                                                                       const uint32_t *__restrict__ order,
                                                                       gs4d_hexplane_layout lay,
                                                                       const float *__restrict__ packed,
                                                                       float *__restrict__ feat) {
    const int G = lay.F / 4;
    const int64_t tid = (int64_t)blockIdx.x * kHexThreads + threadIdx.x;
    const int i = (int)(tid / G), q = (int)(tid % G);
    if (i >= N) return;
    const int n = order ? (int)order[i] : i;
    const float4 p4 = reinterpret_cast<const float4 *>(pts)[n];
    const float pc[4] = {p4.x, p4.y, p4.z, p4.w};
    for (int l = 0; l < lay.levels; l++) {
        float prod[4] = {1.f, 1.f, 1.f, 1.f};
        for (int p = 0; p < 6; p++) {
            const gs4d_hexplane_plane pl = lay.plane[6 * l + p];
            const Tap t = make_tap(pc[kPairC0[p]], pc[kPairC1[p]], pl.W, pl.H);
            const TapVals r = load_taps(packed + pl.offset, t, lay.F, q);
#pragma unroll
            for (int k = 0; k < 4; k++) prod[k] = prod[k] * interp(r, t, k);  // interp_space * interp
        }
        *reinterpret_cast<float4 *>(feat + (size_t)n * lay.levels * lay.F + l * lay.F + 4 * q) =
            make_float4(prod[0], prod[1], prod[2], prod[3]);
    }
}

// Backward.  A workgroup serves NPW consecutive points of the Morton order (hex_points_per_wg: 2048 / F,
// at least one chunk of 256 / (F/4) points, at most 128), so they cover a small box of the field.  Per
// level:
//   1. each point's reverse pass (F/4 lanes) writes its 6 plane gradients dv (F floats each), its
//      bilinear anchor cell (x0, y0) and unnormalised coordinates (ix, iy) to LDS, and reduces its
//      coordinate gradient with shuffles;
//   2. per plane, the points' <= 4 taps (weights as make_tap forms them) are counting-sorted by cell
//      in LDS over the touched box, and every (cell, 4 features) of it sums its taps' w * dv with
//      plain LDS reads and adds the sums to HBM with no-return float atomics.  A plane whose box
//      exceeds kHexMaxCells scatters its points' taps with direct float atomics instead.
// gfx950 executes LDS float atomics (ds_add_f32) at well under one lane per clock per CU: the previous
// version, which summed the taps into LDS windows with them, spent 280 of its 620 us in those atomics.
constexpr int kHexMaxCells = 1024;
constexpr int kHexDvFloats = 2048;   // NPW * F
constexpr int kHexLdsWords = 20480;  // 80 KiB: two workgroups per CU, as the registers allow

__host__ __device__ __forceinline__ int hex_points_per_wg(int F) {
    const int ppc = kHexThreads / (F / 4);
    const int fit = kHexDvFloats / F;
    const int want = fit < 128 ? fit : 128;
    return ppc > want ? ppc : want;  // a whole number of chunks
}
// LDS words of the backward's layout (hexplane_backward_kernel); <= kHexLdsWords for every valid F
__host__ __device__ __forceinline__ int hex_bwd_lds_words(int F) {
    const int npw = hex_points_per_wg(F);
    return 6 * npw * F + 6 * npw * 3 + (kHexMaxCells + 1) + kHexMaxCells / 2 + (kHexMaxCells + 2) / 2 + 4 * npw +
           2 * npw + 6 * 4 + 4 * 6 * 4 + 8;
}

// exclusive prefix sum over the workgroup (256 threads), `tot` = the sum; s_tmp holds 4 ints
__device__ __forceinline__ int block_excl_scan(int v, int *s_tmp, int &tot) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    int x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) s_tmp[wv] = x;
    __syncthreads();
    int base = 0;
    tot = 0;
#pragma unroll
    for (int w = 0; w < kHexThreads / 64; w++) {
        const int t = s_tmp[w];
        if (w < wv) base += t;
        tot += t;
    }
    __syncthreads();
    return base + x - v;
}

// The fixed-point scale 2^e with e chosen so that N max|dfeat| max|param|^5 * 2^e <= 2^61 (mx[0] =
// max|dfeat|, mx[1] = max|param| as float bits, hex_max_kernel); 1 when the bound is 0 or not finite.
__device__ __forceinline__ float hex_scale_of(int N, const uint32_t *mx) {
    const float a = __uint_as_float(mx[0]), m = __uint_as_float(mx[1]);
    const float m2 = m * m;
    const float bound = (float)N * a * (m2 * m2 * m);
    if (!(bound > 0.f) || !(bound < 3.0e38f)) return 1.f;
    int ex;
    (void)frexpf(bound, &ex);  // bound < 2^ex
    return ldexpf(1.f, max(-126, min(127, 61 - ex)));
}
__device__ __forceinline__ unsigned long long hex_fix(float v, float scale) {
    return (unsigned long long)__float2ll_rn(v * scale);  // scale is a power of two: v * scale is exact
}
// max |x| over n floats into *mx (float bits of a non-negative value order like unsigned integers)
__global__ __launch_bounds__(256) void hex_max_kernel(int64_t n, const float *__restrict__ x, uint32_t *__restrict__ mx) {
    float m = 0.f;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) m = fmaxf(m, fabsf(x[i]));
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) m = fmaxf(m, __shfl_xor(m, off));
    __shared__ float s_m[4];
    if ((threadIdx.x & 63) == 0) s_m[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        m = fmaxf(fmaxf(s_m[0], s_m[1]), fmaxf(s_m[2], s_m[3]));
        if (m > 0.f) atomicMax(mx, __float_as_uint(m));
    }
}
// the fixed-point sums back to floats (channels-last packed layout)
__global__ __launch_bounds__(256) void hex_fix_to_float_kernel(int64_t n, int N, const uint32_t *__restrict__ mx,
                                                               const long long *__restrict__ acc,
                                                               float *__restrict__ out) {
    const float inv = 1.f / hex_scale_of(N, mx);
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
        out[i] = (float)acc[i] * inv;
}

// DET: the deterministic sums (fixed rank order in the workgroup, 64-bit fixed-point atomics across
// workgroups, dacc = the fixed-point accumulators); otherwise the reference's kind of sum -- float
// atomics straight into the packed float gradients (dacc), LDS-atomic tap ranks -- which is faster.
template <bool DET>
__global__ __launch_bounds__(kHexThreads) void hexplane_backward_kernel(int N, const float *__restrict__ pts,
                                                                        const uint32_t *__restrict__ order,
                                                                        gs4d_hexplane_layout lay,
                                                                        const float *__restrict__ packed,
                                                                        const float *__restrict__ dfeat,
                                                                        const uint32_t *__restrict__ mx,
                                                                        void *__restrict__ dacc,
                                                                        float *__restrict__ dpts) {
    const float scale = DET ? hex_scale_of(N, mx) : 1.f;
    unsigned long long *const dfix = (unsigned long long *)dacc;
    float *const dflt = (float *)dacc;
    __shared__ float smem[kHexLdsWords];
    const int F = lay.F, G = F / 4, ppc = kHexThreads / G;
    const int npw = hex_points_per_wg(F), cpw = npw / ppc;
    float *s_dv = smem;                                            // [6][npw][F]
    int *s_anc = (int *)(s_dv + 6 * npw * F);                      // [6][npw]: y0 << 16 | x0, -1: none
    float2 *s_ixy = (float2 *)(s_anc + 6 * npw);                   // [6][npw]
    int *s_off = (int *)(s_ixy + 6 * npw);                         // [kHexMaxCells + 1]: cell -> first tap
    uint16_t *s_cells = (uint16_t *)(s_off + kHexMaxCells + 1);    // [kHexMaxCells]: touched cells
    uint16_t *s_cstart = s_cells + kHexMaxCells;                   // [kHexMaxCells + 1]: their first taps
    float *s_pw = (float *)(s_off + kHexMaxCells + 1 + kHexMaxCells / 2 + (kHexMaxCells + 2) / 2);  // [4 npw]
    uint16_t *s_pj = (uint16_t *)(s_pw + 4 * npw);                 // [4 npw]: point
    int *s_box = (int *)(s_pj + 4 * npw);                          // [6][4]: ax0, ay0, aw, ah
    int *s_wbox = s_box + 24;                                      // [waves][6][4]
    int *s_tmp = s_wbox + 4 * 24;                                  // [8]
    const int q = threadIdx.x % G, slot = threadIdx.x / G;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int64_t first = (int64_t)blockIdx.x * npw;
    for (int l = 0; l < lay.levels; l++) {
        // 1. reverse passes
        for (int c = 0; c < cpw; c++) {
            const int j = c * ppc + slot;
            const int64_t i = first + j;
            const int n = i < N ? (order ? (int)order[i] : (int)i) : -1;
            if (n < 0) {
                if (q == 0)
                    for (int p = 0; p < 6; p++) s_anc[p * npw + j] = -1;
                continue;
            }
            const float4 p4 = reinterpret_cast<const float4 *>(pts)[n];
            const float pc[4] = {p4.x, p4.y, p4.z, p4.w};
            float gpt[4] = {0.f, 0.f, 0.f, 0.f};
            float v[6][4], pre[6][4];
            for (int p = 0; p < 6; p++) {
                const gs4d_hexplane_plane pl = lay.plane[6 * l + p];
                const Tap t = make_tap(pc[kPairC0[p]], pc[kPairC1[p]], pl.W, pl.H);
                const TapVals r = load_taps(packed + pl.offset, t, F, q);
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    v[p][k] = interp(r, t, k);
                    pre[p][k] = (p == 0 ? 1.f : pre[p - 1][k]) * v[p][k];  // left-to-right product
                }
            }
            const float4 d4 = *reinterpret_cast<const float4 *>(dfeat + (size_t)n * lay.levels * F + l * F + 4 * q);
            float g[4] = {d4.x, d4.y, d4.z, d4.w};
            for (int p = 5; p >= 0; p--) {
                // autograd of prod_p = prod_{p-1} * v_p: dv_p = g * prod_{p-1}, g <- g * v_p
                float dv[4];
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    dv[k] = g[k] * (p == 0 ? 1.f : pre[p - 1][k]);
                    g[k] = g[k] * v[p][k];
                }
                const gs4d_hexplane_plane pl = lay.plane[6 * l + p];
                const Tap t = make_tap(pc[kPairC0[p]], pc[kPairC1[p]], pl.W, pl.H);
                const TapVals r = load_taps(packed + pl.offset, t, F, q);
                float gix = 0.f, giy = 0.f;
                const float x1 = (float)(t.x0 + 1), y1 = (float)(t.y0 + 1), x0 = (float)t.x0, y0 = (float)t.y0;
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    const float go = dv[k];
                    // grid_sampler_2d_backward (bilinear): input gradient and coordinate gradient
                    gix -= sel(r.v00, k) * (y1 - t.iy) * go;
                    giy -= sel(r.v00, k) * (x1 - t.ix) * go;
                    gix += sel(r.v10, k) * (y1 - t.iy) * go;
                    giy -= sel(r.v10, k) * (t.ix - x0) * go;
                    gix -= sel(r.v01, k) * (t.iy - y0) * go;
                    giy += sel(r.v01, k) * (x1 - t.ix) * go;
                    gix += sel(r.v11, k) * (t.iy - y0) * go;
                    giy += sel(r.v11, k) * (t.ix - x0) * go;
                }
                *reinterpret_cast<float4 *>(s_dv + (p * npw + j) * F + 4 * q) = make_float4(dv[0], dv[1], dv[2], dv[3]);
                if (q == 0) {
                    const bool ok = t.x0 >= 0 && t.x0 < pl.W && t.y0 >= 0 && t.y0 < pl.H;  // false for NaN
                    s_anc[p * npw + j] = ok ? (t.y0 << 16) | t.x0 : -1;
                    s_ixy[p * npw + j] = make_float2(t.ix, t.iy);
                }
                gpt[kPairC0[p]] += t.gxm * gix;
                gpt[kPairC1[p]] += t.gym * giy;
            }
            // sum the coordinate gradient over the point's lanes; levels accumulate in dpts
#pragma unroll
            for (int k = 0; k < 4; k++)
                for (int off = 1; off < G; off <<= 1) gpt[k] += __shfl_xor(gpt[k], off, G);
            if (q == 0) {
                float4 *o = reinterpret_cast<float4 *>(dpts) + n;
                float4 acc = l == 0 ? make_float4(0.f, 0.f, 0.f, 0.f) : *o;
                acc.x += gpt[0]; acc.y += gpt[1]; acc.z += gpt[2]; acc.w += gpt[3];
                *o = acc;
            }
        }
        __syncthreads();
        // 2a. the anchors' boxes of the 6 planes (wave min/max, then over the waves)
        {
            int bx[6][4];
#pragma unroll
            for (int p = 0; p < 6; p++) {
                const int a = threadIdx.x < npw ? s_anc[p * npw + threadIdx.x] : -1;
                const bool ok = a >= 0;
                bx[p][0] = ok ? (a & 0xFFFF) : INT_MAX;
                bx[p][1] = ok ? (a >> 16) : INT_MAX;
                bx[p][2] = ok ? (a & 0xFFFF) : INT_MIN;
                bx[p][3] = ok ? (a >> 16) : INT_MIN;
            }
#pragma unroll
            for (int o = 32; o >= 1; o >>= 1)
#pragma unroll
                for (int p = 0; p < 6; p++) {
                    bx[p][0] = min(bx[p][0], __shfl_xor(bx[p][0], o, 64));
                    bx[p][1] = min(bx[p][1], __shfl_xor(bx[p][1], o, 64));
                    bx[p][2] = max(bx[p][2], __shfl_xor(bx[p][2], o, 64));
                    bx[p][3] = max(bx[p][3], __shfl_xor(bx[p][3], o, 64));
                }
            if (lane == 0)
#pragma unroll
                for (int p = 0; p < 6; p++)
#pragma unroll
                    for (int k = 0; k < 4; k++) s_wbox[(wv * 6 + p) * 4 + k] = bx[p][k];
        }
        __syncthreads();
        if (threadIdx.x < 6) {
            const int p = threadIdx.x;
            int x0 = INT_MAX, y0 = INT_MAX, x1 = INT_MIN, y1 = INT_MIN;
            for (int w = 0; w < kHexThreads / 64; w++) {
                x0 = min(x0, s_wbox[(w * 6 + p) * 4 + 0]);
                y0 = min(y0, s_wbox[(w * 6 + p) * 4 + 1]);
                x1 = max(x1, s_wbox[(w * 6 + p) * 4 + 2]);
                y1 = max(y1, s_wbox[(w * 6 + p) * 4 + 3]);
            }
            s_box[p * 4 + 0] = x0;
            s_box[p * 4 + 1] = y0;
            s_box[p * 4 + 2] = x1 >= x0 ? x1 - x0 + 1 : 0;
            s_box[p * 4 + 3] = y1 >= y0 ? y1 - y0 + 1 : 0;
        }
        __syncthreads();
        // 2b. per plane: bucket the points by anchor, gather each touched (cell, feature)
        for (int p = 0; p < 6; p++) {
            const gs4d_hexplane_plane pl = lay.plane[6 * l + p];
            const int ax0 = s_box[p * 4 + 0], ay0 = s_box[p * 4 + 1], aw = s_box[p * 4 + 2], ah = s_box[p * 4 + 3];
            const int na = aw * ah;
            if (na == 0) continue;  // uniform
            const float *dvp = s_dv + p * npw * F;
            const int *ancp = s_anc + p * npw;
            const float2 *ixyp = s_ixy + p * npw;
            unsigned long long *dpl = dfix + pl.offset;
            float *dplf = dflt + pl.offset;
            if ((min(ax0 + aw, pl.W - 1) - ax0 + 1) * (min(ay0 + ah, pl.H - 1) - ay0 + 1) > kHexMaxCells) {
                // uniform: a box too large for the cell offsets -- direct atomics per (point, feature)
                for (int e = threadIdx.x; e < npw * F; e += kHexThreads) {
                    const int j = e / F, f = e - j * F;
                    const int a = ancp[j];
                    if (a < 0) continue;
                    const int x0 = a & 0xFFFF, y0 = a >> 16;
                    const float2 ixy = ixyp[j];
                    const float d = dvp[j * F + f];
                    const float xa = (float)(x0 + 1) - ixy.x, xb = ixy.x - (float)x0;
                    const float ya = (float)(y0 + 1) - ixy.y, yb = ixy.y - (float)y0;
                    const bool in_x1 = x0 + 1 < pl.W, in_y1 = y0 + 1 < pl.H;
                    const size_t i0 = ((size_t)y0 * pl.W + x0) * F + f;
                    if (DET) {
                        unsigned long long *b0 = dpl + i0;
                        atomicAdd(b0, hex_fix((xa * ya) * d, scale));
                        if (in_x1) atomicAdd(b0 + F, hex_fix((xb * ya) * d, scale));
                        if (in_y1) atomicAdd(b0 + (size_t)pl.W * F, hex_fix((xa * yb) * d, scale));
                        if (in_x1 && in_y1) atomicAdd(b0 + (size_t)(pl.W + 1) * F, hex_fix((xb * yb) * d, scale));
                    } else {
                        float *b0 = dplf + i0;
                        unsafeAtomicAdd(b0, (xa * ya) * d);
                        if (in_x1) unsafeAtomicAdd(b0 + F, (xb * ya) * d);
                        if (in_y1) unsafeAtomicAdd(b0 + (size_t)pl.W * F, (xa * yb) * d);
                        if (in_x1 && in_y1) unsafeAtomicAdd(b0 + (size_t)(pl.W + 1) * F, (xb * yb) * d);
                    }
                }
                continue;
            }
            // the touched cells' box; each point's <= 4 taps counting-sorted by cell: s_off <- counts,
            // the taps' ranks within their cells kept in registers
            const int cw = min(ax0 + aw, pl.W - 1) - ax0 + 1, ch = min(ay0 + ah, pl.H - 1) - ay0 + 1;
            const int nc = cw * ch;
            for (int e = threadIdx.x; e <= nc; e += kHexThreads) s_off[e] = 0;
            __syncthreads();
            int tc[4] = {-1, -1, -1, -1}, tr[4] = {0, 0, 0, 0};
            float tw[4] = {0.f, 0.f, 0.f, 0.f};
            if (threadIdx.x < npw) {
                const int a = ancp[threadIdx.x];
                if (a >= 0) {
                    const int x0 = a & 0xFFFF, y0 = a >> 16, lx = x0 - ax0, ly = y0 - ay0;
                    const float2 ixy = ixyp[threadIdx.x];
                    // make_tap's weights: w00, w10, w01, w11
                    const float xa = (float)(x0 + 1) - ixy.x, xb = ixy.x - (float)x0;
                    const float ya = (float)(y0 + 1) - ixy.y, yb = ixy.y - (float)y0;
                    const bool in_x1 = x0 + 1 < pl.W, in_y1 = y0 + 1 < pl.H;
                    tc[0] = ly * cw + lx;
                    tw[0] = xa * ya;
                    if (in_x1) tc[1] = tc[0] + 1, tw[1] = xb * ya;
                    if (in_y1) tc[2] = tc[0] + cw, tw[2] = xa * yb;
                    if (in_x1 && in_y1) tc[3] = tc[0] + cw + 1, tw[3] = xb * yb;
                }
            }
            // deterministic ranks of the taps within their cells: tap slot by tap slot, wave by wave in
            // order, lane by lane (peer lanes of a cell found by ballots over its 10 bits), so a cell's taps
            // are summed in the same order on every run
            if (!DET) {
                if (threadIdx.x < npw)
#pragma unroll
                    for (int t = 0; t < 4; t++)
                        if (tc[t] >= 0) tr[t] = atomicAdd(&s_off[tc[t]], 1);
                __syncthreads();
            }
            const uint64_t lt_mask = ((threadIdx.x & 63) == 0) ? 0ull : (~0ull >> (64 - (threadIdx.x & 63)));
            for (int t = 0; t < 4 && DET; t++) {
                for (int w = 0; w * 64 < npw; w++) {
                    if ((int)(threadIdx.x >> 6) == w) {
                        const int c = tc[t];
                        uint64_t peers = __builtin_amdgcn_ballot_w64(c >= 0);
#pragma unroll
                        for (int bit = 0; bit < 10; bit++) {
                            const bool set = (c >> bit) & 1;
                            const uint64_t m = __builtin_amdgcn_ballot_w64(set);
                            peers &= set ? m : ~m;
                        }
                        const int old = c >= 0 ? s_off[c] : 0;
                        __builtin_amdgcn_wave_barrier();
                        if (c >= 0 && (peers & lt_mask) == 0) s_off[c] = old + __popcll(peers);
                        tr[t] = old + __popcll(peers & lt_mask);
                    }
                    __syncthreads();
                }
            }
            int ntouched;
            {
                // exclusive scan of s_off[0, nc) (four entries per thread, nc <= kHexMaxCells), the tap
                // counts in the low 16 bits and the touched-cell flags in the high 16: the cells' first
                // taps and the compact list of touched cells from one scan
                const int e0 = 4 * threadIdx.x;
                int c[4], v = 0;
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    c[u] = e0 + u < nc ? s_off[e0 + u] : 0;
                    v += c[u] + (c[u] > 0 ? 0x10000 : 0);
                }
                int tot;
                int ex = block_excl_scan(v, s_tmp, tot);
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    if (e0 + u < nc) {
                        s_off[e0 + u] = ex & 0xFFFF;
                        if (c[u] > 0) {
                            s_cells[ex >> 16] = (uint16_t)(e0 + u);
                            s_cstart[ex >> 16] = (uint16_t)(ex & 0xFFFF);
                        }
                    }
                    ex += c[u] + (c[u] > 0 ? 0x10000 : 0);
                }
                ntouched = tot >> 16;
                if (threadIdx.x == 0) s_cstart[ntouched] = (uint16_t)(tot & 0xFFFF);
            }
            __syncthreads();
#pragma unroll
            for (int t = 0; t < 4; t++)
                if (tc[t] >= 0) {
                    const int k = s_off[tc[t]] + tr[t];
                    s_pj[k] = (uint16_t)threadIdx.x;
                    s_pw[k] = tw[t];
                }
            __syncthreads();
            // gather: (touched cell, 4 features) per item, over the cell's taps in LDS
            const int nb = F / 4;
            for (int e = threadIdx.x; e < ntouched * nb; e += kHexThreads) {
                const int r = e / nb, b4 = e - r * nb;
                const int cell = s_cells[r], k0 = s_cstart[r], k1 = s_cstart[r + 1];
                // the cell's taps in their deterministic rank order, then one exact fixed-point atomic
                float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
                for (int k = k0; k < k1; k++) {
                    const int j = s_pj[k];
                    const float w = s_pw[k];
                    const float4 d = *reinterpret_cast<const float4 *>(dvp + j * F + 4 * b4);
                    acc.x += w * d.x; acc.y += w * d.y; acc.z += w * d.z; acc.w += w * d.w;
                }
                const int ry = cell / cw, rx = cell - ry * cw;
                const size_t i0 = ((size_t)(ay0 + ry) * pl.W + ax0 + rx) * F + 4 * b4;
                if (DET) {
                    unsigned long long *dst = dpl + i0;
                    if (acc.x != 0.f) atomicAdd(dst + 0, hex_fix(acc.x, scale));
                    if (acc.y != 0.f) atomicAdd(dst + 1, hex_fix(acc.y, scale));
                    if (acc.z != 0.f) atomicAdd(dst + 2, hex_fix(acc.z, scale));
                    if (acc.w != 0.f) atomicAdd(dst + 3, hex_fix(acc.w, scale));
                } else {
                    float *dst = dplf + i0;
                    if (acc.x != 0.f) unsafeAtomicAdd(dst + 0, acc.x);
                    if (acc.y != 0.f) unsafeAtomicAdd(dst + 1, acc.y);
                    if (acc.z != 0.f) unsafeAtomicAdd(dst + 2, acc.z);
                    if (acc.w != 0.f) unsafeAtomicAdd(dst + 3, acc.w);
                }
            }
            __syncthreads();
        }
    }
}

// Morton order of the points (normalised x, y, z in [-1, 1], 8 bits per axis): 24-bit codes and the
// sharded digit histograms of the onesweep sort (radix_sort.h).
__device__ __forceinline__ uint32_t spread3(uint32_t x) {  // bit i -> bit 3i (x < 1024)
    x = (x | (x << 16)) & 0x030000FF;
    x = (x | (x << 8)) & 0x0300F00F;
    x = (x | (x << 4)) & 0x030C30C3;
    x = (x | (x << 2)) & 0x09249249;
    return x;
}
__device__ __forceinline__ uint32_t quant8(float c) {
    const float v = (c + 1.f) * 128.f;
    return v >= 255.f ? 255u : (v > 0.f ? (uint32_t)v : 0u);  // NaN -> 0
}
__global__ __launch_bounds__(kHexThreads) void hex_morton_kernel(int N, const float4 *__restrict__ pts,
                                                                 uint32_t *__restrict__ codes,
                                                                 uint32_t *__restrict__ hist) {
    __shared__ uint32_t s_hist[3][256];
    for (int p = 0; p < 3; p++) s_hist[p][threadIdx.x] = 0;
    __syncthreads();
    const int i = blockIdx.x * kHexThreads + threadIdx.x;
    if (i < N) {
        const float4 p4 = pts[i];
        const uint32_t code = spread3(quant8(p4.x)) | (spread3(quant8(p4.y)) << 1) | (spread3(quant8(p4.z)) << 2);
        codes[i] = code;
#pragma unroll
        for (int p = 0; p < 3; p++) atomicAdd(&s_hist[p][(code >> (8 * p)) & 0xFFu], 1u);
    }
    __syncthreads();
    uint32_t *h = hist + (blockIdx.x % kHistShards) * (kMaxPasses * 256);
#pragma unroll
    for (int p = 0; p < 3; p++)
        if (s_hist[p][threadIdx.x]) atomicAdd(&h[p * 256 + threadIdx.x], s_hist[p][threadIdx.x]);
}
constexpr int kHexSortThreads = 1024, kHexSortItems = 4;
static size_t hex_order_zero_words(int N) {
    return 64 + (size_t)kHistWords + 4 * 256 * (size_t)sort_nblk(N, kHexSortThreads * kHexSortItems);
}

// (1, F, H, W) planes <-> the packed channels-last buffer: a transpose per plane, tiled through LDS so that
// both sides are coalesced.  Workgroup = TC consecutive cells of one plane (all F features; TC = 256 for
// F <= 32, fewer for wider planes: the tile stays <= 33 KiB): the planar side is F rows of TC contiguous
// floats, the packed side TC F contiguous floats (tile row stride TC + 1: the column reads spread over the
// banks).
constexpr int kRepackThreads = 256;
__host__ __device__ inline int repack_cells(int F) { return F <= 32 ? 256 : 8192 / F; }
__device__ __forceinline__ int repack_plane(const gs4d_hexplane_layout &lay, int64_t &tile) {
    const int TC = repack_cells(lay.F);
    int p = 0;
    for (; p < 6 * lay.levels; p++) {
        const int64_t nt = ((int64_t)lay.plane[p].W * lay.plane[p].H + TC - 1) / TC;
        if (tile < nt) break;
        tile -= nt;
    }
    return p;
}
template <bool PACK, int FC>  // FC: the feature count when known at compile time (all loads in flight), else 0
__global__ __launch_bounds__(kRepackThreads) void hexplane_repack_kernel(gs4d_hexplane_layout lay,
                                                                         float *__restrict__ packed) {
    extern __shared__ float s_tile[];  // F x (TC + 1)
    int64_t tile = blockIdx.x;
    const int p = repack_plane(lay, tile);
    if (p >= 6 * lay.levels) return;
    const gs4d_hexplane_plane pl = lay.plane[p];
    const int F = FC ? FC : lay.F, TC = repack_cells(F), TS = TC + 1, t = threadIdx.x;
    const int64_t HW = (int64_t)pl.W * pl.H, c0 = tile * TC;
    const int nc = (int)min((int64_t)TC, HW - c0);
    float *dst = packed + pl.offset + c0 * F;
    if (FC && TC == kRepackThreads) {
        // one cell per thread on the planar side, F values in flight
        if (PACK) {
            float v[FC > 0 ? FC : 1];
#pragma unroll
            for (int f = 0; f < FC; f++) v[f] = t < nc ? pl.param[f * HW + c0 + t] : 0.f;
#pragma unroll
            for (int f = 0; f < FC; f++) s_tile[f * TS + t] = v[f];
            __syncthreads();
#pragma unroll
            for (int j = 0; j < FC; j++) {
                const int k = t + j * kRepackThreads;
                if (k < nc * FC) dst[k] = s_tile[(k % FC) * TS + k / FC];
            }
        } else {
            float v[FC > 0 ? FC : 1];
#pragma unroll
            for (int j = 0; j < FC; j++) {
                const int k = t + j * kRepackThreads;
                v[j] = k < nc * FC ? dst[k] : 0.f;
            }
#pragma unroll
            for (int j = 0; j < FC; j++) {
                const int k = t + j * kRepackThreads;
                s_tile[(k % FC) * TS + k / FC] = v[j];
            }
            __syncthreads();
            if (t < nc) {
#pragma unroll
                for (int f = 0; f < FC; f++) pl.grad[f * HW + c0 + t] = s_tile[f * TS + t];
            }
        }
        return;
    }
    if (PACK) {
        for (int e = t; e < F * nc; e += kRepackThreads) {
            const int f = e / nc, c = e % nc;
            s_tile[f * TS + c] = pl.param[f * HW + c0 + c];
        }
        __syncthreads();
        for (int k = t; k < nc * F; k += kRepackThreads) dst[k] = s_tile[(k % F) * TS + k / F];
    } else {
        for (int k = t; k < nc * F; k += kRepackThreads) s_tile[(k % F) * TS + k / F] = dst[k];
        __syncthreads();
        for (int e = t; e < F * nc; e += kRepackThreads) {
            const int f = e / nc, c = e % nc;
            pl.grad[f * HW + c0 + c] = s_tile[f * TS + c];
        }
    }
}

}  // namespace gs4d

using namespace gs4d;

extern "C" {

int gs4d_hexplane_layout_init(gs4d_hexplane_layout *lay, int levels, int F, const int *W, const int *H) {
    if (!lay || levels < 1 || levels > GS4D_HEXPLANE_MAX_LEVELS || F < 4 || F % 4 != 0 || F > 256) return 1;
    if (((F / 4) & (F / 4 - 1)) != 0) return 1;  // the lanes of a point form an aligned power-of-two group
    lay->levels = levels;
    lay->F = F;
    int64_t off = 0;
    for (int i = 0; i < 6 * levels; i++) {
        if (W[i] < 1 || H[i] < 1 || W[i] > 65535 || H[i] > 65535) return 1;  // anchors pack as 16 + 16 bits
        lay->plane[i].W = W[i];
        lay->plane[i].H = H[i];
        lay->plane[i].offset = off;
        lay->plane[i].param = nullptr;
        lay->plane[i].grad = nullptr;
        off += (int64_t)W[i] * H[i] * F;
    }
    lay->total = off;
    return 0;
}

static int64_t repack_tiles(const gs4d_hexplane_layout &lay) {
    int64_t n = 0;
    const int TC = repack_cells(lay.F);
    for (int p = 0; p < 6 * lay.levels; p++) n += ((int64_t)lay.plane[p].W * lay.plane[p].H + TC - 1) / TC;
    return n;
}

int gs4d_hexplane_pack(const gs4d_hexplane_layout *lay, float *packed, void *stream) {
    if (!lay || !packed) return 1;
    for (int p = 0; p < 6 * lay->levels; p++)
        if (!lay->plane[p].param) return 1;
    const dim3 grid((unsigned)repack_tiles(*lay));
    const size_t lds = 4 * (size_t)lay->F * (repack_cells(lay->F) + 1);
    if (lay->F == 16)
        hipLaunchKernelGGL((hexplane_repack_kernel<true, 16>), grid, dim3(kRepackThreads), lds, (hipStream_t)stream, *lay, packed);
    else if (lay->F == 32)
        hipLaunchKernelGGL((hexplane_repack_kernel<true, 32>), grid, dim3(kRepackThreads), lds, (hipStream_t)stream, *lay, packed);
    else
        hipLaunchKernelGGL((hexplane_repack_kernel<true, 0>), grid, dim3(kRepackThreads), lds, (hipStream_t)stream, *lay, packed);
    return hipGetLastError() == hipSuccess ? 0 : 3;
}

int gs4d_hexplane_unpack(const gs4d_hexplane_layout *lay, const float *packed, void *stream) {
    if (!lay || !packed) return 1;
    for (int p = 0; p < 6 * lay->levels; p++)
        if (!lay->plane[p].grad) return 1;
    const dim3 grid((unsigned)repack_tiles(*lay));
    const size_t lds = 4 * (size_t)lay->F * (repack_cells(lay->F) + 1);
    float *pk = (float *)packed;
    if (lay->F == 16)
        hipLaunchKernelGGL((hexplane_repack_kernel<false, 16>), grid, dim3(kRepackThreads), lds, (hipStream_t)stream, *lay, pk);
    else if (lay->F == 32)
        hipLaunchKernelGGL((hexplane_repack_kernel<false, 32>), grid, dim3(kRepackThreads), lds, (hipStream_t)stream, *lay, pk);
    else
        hipLaunchKernelGGL((hexplane_repack_kernel<false, 0>), grid, dim3(kRepackThreads), lds, (hipStream_t)stream, *lay, pk);
    return hipGetLastError() == hipSuccess ? 0 : 3;
}

size_t gs4d_hexplane_order_scratch_bytes(int N) {
    if (N <= 0) return 256;
    return 4 * hex_order_zero_words(N) + 3 * align_up(4 * (size_t)N, 256) + 1024;
}

int gs4d_hexplane_order(int N, const float *pts, uint32_t *order, void *scratch, void *stream) {
    if (N < 0 || (N > 0 && (!pts || !order || !scratch))) return 1;
    if ((size_t)pts & 15) return 1;
    if (N == 0) return 0;
    hipStream_t s = (hipStream_t)stream;
    char *q = (char *)align_up((size_t)scratch, 256);
    auto take = [&](size_t bytes) {
        char *r = q;
        q += align_up(bytes, 256);
        return r;
    };
    const size_t zw = hex_order_zero_words(N);
    uint32_t *zero = (uint32_t *)take(4 * zw);
    uint32_t *codes[2] = {(uint32_t *)take(4 * (size_t)N), (uint32_t *)take(4 * (size_t)N)};
    uint32_t *spare = (uint32_t *)take(4 * (size_t)N);
    // 3 passes: the sorted values end in vals[1]
    uint32_t *vals[2] = {spare, order};
    uint32_t *err = zero + 8, *hist = zero + 64, *look = zero + 64 + kHistWords;
    if (hipMemsetAsync(zero, 0, 4 * zw, s) != hipSuccess) return 3;
    hipLaunchKernelGGL(hex_morton_kernel, dim3((N + kHexThreads - 1) / kHexThreads), dim3(kHexThreads), 0, s, N,
                       (const float4 *)pts, codes[0], hist);
    const int cur = onesweep_sort<kHexSortThreads, kHexSortItems>(codes, vals, N, nullptr, 24, hist, look, err, s);
    if (cur != 1) return 3;
    return hipGetLastError() == hipSuccess ? 0 : 3;
}

int gs4d_hexplane_forward(int N, const float *pts, const uint32_t *order, const gs4d_hexplane_layout *lay,
                          const float *packed, float *feat, void *stream) {
    if (N < 0 || !lay || (N > 0 && (!pts || !packed || !feat))) return 1;
    if (((size_t)pts & 15) || ((size_t)packed & 15) || ((size_t)feat & 15)) return 1;
    if (N == 0) return 0;
    const int64_t threads = (int64_t)N * (lay->F / 4);
    hipLaunchKernelGGL(hexplane_forward_kernel, dim3((unsigned)((threads + kHexThreads - 1) / kHexThreads)),
                       dim3(kHexThreads), 0, (hipStream_t)stream, N, pts, order, *lay, packed, feat);
    return hipGetLastError() == hipSuccess ? 0 : 3;
}

// backward scratch (deterministic mode): the max words and the 64-bit fixed-point accumulators
size_t gs4d_hexplane_backward_scratch_bytes(int N, const gs4d_hexplane_layout *lay) {
    (void)N;
    if (!lay) return 256;
    return 256 + 8 * (size_t)lay->total + 256;
}

int gs4d_hexplane_backward(int N, const float *pts, const uint32_t *order, const gs4d_hexplane_layout *lay,
                           const float *packed, const float *dfeat, float *dpacked, float *dpts, void *scratch,
                           int deterministic, void *stream) {
    if (N < 0 || !lay || (N > 0 && (!pts || !packed || !dfeat || !dpacked || !dpts))) return 1;
    if (deterministic && N > 0 && !scratch) return 1;
    if (((size_t)pts & 15) || ((size_t)packed & 15) || ((size_t)dfeat & 15) || ((size_t)dpts & 15)) return 1;
    hipStream_t s = (hipStream_t)stream;
    if (N == 0) return hipMemsetAsync(dpacked, 0, 4 * (size_t)lay->total, s) == hipSuccess ? 0 : 3;
    const int64_t per_wg = hex_points_per_wg(lay->F);
    const int64_t nwg = ((int64_t)N + per_wg - 1) / per_wg;
    if (hex_bwd_lds_words(lay->F) > kHexLdsWords) return 1;
    if (!deterministic) {
        if (hipMemsetAsync(dpacked, 0, 4 * (size_t)lay->total, s) != hipSuccess) return 3;
        hipLaunchKernelGGL(hexplane_backward_kernel<false>, dim3((unsigned)nwg), dim3(kHexThreads), 0, s, N, pts, order,
                           *lay, packed, dfeat, nullptr, (void *)dpacked, dpts);
        return hipGetLastError() == hipSuccess ? 0 : 3;
    }
    uint32_t *mx = (uint32_t *)align_up((size_t)scratch, 256);
    unsigned long long *dfix = (unsigned long long *)(mx + 64);
    if (hipMemsetAsync(mx, 0, 256 + 8 * (size_t)lay->total, s) != hipSuccess) return 3;
    const int64_t nfeat = (int64_t)N * lay->levels * lay->F;
    hipLaunchKernelGGL(hex_max_kernel, dim3(256), dim3(256), 0, s, nfeat, dfeat, mx);
    hipLaunchKernelGGL(hex_max_kernel, dim3(256), dim3(256), 0, s, lay->total, packed, mx + 1);
    hipLaunchKernelGGL(hexplane_backward_kernel<true>, dim3((unsigned)nwg), dim3(kHexThreads), 0, s, N, pts, order,
                       *lay, packed, dfeat, mx, (void *)dfix, dpts);
    hipLaunchKernelGGL(hex_fix_to_float_kernel, dim3(1024), dim3(256), 0, s, lay->total, N, mx,
                       (const long long *)dfix, dpacked);
    return hipGetLastError() == hipSuccess ? 0 : 3;
}

}  // extern "C"
