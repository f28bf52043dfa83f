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
//   - grid gradients are summed in LDS over those windows (one window per plane and level, bounding
//     box of the workgroup's taps) and added to HBM once per workgroup with hardware float atomics
//     (no-return); a window that does not fit the LDS budget falls back to direct atomics.  The
//     channels-last gradient buffer is repacked to the (1, F, H, W) parameter layout by one launch.
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

// Backward.  A workgroup serves kHexPointsPerWG consecutive points of the Morton order.  Per level it
// first takes, for each of the 6 planes, the bounding box of the cells its points' bilinear taps
// touch, lays the boxes out in LDS (kHexLdsFloats budget, planes in order; a box that does not fit
// keeps direct atomics), accumulates the plane gradients there with LDS atomics, then adds each box
// to the packed gradient buffer with one no-return float atomic per non-zero element.  Time planes
// get tiny boxes: within one render call every point has the same t, so their taps span two rows.
constexpr int kHexPointsPerWG = 128;
constexpr int kHexLdsFloats = 12288;  // 48 KiB: three workgroups per CU

__global__ __launch_bounds__(kHexThreads) void hexplane_backward_kernel(int N, const float *__restrict__ pts,
                                                                        const uint32_t *__restrict__ order,
                                                                        gs4d_hexplane_layout lay,
                                                                        const float *__restrict__ packed,
                                                                        const float *__restrict__ dfeat,
                                                                        float *__restrict__ dpacked,
                                                                        float *__restrict__ dpts) {
    __shared__ float s_win[kHexLdsFloats];
    __shared__ int s_box[6][4];  // x0, x1, y0, y1 (inclusive) of the plane's touched cells
    __shared__ int s_off[6];     // LDS offset of the plane's box, -1: direct atomics
    __shared__ int s_used;
    const int F = lay.F, G = F / 4, ppc = kHexThreads / G;  // lanes per point, points per chunk
    const int cpw = max(1, kHexPointsPerWG / ppc);
    const int q = threadIdx.x % G, slot = threadIdx.x / G;
    const int64_t first = (int64_t)blockIdx.x * cpw * ppc;
    auto point_of = [&](int c) -> int {
        const int64_t i = first + (int64_t)c * ppc + slot;
        return i < N ? (order ? (int)order[i] : (int)i) : -1;
    };
    for (int l = 0; l < lay.levels; l++) {
        // 1. the planes' touched-cell boxes
        if (threadIdx.x < 6) {
            s_box[threadIdx.x][0] = INT_MAX; s_box[threadIdx.x][1] = INT_MIN;
            s_box[threadIdx.x][2] = INT_MAX; s_box[threadIdx.x][3] = INT_MIN;
        }
        __syncthreads();
        if (q == 0) {
            int bx[6][4];
#pragma unroll
            for (int p = 0; p < 6; p++) { bx[p][0] = INT_MAX; bx[p][1] = INT_MIN; bx[p][2] = INT_MAX; bx[p][3] = INT_MIN; }
            for (int c = 0; c < cpw; c++) {
                const int n = point_of(c);
                if (n < 0) break;
                const float4 p4 = reinterpret_cast<const float4 *>(pts)[n];
                const float pc[4] = {p4.x, p4.y, p4.z, p4.w};
#pragma unroll
                for (int p = 0; p < 6; p++) {
                    const gs4d_hexplane_plane pl = lay.plane[6 * l + p];
                    const Tap t = make_tap(pc[kPairC0[p]], pc[kPairC1[p]], pl.W, pl.H);
                    // taps x0, x0 + 1 (y likewise) clipped to the plane: the cells make_tap keeps
                    bx[p][0] = min(bx[p][0], max(t.x0, 0));
                    bx[p][1] = max(bx[p][1], min(t.x0 + 1, pl.W - 1));
                    bx[p][2] = min(bx[p][2], max(t.y0, 0));
                    bx[p][3] = max(bx[p][3], min(t.y0 + 1, pl.H - 1));
                }
            }
#pragma unroll
            for (int p = 0; p < 6; p++) {
                atomicMin(&s_box[p][0], bx[p][0]); atomicMax(&s_box[p][1], bx[p][1]);
                atomicMin(&s_box[p][2], bx[p][2]); atomicMax(&s_box[p][3], bx[p][3]);
            }
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            int used = 0;
            for (int p = 0; p < 6; p++) {
                const int w = s_box[p][1] - s_box[p][0] + 1, h = s_box[p][3] - s_box[p][2] + 1;
                const int need = (w > 0 && h > 0) ? w * h * F : 0;
                if (need > 0 && used + need <= kHexLdsFloats) {
                    s_off[p] = used;
                    used += need;
                } else {
                    s_off[p] = -1;
                }
            }
            s_used = used;
        }
        __syncthreads();
        const int used = s_used;
        for (int e = threadIdx.x; e < used; e += kHexThreads) s_win[e] = 0.f;
        __syncthreads();
        // 2. gradients
        for (int c = 0; c < cpw; c++) {
            const int n = point_of(c);
            if (n < 0) break;
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
                const int cells[4] = {t.i00, t.i10, t.i01, t.i11};
                const float ws[4] = {t.w00, t.w10, t.w01, t.w11};
                const int off = s_off[p];
                if (off >= 0) {
                    const int bx0 = s_box[p][0], by0 = s_box[p][2], bw = s_box[p][1] - bx0 + 1;
#pragma unroll
                    for (int cc = 0; cc < 4; cc++) {
                        if (cells[cc] < 0) continue;
                        const int cy = cells[cc] / pl.W, cx = cells[cc] - cy * pl.W;
                        float *dst = s_win + off + ((cy - by0) * bw + (cx - bx0)) * F + 4 * q;
#pragma unroll
                        for (int k = 0; k < 4; k++) atomicAdd(dst + k, ws[cc] * dv[k]);
                    }
                } else {
                    float *dpl = dpacked + pl.offset + 4 * q;
#pragma unroll
                    for (int cc = 0; cc < 4; cc++) {
                        if (cells[cc] < 0) continue;
                        float *dst = dpl + (size_t)cells[cc] * F;
#pragma unroll
                        for (int k = 0; k < 4; k++) unsafeAtomicAdd(dst + k, ws[cc] * dv[k]);
                    }
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
        // 3. the boxes to HBM (rows of the box are contiguous cells x F floats in the packed layout)
        for (int p = 0; p < 6; p++) {
            const int off = s_off[p];
            if (off < 0) continue;
            const gs4d_hexplane_plane pl = lay.plane[6 * l + p];
            const int bx0 = s_box[p][0], by0 = s_box[p][2], bw = s_box[p][1] - bx0 + 1;
            const int row = bw * F, cnt = row * (s_box[p][3] - by0 + 1);
            for (int e = threadIdx.x; e < cnt; e += kHexThreads) {
                const float val = s_win[off + e];
                if (val == 0.f) continue;
                const int ry = e / row, rx = e - ry * row;
                unsafeAtomicAdd(dpacked + pl.offset + ((size_t)(by0 + ry) * pl.W + bx0) * F + rx, val);
            }
        }
        __syncthreads();
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

// (1, F, H, W) planes <-> the packed channels-last buffer.  One thread per packed element.
template <bool PACK>
__global__ __launch_bounds__(kHexThreads) void hexplane_repack_kernel(gs4d_hexplane_layout lay,
                                                                      float *__restrict__ packed) {
    const int64_t i = (int64_t)blockIdx.x * kHexThreads + threadIdx.x;
    if (i >= lay.total) return;
    int p = 0;
    while (p + 1 < 6 * lay.levels && lay.plane[p + 1].offset <= i) p++;
    const gs4d_hexplane_plane pl = lay.plane[p];
    const int64_t local = i - pl.offset;  // = cell * F + f
    const int f = (int)(local % lay.F);
    const int64_t cell = local / lay.F;
    const int64_t planar = (int64_t)f * pl.H * pl.W + cell;  // (F, H, W) index
    if (PACK) packed[i] = pl.param[planar];
    else pl.grad[planar] = packed[i];
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
        if (W[i] < 1 || H[i] < 1) return 1;
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

int gs4d_hexplane_pack(const gs4d_hexplane_layout *lay, float *packed, void *stream) {
    if (!lay || !packed) return 1;
    for (int p = 0; p < 6 * lay->levels; p++)
        if (!lay->plane[p].param) return 1;
    const int64_t nb = (lay->total + kHexThreads - 1) / kHexThreads;
    hipLaunchKernelGGL(hexplane_repack_kernel<true>, dim3((unsigned)nb), dim3(kHexThreads), 0, (hipStream_t)stream,
                       *lay, packed);
    return hipGetLastError() == hipSuccess ? 0 : 3;
}

int gs4d_hexplane_unpack(const gs4d_hexplane_layout *lay, const float *packed, void *stream) {
    if (!lay || !packed) return 1;
    for (int p = 0; p < 6 * lay->levels; p++)
        if (!lay->plane[p].grad) return 1;
    const int64_t nb = (lay->total + kHexThreads - 1) / kHexThreads;
    hipLaunchKernelGGL(hexplane_repack_kernel<false>, dim3((unsigned)nb), dim3(kHexThreads), 0, (hipStream_t)stream,
                       *lay, (float *)packed);
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

int gs4d_hexplane_backward(int N, const float *pts, const uint32_t *order, const gs4d_hexplane_layout *lay,
                           const float *packed, const float *dfeat, float *dpacked, float *dpts, void *stream) {
    if (N < 0 || !lay || (N > 0 && (!pts || !packed || !dfeat || !dpacked || !dpts))) return 1;
    if (((size_t)pts & 15) || ((size_t)packed & 15) || ((size_t)dfeat & 15) || ((size_t)dpts & 15)) return 1;
    if (N == 0) return 0;
    const int ppc = kHexThreads / (lay->F / 4);
    const int64_t per_wg = (int64_t)std::max(1, kHexPointsPerWG / ppc) * ppc;
    const int64_t nwg = ((int64_t)N + per_wg - 1) / per_wg;
    hipLaunchKernelGGL(hexplane_backward_kernel, dim3((unsigned)nwg), dim3(kHexThreads), 0, (hipStream_t)stream, N, pts,
                       order, *lay, packed, dfeat, dpacked, dpts);
    return hipGetLastError() == hipSuccess ? 0 : 3;
}

}  // extern "C"
