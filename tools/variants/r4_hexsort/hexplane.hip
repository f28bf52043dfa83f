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
//     reads, then goes to HBM with one no-return float atomic per workgroup; a plane whose anchor box
//     is too large falls back to direct atomics.  The channels-last gradient buffer is repacked to
//     the (1, F, H, W) parameter layout by one launch.
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

// Backward, deterministic: the plane gradients are sums over taps in an order fixed by the data, never
// by the schedule (no float atomics).  Three steps:
//   1. hexplane_dv_kernel, point-major (a point = F/4 lanes, the Morton order of the forward): per
//      level the point's reverse pass -- the 6 plane values recomputed, the left-to-right product's
//      gradients dv (F floats per plane), grid_sampler_2d_backward's coordinate gradients reduced over
//      the point's lanes -- and one ENTRY per (point, plane): dv, the unnormalised coordinates (ix, iy)
//      and the key = the global id of its bilinear anchor cell (y0, x0), with the key's digit histograms
//      for the sort;
//   2. a stable onesweep sort of the entries by key (radix_sort.h), then each cell's [start, end) of
//      the sorted entries (hex_cell_ranges_kernel);
//   3. hexplane_gather_kernel, cell-major: the gradient of cell (cx, cy) sums the taps of the entries
//      anchored at (cx-1, cy-1), (cx, cy-1), (cx-1, cy), (cx, cy) -- bucket by bucket, each bucket in
//      sorted (= Morton point) order -- with make_tap's weights, the taps split over the lanes of a wave
//      and summed by a fixed shuffle tree, and writes the cell's F features to the packed buffer
//      (every cell, zeros included: no zero-fill).
// A cell of a time plane collects the taps of every point at the view's timestamp (thousands): the taps
// of a cell are spread over the wave's lanes, so a long bucket costs iterations, not a serial walk.
constexpr int kHexGatherThreads = 256;
constexpr int kHexSortThreads = 1024, kHexSortItems = 4;
constexpr int kHexKeyBits = 24;  // 3 onesweep passes: cell ids < 2^24 (the invalid key 0xFFFFFFFF sorts last)

__global__ __launch_bounds__(kHexThreads) void hexplane_dv_kernel(int N, const float *__restrict__ pts,
                                                                  const uint32_t *__restrict__ order,
                                                                  gs4d_hexplane_layout lay,
                                                                  const float *__restrict__ packed,
                                                                  const float *__restrict__ dfeat,
                                                                  float *__restrict__ dv_out,
                                                                  float2 *__restrict__ ixy_out,
                                                                  uint32_t *__restrict__ keys,
                                                                  uint32_t *__restrict__ hist,
                                                                  float *__restrict__ dpts) {
    __shared__ uint32_t s_hist[3][256];
    for (int k = threadIdx.x; k < 3 * 256; k += kHexThreads) (&s_hist[0][0])[k] = 0;
    __syncthreads();
    const int F = lay.F, G = F / 4, NP = 6 * lay.levels;
    const int64_t tid = (int64_t)blockIdx.x * kHexThreads + threadIdx.x;
    const int i = (int)(tid / G), q = (int)(tid % G);
    if (i < N) {
        const int n = order ? (int)order[i] : i;
        const float4 p4 = reinterpret_cast<const float4 *>(pts)[n];
        const float pc[4] = {p4.x, p4.y, p4.z, p4.w};
        float gpt[4] = {0.f, 0.f, 0.f, 0.f};
        for (int l = 0; l < lay.levels; l++) {
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
                const int lp = 6 * l + p;
                const gs4d_hexplane_plane pl = lay.plane[lp];
                const Tap t = make_tap(pc[kPairC0[p]], pc[kPairC1[p]], pl.W, pl.H);
                const TapVals r = load_taps(packed + pl.offset, t, F, q);
                float gix = 0.f, giy = 0.f;
                const float x1 = (float)(t.x0 + 1), y1 = (float)(t.y0 + 1), x0 = (float)t.x0, y0 = (float)t.y0;
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    const float go = dv[k];
                    // grid_sampler_2d_backward (bilinear): coordinate gradient
                    gix -= sel(r.v00, k) * (y1 - t.iy) * go;
                    giy -= sel(r.v00, k) * (x1 - t.ix) * go;
                    gix += sel(r.v10, k) * (y1 - t.iy) * go;
                    giy -= sel(r.v10, k) * (t.ix - x0) * go;
                    gix -= sel(r.v01, k) * (t.iy - y0) * go;
                    giy += sel(r.v01, k) * (x1 - t.ix) * go;
                    gix += sel(r.v11, k) * (t.iy - y0) * go;
                    giy += sel(r.v11, k) * (t.ix - x0) * go;
                }
                const size_t e = (size_t)i * NP + lp;
                *reinterpret_cast<float4 *>(dv_out + e * F + 4 * q) = make_float4(dv[0], dv[1], dv[2], dv[3]);
                if (q == 0) {
                    const bool ok = t.x0 >= 0 && t.x0 < pl.W && t.y0 >= 0 && t.y0 < pl.H;  // false for NaN
                    const uint32_t key = ok ? (uint32_t)(pl.offset / F) + (uint32_t)(t.y0 * pl.W + t.x0) : 0xFFFFFFFFu;
                    keys[e] = key;
                    ixy_out[e] = make_float2(t.ix, t.iy);
#pragma unroll
                    for (int d = 0; d < 3; d++) atomicAdd(&s_hist[d][(key >> (8 * d)) & 0xFFu], 1u);
                }
                gpt[kPairC0[p]] += t.gxm * gix;
                gpt[kPairC1[p]] += t.gym * giy;
            }
        }
        // the coordinate gradient summed over the point's lanes (levels in order, as the reference's sum)
#pragma unroll
        for (int k = 0; k < 4; k++)
            for (int off = 1; off < G; off <<= 1) gpt[k] += __shfl_xor(gpt[k], off, G);
        if (q == 0) reinterpret_cast<float4 *>(dpts)[n] = make_float4(gpt[0], gpt[1], gpt[2], gpt[3]);
    }
    __syncthreads();
    uint32_t *h = hist + (blockIdx.x % kHistShards) * (kMaxPasses * 256);
    for (int k = threadIdx.x; k < 3 * 256; k += kHexThreads) {
        const uint32_t c = (&s_hist[0][0])[k];
        if (c) atomicAdd(&h[(k >> 8) * 256 + (k & 255)], c);
    }
}

// [start, end) of every cell's run of sorted entries (cells without entries keep the zero fill)
__global__ __launch_bounds__(256) void hex_cell_ranges_kernel(int64_t NE, uint32_t NC, const uint32_t *__restrict__ skeys,
                                                              uint2 *__restrict__ ranges) {
    const int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (k >= NE) return;
    const uint32_t key = skeys[k];
    if (key >= NC) return;
    if (k == 0 || skeys[k - 1] != key) ranges[key].x = (uint32_t)k;
    if (k == NE - 1 || skeys[k + 1] != key) ranges[key].y = (uint32_t)(k + 1);
}

// The gather is balanced by CHUNKS of at most kHexChunk taps: a cell with K taps (its 4 anchor buckets)
// owns ceil(K / kHexChunk) chunks (one when empty).  hex_chunk_plan_kernel numbers the chunks in cell
// order (a block scan + decoupled block prefixes) and records, per chunk, its cell; hexplane_gather_kernel
// (a fixed grid looping over the chunks) sums a chunk's taps -- lane = (tap slot s, feature group q):
// G = F/4 groups, S = 64/G slots, slot s takes taps s, s + S, ... of the chunk, summed by a fixed xor
// tree -- and writes a one-chunk cell's F features straight to the packed buffer, a longer cell's
// partial to its chunk slot; hex_combine_kernel then adds each long cell's partials in chunk order.
// A cell of a time plane collects the taps of every point at the view's timestamp (thousands): its work
// is spread over many waves instead of one serial walk, and the sums stay in a data-fixed order.
constexpr int kHexChunk = 64;
constexpr int kHexPlanThreads = 256;

struct HexCell {
    uint32_t base;  // first cell id of the plane
    int W, cx, cy;
};
__device__ __forceinline__ HexCell hex_cell(const gs4d_hexplane_layout &lay, uint32_t c) {
    const int F = lay.F, NP = 6 * lay.levels;
    int lp = 0;
    while (lp + 1 < NP && (uint32_t)(lay.plane[lp + 1].offset / F) <= c) lp++;
    HexCell h;
    h.base = (uint32_t)(lay.plane[lp].offset / F);
    h.W = lay.plane[lp].W;
    const uint32_t loc = c - h.base;
    h.cy = (int)(loc / (uint32_t)h.W);
    h.cx = (int)(loc - (uint32_t)h.cy * h.W);
    return h;
}
// the 4 anchor buckets of a cell: (cx - 1, cy - 1), (cx, cy - 1), (cx - 1, cy), (cx, cy)
__device__ __forceinline__ uint32_t hex_buckets(const HexCell &h, const uint2 *__restrict__ ranges, uint32_t bs[4],
                                                uint32_t bn[4]) {
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int ax = h.cx - 1 + (k & 1), ay = h.cy - 1 + (k >> 1);
        const uint2 r = (ax >= 0 && ay >= 0) ? ranges[h.base + (uint32_t)(ay * h.W + ax)] : make_uint2(0u, 0u);
        bs[k] = r.x;
        bn[k] = r.y - r.x;
    }
    return bn[0] + bn[1] + bn[2] + bn[3];
}

// plan: per cell its chunk count; cell_chunk[c] = its first chunk, chunk_cell[ch] = the chunk's cell,
// long[] = the cells of more than one chunk (appended in any order), cnt[0] = chunks, cnt[1] = long cells
__global__ __launch_bounds__(kHexPlanThreads) void hex_chunk_plan_kernel(gs4d_hexplane_layout lay, uint32_t NC,
                                                                         const uint2 *__restrict__ ranges,
                                                                         uint32_t *__restrict__ cell_chunk,
                                                                         uint32_t *__restrict__ chunk_cell,
                                                                         uint32_t *__restrict__ long_cells,
                                                                         uint32_t *__restrict__ cnt,
                                                                         uint32_t *__restrict__ look,
                                                                         uint32_t *__restrict__ err) {
    __shared__ uint32_t s_w[kHexPlanThreads / 64], s_tmp[4];
    const uint32_t c = blockIdx.x * kHexPlanThreads + threadIdx.x;
    uint32_t nch = 0;
    if (c < NC) {
        const HexCell h = hex_cell(lay, c);
        uint32_t bs[4], bn[4];
        const uint32_t K = hex_buckets(h, ranges, bs, bn);
        nch = K == 0 ? 1u : (K + kHexChunk - 1) / kHexChunk;
        if (nch > 1) long_cells[atomicAdd(&cnt[1], 1u)] = c;
    }
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint32_t incl = wave_incl_sum(nch);
    if (lane == 63) s_w[w] = incl;
    __syncthreads();
    uint32_t wbase = 0, tot = 0;
#pragma unroll
    for (int k = 0; k < kHexPlanThreads / 64; k++) {
        if (k < w) wbase += s_w[k];
        tot += s_w[k];
    }
    const uint32_t base = block_prefix(look, blockIdx.x, tot, err, s_tmp);
    const uint32_t off = base + wbase + incl - nch;
    if (c < NC) {
        cell_chunk[c] = off;
        for (uint32_t j = 0; j < nch; j++) chunk_cell[off + j] = c;
    }
    if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) {
        store_word(&cnt[0], base + tot);
        cell_chunk[NC] = base + tot;
    }
}

__global__ __launch_bounds__(kHexGatherThreads) void hexplane_gather_kernel(gs4d_hexplane_layout lay,
                                                                           const uint32_t *__restrict__ cnt,
                                                                           const uint32_t *__restrict__ chunk_cell,
                                                                           const uint32_t *__restrict__ cell_chunk,
                                                                           const uint2 *__restrict__ ranges,
                                                                           const uint32_t *__restrict__ svals,
                                                                           const float *__restrict__ dv,
                                                                           const float2 *__restrict__ ixy,
                                                                           float *__restrict__ part,
                                                                           float *__restrict__ dpacked) {
    const int F = lay.F, G = F / 4, S = 64 / G;
    const int lane = threadIdx.x & 63, q = lane % G, slot = lane / G;
    const uint32_t nchunks = __builtin_amdgcn_readfirstlane(*cnt);
    const uint32_t nwaves = gridDim.x * (kHexGatherThreads / 64);
    // XCD-contiguous waves (the grid is a multiple of 8): neighbouring chunks -- neighbouring cells, which
    // read the same anchors' dv -- run on one XCD and share its L2 (a speed-only assumption)
    const uint32_t per_xcd = gridDim.x / 8, b = (blockIdx.x % 8) * per_xcd + blockIdx.x / 8;
    const uint32_t wave = b * (kHexGatherThreads / 64) + (threadIdx.x >> 6);
    const uint32_t per_wave = (nchunks + nwaves - 1) / nwaves;
    const uint32_t ch0 = wave * per_wave, ch1 = min(nchunks, ch0 + per_wave);
    for (uint32_t ch = ch0; ch < ch1; ch++) {
        const uint32_t c = __builtin_amdgcn_readfirstlane(chunk_cell[ch]);
        const uint32_t j0 = (ch - __builtin_amdgcn_readfirstlane(cell_chunk[c])) * kHexChunk;
        const HexCell h = hex_cell(lay, c);
        uint32_t bs[4], bn[4];
        const uint32_t K = hex_buckets(h, ranges, bs, bn);
        const uint32_t j1 = min(K, j0 + kHexChunk);
        float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
        for (uint32_t t = j0 + slot; t < j1; t += S) {
            int k = 0;
            uint32_t jj = t;
            while (k < 3 && jj >= bn[k]) {
                jj -= bn[k];
                k++;
            }
            const uint32_t e = svals[bs[k] + jj];
            const float2 p = ixy[e];
            const int ax = h.cx - 1 + (k & 1), ay = h.cy - 1 + (k >> 1);
            // make_tap's weights: this cell is the anchor's (x1 | x0, y1 | y0) corner
            const float wx = (k & 1) ? (float)(ax + 1) - p.x : p.x - (float)ax;
            const float wy = (k >> 1) ? (float)(ay + 1) - p.y : p.y - (float)ay;
            const float w = wx * wy;
            const float4 d = *reinterpret_cast<const float4 *>(dv + (size_t)e * F + 4 * q);
            acc.x += w * d.x;
            acc.y += w * d.y;
            acc.z += w * d.z;
            acc.w += w * d.w;
        }
        for (int off = G; off < 64; off <<= 1) {
            acc.x += __shfl_xor(acc.x, off);
            acc.y += __shfl_xor(acc.y, off);
            acc.z += __shfl_xor(acc.z, off);
            acc.w += __shfl_xor(acc.w, off);
        }
        if (slot == 0) {
            float *dst = K <= kHexChunk ? dpacked + (size_t)c * F : part + (size_t)ch * F;
            *reinterpret_cast<float4 *>(dst + 4 * q) = acc;
        }
    }
}

// the cells of more than one chunk: their partials added in chunk order (lane = feature)
__global__ __launch_bounds__(256) void hex_combine_kernel(gs4d_hexplane_layout lay, const uint32_t *__restrict__ cnt,
                                                          const uint32_t *__restrict__ long_cells,
                                                          const uint32_t *__restrict__ cell_chunk,
                                                          const float *__restrict__ part, float *__restrict__ dpacked) {
    const int F = lay.F;
    const uint32_t nlong = __builtin_amdgcn_readfirstlane(cnt[1]);
    const uint32_t nwaves = gridDim.x * 4, wave = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    for (uint32_t i = wave; i < nlong; i += nwaves) {
        const uint32_t c = long_cells[i];
        const uint32_t ch0 = cell_chunk[c], ch1 = cell_chunk[c + 1];
        for (int f = lane; f < F; f += 64) {
            float acc = 0.f;
            for (uint32_t ch = ch0; ch < ch1; ch++) acc += part[(size_t)ch * F + f];
            dpacked[(size_t)c * F + f] = acc;
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

// backward scratch: zero region (err, digit histograms, look-back words, cell ranges) | dv (NE x F) |
// ixy (NE) | keys x 2 | vals x 2, NE = N x 6 levels entries
struct HexBwdScratch {
    uint32_t *zero, *err, *hist, *look, *plan_look, *cnt;
    uint2 *ranges;
    float *dv, *part;
    float2 *ixy;
    uint32_t *keys[2], *vals[2], *cell_chunk, *chunk_cell, *long_cells;
    size_t zero_bytes, total;
    int plan_blocks;
};
// chunks of the gather: each cell at most 1 + K / kHexChunk, K summing to 4 taps per entry
static size_t hex_max_chunks(size_t NE, size_t NC) { return NC + 4 * NE / kHexChunk + 1; }
static HexBwdScratch hex_bwd_scratch(int N, const gs4d_hexplane_layout &lay, char *base) {
    HexBwdScratch h;
    const size_t NE = (size_t)N * 6 * lay.levels, NC = (size_t)(lay.total / lay.F);
    const int nblk = sort_nblk((int)NE, kHexSortThreads * kHexSortItems);
    char *q = (char *)align_up((size_t)base, 256);
    char *q0 = q;
    auto take = [&](size_t bytes) {
        char *r = q;
        q += align_up(bytes, 256);
        return r;
    };
    h.plan_blocks = (int)((NC + kHexPlanThreads - 1) / kHexPlanThreads);
    h.zero = (uint32_t *)take(4 * (64 + (size_t)kHistWords + 256 * 3 * (size_t)nblk + (size_t)h.plan_blocks) + 8 * NC);
    h.err = h.zero + 8;
    h.cnt = h.zero + 16;  // [0] chunks, [1] long cells
    h.hist = h.zero + 64;
    h.look = h.hist + kHistWords;
    h.plan_look = h.look + 256 * 3 * (size_t)nblk;
    h.ranges = (uint2 *)(h.plan_look + h.plan_blocks);
    h.zero_bytes = (size_t)(q - q0);
    const size_t MC = hex_max_chunks(NE, NC);
    h.cell_chunk = (uint32_t *)take(4 * (NC + 1));
    h.chunk_cell = (uint32_t *)take(4 * MC);
    h.long_cells = (uint32_t *)take(4 * NC);
    h.part = (float *)take(4 * MC * lay.F);
    h.dv = (float *)take(4 * NE * lay.F);
    h.ixy = (float2 *)take(8 * NE);
    for (int k = 0; k < 2; k++) {
        h.keys[k] = (uint32_t *)take(4 * NE);
        h.vals[k] = (uint32_t *)take(4 * NE);
    }
    h.total = (size_t)(q - base) + 256;
    return h;
}

size_t gs4d_hexplane_backward_scratch_bytes(int N, const gs4d_hexplane_layout *lay) {
    if (N <= 0 || !lay) return 256;
    return hex_bwd_scratch(N, *lay, nullptr).total;
}

int gs4d_hexplane_backward(int N, const float *pts, const uint32_t *order, const gs4d_hexplane_layout *lay,
                           const float *packed, const float *dfeat, float *dpacked, float *dpts, void *scratch,
                           void *stream) {
    if (N < 0 || !lay || (N > 0 && (!pts || !packed || !dfeat || !dpacked || !dpts || !scratch))) return 1;
    if (((size_t)pts & 15) || ((size_t)packed & 15) || ((size_t)dfeat & 15) || ((size_t)dpts & 15) ||
        ((size_t)dpacked & 15))
        return 1;
    const int64_t NE = (int64_t)N * 6 * lay->levels, NC = lay->total / lay->F;
    if (NE >= ((int64_t)1 << 30) || NC >= ((int64_t)1 << kHexKeyBits)) return 1;
    hipStream_t s = (hipStream_t)stream;
    if (N == 0) {
        // no points: every plane gradient is zero
        return hipMemsetAsync(dpacked, 0, 4 * (size_t)lay->total, s) == hipSuccess ? 0 : 3;
    }
    HexBwdScratch h = hex_bwd_scratch(N, *lay, (char *)scratch);
    if (hipMemsetAsync(h.zero, 0, h.zero_bytes, s) != hipSuccess) return 3;
    const int64_t threads = (int64_t)N * (lay->F / 4);
    hipLaunchKernelGGL(hexplane_dv_kernel, dim3((unsigned)((threads + kHexThreads - 1) / kHexThreads)), dim3(kHexThreads),
                       0, s, N, pts, order, *lay, packed, dfeat, h.dv, h.ixy, h.keys[0], h.hist, dpts);
    const int cur = onesweep_sort<kHexSortThreads, kHexSortItems>(h.keys, h.vals, (int)NE, nullptr, kHexKeyBits,
                                                                  h.hist, h.look, h.err, s);
    hipLaunchKernelGGL(hex_cell_ranges_kernel, dim3((unsigned)((NE + 255) / 256)), dim3(256), 0, s, NE, (uint32_t)NC,
                       h.keys[cur], h.ranges);
    hipLaunchKernelGGL(hex_chunk_plan_kernel, dim3((unsigned)h.plan_blocks), dim3(kHexPlanThreads), 0, s, *lay,
                       (uint32_t)NC, h.ranges, h.cell_chunk, h.chunk_cell, h.long_cells, h.cnt, h.plan_look, h.err);
    // a fixed grid (a multiple of 8 for the XCD-contiguous order): ~4 waves per SIMD of the chip
    hipLaunchKernelGGL(hexplane_gather_kernel, dim3(1024), dim3(kHexGatherThreads), 0, s, *lay, h.cnt, h.chunk_cell,
                       h.cell_chunk, h.ranges, h.vals[cur], h.dv, h.ixy, h.part, dpacked);
    hipLaunchKernelGGL(hex_combine_kernel, dim3(256), dim3(256), 0, s, *lay, h.cnt, h.long_cells, h.cell_chunk, h.part,
                       dpacked);
    return hipGetLastError() == hipSuccess ? 0 : 3;
}

}  // extern "C"
