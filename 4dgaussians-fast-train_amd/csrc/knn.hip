// knn.hip -- initial-scale kNN: mean squared distance from every point to its 3 nearest other points.
//
// Replaces simple_knn._C.distCUDA2 (submodules/simple-knn/spatial.cu:15-25, simple_knn.cu:187-223),
// which scene/gaussian_model.py:148-149 calls once per scene to initialise the Gaussian scales.
// The reference's algorithm, kept here because its result is defined by it:
//   1. bounding box of the points, reduced WITH the origin as the initial value (cub Reduce with
//      init {0,0,0}, simple_knn.cu:193-202): minn <= 0 <= maxx on every axis;
//   2. 30-bit Morton code of each point on a 1023^3 grid over that box (:47-63);
//   3. stable radix sort of (code, index) (:212-215);
//   4. boxes of 1024 consecutive sorted points with their min/max corners (:80-119);
//   5. per point: the 3 best squared distances among its +-3 sorted neighbours give a rejection
//      radius; then every box closer than both that radius and the current 3rd best is scanned
//      (:149-185).  The box tests only prune, so the result is the exact 3-nearest-neighbour mean
//      (self excluded by index; duplicates count at distance 0; fewer than 3 others -> FLT_MAX terms).
// MI355X mapping: one pass per stage over coalesced SoA/float4 arrays; the bounds are reduced by
// wave shuffles and one order-preserving integer atomic per workgroup; the Morton pass builds the
// sort's sharded digit histograms (no separate histogram pass); the sort is the library's onesweep
// LSD sort (radix_sort.h); the box pass also lays the points out in sorted order (float4) so the
// distance pass reads them contiguously; the distance pass keeps all box corners of its workgroup's
// slice in LDS and prunes inside a passing box by sub-boxes of 32 points (the same test one level
// finer: it skips only points that cannot enter the 3 best, so the result is unchanged).  Distances are evaluated as (dx*dx + dy*dy) + dz*dz without contraction (compiled
// with -ffp-contract=off), identically in the oracle.
#include <algorithm>
#include <cfloat>

#include "radix_sort.h"

namespace gs4d {

constexpr int kKnnBox = 1024;       // points per box (BOX_SIZE, simple_knn.cu:12)
constexpr int kKnnThreads = 256;
constexpr int kKnnSortThreads = 1024;  // Morton-sort workgroup
constexpr int kKnnSortItems = 4;       // keys per lane of the Morton sort (4096 per workgroup)
constexpr int kKnnLdsBoxes = 2048;  // box corners staged in LDS per slice (64 KiB)
constexpr int kKnnSub = 32;         // points per sub-box: the distance pass prunes inside a passing box by these

// order-preserving float <-> u32 map for integer atomic min/max
__device__ __forceinline__ uint32_t f2ord(float f) {
    const uint32_t u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float ord2f(uint32_t u) {
    return __uint_as_float((u & 0x80000000u) ? (u & 0x7FFFFFFFu) : ~u);
}

// bounds[0..2] = ord(min), bounds[3..5] = ord(max); pre-set to ord(0.0f) = 0x80000000 (the origin
// is the reduction's initial value).  NaN coordinates are ignored, as CUDA's min/max do.
__global__ __launch_bounds__(kKnnThreads) void knn_bounds_kernel(int P, const float *__restrict__ pts,
                                                                 uint32_t *__restrict__ bounds) {
    float mn[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, mx[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
    for (int i = blockIdx.x * kKnnThreads + threadIdx.x; i < P; i += gridDim.x * kKnnThreads) {
#pragma unroll
        for (int c = 0; c < 3; c++) {
            const float v = pts[3 * (size_t)i + c];
            mn[c] = fminf(mn[c], v);
            mx[c] = fmaxf(mx[c], v);
        }
    }
    __shared__ float s[6][kKnnThreads / 64];
#pragma unroll
    for (int c = 0; c < 3; c++) {
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            mn[c] = fminf(mn[c], __shfl_xor(mn[c], off));
            mx[c] = fmaxf(mx[c], __shfl_xor(mx[c], off));
        }
    }
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
#pragma unroll
        for (int c = 0; c < 3; c++) {
            s[c][w] = mn[c];
            s[3 + c][w] = mx[c];
        }
    }
    __syncthreads();
    if (threadIdx.x < 6) {
        const int c = threadIdx.x;
        float v = s[c][0];
        for (int q = 1; q < kKnnThreads / 64; q++) v = c < 3 ? fminf(v, s[c][q]) : fmaxf(v, s[c][q]);
        if (c < 3) atomicMin(&bounds[c], f2ord(v));
        else atomicMax(&bounds[c], f2ord(v));
    }
}

// simple_knn.cu:47-54
__device__ __forceinline__ uint32_t prep_morton(uint32_t x) {
    x = (x | (x << 16)) & 0x030000FF;
    x = (x | (x << 8)) & 0x0300F00F;
    x = (x | (x << 4)) & 0x030C30C3;
    x = (x | (x << 2)) & 0x09249249;
    return x;
}
// simple_knn.cu:56-63; the float -> u32 conversion truncates, and a degenerate axis (0/0 = NaN)
// converts to 0 as the CUDA conversion does
__device__ __forceinline__ uint32_t grid_coord(float c, float mn, float mx) {
    const float v = ((c - mn) / (mx - mn)) * (float)((1 << 10) - 1);
    return v >= 0.f ? (uint32_t)v : 0u;
}

__global__ __launch_bounds__(kKnnThreads) void knn_morton_kernel(int P, const float *__restrict__ pts,
                                                                 const uint32_t *__restrict__ bounds,
                                                                 uint32_t *__restrict__ codes,
                                                                 uint32_t *__restrict__ hist) {
    __shared__ uint32_t s_hist[4][256];
    for (int p = 0; p < 4; p++) s_hist[p][threadIdx.x] = 0;
    __syncthreads();
    const int i = blockIdx.x * kKnnThreads + threadIdx.x;
    if (i < P) {
        float mn[3], mx[3];
#pragma unroll
        for (int c = 0; c < 3; c++) {
            mn[c] = ord2f(bounds[c]);
            mx[c] = ord2f(bounds[3 + c]);
        }
        const uint32_t x = prep_morton(grid_coord(pts[3 * (size_t)i], mn[0], mx[0]));
        const uint32_t y = prep_morton(grid_coord(pts[3 * (size_t)i + 1], mn[1], mx[1]));
        const uint32_t z = prep_morton(grid_coord(pts[3 * (size_t)i + 2], mn[2], mx[2]));
        const uint32_t code = x | (y << 1) | (z << 2);
        codes[i] = code;
#pragma unroll
        for (int p = 0; p < 4; p++) atomicAdd(&s_hist[p][(code >> (8 * p)) & 0xFFu], 1u);
    }
    __syncthreads();
    uint32_t *h = hist + (blockIdx.x % kHistShards) * (kMaxPasses * 256);
#pragma unroll
    for (int p = 0; p < 4; p++)
        if (s_hist[p][threadIdx.x]) atomicAdd(&h[p * 256 + threadIdx.x], s_hist[p][threadIdx.x]);
}

struct KnnBox {
    float4 mn, mx;
};

// simple_knn.cu:80-119, plus the points laid out in sorted order
__global__ __launch_bounds__(kKnnThreads) void knn_boxes_kernel(int P, const float *__restrict__ pts,
                                                                const uint32_t *__restrict__ order,
                                                                float4 *__restrict__ sorted, KnnBox *__restrict__ boxes) {
    float mn[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, mx[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
    const int base = blockIdx.x * kKnnBox;
#pragma unroll
    for (int k = 0; k < kKnnBox / kKnnThreads; k++) {
        const int i = base + k * kKnnThreads + threadIdx.x;
        if (i < P) {
            const uint32_t id = order[i];
            const float4 p = make_float4(pts[3 * (size_t)id], pts[3 * (size_t)id + 1], pts[3 * (size_t)id + 2], 0.f);
            sorted[i] = p;
            mn[0] = fminf(mn[0], p.x); mn[1] = fminf(mn[1], p.y); mn[2] = fminf(mn[2], p.z);
            mx[0] = fmaxf(mx[0], p.x); mx[1] = fmaxf(mx[1], p.y); mx[2] = fmaxf(mx[2], p.z);
        }
    }
#pragma unroll
    for (int c = 0; c < 3; c++) {
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            mn[c] = fminf(mn[c], __shfl_xor(mn[c], off));
            mx[c] = fmaxf(mx[c], __shfl_xor(mx[c], off));
        }
    }
    __shared__ float s[6][kKnnThreads / 64];
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
#pragma unroll
        for (int c = 0; c < 3; c++) {
            s[c][w] = mn[c];
            s[3 + c][w] = mx[c];
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        KnnBox b;
        float r[6];
#pragma unroll
        for (int c = 0; c < 6; c++) {
            float v = s[c][0];
            for (int q = 1; q < kKnnThreads / 64; q++) v = c < 3 ? fminf(v, s[c][q]) : fmaxf(v, s[c][q]);
            r[c] = v;
        }
        b.mn = make_float4(r[0], r[1], r[2], 0.f);
        b.mx = make_float4(r[3], r[4], r[5], 0.f);
        boxes[blockIdx.x] = b;
    }
}

__device__ __forceinline__ float sqdist(const float4 &a, const float4 &b) {
    const float dx = b.x - a.x, dy = b.y - a.y, dz = b.z - a.z;
    return dx * dx + dy * dy + dz * dz;
}
// simple_knn.cu:121-131
__device__ __forceinline__ float box_dist(const float4 &mn, const float4 &mx, const float4 &p) {
    float dx = 0.f, dy = 0.f, dz = 0.f;
    if (p.x < mn.x || p.x > mx.x) dx = fminf(fabsf(p.x - mn.x), fabsf(p.x - mx.x));
    if (p.y < mn.y || p.y > mx.y) dy = fminf(fabsf(p.y - mn.y), fabsf(p.y - mx.y));
    if (p.z < mn.z || p.z > mx.z) dz = fminf(fabsf(p.z - mn.z), fabsf(p.z - mx.z));
    return dx * dx + dy * dy + dz * dz;
}
// simple_knn.cu:133-147: insertion into the ascending 3-best list
__device__ __forceinline__ void update3(float best[3], float d) {
#pragma unroll
    for (int j = 0; j < 3; j++) {
        if (best[j] > d) {
            const float t = best[j];
            best[j] = d;
            d = t;
        }
    }
}

// Corners of every run of kKnnSub consecutive sorted points (a second, finer level of the reference's
// boxes: a box that passes the distance test is scanned sub-box by sub-box, each with the same test).
__global__ __launch_bounds__(kKnnThreads) void knn_subboxes_kernel(int P, const float4 *__restrict__ sorted,
                                                                   KnnBox *__restrict__ sub) {
    const int i = blockIdx.x * kKnnThreads + threadIdx.x;
    const bool valid = i < P;
    const float4 p = valid ? sorted[i] : make_float4(0.f, 0.f, 0.f, 0.f);
    float mn[3] = {valid ? p.x : FLT_MAX, valid ? p.y : FLT_MAX, valid ? p.z : FLT_MAX};
    float mx[3] = {valid ? p.x : -FLT_MAX, valid ? p.y : -FLT_MAX, valid ? p.z : -FLT_MAX};
#pragma unroll
    for (int c = 0; c < 3; c++) {
#pragma unroll
        for (int off = kKnnSub / 2; off > 0; off >>= 1) {  // inside 32-lane groups
            mn[c] = fminf(mn[c], __shfl_xor(mn[c], off));
            mx[c] = fmaxf(mx[c], __shfl_xor(mx[c], off));
        }
    }
    if (valid && (i % kKnnSub) == 0) {
        KnnBox b;
        b.mn = make_float4(mn[0], mn[1], mn[2], 0.f);
        b.mx = make_float4(mx[0], mx[1], mx[2], 0.f);
        sub[i / kKnnSub] = b;
    }
}

__global__ __launch_bounds__(kKnnThreads) void knn_dist_kernel(int P, const float4 *__restrict__ sorted,
                                                               const uint32_t *__restrict__ order,
                                                               const KnnBox *__restrict__ boxes, int nbox,
                                                               const KnnBox *__restrict__ sub,
                                                               float *__restrict__ mean_dists) {
    __shared__ KnnBox s_box[kKnnLdsBoxes];
    const int idx = blockIdx.x * kKnnThreads + threadIdx.x;
    const bool live = idx < P;
    const float4 p = live ? sorted[idx] : make_float4(0.f, 0.f, 0.f, 0.f);
    float best[3] = {FLT_MAX, FLT_MAX, FLT_MAX};
    if (live) {
        for (int i = max(0, idx - 3); i <= min(P - 1, idx + 3); i++)
            if (i != idx) update3(best, sqdist(p, sorted[i]));
    }
    const float reject = best[2];
    best[0] = best[1] = best[2] = FLT_MAX;
    for (int b0 = 0; b0 < nbox; b0 += kKnnLdsBoxes) {
        const int nb = min(kKnnLdsBoxes, nbox - b0);
        __syncthreads();
        for (int k = threadIdx.x; k < nb; k += kKnnThreads) s_box[k] = boxes[b0 + k];
        __syncthreads();
        if (!live) continue;
        for (int k = 0; k < nb; k++) {
            const float d = box_dist(s_box[k].mn, s_box[k].mx, p);
            if (d > reject || d > best[2]) continue;
            // the box's points, sub-box by sub-box (simple_knn.cu:177-184 scans all 1024; the finer test
            // only skips points that cannot enter the 3 best)
            const int lo = (b0 + k) * kKnnBox, hi = min(P, lo + kKnnBox);
            for (int s0 = lo; s0 < hi; s0 += kKnnSub) {
                const KnnBox sb = sub[s0 / kKnnSub];
                const float ds = box_dist(sb.mn, sb.mx, p);
                if (ds > reject || ds > best[2]) continue;
                const int s1 = min(hi, s0 + kKnnSub);
                for (int i = s0; i < s1; i++)
                    if (i != idx) update3(best, sqdist(p, sorted[i]));
            }
        }
    }
    if (live) mean_dists[order[idx]] = (best[0] + best[1] + best[2]) / 3.0f;
}

size_t knn_scratch_bytes(int P) {
    const size_t nblk = (size_t)sort_nblk(P, kKnnSortThreads * kKnnSortItems);
    const size_t nbox = ((size_t)P + kKnnBox - 1) / kKnnBox;
    size_t b = 0;
    b += align_up(4 * (64 + (size_t)kHistWords + 4 * 256 * nblk), 256);  // bounds | hist | look-back
    b += 4 * align_up(4 * (size_t)P, 256);                               // codes x2, order x2
    b += align_up(16 * (size_t)P, 256);                                  // sorted points
    b += align_up(sizeof(KnnBox) * nbox, 256);
    b += align_up(sizeof(KnnBox) * (((size_t)P + kKnnSub - 1) / kKnnSub), 256);
    return b + 256;
}

hipError_t launch_knn(int P, const float *pts, float *mean_dists, char *scratch, hipStream_t s) {
    const int nblk = sort_nblk(P, kKnnSortThreads * kKnnSortItems);
    const int nbox = (P + kKnnBox - 1) / kKnnBox;
    char *q = (char *)align_up((size_t)scratch, 256);
    auto take = [&](size_t bytes) {
        char *r = q;
        q += align_up(bytes, 256);
        return r;
    };
    const size_t zero_words = 64 + (size_t)kHistWords + 4 * 256 * (size_t)nblk;
    uint32_t *zero = (uint32_t *)take(4 * zero_words);
    uint32_t *codes[2] = {(uint32_t *)take(4 * (size_t)P), (uint32_t *)take(4 * (size_t)P)};
    uint32_t *order[2] = {(uint32_t *)take(4 * (size_t)P), (uint32_t *)take(4 * (size_t)P)};
    float4 *sorted = (float4 *)take(16 * (size_t)P);
    KnnBox *boxes = (KnnBox *)take(sizeof(KnnBox) * nbox);
    KnnBox *sub = (KnnBox *)take(sizeof(KnnBox) * (((size_t)P + kKnnSub - 1) / kKnnSub));
    uint32_t *bounds = zero, *err = zero + 8, *hist = zero + 64, *look = zero + 64 + kHistWords;

    hipError_t e = hipMemsetAsync(zero, 0, 4 * zero_words, s);
    if (e != hipSuccess) return e;
    e = hipMemsetD32Async((hipDeviceptr_t)bounds, 0x80000000u, 6, s);  // ord(0.0f): the origin
    if (e != hipSuccess) return e;
    const int gb = std::min(1024, (P + kKnnThreads - 1) / kKnnThreads);
    hipLaunchKernelGGL(knn_bounds_kernel, dim3(gb), dim3(kKnnThreads), 0, s, P, pts, bounds);
    hipLaunchKernelGGL(knn_morton_kernel, dim3((P + kKnnThreads - 1) / kKnnThreads), dim3(kKnnThreads), 0, s, P, pts,
                       bounds, codes[0], hist);
    const int cur = onesweep_sort<kKnnSortThreads, kKnnSortItems>(codes, order, P, nullptr, 30, hist, look, err, s);
    hipLaunchKernelGGL(knn_boxes_kernel, dim3(nbox), dim3(kKnnThreads), 0, s, P, pts, order[cur], sorted, boxes);
    hipLaunchKernelGGL(knn_subboxes_kernel, dim3((P + kKnnThreads - 1) / kKnnThreads), dim3(kKnnThreads), 0, s, P,
                       sorted, sub);
    hipLaunchKernelGGL(knn_dist_kernel, dim3((P + kKnnThreads - 1) / kKnnThreads), dim3(kKnnThreads), 0, s, P, sorted,
                       order[cur], boxes, nbox, sub, mean_dists);
    return hipGetLastError();
}

}  // namespace gs4d
