// binning.hip -- (tile, depth) key duplication (K3), stable LSD radix sort (K4) and tile ranges (K5).
//
// Reference: cuda_rasterizer/rasterizer_impl.cu:70-111 (duplicateWithKeys), :116-138
// (identifyTileRanges), :301-318 (cub::DeviceRadixSort::SortPairs on bits [0, 32+msb(T)), memset).
//
// The sort is this library's own wave64 LSD radix sort: 8-bit digits, reduce-then-scan per pass
// (digit histogram per workgroup -> one exclusive scan over [digit][workgroup] -> stable scatter
// ranked with 64-lane ballots).  It sorts (key, unsorted position) pairs, which is the same
// permutation CUB's stable sort produces for (key, Gaussian id) pairs; the Gaussian ids are
// gathered afterwards in the tile-range pass.
#include "gs4d_internal.h"

namespace gs4d {

// ---------------------------------------------------------------------------------------------
// K3: one workgroup per 256 Gaussians (the same partition as the preprocess block sums).  The
// workgroup re-derives its local exclusive scan of tiles_touched, then emits its instances with a
// load-balanced loop: output slot k of the workgroup finds its Gaussian by binary search over the
// local inclusive scan, so every lane writes one contiguous key per iteration regardless of how
// unevenly the tile counts are spread over Gaussians.
__global__ __launch_bounds__(kPreprocessBlock) void duplicate_kernel(Args a, GeomState g, const int *__restrict__ radii,
                                                                     BinningState b) {
    __shared__ uint32_t s_incl[kPreprocessBlock];
    __shared__ int4 s_rect[kPreprocessBlock];     // x0, y0, width, depth bits
    __shared__ uint32_t s_wave[kPreprocessBlock / 64];
    const int tid = threadIdx.x;
    const int idx = blockIdx.x * kPreprocessBlock + tid;
    uint32_t t = 0;
    int4 rect = make_int4(0, 0, 1, 0);
    if (idx < a.P) {
        t = g.tiles_touched[idx];
        if (t > 0) {
            int x0, y0, x1, y1;
            float2 p = g.xy[idx];
            getRect(p.x, p.y, radii[idx], a.gx, a.gy, x0, y0, x1, y1);
            rect = make_int4(x0, y0, x1 - x0, __float_as_int(g.depths[idx]));
        }
    }
    // workgroup inclusive scan of t
    const int lane = tid & 63, w = tid >> 6;
    uint32_t x = t;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        uint32_t y = __shfl_up(x, off);
        if (lane >= off) x += y;
    }
    if (lane == 63) s_wave[w] = x;
    __syncthreads();
    uint32_t wbase = 0;
    for (int i = 0; i < w; i++) wbase += s_wave[i];
    x += wbase;
    s_incl[tid] = x;
    s_rect[tid] = rect;
    const uint32_t block_off = g.block_sums[blockIdx.x];
    if (idx < a.P) g.point_offsets[idx] = block_off + x - t;
    __syncthreads();
    const uint32_t total = s_incl[kPreprocessBlock - 1];
    for (uint32_t k = tid; k < total; k += kPreprocessBlock) {
        // first i with s_incl[i] > k
        int lo = 0, hi = kPreprocessBlock - 1;
        while (lo < hi) {
            int mid = (lo + hi) >> 1;
            if (s_incl[mid] > k) hi = mid; else lo = mid + 1;
        }
        const uint32_t start = lo ? s_incl[lo - 1] : 0;
        const uint32_t local = k - start;
        const int4 r = s_rect[lo];
        const uint32_t ty = r.y + local / (uint32_t)r.z;
        const uint32_t tx = r.x + local % (uint32_t)r.z;
        const uint64_t key = ((uint64_t)(ty * a.gx + tx) << 32) | (uint32_t)r.w;
        const uint32_t upos = block_off + k;
        b.keys[0][upos] = key;
        b.vals[0][upos] = upos;
        b.gid_by_upos[upos] = blockIdx.x * kPreprocessBlock + lo;
    }
}

hipError_t launch_duplicate(const Args &a, GeomState g, const int *radii, BinningState b, hipStream_t s) {
    const int nblk = (a.P + kPreprocessBlock - 1) / kPreprocessBlock;
    hipLaunchKernelGGL(duplicate_kernel, dim3(nblk), dim3(kPreprocessBlock), 0, s, a, g, radii, b);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// K4: LSD radix sort, 8 bits per pass.
constexpr int kSortThreads = 256;
constexpr int kSortRounds = kSortBlockItems / kSortThreads;  // 16

__global__ __launch_bounds__(kSortThreads) void radix_hist_kernel(const uint64_t *__restrict__ keys, int n, int shift,
                                                                  uint32_t *__restrict__ hist, int nblk) {
    __shared__ uint32_t s_h[256];
    const int tid = threadIdx.x;
    s_h[tid] = 0;
    __syncthreads();
    const size_t base = (size_t)blockIdx.x * kSortBlockItems;
#pragma unroll 4
    for (int r = 0; r < kSortRounds; r++) {
        size_t i = base + r * kSortThreads + tid;
        if (i < (size_t)n) atomicAdd(&s_h[(uint32_t)(keys[i] >> shift) & 0xFFu], 1u);
    }
    __syncthreads();
    hist[(size_t)tid * nblk + blockIdx.x] = s_h[tid];
}

// exclusive scan over hist[0 .. n) in place (digit-major so the result is each (digit, block)'s
// global output offset); one workgroup of 1024 threads.
__global__ __launch_bounds__(1024) void radix_scan_kernel(uint32_t *__restrict__ h, int n) {
    __shared__ uint32_t s_tot[1024 / 64];
    const int tid = threadIdx.x;
    const int chunk = (n + 1023) / 1024;
    const int b = tid * chunk, e = min(n, b + chunk);
    uint32_t local = 0;
    for (int i = b; i < e; i++) local += h[i];
    const int lane = tid & 63;
    uint32_t x = local;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        uint32_t y = __shfl_up(x, off);
        if (lane >= off) x += y;
    }
    if (lane == 63) s_tot[tid >> 6] = x;
    __syncthreads();
    uint32_t run = x - local;
    for (int w = 0; w < (tid >> 6); w++) run += s_tot[w];
    for (int i = b; i < e; i++) {
        uint32_t v = h[i];
        h[i] = run;
        run += v;
    }
}

__global__ __launch_bounds__(kSortThreads) void radix_scatter_kernel(const uint64_t *__restrict__ kin,
                                                                     const uint32_t *__restrict__ vin,
                                                                     uint64_t *__restrict__ kout,
                                                                     uint32_t *__restrict__ vout, int n, int shift,
                                                                     const uint32_t *__restrict__ hist, int nblk) {
    __shared__ uint32_t s_base[256];
    __shared__ uint32_t s_w[kSortThreads / 64][256];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    s_base[tid] = hist[(size_t)tid * nblk + blockIdx.x];
    const uint64_t lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    const size_t base = (size_t)blockIdx.x * kSortBlockItems;
    for (int r = 0; r < kSortRounds; r++) {
        const size_t i = base + r * kSortThreads + tid;
        const bool valid = i < (size_t)n;
        uint64_t key = 0;
        uint32_t val = 0;
        uint32_t d = 0;
        if (valid) {
            key = kin[i];
            val = vin[i];
            d = (uint32_t)(key >> shift) & 0xFFu;
        }
        // lanes of this wave with the same digit
        uint64_t peers = __ballot(valid);
#pragma unroll
        for (int bit = 0; bit < 8; bit++) {
            const bool set = (d >> bit) & 1u;
            const uint64_t m = __ballot(set);
            peers &= set ? m : ~m;
        }
        const uint32_t rank = __popcll(peers & lt_mask);
#pragma unroll
        for (int q = 0; q < kSortThreads / 64; q++) s_w[q][tid] = 0;
        __syncthreads();
        if (valid && rank == 0) s_w[w][d] = __popcll(peers);
        __syncthreads();
        {
            // per digit (thread tid): exclusive prefix over waves, advance the running base
            uint32_t run = s_base[tid];
#pragma unroll
            for (int q = 0; q < kSortThreads / 64; q++) {
                uint32_t c = s_w[q][tid];
                s_w[q][tid] = run;
                run += c;
            }
            s_base[tid] = run;
        }
        __syncthreads();
        if (valid) {
            const uint32_t pos = s_w[w][d] + rank;
            kout[pos] = key;
            vout[pos] = val;
        }
        __syncthreads();
    }
}

hipError_t launch_radix_sort(BinningState b, int L, int nbits, int *result_buf, hipStream_t s) {
    const int nblk = (L + kSortBlockItems - 1) / kSortBlockItems;
    int cur = 0;
    for (int shift = 0; shift < nbits; shift += 8) {
        hipLaunchKernelGGL(radix_hist_kernel, dim3(nblk), dim3(kSortThreads), 0, s, b.keys[cur], L, shift, b.hist, nblk);
        hipLaunchKernelGGL(radix_scan_kernel, dim3(1), dim3(1024), 0, s, b.hist, 256 * nblk);
        hipLaunchKernelGGL(radix_scatter_kernel, dim3(nblk), dim3(kSortThreads), 0, s, b.keys[cur], b.vals[cur],
                           b.keys[cur ^ 1], b.vals[cur ^ 1], L, shift, b.hist, nblk);
        cur ^= 1;
    }
    *result_buf = cur;
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// K5: tile ranges + gather of the Gaussian id of each sorted instance (render order).
__global__ void tile_ranges_kernel(const uint64_t *__restrict__ keys, const uint32_t *__restrict__ upos, int L,
                                   const uint32_t *__restrict__ gid_by_upos, uint32_t *__restrict__ point_list,
                                   uint2 *__restrict__ ranges) {
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= L) return;
    const uint32_t cur = (uint32_t)(keys[idx] >> 32);
    if (idx == 0) {
        ranges[cur].x = 0;
    } else {
        const uint32_t prev = (uint32_t)(keys[idx - 1] >> 32);
        if (cur != prev) {
            ranges[prev].y = idx;
            ranges[cur].x = idx;
        }
    }
    if (idx == L - 1) ranges[cur].y = L;
    point_list[idx] = gid_by_upos[upos[idx]];
}

hipError_t launch_tile_ranges(BinningState b, int L, int buf, ImageState img, int T, hipStream_t s) {
    hipError_t e = hipMemsetAsync(img.ranges, 0, sizeof(uint2) * (size_t)T, s);
    if (e != hipSuccess) return e;
    if (L > 0)
        hipLaunchKernelGGL(tile_ranges_kernel, dim3((L + 255) / 256), dim3(256), 0, s, b.keys[buf], b.vals[buf], L,
                           b.gid_by_upos, b.point_list, img.ranges);
    return hipGetLastError();
}

}  // namespace gs4d
