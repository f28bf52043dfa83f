// binning.hip -- depth ordering, (tile, depth) instance keys (K3), radix sort (K4) and tile ranges (K5).
//
// Reference: cuda_rasterizer/rasterizer_impl.cu:70-111 (duplicateWithKeys), :116-138
// (identifyTileRanges), :301-318 (cub::DeviceRadixSort::SortPairs of (tile<<32 | depth_bits, id)
// on bits [0, 32+msb(T)), stable).
//
// MI355X design (this library's own): the reference sorts L ~ 1.4M 64-bit keys with 32-bit values
// over 45 bits.  Here the P Gaussians are first sorted by depth bits (a P-sized, 32-bit stable radix
// sort, ties by id), which gives every Gaussian a depth RANK; each instance then carries the key
// (tile << R) | rank with R = bits(P-1).  That key is <= 32 bits at every BASELINE config, so the L
// instances are sorted keys-only as u32 in ceil((R+msb(T))/8) passes (4 instead of 6 at the metric
// config) and 4 bytes instead of 12 move per instance per pass.  The resulting order -- by tile, then
// depth bits, then Gaussian id -- is exactly the reference's stable (tile, depth) order.  When the
// key would exceed 32 bits (very large P x T) the same code runs on u64 keys.
//
// Each radix pass is reduce-then-scan, with no inter-workgroup hand-off: a per-workgroup digit
// histogram, a two-kernel exclusive scan over [digit][workgroup], and a stable scatter.  In the
// scatter each wave ranks its own contiguous chunk of keys round by round (64-lane ballot matching +
// per-wave digit counters in LDS, which a wave reads and bumps in program order), so a workgroup
// needs only two barriers regardless of how many keys it owns.
#include "gs4d_internal.h"

namespace gs4d {

constexpr int kSortThreads = 256;
constexpr int kScanItems = 4096;  // per scan workgroup (256 threads x 16)
constexpr int kItemsL = 16;       // keys per lane for the instance sort (4096 per workgroup)
constexpr int kItemsP = 4;        // keys per lane for the Gaussian depth sort (1024 per workgroup)

// ---------------------------------------------------------------------------------------------
// device-wide exclusive scan of u32 (two launches: per-workgroup totals, then scan + offset)
__global__ __launch_bounds__(256) void scan_reduce_kernel(const uint32_t *__restrict__ data, int n,
                                                          uint32_t *__restrict__ partials) {
    __shared__ uint32_t s_w[4];
    const int tid = threadIdx.x;
    const size_t base = (size_t)blockIdx.x * kScanItems;
    uint32_t v = 0;
#pragma unroll
    for (int r = 0; r < kScanItems / 256; r++) {
        size_t i = base + r * 256 + tid;
        if (i < (size_t)n) v += data[i];
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    if ((tid & 63) == 0) s_w[tid >> 6] = v;
    __syncthreads();
    if (tid == 0) partials[blockIdx.x] = s_w[0] + s_w[1] + s_w[2] + s_w[3];
}

__global__ __launch_bounds__(256) void scan_apply_kernel(uint32_t *__restrict__ data, int n,
                                                         const uint32_t *__restrict__ partials) {
    __shared__ uint32_t s_w[4];
    __shared__ uint32_t s_base;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    uint32_t pb = 0;
    for (int i = tid; i < (int)blockIdx.x; i += 256) pb += partials[i];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) pb += __shfl_xor(pb, off);
    if (lane == 0) s_w[w] = pb;
    __syncthreads();
    if (tid == 0) s_base = s_w[0] + s_w[1] + s_w[2] + s_w[3];
    __syncthreads();
    const size_t base = (size_t)blockIdx.x * kScanItems + (size_t)tid * 16;
    uint32_t v[16];
    uint32_t sum = 0;
#pragma unroll
    for (int i = 0; i < 16; i++) {
        v[i] = (base + i < (size_t)n) ? data[base + i] : 0u;
        sum += v[i];
    }
    uint32_t x = sum;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        uint32_t y = __shfl_up(x, off);
        if (lane >= off) x += y;
    }
    __syncthreads();
    if (lane == 63) s_w[w] = x;
    __syncthreads();
    uint32_t run = s_base + x - sum;
    for (int q = 0; q < w; q++) run += s_w[q];
#pragma unroll
    for (int i = 0; i < 16; i++) {
        if (base + i < (size_t)n) data[base + i] = run;
        run += v[i];
    }
}

static void exclusive_scan(uint32_t *data, int n, uint32_t *partials, hipStream_t s) {
    const int nb = (n + kScanItems - 1) / kScanItems;
    hipLaunchKernelGGL(scan_reduce_kernel, dim3(nb), dim3(256), 0, s, data, n, partials);
    hipLaunchKernelGGL(scan_apply_kernel, dim3(nb), dim3(256), 0, s, data, n, partials);
}

// scratch for a sort of n keys, sized for the smallest workgroup chunk in use
size_t radix_scratch_words(int n) {
    const int nblk = (n + kSortThreads * kItemsP - 1) / (kSortThreads * kItemsP);
    const size_t m = 256 * (size_t)nblk;
    return m + (m + kScanItems - 1) / kScanItems + 64;
}

// ---------------------------------------------------------------------------------------------
// LSD radix sort, 8 bits per pass.  Workgroup b owns keys [b*256*ITEMS, (b+1)*256*ITEMS); wave w of
// it owns the contiguous sub-chunk [w*64*ITEMS, (w+1)*64*ITEMS), read 64 keys per round.
template <typename K, int ITEMS>
__global__ __launch_bounds__(kSortThreads) void radix_hist_kernel(const K *__restrict__ keys, int n, int shift,
                                                                  uint32_t *__restrict__ hist, int nblk) {
    __shared__ uint32_t s_h[256];
    const int tid = threadIdx.x;
    s_h[tid] = 0;
    __syncthreads();
    const size_t base = (size_t)blockIdx.x * (kSortThreads * ITEMS);
#pragma unroll
    for (int r = 0; r < ITEMS; r++) {
        size_t i = base + r * kSortThreads + tid;
        if (i < (size_t)n) atomicAdd(&s_h[(uint32_t)(keys[i] >> shift) & 0xFFu], 1u);
    }
    __syncthreads();
    hist[(size_t)tid * nblk + blockIdx.x] = s_h[tid];
}

// VALS: carry 32-bit values (vin == nullptr -> identity values).  rank_out != nullptr:
// additionally write rank_out[value] = sorted position (used by the last depth-sort pass).
template <typename K, int ITEMS, bool VALS>
__global__ __launch_bounds__(kSortThreads) void radix_scatter_kernel(const K *__restrict__ kin,
                                                                     const uint32_t *__restrict__ vin,
                                                                     K *__restrict__ kout, uint32_t *__restrict__ vout,
                                                                     int n, int shift,
                                                                     const uint32_t *__restrict__ hist, int nblk,
                                                                     uint32_t *__restrict__ rank_out) {
    __shared__ uint32_t s_cnt[kSortThreads / 64][256];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
#pragma unroll
    for (int q = 0; q < kSortThreads / 64; q++) s_cnt[q][tid] = 0;
    __syncthreads();
    const uint64_t lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    const size_t wbase = (size_t)blockIdx.x * (kSortThreads * ITEMS) + (size_t)w * (64 * ITEMS);
    K key[ITEMS];
    uint32_t val[ITEMS], lrank[ITEMS];
#pragma unroll
    for (int r = 0; r < ITEMS; r++) {
        const size_t i = wbase + (size_t)r * 64 + lane;
        const bool valid = i < (size_t)n;
        key[r] = valid ? kin[i] : (K)0;
        if (VALS) val[r] = valid ? (vin ? vin[i] : (uint32_t)i) : 0u;
        const uint32_t d = (uint32_t)(key[r] >> shift) & 0xFFu;
        uint64_t peers = __ballot(valid);
#pragma unroll
        for (int bit = 0; bit < 8; bit++) {
            const bool set = (d >> bit) & 1u;
            const uint64_t m = __ballot(set);
            peers &= set ? m : ~m;
        }
        const uint32_t below = __popcll(peers & lt_mask);
        // every lane reads its digit's running count, then the group leader bumps it; the wave's LDS
        // accesses execute in program order, so all lanes see the value before the bump
        const uint32_t old = valid ? s_cnt[w][d] : 0u;
        if (valid && below == 0) s_cnt[w][d] = old + (uint32_t)__popcll(peers);
        lrank[r] = old + below;
    }
    __syncthreads();
    {
        uint32_t run = hist[(size_t)tid * nblk + blockIdx.x];
#pragma unroll
        for (int q = 0; q < kSortThreads / 64; q++) {
            const uint32_t c = s_cnt[q][tid];
            s_cnt[q][tid] = run;
            run += c;
        }
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < ITEMS; r++) {
        const size_t i = wbase + (size_t)r * 64 + lane;
        if (i < (size_t)n) {
            const uint32_t d = (uint32_t)(key[r] >> shift) & 0xFFu;
            const uint32_t pos = s_cnt[w][d] + lrank[r];
            kout[pos] = key[r];
            if (VALS) {
                vout[pos] = val[r];
                if (rank_out) rank_out[val[r]] = pos;
            }
        }
    }
}

// Keys-only sort of keys[0] on bits [0, nbits); returns the index of the buffer holding the result.
template <typename K, int ITEMS>
static int radix_sort_keys(K *keys[2], int n, int nbits, uint32_t *scratch, hipStream_t s) {
    const int chunk = kSortThreads * ITEMS;
    const int nblk = (n + chunk - 1) / chunk;
    uint32_t *hist = scratch;
    uint32_t *partials = scratch + 256 * (size_t)nblk;
    int cur = 0;
    for (int shift = 0; shift < nbits; shift += 8) {
        hipLaunchKernelGGL((radix_hist_kernel<K, ITEMS>), dim3(nblk), dim3(kSortThreads), 0, s, keys[cur], n, shift,
                           hist, nblk);
        exclusive_scan(hist, 256 * nblk, partials, s);
        hipLaunchKernelGGL((radix_scatter_kernel<K, ITEMS, false>), dim3(nblk), dim3(kSortThreads), 0, s, keys[cur],
                           nullptr, keys[cur ^ 1], nullptr, n, shift, hist, nblk, nullptr);
        cur ^= 1;
    }
    return cur;
}

// ---------------------------------------------------------------------------------------------
// Depth order of the Gaussians.  The preprocess wrote dkeys[0] = depth bits (culled: ~0u).
hipError_t launch_depth_order(const Args &a, GeomState g, hipStream_t s) {
    uint32_t *keys[2] = {g.dkeys[0], g.dkeys[1]};
    // pass 0 reads identity values (nullptr) and writes dvals[1]; passes ping-pong afterwards
    const int chunk = kSortThreads * kItemsP;
    const int nblk = (a.P + chunk - 1) / chunk;
    uint32_t *hist = g.sort_scratch;
    uint32_t *partials = g.sort_scratch + 256 * (size_t)nblk;
    int cur = 0;
    for (int shift = 0; shift < 32; shift += 8) {
        hipLaunchKernelGGL((radix_hist_kernel<uint32_t, kItemsP>), dim3(nblk), dim3(kSortThreads), 0, s, keys[cur],
                           a.P, shift, hist, nblk);
        exclusive_scan(hist, 256 * nblk, partials, s);
        const uint32_t *vin = shift == 0 ? nullptr : (cur == 0 ? g.dvals[0] : g.dvals[1]);
        uint32_t *vout = cur == 0 ? g.dvals[1] : g.dvals[0];
        hipLaunchKernelGGL((radix_scatter_kernel<uint32_t, kItemsP, true>), dim3(nblk), dim3(kSortThreads), 0, s,
                           keys[cur], vin, keys[cur ^ 1], vout, a.P, shift, hist, nblk,
                           shift == 24 ? g.rank : nullptr);
        cur ^= 1;
    }
    // 4 passes: dvals[0] = Gaussian id by depth rank, rank[id] = depth rank
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// K3: one workgroup per 256 Gaussians (the partition of the preprocess block sums).  The workgroup
// re-derives its local exclusive scan of tiles_touched, then emits its instances with a
// load-balanced loop: slot k finds its Gaussian by binary search over the local inclusive scan, so
// every lane writes one key per iteration however unevenly tile counts are spread.
template <typename K>
__global__ __launch_bounds__(kPreprocessBlock) void duplicate_kernel(Args a, GeomState g, const int *__restrict__ radii,
                                                                     K *__restrict__ keys, int rank_bits) {
    __shared__ uint32_t s_incl[kPreprocessBlock];
    __shared__ int4 s_rect[kPreprocessBlock];  // x0, y0, width, rank
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
            rect = make_int4(x0, y0, x1 - x0, (int)g.rank[idx]);
        }
    }
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
        int lo = 0, hi = kPreprocessBlock - 1;
        while (lo < hi) {
            int mid = (lo + hi) >> 1;
            if (s_incl[mid] > k) hi = mid; else lo = mid + 1;
        }
        const uint32_t local = k - (lo ? s_incl[lo - 1] : 0);
        const int4 r = s_rect[lo];
        const uint32_t ty = r.y + local / (uint32_t)r.z;
        const uint32_t tx = r.x + local % (uint32_t)r.z;
        keys[block_off + k] = ((K)(ty * a.gx + tx) << rank_bits) | (K)(uint32_t)r.w;
    }
}

// ---------------------------------------------------------------------------------------------
// K5: tile ranges, the render-order Gaussian ids, and each sorted instance's unsorted position
// (point_offsets[g] + k, k = row-major index inside g's tile rect, as duplicateWithKeys emits them)
// where the render backward stores its gradient record.
template <typename K>
__global__ void tile_ranges_kernel(Args a, GeomState g, const int *__restrict__ radii, const K *__restrict__ keys,
                                   int L, int rank_bits, uint32_t *__restrict__ point_list,
                                   uint32_t *__restrict__ upos, uint2 *__restrict__ ranges) {
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= L) return;
    const K key = keys[idx];
    const uint32_t cur = (uint32_t)(key >> rank_bits);
    if (idx == 0) {
        ranges[cur].x = 0;
    } else {
        const uint32_t prev = (uint32_t)(keys[idx - 1] >> rank_bits);
        if (cur != prev) {
            ranges[prev].y = idx;
            ranges[cur].x = idx;
        }
    }
    if (idx == L - 1) ranges[cur].y = L;
    const uint32_t rank = (uint32_t)(key & (((K)1 << rank_bits) - 1));
    const uint32_t gid = g.dvals[0][rank];
    point_list[idx] = gid;
    int x0, y0, x1, y1;
    const float2 p = g.xy[gid];
    getRect(p.x, p.y, radii[gid], a.gx, a.gy, x0, y0, x1, y1);
    const uint32_t tx = cur % (uint32_t)a.gx, ty = cur / (uint32_t)a.gx;
    upos[idx] = g.point_offsets[gid] + (ty - y0) * (uint32_t)(x1 - x0) + (tx - x0);
}

template <typename K>
static hipError_t binning_impl(const Args &a, GeomState g, const int *radii, BinningState b, int L, ImageState img,
                               hipStream_t s) {
    const int T = a.gx * a.gy;
    hipError_t e = hipMemsetAsync(img.ranges, 0, sizeof(uint2) * (size_t)T, s);
    if (e != hipSuccess || L == 0) return e;
    K *keys[2] = {(K *)b.keys[0], (K *)b.keys[1]};
    const int nblkP = (a.P + kPreprocessBlock - 1) / kPreprocessBlock;
    hipLaunchKernelGGL((duplicate_kernel<K>), dim3(nblkP), dim3(kPreprocessBlock), 0, s, a, g, radii, keys[0],
                       b.rank_bits);
    const int buf = radix_sort_keys<K, kItemsL>(keys, L, b.key_bits, b.scratch, s);
    hipLaunchKernelGGL((tile_ranges_kernel<K>), dim3((L + 255) / 256), dim3(256), 0, s, a, g, radii, keys[buf], L,
                       b.rank_bits, b.point_list, b.upos, img.ranges);
    return hipGetLastError();
}

hipError_t launch_binning(const Args &a, GeomState g, const int *radii, BinningState b, int L, ImageState img,
                          hipStream_t s) {
    return b.wide ? binning_impl<uint64_t>(a, g, radii, b, L, img, s)
                  : binning_impl<uint32_t>(a, g, radii, b, L, img, s);
}

}  // namespace gs4d
