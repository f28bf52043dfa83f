// binning.hip -- depth order, culled (tile, Gaussian) instance emission (K3), radix sort (K4) and tile
// ranges (K5).
//
// Reference: cuda_rasterizer/rasterizer_impl.cu:70-111 (duplicateWithKeys), :116-138
// (identifyTileRanges), :301-318 (cub::DeviceRadixSort::SortPairs of (tile<<32 | depth_bits, id)
// on bits [0, 32+msb(T)), stable).
//
// MI355X design (this library's own).  The reference sorts L ~ 1.4M 64-bit (tile, depth) keys over
// 45 bits.  Here:
//   1. the P Gaussians are sorted by depth bits (32-bit stable radix sort, ties by id -> the same
//      tie order as the reference's stable sort of instances emitted in id order);
//   2. the candidate instances (each Gaussian's 3-sigma tile rectangle, row-major, Gaussians in depth
//      order) are numbered by a prefix sum of the rectangle areas, and emitted -- only for tiles the
//      splat actually reaches (tile_reached, gs4d_internal.h) -- in one load-balanced stream
//      compaction pass: every workgroup takes a fixed number of candidates, whatever the splat sizes;
//   3. the emitted sequence is already depth-ordered, so a STABLE sort by tile id alone yields the
//      reference's (tile, depth, id) order: ceil(msb(T)/8) passes over u32 keys (2 at the metric
//      config instead of 6 over 12-byte pairs).
// Scan, compaction and every sort pass are single launches that chain workgroups by decoupled
// look-back: workgroups take chunk ids from an atomic counter in launch order, publish their chunk
// aggregate, and find their global offset from lower chunk ids only (one 32-bit status+count word per
// chunk (and digit), stored and polled with agent-scope relaxed atomics, so each word is its own
// flag; a chunk only waits on chunks that already started, and spins are bounded).
#include "gs4d_internal.h"

namespace gs4d {

constexpr int kSortThreads = 256;
constexpr int kItemsL = 8;     // keys per lane for the instance sort (2048 per workgroup)
constexpr int kItemsP = 4;     // keys per lane for the Gaussian depth sort (1024 per workgroup)
constexpr int kMaxPasses = 4;  // u32 keys
constexpr int kScanItems = 4;  // area scan: 1024 per workgroup
constexpr int kEmitItems = 8;  // candidates per lane in the emission pass (2048 per workgroup)
constexpr int kEmitChunk = 256 * kEmitItems;
constexpr uint32_t kAgg = 1u << 30, kPrefix = 2u << 30, kValMask = (1u << 30) - 1;
constexpr uint32_t kSpinLimit = 1u << 22;

__device__ __forceinline__ void store_word(uint32_t *p, uint32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t load_word(const uint32_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// element count: host value, or a device word when it is only known on the GPU
__device__ __forceinline__ int count_of(int n_host, const uint32_t *n_dev) {
    return n_dev ? (int)__builtin_amdgcn_readfirstlane(*n_dev) : n_host;
}

// Decoupled look-back for one value of chunk b (words look[p * stride]): publishes c, returns the
// exclusive prefix over chunks 0..b-1.
__device__ __forceinline__ uint32_t look_back(uint32_t *look, size_t stride, uint32_t b, uint32_t c, uint32_t *err) {
    uint32_t *mine = look + (size_t)b * stride;
    if (b == 0) {
        store_word(mine, kPrefix | c);
        return 0;
    }
    store_word(mine, kAgg | c);
    uint32_t excl = 0, spins = 0;
    for (int p = (int)b - 1; p >= 0;) {
        const uint32_t v = load_word(look + (size_t)p * stride);
        if ((v & ~kValMask) == 0) {
            if (++spins > kSpinLimit) {
                atomicOr(err, 1u);
                break;
            }
            __builtin_amdgcn_s_sleep(1);
            continue;
        }
        excl += v & kValMask;
        if (v & kPrefix) break;
        p--;
    }
    store_word(mine, kPrefix | (excl + c));
    return excl;
}

// ---------------------------------------------------------------------------------------------
// Scratch layouts (u32 words, each zeroed by one memset).
// Sort: 256*kMaxPasses digit histograms | kMaxPasses chunk counters | error flag | pad |
//       npass x (nblk*256) look-back words
static int sort_nblk(int n, int items) { return (n + kSortThreads * items - 1) / (kSortThreads * items); }
static size_t sort_header_words() { return 256 * kMaxPasses + kMaxPasses + 60; }
static size_t sort_words(int n, int items, int npass) {
    return sort_header_words() + (size_t)npass * 256 * (size_t)sort_nblk(n, items);
}
struct SortScratch {
    uint32_t *ghist, *counters, *err, *look;
    int nblk;
};
static SortScratch sort_scratch(uint32_t *base, int n, int items) {
    SortScratch s;
    s.ghist = base;
    s.counters = base + 256 * kMaxPasses;
    s.err = s.counters + kMaxPasses;
    s.look = base + sort_header_words();
    s.nblk = sort_nblk(n, items);
    return s;
}
// Chained single-pass kernels (scan, emission): [0] chunk counter | [1] error flag | pad |
// [64 + j] word of chunk j.
static size_t chain_words(int nchunks) { return 64 + (size_t)nchunks; }

// Geometry scratch: [area scan chain | depth sort], zeroed together before the depth sort.
size_t geom_scratch_words(int P) {
    return chain_words((P + 256 * kScanItems - 1) / (256 * kScanItems)) + sort_words(P, kItemsP, 4) + 64;
}
// Binning scratch: [counters (L' at [0]) | emission chain | instance sort], zeroed together.
size_t binning_scratch_words(int L) {
    return 64 + chain_words((L + kEmitChunk - 1) / kEmitChunk) + sort_words(L, kItemsL, kMaxPasses) + 64;
}

// ---------------------------------------------------------------------------------------------
// One read of the keys: the global histogram of every 8-bit digit position of the sort.
template <int ITEMS>
__global__ __launch_bounds__(kSortThreads) void global_hist_kernel(const uint32_t *__restrict__ keys, int n_host,
                                                                   const uint32_t *__restrict__ n_dev, int npass,
                                                                   uint32_t *__restrict__ ghist) {
    __shared__ uint32_t s_h[kMaxPasses][256];
    const int tid = threadIdx.x;
    const int n = count_of(n_host, n_dev);
    for (int p = 0; p < npass; p++) s_h[p][tid] = 0;
    __syncthreads();
    const size_t base = (size_t)blockIdx.x * (kSortThreads * ITEMS);
#pragma unroll
    for (int r = 0; r < ITEMS; r++) {
        const size_t i = base + (size_t)r * kSortThreads + tid;
        if (i < (size_t)n) {
            const uint32_t k = keys[i];
            for (int p = 0; p < npass; p++) atomicAdd(&s_h[p][(k >> (8 * p)) & 0xFFu], 1u);
        }
    }
    __syncthreads();
    for (int p = 0; p < npass; p++)
        if (s_h[p][tid]) atomicAdd(&ghist[p * 256 + tid], s_h[p][tid]);
}

enum Epilogue { kEpiDepth = 1, kEpiInstances = 2 };
// Last-pass side outputs (see onesweep_kernel); o2 == nullptr disables them.
struct EpiPtrs {
    uint32_t *o0;
    const uint32_t *i1;
    uint32_t *o2, *o3;
};

// One LSD pass over 8 bits at `shift`.  Values: vin == nullptr -> identity (the item's index).
// Epilogue on the last pass:
//   kEpiDepth:     o2[pos] = i1[value] (rect area by depth rank), o3[value] = 0 (reached-tile count)
//   kEpiInstances: o0[pos] = i1[value] (Gaussian id, render order), o2[pos] = value (emission slot,
//                  where the backward stores the instance's gradient record)
template <int ITEMS, int EPI>
__global__ __launch_bounds__(kSortThreads) void onesweep_kernel(const uint32_t *__restrict__ kin,
                                                                const uint32_t *__restrict__ vin,
                                                                uint32_t *__restrict__ kout,
                                                                uint32_t *__restrict__ vout, int n_host,
                                                                const uint32_t *__restrict__ n_dev, int shift,
                                                                const uint32_t *__restrict__ ghist,
                                                                uint32_t *__restrict__ look,
                                                                uint32_t *__restrict__ counter,
                                                                uint32_t *__restrict__ err, EpiPtrs e) {
    __shared__ uint32_t s_cnt[kSortThreads / 64][256];
    __shared__ uint32_t s_wsum[kSortThreads / 64];
    __shared__ uint32_t s_bid;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int n = count_of(n_host, n_dev);
    if (tid == 0) s_bid = atomicAdd(counter, 1u);
#pragma unroll
    for (int q = 0; q < kSortThreads / 64; q++) s_cnt[q][tid] = 0;
    // exclusive scan of the global digit histogram (thread tid <-> digit tid)
    const uint32_t gcount = ghist[tid];
    uint32_t gx = gcount;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t y = __shfl_up(gx, off);
        if (lane >= off) gx += y;
    }
    if (lane == 63) s_wsum[w] = gx;
    __syncthreads();
    uint32_t gbase = gx - gcount;
    for (int q = 0; q < w; q++) gbase += s_wsum[q];
    const uint32_t b = s_bid;
    const uint64_t lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    const size_t wbase = (size_t)b * (kSortThreads * ITEMS) + (size_t)w * (64 * ITEMS);
    uint32_t key[ITEMS], val[ITEMS], lrank[ITEMS];
    // issue every load of the chunk before ranking
#pragma unroll
    for (int r = 0; r < ITEMS; r++) {
        const size_t i = wbase + (size_t)r * 64 + lane;
        const bool valid = i < (size_t)n;
        key[r] = valid ? kin[i] : 0u;
        val[r] = valid ? (vin ? vin[i] : (uint32_t)i) : 0u;
    }
#pragma unroll
    for (int r = 0; r < ITEMS; r++) {
        const bool valid = wbase + (size_t)r * 64 + lane < (size_t)n;
        const uint32_t d = (key[r] >> shift) & 0xFFu;
        uint64_t peers = __ballot(valid);
#pragma unroll
        for (int bit = 0; bit < 8; bit++) {
            const bool set = (d >> bit) & 1u;
            const uint64_t m = __ballot(set);
            peers &= set ? m : ~m;
        }
        const uint32_t below = __popcll(peers & lt_mask);
        const uint32_t old = valid ? s_cnt[w][d] : 0u;
        if (valid && below == 0) s_cnt[w][d] = old + (uint32_t)__popcll(peers);
        lrank[r] = old + below;
    }
    __syncthreads();
    // thread tid <-> digit tid: chunk count, look-back, global offset
    uint32_t c = 0;
#pragma unroll
    for (int q = 0; q < kSortThreads / 64; q++) c += s_cnt[q][tid];
    const uint32_t excl = look_back(look + tid, 256, b, c, err);
    {
        uint32_t run = gbase + excl;
#pragma unroll
        for (int q = 0; q < kSortThreads / 64; q++) {
            const uint32_t cq = s_cnt[q][tid];
            s_cnt[q][tid] = run;
            run += cq;
        }
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < ITEMS; r++) {
        const size_t i = wbase + (size_t)r * 64 + lane;
        if (i < (size_t)n) {
            const uint32_t d = (key[r] >> shift) & 0xFFu;
            const uint32_t pos = s_cnt[w][d] + lrank[r];
            kout[pos] = key[r];
            if (vout) vout[pos] = val[r];
            if (EPI == kEpiDepth && e.o2) {
                e.o2[pos] = e.i1[val[r]];
                e.o3[val[r]] = 0u;
            }
            if (EPI == kEpiInstances && e.o2) {
                e.o0[pos] = e.i1[val[r]];
                e.o2[pos] = val[r];
            }
        }
    }
}

// Stable LSD sort of u32 keys[0] (+ values, identity in pass 0) on bits [0, nbits): one histogram
// launch and one onesweep launch per pass over `scratch` (already zeroed by the caller).  n = n_host,
// or *n_dev when n_dev != nullptr (then n_host is only the grid-sizing upper bound).  Returns the
// buffer index holding the sorted keys.
template <int ITEMS, int EPI>
static int onesweep_sort(uint32_t *keys[2], uint32_t *vals[2], int n_host, const uint32_t *n_dev, int nbits,
                         uint32_t *scratch, EpiPtrs epi, hipStream_t s) {
    const int npass = (nbits + 7) / 8;
    SortScratch ss = sort_scratch(scratch, n_host, ITEMS);
    hipLaunchKernelGGL((global_hist_kernel<ITEMS>), dim3(ss.nblk), dim3(kSortThreads), 0, s, keys[0], n_host, n_dev,
                       npass, ss.ghist);
    int cur = 0;
    const EpiPtrs none = {nullptr, nullptr, nullptr, nullptr};
    for (int p = 0; p < npass; p++) {
        const bool last = p == npass - 1;
        // the instance sort's last pass writes render-order ids instead of sorted values
        uint32_t *vout = (last && EPI == kEpiInstances) ? nullptr : vals[cur ^ 1];
        hipLaunchKernelGGL((onesweep_kernel<ITEMS, EPI>), dim3(ss.nblk), dim3(kSortThreads), 0, s, keys[cur],
                           p == 0 ? nullptr : vals[cur], keys[cur ^ 1], vout, n_host, n_dev, 8 * p,
                           ss.ghist + 256 * p, ss.look + (size_t)p * 256 * ss.nblk, ss.counters + p, ss.err,
                           last ? epi : none);
        cur ^= 1;
    }
    return cur;
}

// ---------------------------------------------------------------------------------------------
// Exclusive scan of the rect areas in depth-rank order: cand_off[r] = first candidate of rank r,
// cand_off[P] = num_rendered.  Single pass, chained by look-back.
__global__ __launch_bounds__(256) void area_scan_kernel(const uint32_t *__restrict__ in, uint32_t *__restrict__ out,
                                                        int n, uint32_t *__restrict__ chain) {
    __shared__ uint32_t s_w[4];
    __shared__ uint32_t s_bid, s_prefix;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    if (tid == 0) s_bid = atomicAdd(chain, 1u);
    __syncthreads();
    const uint32_t b = s_bid;
    const size_t base = (size_t)b * (256 * kScanItems) + (size_t)tid * kScanItems;
    uint32_t v[kScanItems], t = 0;
#pragma unroll
    for (int i = 0; i < kScanItems; i++) {
        v[i] = base + i < (size_t)n ? in[base + i] : 0u;
        t += v[i];
    }
    uint32_t x = t;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t y = __shfl_up(x, off);
        if (lane >= off) x += y;
    }
    if (lane == 63) s_w[w] = x;
    __syncthreads();
    uint32_t before = 0, total = 0;
#pragma unroll
    for (int q = 0; q < 4; q++) {
        before += q < w ? s_w[q] : 0u;
        total += s_w[q];
    }
    if (tid == 0) s_prefix = look_back(chain + 64, 1, b, total, chain + 1);
    __syncthreads();
    uint32_t run = s_prefix + before + x - t;
#pragma unroll
    for (int i = 0; i < kScanItems; i++) {
        if (base + i < (size_t)n) out[base + i] = run;
        run += v[i];
    }
    if (base < (size_t)n && base + kScanItems >= (size_t)n) out[n] = run;
}

hipError_t launch_depth_order(const Args &a, GeomState g, hipStream_t s) {
    const int nchunk = (a.P + 256 * kScanItems - 1) / (256 * kScanItems);
    uint32_t *chain = g.sort_scratch;
    uint32_t *sort_base = chain + chain_words(nchunk);
    hipError_t e = hipMemsetAsync(g.sort_scratch, 0, 4 * geom_scratch_words(a.P), s);
    if (e != hipSuccess) return e;
    // dkeys[0] = depth bits (unbinned: ~0u, last); afterwards dvals[0] = Gaussian id by depth rank,
    // area_rank[r] = tiles_touched of rank r, n_inst = 0
    uint32_t *keys[2] = {g.dkeys[0], g.dkeys[1]};
    uint32_t *vals[2] = {g.dvals[0], g.dvals[1]};
    const EpiPtrs epi = {nullptr, g.tiles_touched, g.area_rank, g.n_inst};
    onesweep_sort<kItemsP, kEpiDepth>(keys, vals, a.P, nullptr, 32, sort_base, epi, s);
    hipLaunchKernelGGL(area_scan_kernel, dim3(nchunk), dim3(256), 0, s, g.area_rank, g.cand_off, a.P, chain);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// K3: load-balanced emission.  Workgroup (chunk) j takes candidates [j*2048, +2048) of the
// depth-ordered candidate sequence, tests each with tile_reached, and compacts the reached ones in
// candidate order: keys[e] = tile, gid_by_e[e] = Gaussian.  Emission offsets are chained by
// look-back; the last chunk stores L' = the number of emitted instances.  n_inst[g] (zeroed by the
// depth sort) receives each Gaussian's count with integer atomics.  The first T threads of the grid
// also zero the tile ranges.
__global__ __launch_bounds__(256) void emit_instances_kernel(Args a, GeomState g, const int *__restrict__ radii,
                                                             int L, uint32_t *__restrict__ keys,
                                                             uint32_t *__restrict__ gid_by_e,
                                                             uint32_t *__restrict__ counters,
                                                             uint32_t *__restrict__ chain, uint2 *__restrict__ ranges) {
    __shared__ uint32_t s_off[kEmitChunk + 1];
    __shared__ uint32_t s_n[kEmitChunk];
    __shared__ uint32_t s_cnt[kEmitItems][4];
    __shared__ uint32_t s_bid, s_prefix;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    {
        const int gt = blockIdx.x * 256 + tid;
        if (gt < a.gx * a.gy) ranges[gt] = make_uint2(0u, 0u);
    }
    if (tid == 0) s_bid = atomicAdd(chain, 1u);
    __syncthreads();
    const uint32_t b = s_bid;
    const uint32_t c0 = b * kEmitChunk;
    if (c0 >= (uint32_t)L) return;  // grid padding for the range zeroing
    const uint32_t c1 = min((uint32_t)L, c0 + kEmitChunk);
    const uint32_t *__restrict__ off = g.cand_off;
    // ranks owning candidates c0 and c1-1: the last r with off[r] <= x (256-ary search, off[P] = L)
    int lo0 = 0, hi0 = a.P, lo1 = 0, hi1 = a.P;
    while (hi0 - lo0 > 1 || hi1 - lo1 > 1) {
        const int st0 = (hi0 - lo0 + 255) / 256, st1 = (hi1 - lo1 + 255) / 256;
        const int p0 = lo0 + tid * st0, p1 = lo1 + tid * st1;
        const int n0 = __syncthreads_count(tid > 0 && p0 < hi0 && off[p0] <= c0);
        const int n1 = __syncthreads_count(tid > 0 && p1 < hi1 && off[p1] <= c1 - 1);
        lo0 += n0 * st0;
        hi0 = min(hi0, lo0 + st0);
        lo1 += n1 * st1;
        hi1 = min(hi1, lo1 + st1);
    }
    // unbinned Gaussians (area 0) sort last, so every rank in [lo0, lo1] has area >= 1: nr <= 2048
    const int rlo = lo0, nr = lo1 - lo0 + 1;
    for (int i = tid; i <= nr; i += 256) s_off[i] = off[rlo + i];
    for (int i = tid; i < nr; i += 256) s_n[i] = 0;
    __syncthreads();
    uint32_t tile[kEmitItems], gid[kEmitItems];
    uint64_t kept[kEmitItems];
#pragma unroll
    for (int it = 0; it < kEmitItems; it++) {
        const uint32_t c = c0 + it * 256 + tid;
        bool keep = false;
        tile[it] = 0;
        gid[it] = 0;
        if (c < c1) {
            int l = 0, h = nr - 1;  // last j with s_off[j] <= c
            while (l < h) {
                const int m = (l + h + 1) >> 1;
                if (s_off[m] <= c) l = m; else h = m - 1;
            }
            const uint32_t id = g.dvals[0][rlo + l];
            const float2 p = g.xy[id];
            int x0, y0, x1, y1;
            getRect(p.x, p.y, radii[id], a.gx, a.gy, x0, y0, x1, y1);
            const uint32_t local = c - s_off[l], wdt = (uint32_t)(x1 - x0);
            const int ty = y0 + (int)(local / wdt), tx = x0 + (int)(local % wdt);
            const uint32_t area = s_off[l + 1] - s_off[l];
            keep = area > kTightMaxArea || tile_reached(p.x, p.y, g.conic_opacity[id], tx, ty, a.W, a.H);
            tile[it] = (uint32_t)(ty * a.gx + tx);
            gid[it] = id;
            if (keep) atomicAdd(&s_n[l], 1u);
        }
        kept[it] = __ballot(keep);
        if (lane == 0) s_cnt[it][w] = (uint32_t)__popcll(kept[it]);
    }
    __syncthreads();
    if (tid == 0) {
        uint32_t total = 0;
        for (int it = 0; it < kEmitItems; it++)
            for (int q = 0; q < 4; q++) total += s_cnt[it][q];
        s_prefix = look_back(chain + 64, 1, b, total, chain + 1);
        if (c1 == (uint32_t)L) counters[0] = s_prefix + total;
    }
    __syncthreads();
    const uint64_t lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    uint32_t run = s_prefix;
#pragma unroll
    for (int it = 0; it < kEmitItems; it++) {
        uint32_t before = 0, step = 0;
#pragma unroll
        for (int q = 0; q < 4; q++) {
            before += q < w ? s_cnt[it][q] : 0u;
            step += s_cnt[it][q];
        }
        if ((kept[it] >> lane) & 1ull) {
            const uint32_t e = run + before + (uint32_t)__popcll(kept[it] & lt_mask);
            keys[e] = tile[it];
            gid_by_e[e] = gid[it];
        }
        run += step;
    }
    for (int i = tid; i < nr; i += 256)
        if (s_n[i]) atomicAdd(&g.n_inst[g.dvals[0][rlo + i]], s_n[i]);
}

// K5: tile ranges from the sorted tile keys (rasterizer_impl.cu:116-138); tiles without instances
// keep the emission pass's (0, 0).
__global__ void tile_ranges_kernel(const uint32_t *__restrict__ keys, const uint32_t *__restrict__ n_dev,
                                   uint2 *__restrict__ ranges) {
    const int L = (int)*n_dev;
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= L) return;
    const uint32_t cur = keys[idx];
    if (idx == 0) {
        ranges[cur].x = 0;
    } else {
        const uint32_t prev = keys[idx - 1];
        if (cur != prev) {
            ranges[prev].y = idx;
            ranges[cur].x = idx;
        }
    }
    if (idx == L - 1) ranges[cur].y = L;
}

hipError_t launch_binning(const Args &a, GeomState g, const int *radii, BinningState b, int L, ImageState img,
                          hipStream_t s) {
    const int T = a.gx * a.gy;
    hipError_t e = hipMemsetAsync(b.scratch, 0, 4 * binning_scratch_words(L), s);
    if (e != hipSuccess) return e;
    if (L == 0) return hipMemsetAsync(img.ranges, 0, sizeof(uint2) * (size_t)T, s);
    uint32_t *counters = b.scratch;
    uint32_t *chain = counters + 64;
    const int nchunk = (L + kEmitChunk - 1) / kEmitChunk;
    const int nblk = max(nchunk, (T + 255) / 256);
    hipLaunchKernelGGL(emit_instances_kernel, dim3(nblk), dim3(256), 0, s, a, g, radii, L, b.keys[0], b.gid_by_e,
                       counters, chain, img.ranges);
    const uint32_t *n_dev = counters;  // L' <= L reached instances
    uint32_t *keys[2] = {b.keys[0], b.keys[1]};
    uint32_t *vals[2] = {b.vals[0], b.vals[1]};
    const EpiPtrs epi = {b.point_list, b.gid_by_e, b.upos, nullptr};
    const int buf = onesweep_sort<kItemsL, kEpiInstances>(keys, vals, L, n_dev, b.key_bits,
                                                          chain + chain_words(nchunk), epi, s);
    hipLaunchKernelGGL(tile_ranges_kernel, dim3((L + 255) / 256), dim3(256), 0, s, keys[buf], n_dev, img.ranges);
    return hipGetLastError();
}

}  // namespace gs4d
