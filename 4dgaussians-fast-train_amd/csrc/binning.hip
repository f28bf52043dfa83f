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
constexpr int kItemsL = 16;   // keys per lane for the instance sort (4096 per workgroup)
constexpr int kItemsP = 4;    // keys per lane for the Gaussian depth sort (1024 per workgroup)
constexpr int kMaxPasses = 8; // 64-bit keys
// decoupled look-back words: 2 status bits + 30-bit count (so every sort holds < 2^30 keys)
constexpr uint32_t kAgg = 1u << 30, kPrefix = 2u << 30, kValMask = (1u << 30) - 1;
constexpr uint32_t kSpinLimit = 1u << 22;

// Sort scratch layout (u32 words), zeroed by one memset per sort:
//   [0, 256*kMaxPasses)            global digit histograms, one per pass
//   [+0, +kMaxPasses)              dynamic workgroup counters, one per pass
//   [+kMaxPasses]                  error flag (look-back spin limit reached)
//   then kMaxPasses x (nblk*256)   look-back status words
struct SortScratch {
    uint32_t *ghist, *counters, *err, *look;
    int nblk;
};
static int sort_nblk(int n, int items) { return (n + kSortThreads * items - 1) / (kSortThreads * items); }
static size_t sort_header_words() { return 256 * kMaxPasses + kMaxPasses + 16; }
size_t radix_scratch_words(int n) {
    return sort_header_words() + (size_t)kMaxPasses * 256 * (size_t)sort_nblk(n, kItemsP) + 64;
}
static SortScratch sort_scratch(uint32_t *base, int n, int items) {
    SortScratch s;
    s.ghist = base;
    s.counters = base + 256 * kMaxPasses;
    s.err = s.counters + kMaxPasses;
    s.look = base + sort_header_words();
    s.nblk = sort_nblk(n, items);
    return s;
}

__device__ __forceinline__ void store_word(uint32_t *p, uint32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t load_word(const uint32_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ---------------------------------------------------------------------------------------------
// One read of the keys: the global histogram of every 8-bit digit position the sort will use.
template <typename K, int ITEMS>
__global__ __launch_bounds__(kSortThreads) void global_hist_kernel(const K *__restrict__ keys, int n, int npass,
                                                                   uint32_t *__restrict__ ghist) {
    __shared__ uint32_t s_h[kMaxPasses][256];
    const int tid = threadIdx.x;
    for (int p = 0; p < npass; p++) s_h[p][tid] = 0;
    __syncthreads();
    const size_t base = (size_t)blockIdx.x * (kSortThreads * ITEMS);
#pragma unroll
    for (int r = 0; r < ITEMS; r++) {
        const size_t i = base + (size_t)r * kSortThreads + tid;
        if (i < (size_t)n) {
            const K k = keys[i];
            for (int p = 0; p < npass; p++) atomicAdd(&s_h[p][(uint32_t)(k >> (8 * p)) & 0xFFu], 1u);
        }
    }
    __syncthreads();
    for (int p = 0; p < npass; p++)
        if (s_h[p][tid]) atomicAdd(&ghist[p * 256 + tid], s_h[p][tid]);
}

// ---------------------------------------------------------------------------------------------
// One LSD pass (8 bits at `shift`), single launch ("onesweep"): workgroups take chunk ids from an
// atomic counter in launch order, rank their keys locally (each wave ranks its contiguous
// sub-chunk round by round with 64-lane ballot matching and per-wave digit counters in LDS), publish
// per-digit counts, and find their global offsets by decoupled look-back over the status words of
// lower chunk ids (one 32-bit word per (chunk, digit) = status + count, stored and polled with
// agent-scope relaxed atomics, so a word is its own flag).  A chunk only ever waits on chunks that
// already started, so the look-back cannot deadlock; spins are bounded regardless.
// VALS: carry 32-bit values (vin == nullptr -> identity values); rank_out[value] = position.
template <typename K, int ITEMS, bool VALS>
__global__ __launch_bounds__(kSortThreads) void onesweep_kernel(const K *__restrict__ kin,
                                                                const uint32_t *__restrict__ vin,
                                                                K *__restrict__ kout, uint32_t *__restrict__ vout,
                                                                int n, int shift, const uint32_t *__restrict__ ghist,
                                                                uint32_t *__restrict__ look,
                                                                uint32_t *__restrict__ counter,
                                                                uint32_t *__restrict__ err,
                                                                uint32_t *__restrict__ rank_out) {
    __shared__ uint32_t s_cnt[kSortThreads / 64][256];
    __shared__ uint32_t s_wsum[kSortThreads / 64];
    __shared__ uint32_t s_bid;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
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
        // every lane reads its digit's running count, then the group leader bumps it; a wave's LDS
        // accesses execute in program order, so all lanes see the value before the bump
        const uint32_t old = valid ? s_cnt[w][d] : 0u;
        if (valid && below == 0) s_cnt[w][d] = old + (uint32_t)__popcll(peers);
        lrank[r] = old + below;
    }
    __syncthreads();
    // thread tid <-> digit tid: chunk count, look-back, global offset
    uint32_t c = 0;
#pragma unroll
    for (int q = 0; q < kSortThreads / 64; q++) c += s_cnt[q][tid];
    uint32_t *mine = look + (size_t)b * 256 + tid;
    uint32_t excl = 0;
    if (b == 0) {
        store_word(mine, kPrefix | c);
    } else {
        store_word(mine, kAgg | c);
        uint32_t spins = 0;
        for (int p = (int)b - 1; p >= 0;) {
            const uint32_t v = load_word(look + (size_t)p * 256 + tid);
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
    }
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

// Full LSD sort of keys[0] on bits [0, nbits): memset + histogram + one onesweep launch per pass.
// vals: nullptr (keys only) or {nullptr -> identity in pass 0, ping, pong}.  Returns the index of
// the key/value buffers holding the result.
template <typename K, int ITEMS, bool VALS>
static int onesweep_sort(K *keys[2], uint32_t *vals[2], int n, int nbits, uint32_t *scratch, uint32_t *rank_out,
                         hipStream_t s) {
    const int npass = (nbits + 7) / 8;
    SortScratch ss = sort_scratch(scratch, n, ITEMS);
    (void)hipMemsetAsync(scratch, 0, 4 * (sort_header_words() + (size_t)npass * 256 * ss.nblk), s);
    hipLaunchKernelGGL((global_hist_kernel<K, ITEMS>), dim3(ss.nblk), dim3(kSortThreads), 0, s, keys[0], n, npass,
                       ss.ghist);
    int cur = 0;
    for (int p = 0; p < npass; p++) {
        const uint32_t *vin = nullptr;
        uint32_t *vout = nullptr;
        if (VALS) {
            vin = (p == 0) ? nullptr : vals[cur];
            vout = vals[cur ^ 1];
        }
        hipLaunchKernelGGL((onesweep_kernel<K, ITEMS, VALS>), dim3(ss.nblk), dim3(kSortThreads), 0, s, keys[cur], vin,
                           keys[cur ^ 1], vout, n, 8 * p, ss.ghist + 256 * p, ss.look + (size_t)p * 256 * ss.nblk,
                           ss.counters + p, ss.err, (p == npass - 1) ? rank_out : nullptr);
        cur ^= 1;
    }
    return cur;
}

// ---------------------------------------------------------------------------------------------
// Depth order of the Gaussians.  The preprocess wrote dkeys[0] = depth bits (unbinned: ~0u).
// After 4 passes dvals[0] = Gaussian id by depth rank and rank[id] = its depth rank.
hipError_t launch_depth_order(const Args &a, GeomState g, hipStream_t s) {
    uint32_t *keys[2] = {g.dkeys[0], g.dkeys[1]};
    uint32_t *vals[2] = {g.dvals[0], g.dvals[1]};
    onesweep_sort<uint32_t, kItemsP, true>(keys, vals, a.P, 32, g.sort_scratch, g.rank, s);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// K3: one workgroup per 256 Gaussians (the partition of the preprocess block sums).  The workgroup
// enumerates its Gaussians' candidate tiles (3-sigma rects, duplicateWithKeys' row-major order) with
// a load-balanced loop -- candidate slot k finds its Gaussian by binary search over the local
// inclusive scan of rect areas -- tests each with tile_reached(), and compacts the survivors in
// slot order (ballot prefix inside each wave + a running workgroup offset).  A survivor's output
// position is therefore point_offsets[g] + (its rank among g's survivors), the "unsorted position"
// the backward's per-Gaussian reduction uses.
template <typename K>
__global__ __launch_bounds__(kPreprocessBlock) void duplicate_kernel(Args a, GeomState g, const int *__restrict__ radii,
                                                                     K *__restrict__ keys, int rank_bits) {
    __shared__ uint32_t s_incl[kPreprocessBlock];   // inclusive scan of candidate counts (rect areas)
    __shared__ int4 s_rect[kPreprocessBlock];       // x0, y0, width, rank
    __shared__ float2 s_xy[kPreprocessBlock];
    __shared__ float4 s_co[kPreprocessBlock];
    __shared__ uint32_t s_wave[kPreprocessBlock / 64];
    __shared__ uint32_t s_cnt[kPreprocessBlock / 64];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int idx = blockIdx.x * kPreprocessBlock + tid;
    uint32_t area = 0, ninst = 0;
    int4 rect = make_int4(0, 0, 1, 0);
    float2 p = make_float2(0.f, 0.f);
    float4 co = make_float4(0.f, 0.f, 0.f, 0.f);
    if (idx < a.P) {
        ninst = g.n_inst[idx];
        if (ninst > 0) {
            int x0, y0, x1, y1;
            p = g.xy[idx];
            co = g.conic_opacity[idx];
            getRect(p.x, p.y, radii[idx], a.gx, a.gy, x0, y0, x1, y1);
            rect = make_int4(x0, y0, x1 - x0, (int)g.rank[idx]);
            area = (uint32_t)((x1 - x0) * (y1 - y0));
        }
    }
    // inclusive workgroup scans of candidate counts and of instance counts
    uint32_t x = area, xi = ninst;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t y = __shfl_up(x, off), yi = __shfl_up(xi, off);
        if (lane >= off) {
            x += y;
            xi += yi;
        }
    }
    if (lane == 63) {
        s_wave[w] = x;
        s_cnt[w] = xi;
    }
    __syncthreads();
    uint32_t wbase = 0, wbase_i = 0;
    for (int i = 0; i < w; i++) {
        wbase += s_wave[i];
        wbase_i += s_cnt[i];
    }
    x += wbase;
    s_incl[tid] = x;
    s_rect[tid] = rect;
    s_xy[tid] = p;
    s_co[tid] = co;
    const uint32_t block_off = g.block_sums[blockIdx.x];
    if (idx < a.P) g.point_offsets[idx] = block_off + wbase_i + xi - ninst;
    __syncthreads();
    const uint32_t total = s_incl[kPreprocessBlock - 1];
    const uint64_t lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    uint32_t out = block_off;  // running output position (uniform)
    for (uint32_t k0 = 0; k0 < total; k0 += kPreprocessBlock) {
        const uint32_t k = k0 + tid;
        bool keep = false;
        K key = 0;
        if (k < total) {
            int lo = 0, hi = kPreprocessBlock - 1;
            while (lo < hi) {
                const int mid = (lo + hi) >> 1;
                if (s_incl[mid] > k) hi = mid; else lo = mid + 1;
            }
            const uint32_t local = k - (lo ? s_incl[lo - 1] : 0);
            const int4 r = s_rect[lo];
            const int ty = r.y + (int)(local / (uint32_t)r.z);
            const int tx = r.x + (int)(local % (uint32_t)r.z);
            const uint32_t rarea = (lo ? s_incl[lo] - s_incl[lo - 1] : s_incl[lo]);
            const float2 sp = s_xy[lo];
            keep = rarea > kTightMaxArea || tile_reached(sp.x, sp.y, s_co[lo], tx, ty, a.W, a.H);
            key = ((K)(uint32_t)(ty * a.gx + tx) << rank_bits) | (K)(uint32_t)r.w;
        }
        const uint64_t m = __ballot(keep);
        if (lane == 0) s_cnt[w] = (uint32_t)__popcll(m);
        __syncthreads();
        uint32_t before = 0, step = 0;
#pragma unroll
        for (int q = 0; q < kPreprocessBlock / 64; q++) {
            const uint32_t c = s_cnt[q];
            before += (q < w) ? c : 0u;
            step += c;
        }
        if (keep) keys[out + before + __popcll(m & lt_mask)] = key;
        out += step;
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------------------------
// K5: tile ranges, the render-order Gaussian ids, and each sorted instance's unsorted position
// point_offsets[g] + (rank of this tile among g's reached tiles in row-major rect order) -- where the
// render backward stores its gradient record.
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
    const int tx = (int)(cur % (uint32_t)a.gx), ty = (int)(cur / (uint32_t)a.gx);
    uint32_t k = (uint32_t)((ty - y0) * (x1 - x0) + (tx - x0));
    if ((uint32_t)((x1 - x0) * (y1 - y0)) <= kTightMaxArea) {
        const float4 co = g.conic_opacity[gid];
        k = 0;
        for (int yy = y0; yy <= ty; yy++)
            for (int xx = x0; xx < x1; xx++) {
                if (yy == ty && xx == tx) break;
                k += tile_reached(p.x, p.y, co, xx, yy, a.W, a.H) ? 1u : 0u;
            }
    }
    upos[idx] = g.point_offsets[gid] + k;
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
    const int buf = onesweep_sort<K, kItemsL, false>(keys, nullptr, L, b.key_bits, b.scratch, nullptr, s);
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
