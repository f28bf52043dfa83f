// radix_sort.h -- decoupled chunk prefixes and the stable onesweep LSD radix sort shared by the
// binning (depth and tile sorts) and the kNN initialiser (Morton sort).  The reference uses
// cub::DeviceRadixSort::SortPairs (rasterizer_impl.cu:304-309, simple_knn.cu:212-215): a stable
// ascending sort; this is the same contract, built for gfx950 (see binning.hip for the design).
#pragma once
#include "gs4d_internal.h"

namespace gs4d {

constexpr uint32_t kAgg = 1u << 30, kValMask = (1u << 30) - 1;

// Wave-wide inclusive scans by DPP moves (row_shr 1/2/4/8 inside rows of 16, then row_bcast:15 into rows
// 1 and 3 and row_bcast:31 into rows 2 and 3): plain VALU, no LDS round trips as __shfl_up's bpermutes.
// Lanes without a source read 0, the identity of both operations (unsigned values).
template <int CTRL, int RM>
__device__ __forceinline__ uint32_t dpp_src(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, RM, 0xF, false);
}
__device__ __forceinline__ uint32_t wave_incl_sum(uint32_t x) {
    x += dpp_src<0x111, 0xF>(x);
    x += dpp_src<0x112, 0xF>(x);
    x += dpp_src<0x114, 0xF>(x);
    x += dpp_src<0x118, 0xF>(x);
    x += dpp_src<0x142, 0xA>(x);
    x += dpp_src<0x143, 0xC>(x);
    return x;
}
__device__ __forceinline__ uint32_t wave_incl_max(uint32_t x) {
    x = max(x, dpp_src<0x111, 0xF>(x));
    x = max(x, dpp_src<0x112, 0xF>(x));
    x = max(x, dpp_src<0x114, 0xF>(x));
    x = max(x, dpp_src<0x118, 0xF>(x));
    x = max(x, dpp_src<0x142, 0xA>(x));
    x = max(x, dpp_src<0x143, 0xC>(x));
    return x;
}
constexpr uint32_t kSpinLimit = 1u << 20;

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

// Chunk prefixes without a chain.  Every chunk publishes its count as soon as it is known (status
// bit kAgg | count, agent-scope store); a chunk then sums the published counts of ALL lower chunks
// directly, many loads in flight at once.  Chained look-back makes the last of N chunks wait
// ~N/window round trips; this waits ~1, for O(N) loads per chunk (N is at most a few hundred here).
// Lower chunks publish before they wait on anything, and the dispatcher starts them first, so the
// waits terminate; they are bounded anyway (err).
__device__ __forceinline__ uint32_t sum_published(const uint32_t *look, size_t stride, int b, int first, int step,
                                                  uint32_t *err) {
    constexpr int kBatch = 16;
    uint32_t sum = 0;
    for (int p0 = first; p0 < b; p0 += kBatch * step) {
        uint32_t v[kBatch];
        bool ready = true;
#pragma unroll
        for (int i = 0; i < kBatch; i++) {
            const int p = p0 + i * step;
            v[i] = p < b ? load_word(look + (size_t)p * stride) : kAgg;
        }
#pragma unroll
        for (int i = 0; i < kBatch; i++) ready &= (v[i] & kAgg) != 0;
        if (!ready) {
            // slow path: poll the words one by one (reloaded: v[] must not be indexed dynamically)
#pragma nounroll
            for (int i = 0; i < kBatch; i++) {
                const int p = p0 + i * step;
                if (p >= b) break;
                uint32_t w = load_word(look + (size_t)p * stride), spins = 0;
                while ((w & kAgg) == 0) {
                    if (++spins > kSpinLimit) {
                        atomicOr(err, 1u);
                        w = kAgg;
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                    w = load_word(look + (size_t)p * stride);
                }
                sum += w & kValMask;
            }
        } else {
#pragma unroll
            for (int i = 0; i < kBatch; i++) sum += v[i] & kValMask;
        }
    }
    return sum;
}

// Exclusive prefix of chunk b's count c over a 256-thread workgroup (call from every thread).
__device__ __forceinline__ uint32_t block_prefix(uint32_t *look, uint32_t b, uint32_t c, uint32_t *err,
                                                 uint32_t *s_tmp /* 4 words of LDS */) {
    const int tid = threadIdx.x;
    if (tid == 0) store_word(look + b, kAgg | c);
    uint32_t x = sum_published(look, 1, (int)b, tid, 256, err);
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off);
    __syncthreads();
    if ((tid & 63) == 0) s_tmp[tid >> 6] = x;
    __syncthreads();
    return s_tmp[0] + s_tmp[1] + s_tmp[2] + s_tmp[3];
}

static inline int sort_nblk(int n, int chunk) { return (n + chunk - 1) / chunk; }

// One LSD pass over 8 bits at `shift` (chunk = blockIdx.x).  Values: vin == nullptr -> identity (the
// item's index).  hist: the 8 shards of the producer's digit histogram for this pass.
// MODE: diagnostic knob for tools/bench/sortbench.hip only (0 in the library): 1 skips the chunk
// prefix sums (wrong order, in-bounds positions: timing only).
template <int THREADS, int ITEMS, int MODE = 0>
__global__ __launch_bounds__(THREADS) void onesweep_kernel(const uint32_t *__restrict__ kin,
                                                           const uint32_t *__restrict__ vin,
                                                           uint32_t *__restrict__ kout, uint32_t *__restrict__ vout,
                                                           int n_host, const uint32_t *__restrict__ n_dev, int shift,
                                                           const uint32_t *__restrict__ hist,
                                                           uint32_t *__restrict__ look, uint32_t *__restrict__ err) {
    constexpr int NW = THREADS / 64;
    __shared__ uint32_t s_cnt[NW][256];
    __shared__ uint32_t s_wsum[4], s_lsum[4];
    __shared__ uint32_t s_delta[256], s_lexc[256], s_c[256];
    __shared__ uint32_t s_part[THREADS / 256][256];
    __shared__ uint32_t s_key[THREADS * ITEMS], s_val[THREADS * ITEMS];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int n = count_of(n_host, n_dev);
    const uint32_t b = blockIdx.x;
    // a chunk past the device count (the grid is sized by the host's upper bound) has no items, and
    // no chunk with items reads its look-back words (they only read lower chunks)
    if ((size_t)b * (THREADS * ITEMS) >= (size_t)n && n_dev) return;
    const size_t wbase = (size_t)b * (THREADS * ITEMS) + (size_t)w * (64 * ITEMS);
    uint32_t key[ITEMS], val[ITEMS], lrank[ITEMS];
    // issue every load of the chunk first
#pragma unroll
    for (int r = 0; r < ITEMS; r++) {
        const size_t i = wbase + (size_t)r * 64 + lane;
        const bool valid = i < (size_t)n;
        key[r] = valid ? kin[i] : 0u;
        val[r] = valid ? (vin ? vin[i] : (uint32_t)i) : 0u;
    }
    // threads 0..255 <-> digits: global digit count and its exclusive scan
    uint32_t gcount = 0, gx = 0;
    if (tid < 256) {
#pragma unroll
        for (int s = 0; s < kHistShards; s++) gcount += hist[s * (kMaxPasses * 256) + tid];
        gx = gcount;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const uint32_t y = __shfl_up(gx, off);
            if (lane >= off) gx += y;
        }
        if (lane == 63) s_wsum[w] = gx;
    }
    for (int i = tid; i < NW * 256; i += THREADS) (&s_cnt[0][0])[i] = 0;
    __syncthreads();
    uint32_t gbase = gx - gcount;
    if (tid < 256)
        for (int q = 0; q < w; q++) gbase += s_wsum[q];
    const uint64_t lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
#pragma unroll
    for (int r = 0; r < ITEMS; r++) {
        const bool valid = wbase + (size_t)r * 64 + lane < (size_t)n;
        const uint32_t d = (key[r] >> shift) & 0xFFu;
        uint64_t peers = __builtin_amdgcn_ballot_w64(valid);
#pragma unroll
        for (int bit = 0; bit < 8; bit++) {
            const bool set = (d >> bit) & 1u;
            const uint64_t m = __builtin_amdgcn_ballot_w64(set);
            peers &= set ? m : ~m;
        }
        const uint32_t below = __popcll(peers & lt_mask);
        const uint32_t old = valid ? s_cnt[w][d] : 0u;
        if (valid && below == 0) s_cnt[w][d] = old + (uint32_t)__popcll(peers);
        lrank[r] = old + below;
    }
    __syncthreads();
    // digit threads publish the chunk's digit counts; every thread then sums a strided share of the
    // lower chunks' published counts of digit tid & 255
    constexpr int PARTS = THREADS / 256;
    if (tid < 256) {
        uint32_t c = 0;
#pragma unroll
        for (int q = 0; q < NW; q++) c += s_cnt[q][tid];
        s_c[tid] = c;
        store_word(look + (size_t)b * 256 + tid, kAgg | c);
    }
    s_part[tid >> 8][tid & 255] = (MODE & 1) ? 0u : sum_published(look + (tid & 255), 256, (int)b, tid >> 8, PARTS, err);
    __syncthreads();
    // for every wave's run of the digit: its start in the chunk's locally sorted order; delta[d] maps a
    // local position of digit d to its global one
    if (tid < 256) {
        const uint32_t c = s_c[tid];
        uint32_t excl = 0;
#pragma unroll
        for (int k = 0; k < PARTS; k++) excl += s_part[k][tid];
        uint32_t x = c;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const uint32_t y = __shfl_up(x, off);
            if (lane >= off) x += y;
        }
        s_lsum[w] = x;
        s_delta[tid] = gbase + excl;  // global start of this chunk's run of digit tid
        s_lexc[tid] = x - c;          // wave-local exclusive part
    }
    __syncthreads();
    if (tid < 256) {
        uint32_t lbase = s_lexc[tid];
        for (int q = 0; q < w; q++) lbase += s_lsum[q];
        s_delta[tid] -= lbase;
        uint32_t run = lbase;
#pragma unroll
        for (int q = 0; q < NW; q++) {
            const uint32_t cq = s_cnt[q][tid];
            s_cnt[q][tid] = run;
            run += cq;
        }
    }
    __syncthreads();
    // stage the chunk in digit order in LDS, then write it out with consecutive lanes on consecutive
    // global positions (each digit's run is contiguous in the output)
#pragma unroll
    for (int r = 0; r < ITEMS; r++) {
        if (wbase + (size_t)r * 64 + lane < (size_t)n) {
            const uint32_t lp = s_cnt[w][(key[r] >> shift) & 0xFFu] + lrank[r];
            s_key[lp] = key[r];
            s_val[lp] = val[r];
        }
    }
    __syncthreads();
    const int nvalid = (int)min((size_t)(THREADS * ITEMS), (size_t)n - min((size_t)n, (size_t)b * (THREADS * ITEMS)));
    uint32_t pos[ITEMS];
    bool ok[ITEMS];
#pragma unroll
    for (int r = 0; r < ITEMS; r++) {
        const int lp = r * THREADS + tid;
        ok[r] = lp < nvalid;
        key[r] = ok[r] ? s_key[lp] : 0u;
        val[r] = ok[r] ? s_val[lp] : 0u;
        pos[r] = lp + s_delta[(key[r] >> shift) & 0xFFu];
    }
#pragma unroll
    for (int r = 0; r < ITEMS; r++) {
        if (!ok[r]) continue;
        kout[pos[r]] = key[r];
        if (vout) vout[pos[r]] = val[r];
    }
}

// Stable LSD sort of u32 keys[0] (+ values, identity in pass 0) on bits [0, nbits): one onesweep
// launch per pass.  hist = the producer's sharded digit histograms, look = zeroed look-back words.
// n = n_host, or *n_dev when n_dev != nullptr (then n_host is only the grid-sizing upper bound).
// Returns the buffer index holding the sorted keys.
template <int THREADS, int ITEMS, int MODE = 0>
static int onesweep_sort(uint32_t *keys[2], uint32_t *vals[2], int n_host, const uint32_t *n_dev, int nbits,
                         const uint32_t *hist, uint32_t *look, uint32_t *err, hipStream_t s) {
    const int npass = (nbits + 7) / 8;
    const int nblk = sort_nblk(n_host, THREADS * ITEMS);
    int cur = 0;
    for (int p = 0; p < npass; p++) {
        uint32_t *vout = vals[cur ^ 1];
        hipLaunchKernelGGL((onesweep_kernel<THREADS, ITEMS, MODE>), dim3(nblk), dim3(THREADS), 0, s, keys[cur],
                           p == 0 ? nullptr : vals[cur], keys[cur ^ 1], vout, n_host, n_dev, 8 * p, hist + 256 * p,
                           look + (size_t)p * 256 * nblk, err);
        cur ^= 1;
    }
    return cur;
}

}  // namespace gs4d
