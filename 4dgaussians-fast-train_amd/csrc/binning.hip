// binning.hip -- instance emission (K3), tile binning and the per-tile depth sort (K4), tile ranges (K5).
//
// Reference: cuda_rasterizer/rasterizer_impl.cu:70-111 (duplicateWithKeys), :116-138
// (identifyTileRanges), :301-318 (cub::DeviceRadixSort::SortPairs of (tile<<32 | depth_bits, id)
// on bits [0, 32+msb(T)), stable over instances emitted in Gaussian-id order).
//
// MI355X design (this library's own).  The reference sorts L ~ 1.4M 64-bit (tile, depth) keys over
// 45 bits (6 radix passes over 12-byte pairs).  Its order is: by tile, then by depth bits, ties by
// Gaussian id.  Here:
//   1. visible_scan: one pass over the Gaussians in id order compacts the visible ones (tiles_touched
//      > 0) and numbers their candidate instances (the 3-sigma tile rectangles, row-major) by a prefix
//      sum of the rectangle areas -- two chunk-prefix chains in one launch;
//   2. emission: one load-balanced pass over the L candidates (a fixed number per workgroup, whatever
//      the splat sizes) keeps only the (tile, splat) pairs the splat reaches (half_reach,
//      gs4d_internal.h) and compacts them in candidate order (so a Gaussian's instances are
//      consecutive: the backward reduces its gradient records by segment);
//   3. a counting sort of the emitted instances by tile id alone (tile_count / tile_scan /
//      tile_scatter: per-chunk tile counts in LDS, their (tile, chunk) exclusive offsets, an LDS
//      fetch-add per instance; the tile ranges fall out of the offsets).  The order inside a tile's
//      run is left arbitrary: step 4 sorts every run by a key unique in the tile, so the result is the
//      same whatever it was.  Tile grids beyond kCountMaxT tiles, or more chunks than the column scan
//      holds, take a STABLE LSD radix sort by tile id instead (ceil(msb(T)/8) passes over u32 keys,
//      digit histograms built by the emission) and tile ranges from the sorted keys;
//   4. tile_sort: each tile's run is sorted by the 64-bit key (depth bits, Gaussian id) -- exactly the
//      reference's within-tile order (the key is unique inside a tile).  Runs of up to kWaveSortMax
//      (256) are sorted by the render forward itself, in registers, before it blends them
//      (render.hip); here runs of up to 2048 by one workgroup in LDS (register sorts + merge path),
//      longer ones as LDS-sorted 2048-runs merged by the bitonic network's global steps.
// The P Gaussians are never sorted by depth globally (the reference's 45-bit key needs 6 passes; a
// global depth sort needs 4 more over the Gaussians).  Prefix sums publish per-chunk counts (one
// 32-bit status+count word per chunk, agent-scope relaxed atomics) and sum the lower chunks' words
// directly (radix_sort.h).
#include <algorithm>
#include <cstdlib>
#include <cstring>

#include "radix_sort.h"

namespace gs4d {

constexpr int kEmitPer = kEmitChunk / 256;  // candidates per lane in the emission pass
constexpr int kEmitStage = 256;             // Gaussians per emission chunk staged in LDS (see the kernel)
constexpr int kSortThreads = 1024;          // radix-sort workgroup: 16 waves rank one chunk together
constexpr int kItemsL = 8;                  // keys per lane for the instance sort (8192 per workgroup)
constexpr int kSortCap = 2048;              // tile runs sorted in LDS by one workgroup (see tile_sort_kernel)

// ---------------------------------------------------------------------------------------------
// Zero-region layouts (u32 words).
constexpr int kScanPer = 4;  // Gaussians per thread of the visible scan (1024 per workgroup)
__host__ __device__ static size_t nchunk_scan(int P) { return ((size_t)P + 256 * kScanPer - 1) / (256 * kScanPer); }
__host__ __device__ static size_t nchunk_emit(int L) { return ((size_t)L + kEmitChunk - 1) / kEmitChunk; }
// geometry: counters | visible-count chain (+ err) | area chain (+ err) | the emission's tile-digit
// histograms (zeroed by the forward's one memset, before the preprocess)
__host__ __device__ static size_t geom_vis_chain_off() { return 64; }
__host__ __device__ static size_t geom_area_chain_off(int P) { return 64 + nchunk_scan(P) + 64; }
__host__ __device__ static size_t geom_hist_off(int P) { return geom_area_chain_off(P) + nchunk_scan(P) + 64; }
// rounded to 256 B so that one fill clears each region
size_t geom_zero_words(int P) { return align_up(geom_hist_off(P) + kHistWords, 64); }
// binning: counters ([0] = L', written by the last emission chunk) | the tile sort's look-back words
// (zeroed by the emission kernel, which runs before the sort): the binning buffer needs no memset
static size_t bin_look_off() { return 64; }
size_t binning_zero_words(int L, int T) {
    (void)T;
    return align_up(bin_look_off() + (size_t)kMaxPasses * 256 * sort_nblk(L, kSortThreads * kItemsL), 64);
}
size_t max_emit_chunks(int P, int T) {
    // L < 2^30 is enforced by the caller
    const size_t bound = ((size_t)P * (size_t)T + kEmitChunk - 1) / kEmitChunk;
    return std::min<size_t>(bound, ((size_t)1 << 30) / kEmitChunk) + 1;
}

// Counting binning (see the header): chunks of kCountThreads * ITEMS emission slots.
constexpr int kCountThreads = 1024;
constexpr int kCountMaxT = 16384;  // LDS bins of one chunk (64 KiB)
constexpr int kColWaves = 16, kColPer = 32;  // column scan: 16 waves x 32 chunks per lane
int count_items(int L, int T) {
    // GS4D_BINNING=radix: the radix-sort binning everywhere (A/B diagnostics; read once per process,
    // so a forward and its backward always agree on the buffer layout)
    static const char *force = getenv("GS4D_BINNING");
    static const char *min_items = getenv("GS4D_COUNT_MIN_ITEMS");  // A/B diagnostics: 4, 8 (default), 16
    if (force && strcmp(force, "radix") == 0) return 0;
    if (min_items && atoi(min_items) != 4 && atoi(min_items) != 8 && atoi(min_items) != 16) return 0;
    if (T > kCountMaxT || L <= 0) return 0;
    for (int items = min_items ? atoi(min_items) : 8; items <= 16; items *= 2)
        if (sort_nblk(L, kCountThreads * items) <= kColWaves * kColPer) return items;
    return 0;
}
size_t tile_hist_words(int L, int T) {
    const int items = count_items(L, T);
    return items ? (size_t)sort_nblk(L, kCountThreads * items) * (size_t)T : 0;
}

// Exclusive 256-thread workgroup scan: returns this thread's exclusive prefix inside the workgroup
// and (in *total) the workgroup sum.
__device__ __forceinline__ uint32_t wg_exclusive(uint32_t v, uint32_t *s_w, uint32_t *total) {
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const uint32_t x = wave_incl_sum(v);
    __syncthreads();
    if (lane == 63) s_w[w] = x;
    __syncthreads();
    uint32_t before = 0, t = 0;
#pragma unroll
    for (int q = 0; q < 4; q++) {
        before += q < w ? s_w[q] : 0u;
        t += s_w[q];
    }
    *total = t;
    return before + x - v;
}

// K2 replacement: visible Gaussians in id order and their candidate numbering.
// vis_gid[v] = id of the v-th visible Gaussian; cand_off[v] = its first candidate (cand_off[V] = L);
// first_vis[j] = the visible index owning candidate j * kEmitChunk.
__global__ __launch_bounds__(256) void visible_scan_kernel(GeomState g, int P, uint32_t jmax) {
    __shared__ uint32_t s_w[4], s_tmp[4];
    const uint32_t b = blockIdx.x;
    const int i0 = ((int)b * 256 + threadIdx.x) * kScanPer;  // this thread's kScanPer consecutive Gaussians
    uint32_t t[kScanPer], vsum = 0, asum = 0;
#pragma unroll
    for (int k = 0; k < kScanPer; k++) {
        t[k] = i0 + k < P ? g.tiles_touched[i0 + k] : 0u;
        vsum += t[k] > 0;
        asum += t[k];
    }
    uint32_t vtot, atot;
    const uint32_t vx = wg_exclusive(vsum, s_w, &vtot);
    const uint32_t ax = wg_exclusive(asum, s_w, &atot);
    uint32_t *vchain = g.zero + geom_vis_chain_off(), *achain = g.zero + geom_area_chain_off(P);
    const uint32_t vpre = block_prefix(vchain + 64, b, vtot, vchain + 1, s_tmp);
    const uint32_t apre = block_prefix(achain + 64, b, atot, achain + 1, s_tmp);
    uint32_t v = vpre + vx, run = apre + ax;
#pragma unroll
    for (int k = 0; k < kScanPer; k++) {
        const int idx = i0 + k;
        if (idx >= P) break;
        if (t[k] > 0) {
            g.vis_gid[v] = (uint32_t)idx;
            g.cand_off[v] = run;
            // emission chunks starting inside this Gaussian's candidates
            for (uint32_t j = (run + kEmitChunk - 1) / kEmitChunk; j * (uint32_t)kEmitChunk < run + t[k] && j < jmax;
                 j++)
                g.first_vis[j] = v;
            v++;
        }
        run += t[k];
        if (idx == P - 1) {
            g.cand_off[v] = run;  // cand_off[V] = num_rendered
            g.zero[kZeroV] = v;   // V
        }
    }
    // the last workgroup knows L (its inclusive area prefix): it clears the emission's chunk-prefix
    // chain for the nchunk_emit(L) chunks of this call (the emission runs after this kernel)
    if (b == gridDim.x - 1) {
        const uint32_t L = apre + atot;
        const uint32_t n = min((uint32_t)((L + kEmitChunk - 1) / kEmitChunk), jmax) + 64;
        for (uint32_t i = threadIdx.x; i < n; i += 256) g.emit_chain[i] = 0u;
    }
}

hipError_t launch_visible_scan(const Args &a, GeomState g, hipStream_t s) {
    hipLaunchKernelGGL(visible_scan_kernel, dim3((unsigned)nchunk_scan(a.P)), dim3(256), 0, s, g, a.P,
                       (uint32_t)max_emit_chunks(a.P, a.gx * a.gy));
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// K3: load-balanced emission.  Workgroup j takes candidates [j*2048, +2048) of the candidate sequence
// (visible Gaussians in id order, each its rectangle row-major); lane t owns 8 consecutive ones.
// Their owning Gaussians come from a load-balancing search in LDS: each Gaussian starting inside the
// chunk marks its first slot, and a max-scan spreads the marks.  Each candidate is tested with
// half_reach; the reached ones are compacted in candidate order: keys[e] = tile, gid_by_e[e] =
// Gaussian | reach bits.  Emission offsets are chained by look-back; the last chunk stores L'.  Also
// accumulated: n_inst[g] and the per-tile instance counts (integer atomics).
__global__ __launch_bounds__(256) void emit_instances_kernel(Args a, GeomState g, const int *__restrict__ radii,
                                                             int L, int npass, uint32_t *__restrict__ keys,
                                                             uint32_t *__restrict__ gid_by_e,
                                                             uint32_t *__restrict__ zero, uint2 *__restrict__ ranges,
                                                             int T, uint32_t *__restrict__ look, int nlook) {
    // the tile ranges start empty (tile_ranges_kernel writes the non-empty ones) and the tile sort's
    // look-back words start at zero: both cleared here instead of by memset launches of their own
    for (int i = blockIdx.x * 256 + threadIdx.x; i < T; i += gridDim.x * 256) ranges[i] = make_uint2(0u, 0u);
    for (int i = blockIdx.x * 256 + threadIdx.x; i < nlook; i += gridDim.x * 256) look[i] = 0u;
    __shared__ uint32_t s_own[kEmitChunk];
    __shared__ uint32_t s_off[kEmitChunk + 2];
    // s_n: kept candidates before each candidate of the chunk (after the tests); during the tests the same
    // words hold the chunk's Gaussians' attributes when there are at most kEmitStage of them (the common
    // case: each candidate then reads its Gaussian from LDS, not by two dependent global gathers)
    __shared__ __attribute__((aligned(16))) uint32_t s_n[kEmitChunk + 4];
    __shared__ uint32_t s_ggid[kEmitStage];
    float4 *s_gco = reinterpret_cast<float4 *>(s_n);                  // [kEmitStage]
    float2 *s_gxy = reinterpret_cast<float2 *>(s_gco + kEmitStage);   // [kEmitStage]
    int *s_grad = reinterpret_cast<int *>(s_gxy + kEmitStage);        // [kEmitStage]
    __shared__ uint32_t s_hist[kMaxPasses][256];
    __shared__ uint32_t s_w[4], s_tmp[4];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const uint32_t b = blockIdx.x;
    const uint32_t c0 = b * kEmitChunk;
    const uint32_t c1 = min((uint32_t)L, c0 + kEmitChunk);
    const int V = (int)(g.zero[kZeroV]);
    const int rlo = (int)g.first_vis[b];
    // the chunk's Gaussians: first_vis[b] .. first_vis[b + 1] (the owner of candidate c1); the last
    // chunk's run to V.  Visible Gaussians starting at or after c1 are ignored.
    const int rhi = c1 < (uint32_t)L ? (int)g.first_vis[b + 1] + 1 : V;
    const int nr = min(rhi - rlo, kEmitChunk + 1);
    const bool staged = nr <= kEmitStage;  // workgroup-uniform
    for (int i = tid; i < kEmitChunk; i += 256) s_own[i] = 0;
    for (int i = tid; i < kMaxPasses * 256; i += 256) (&s_hist[0][0])[i] = 0;
    __syncthreads();
    for (int i = tid; i < nr; i += 256) {
        const uint32_t st = g.cand_off[rlo + i];
        s_off[i] = st;
        if (st > c0 && st < c1) s_own[st - c0] = (uint32_t)i;
        if (staged) {
            const uint32_t gi = g.vis_gid[rlo + i];
            s_ggid[i] = gi;
            s_gxy[i] = g.xy[gi];
            s_gco[i] = g.conic_opacity[gi];
            s_grad[i] = radii[gi];
        }
    }
    if (tid == 0) s_off[nr] = g.cand_off[rlo + nr];
    __syncthreads();
    // inclusive max-scan of the marks over the lane's 8 slots, then across lanes
    uint32_t own[kEmitPer];
    uint32_t mx = 0;
#pragma unroll
    for (int k = 0; k < kEmitPer; k++) {
        mx = max(mx, s_own[tid * kEmitPer + k]);
        own[k] = mx;
    }
    {
        const uint32_t x = wave_incl_max(mx);
        if (lane == 63) s_w[w] = x;
        __syncthreads();
        uint32_t carry = dpp_src<0x138, 0xF>(x);  // wave_shr:1 (lane 0 reads 0)
        for (int q = 0; q < w; q++) carry = max(carry, s_w[q]);
#pragma unroll
        for (int k = 0; k < kEmitPer; k++) own[k] = max(own[k], carry);
    }
    // test the candidates (every gather issued before the first test)
    float2 xy[kEmitPer];
    float4 co[kEmitPer];
    int rad[kEmitPer];
    uint32_t gid[kEmitPer];
    if (staged) {
#pragma unroll
        for (int k = 0; k < kEmitPer; k++) {
            const int i = min((int)own[k], nr - 1);
            gid[k] = s_ggid[i];
            xy[k] = s_gxy[i];
            co[k] = s_gco[i];
            rad[k] = s_grad[i];
        }
    } else {
#pragma unroll
        for (int k = 0; k < kEmitPer; k++) {
            gid[k] = g.vis_gid[min(rlo + (int)own[k], V - 1)];
            xy[k] = g.xy[gid[k]];
            co[k] = g.conic_opacity[gid[k]];
            rad[k] = radii[gid[k]];
        }
    }
    uint32_t tile[kEmitPer], reach[kEmitPer];
    uint32_t keep = 0;
#pragma unroll
    for (int k = 0; k < kEmitPer; k++) {
        const uint32_t c = c0 + tid * kEmitPer + k;
        tile[k] = 0;
        reach[k] = 0;
        if (c < c1) {
            const int i = (int)own[k];
            int x0, y0, x1, y1;
            getRect(xy[k].x, xy[k].y, rad[k], a.gx, a.gy, x0, y0, x1, y1);
            // row-major position in the rect: local = qd * wdt + rm by a float reciprocal and one
            // correction step (exact for local < 2^20, i.e. for grids of fewer than 2^20 tiles; larger
            // grids take the integer division)
            const int local = (int)(c - s_off[i]), wdt = x1 - x0;
            int qd, rm;
            if (a.exact_div) {
                qd = local / wdt;
                rm = local - qd * wdt;
            } else {
                qd = (int)((float)local * __builtin_amdgcn_rcpf((float)wdt));
                rm = local - qd * wdt;
                if (rm < 0) { qd--; rm += wdt; }
                else if (rm >= wdt) { qd++; rm -= wdt; }
            }
            const int ty = y0 + qd, tx = x0 + rm;
            reach[k] = half_reach(xy[k].x, xy[k].y, co[k], tx, ty, a.W, a.H);
            if (reach[k] != 0) {
                keep |= 1u << k;
                tile[k] = (uint32_t)(ty * a.gx + tx);
                for (int p = 0; p < npass; p++) atomicAdd(&s_hist[p][(tile[k] >> (8 * p)) & 0xFFu], 1u);
            }
        }
    }
    // compaction offsets: exclusive scan of the per-lane counts, chunk total chained by look-back
    const uint32_t cnt = __popc(keep);
    const uint32_t x = wave_incl_sum(cnt);
    __syncthreads();
    if (lane == 63) s_w[w] = x;
    __syncthreads();
    uint32_t before = 0, total = 0;
#pragma unroll
    for (int q = 0; q < 4; q++) {
        before += q < w ? s_w[q] : 0u;
        total += s_w[q];
    }
    uint32_t *chain = g.emit_chain;  // cleared by visible_scan
    const uint32_t prefix = block_prefix(chain + 64, b, total, chain + 1, s_tmp);
    if (tid == 0 && c1 == (uint32_t)L) zero[0] = prefix + total;  // L'
    uint32_t e = prefix + before + x - cnt;
#pragma unroll
    for (int k = 0; k < kEmitPer; k++) {
        if ((keep >> k) & 1u) {
            keys[e] = tile[k];
            gid_by_e[e] = gid[k] | (reach[k] << kReachShift);
            e++;
        }
    }
    // n_inst: a Gaussian's candidates are consecutive, so its kept count in this chunk is a difference
    // of the chunk-local kept prefix at the ends of its candidate range (no per-candidate atomics)
    {
        uint32_t run = before + x - cnt;
#pragma unroll
        for (int k = 0; k < kEmitPer; k++) {
            s_n[tid * kEmitPer + k] = run;
            run += (keep >> k) & 1u;
        }
        if (tid == 255) s_n[kEmitChunk] = run;  // the chunk total
    }
    __syncthreads();
    for (int i = tid; i < nr; i += 256) {
        const uint32_t lo = max(s_off[i], c0) - c0, hi = min(s_off[i + 1], c1) - c0;
        const uint32_t n = hi > lo ? s_n[hi] - s_n[lo] : 0u;
        if (n) atomicAdd(&g.n_inst[staged ? s_ggid[i] : g.vis_gid[rlo + i]], n);
    }
    uint32_t *hist = g.zero + geom_hist_off(a.P) + (b % kHistShards) * (kMaxPasses * 256);
    for (int p = 0; p < npass; p++)
        if (s_hist[p][tid]) atomicAdd(&hist[p * 256 + tid], s_hist[p][tid]);
}

// K5: tile ranges from the sorted tile keys (rasterizer_impl.cu:116-138); tiles without instances keep
// the (0, 0) of the memset.
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

// ---- Counting binning ---------------------------------------------------------------------------
// tile_count: chunk c's tile histogram, hist[c][t] (chunks past L' exit at once).
template <int ITEMS>
__global__ __launch_bounds__(kCountThreads) void tile_count_kernel(const uint32_t *__restrict__ keys,
                                                                   const uint32_t *__restrict__ n_dev, int T,
                                                                   uint32_t *__restrict__ hist) {
    extern __shared__ uint32_t s_bin[];
    const int n = count_of(0, n_dev), tid = threadIdx.x;
    const size_t c0 = (size_t)blockIdx.x * (kCountThreads * ITEMS);
    if (c0 >= (size_t)n) return;
    uint32_t key[ITEMS];
#pragma unroll
    for (int r = 0; r < ITEMS; r++) {
        const size_t i = c0 + (size_t)r * kCountThreads + tid;
        key[r] = i < (size_t)n ? keys[i] : ~0u;
    }
    for (int t = tid; t < T; t += kCountThreads) s_bin[t] = 0;
    __syncthreads();
#pragma unroll
    for (int r = 0; r < ITEMS; r++)
        if (key[r] != ~0u) atomicAdd(&s_bin[key[r]], 1u);
    __syncthreads();
    uint32_t *h = hist + (size_t)blockIdx.x * T;
    for (int t = tid; t < T; t += kCountThreads) h[t] = s_bin[t];
}

// tile_scan: workgroup g owns tiles [64 g, 64 g + 64), lane l tile 64 g + l; wave w the chunks
// [w per, (w + 1) per).  Rewrites hist[c][t] in place as the exclusive offset of (t, c) in
// tile-major order -- the global start of chunk c's share of tile t -- and writes ranges[t]
// (rasterizer_impl.cu:116-138's result; empty tiles (0, 0)).  The tile groups' totals are chained
// by the published-count prefix of radix_sort.h (look: zeroed words, one per group).
__global__ __launch_bounds__(kCountThreads) void tile_scan_kernel(uint32_t *__restrict__ hist,
                                                                  const uint32_t *__restrict__ n_dev, int T, int chunk,
                                                                  uint2 *__restrict__ ranges,
                                                                  uint32_t *__restrict__ look, uint32_t *__restrict__ err) {
    __shared__ uint32_t s_col[kColWaves][64];
    __shared__ uint32_t s_base[64];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int n = count_of(0, n_dev);
    const int nc = (n + chunk - 1) / chunk;
    const int t = blockIdx.x * 64 + lane;
    const bool tv = t < T;
    const int per = (nc + kColWaves - 1) / kColWaves;
    const int cb = w * per;
    uint32_t v[kColPer];
#pragma unroll
    for (int k = 0; k < kColPer; k++) {
        const int c = cb + k;
        v[k] = (k < per && c < nc && tv) ? hist[(size_t)c * T + t] : 0u;
    }
    uint32_t run = 0;
#pragma unroll
    for (int k = 0; k < kColPer; k++) {
        const uint32_t x = v[k];
        v[k] = run;
        run += x;
    }
    s_col[w][lane] = run;
    __syncthreads();
    uint32_t before = 0, tot = 0;
#pragma unroll
    for (int q = 0; q < kColWaves; q++) {
        const uint32_t x = s_col[q][lane];
        before += q < w ? x : 0u;
        tot += x;
    }
    if (w == 0) {
        const uint32_t x = wave_incl_sum(tot);  // inclusive scan of the group's tile totals
        const uint32_t gsum = __shfl(x, 63);
        if (lane == 0) store_word(look + blockIdx.x, kAgg | gsum);
        uint32_t lower = sum_published(look, 1, (int)blockIdx.x, lane, 64, err);
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) lower += __shfl_xor(lower, off);
        const uint32_t base = lower + x - tot;
        s_base[lane] = base;
        if (tv) ranges[t] = tot ? make_uint2(base, base + tot) : make_uint2(0u, 0u);
    }
    __syncthreads();
    const uint32_t base = s_base[lane] + before;
#pragma unroll
    for (int k = 0; k < kColPer; k++) {
        const int c = cb + k;
        if (k < per && c < nc && tv) hist[(size_t)c * T + t] = base + v[k];
    }
}

// tile_scatter: chunk c's offsets into LDS, one fetch-add per instance places its emission slot in
// its tile's run (the order inside the run is the arbitrary order of the LDS atomics: see the header).
// A tile's run holds each chunk's share (~1.5 slots at the metric config) in chunk order, so with chunk =
// workgroup the 4-byte writes of one 64-byte line came from workgroups dealt round-robin to all 8 XCDs,
// each L2 writing its partial line back (~8x write amplification).  Chunks are mapped so that each XCD
// takes one contiguous range of them (workgroups b and b + 8 share an XCD: MI355X_MICROARCH.md, dispatch;
// speed only, any mapping is correct): a tile's run is then written by at most 8 XCDs in 8 pieces.
__device__ __forceinline__ int xcd_chunk(int b, int nblk) {
    const int q = nblk >> 3, r = nblk & 7, x = b & 7, j = b >> 3;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + j;
}
template <int ITEMS>
__global__ __launch_bounds__(kCountThreads) void tile_scatter_kernel(const uint32_t *__restrict__ keys,
                                                                     const uint32_t *__restrict__ n_dev, int T,
                                                                     const uint32_t *__restrict__ offs,
                                                                     uint32_t *__restrict__ upos) {
    extern __shared__ uint32_t s_off[];
    const int n = count_of(0, n_dev), tid = threadIdx.x;
    const int chunk = xcd_chunk((int)blockIdx.x, (int)gridDim.x);
    const size_t c0 = (size_t)chunk * (kCountThreads * ITEMS);
    if (c0 >= (size_t)n) return;
    uint32_t key[ITEMS];
#pragma unroll
    for (int r = 0; r < ITEMS; r++) {
        const size_t i = c0 + (size_t)r * kCountThreads + tid;
        key[r] = i < (size_t)n ? keys[i] : ~0u;
    }
    const uint32_t *h = offs + (size_t)chunk * T;
    for (int t = tid; t < T; t += kCountThreads) s_off[t] = h[t];
    __syncthreads();
#pragma unroll
    for (int r = 0; r < ITEMS; r++)
        if (key[r] != ~0u) upos[atomicAdd(&s_off[key[r]], 1u)] = (uint32_t)(c0 + (size_t)r * kCountThreads + tid);
}

template <int ITEMS>
static void launch_counting(const BinningState &b, int L, int T, ImageState img, uint32_t *look, uint32_t *err,
                            hipStream_t s) {
    constexpr int C = kCountThreads * ITEMS;
    const int nblk = sort_nblk(L, C);
    const uint32_t *n_dev = b.scratch;
    const size_t lds = 4 * (size_t)T;
    hipLaunchKernelGGL(tile_count_kernel<ITEMS>, dim3(nblk), dim3(kCountThreads), lds, s, b.keys[0], n_dev, T,
                       b.tile_hist);
    hipLaunchKernelGGL(tile_scan_kernel, dim3((T + 63) / 64), dim3(kCountThreads), 0, s, b.tile_hist, n_dev, T, C,
                       img.ranges, look, err);
    hipLaunchKernelGGL(tile_scatter_kernel<ITEMS>, dim3(nblk), dim3(kCountThreads), lds, s, b.keys[0], n_dev, T,
                       b.tile_hist, b.upos);
}

// ---- K4: per-tile sort by (depth bits, Gaussian id) -------------------------------------------------
// Bitonic network in its all-ascending ("flip") form: for k = 2, 4, ..: compare i with i ^ (k-1)
// (flip), then for j = k/4 .. 1 with i ^ j.  Every comparison sends the smaller key to the lower
// index, so a length n that is not a power of two is padded virtually with +inf: a pair whose
// partner lies at or beyond n is left alone.
struct TileSortLds {
    uint64_t key[kSortCap];
    uint32_t val[kSortCap];
};

__device__ __forceinline__ uint64_t inst_key(uint32_t e, const uint32_t *__restrict__ gid_by_e,
                                             const float *__restrict__ depths) {
    const uint32_t gid = gid_by_e[e] & kGidMask;
    return ((uint64_t)__float_as_uint(depths[gid]) << 32) | gid;  // positive depths order as their bits
}

// Steps (k, j) for k = k_lo .. k_hi (j from j_top for the first k, from k/2 otherwise) over an
// LDS-resident index space of `space` (a power of two) holding n valid elements.
__device__ void lds_network(TileSortLds &s, int n, int space, int k_lo, int k_hi, int j_top) {
    for (int k = k_lo; k <= k_hi; k <<= 1) {
        for (int j = (k == k_lo ? j_top : k >> 1); j >= 1; j >>= 1) {
            const bool flip = j == (k >> 1);
            for (int p = threadIdx.x; p < (space >> 1); p += blockDim.x) {
                const int i = (p / j) * 2 * j + (p % j);  // bit j of i clear
                const int q = flip ? (i ^ (k - 1)) : (i + j);
                if (q >= n) continue;
                const uint64_t a = s.key[i], b = s.key[q];
                if (b < a) {
                    s.key[i] = b;
                    s.key[q] = a;
                    const uint32_t t = s.val[i];
                    s.val[i] = s.val[q];
                    s.val[q] = t;
                }
            }
            __syncthreads();
        }
    }
}

// Runs of kWaveSortMax < n <= 2048 instances (one 256-thread workgroup): each wave sorts 256-key chunks
// in registers (the bitonic network of the forward's short-run sort, lane l holding chunk positions
// l, 64 + l, ..), then merge-path rounds in LDS double the sorted runs up to the power of two >= n:
// every thread emits total / 256 consecutive outputs of its pair of runs, its start found by a binary
// search on its diagonal, the last round straight into the segment.  Chunks past n are +inf keys
// (already in order).  O(n log n) compare-selects against the bitonic network's O(n log^2 n): a bitonic
// block sort at n = 2048 spent 66 network steps of 8 registers per thread.
__device__ __forceinline__ void wave_sort256(uint64_t key[4], int lane) {
#pragma unroll
    for (int k = 2; k <= 256; k <<= 1) {
#pragma unroll
        for (int j = k >> 1; j >= 1; j >>= 1) {
            const int mask = j == (k >> 1) ? k - 1 : j;  // flip, then half-cleaners
            const int lx = mask & 63, rx = mask >> 6;
            uint64_t pk[4];
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const int rq = r ^ rx;
                if (lx == 0) {
                    pk[r] = key[rq];
                } else {
                    const uint32_t hi = xor_lane((uint32_t)(key[rq] >> 32), lx);
                    const uint32_t lo = xor_lane((uint32_t)key[rq], lx);
                    pk[r] = ((uint64_t)hi << 32) | lo;
                }
            }
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const bool lower = ((r * 64 + lane) & j) == 0;
                const uint64_t kr = key[r];
                key[r] = lower ? (pk[r] < kr ? pk[r] : kr) : (pk[r] > kr ? pk[r] : kr);
            }
        }
    }
}

__device__ void merge_sort_run(uint32_t *__restrict__ seg, int n, const uint32_t *__restrict__ gid_by_e,
                               const float *__restrict__ depths, uint64_t *__restrict__ s_x) {
    const int lane = threadIdx.x & 63, w = (int)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    int total = 512;
    while (total < n) total <<= 1;  // 512, 1024 or 2048
    uint64_t *src = s_x, *dst = s_x + 2048;
    for (int c = w; c < total / 256; c += 4) {
        uint64_t key[4];
#pragma unroll
        for (int r = 0; r < 4; r++) {
            const int i = c * 256 + r * 64 + lane;
            const uint32_t e = i < n ? seg[i] : 0u;
            const uint32_t gid = i < n ? gid_by_e[e] & kGidMask : 0u;
            key[r] = i < n ? ((uint64_t)__float_as_uint(depths[gid]) << 32) | e : ~0ull;  // depths > 0.2
        }
        if (c * 256 < n) wave_sort256(key, lane);
#pragma unroll
        for (int r = 0; r < 4; r++) src[c * 256 + r * 64 + lane] = key[r];
    }
    __syncthreads();
    const int per = total >> 8;  // outputs per thread
    const int o0 = threadIdx.x * per;
    for (int wd = 256; wd < total; wd <<= 1) {
        const bool last = 2 * wd == total;
        const int p0 = o0 & ~(2 * wd - 1), d = o0 - p0;  // this thread's pair of runs, its diagonal
        const uint64_t *r1 = src + p0, *r2 = src + p0 + wd;
        int lo = max(0, d - wd), hi = min(d, wd);
        while (lo < hi) {  // ties (the +inf padding only) go to the first run, as below
            const int mid = (lo + hi) >> 1;
            if (r1[mid] > r2[d - 1 - mid]) hi = mid;
            else lo = mid + 1;
        }
        int i = lo, j = d - lo;
        uint64_t x = i < wd ? r1[i] : ~0ull, y = j < wd ? r2[j] : ~0ull;
        for (int k = 0; k < per; k++) {
            const bool first = x <= y;
            const uint64_t v = first ? x : y;
            if (last) {
                if (o0 + k < n) seg[o0 + k] = (uint32_t)v;
            } else {
                dst[o0 + k] = v;
            }
            if (first) {
                i++;
                x = i < wd ? r1[i] : ~0ull;
            } else {
                j++;
                y = j < wd ? r2[j] : ~0ull;
            }
        }
        __syncthreads();
        uint64_t *t = src;
        src = dst;
        dst = t;
    }
}

// The blend kernels run one wave per tile, more waves than fit on the chip at once: the last ones to
// start run at low occupancy, so a long tile started late ends the kernel late.  tile_order_kernel
// (one workgroup) orders the tiles longest run first (a counting sort on min(run, 1023), the order
// inside a length arbitrary: it only schedules, every tile's result is its own).
constexpr int kOrderBins = 1024, kOrderBatch = 8;
__device__ void order_tiles(const uint2 *__restrict__ ranges, int T, uint32_t *__restrict__ order, uint32_t *s_bin) {
    const int tid = threadIdx.x, nt = blockDim.x;
    for (int i = tid; i < kOrderBins; i += nt) s_bin[i] = 0;
    __syncthreads();
    // kOrderBatch tiles per thread per round, their loads all in flight before the first use
    auto bins_of = [&](int base, int bin[kOrderBatch]) {
        uint2 r[kOrderBatch];
#pragma unroll
        for (int k = 0; k < kOrderBatch; k++) {
            const int t = base + k * nt + tid;
            r[k] = t < T ? ranges[t] : make_uint2(0u, 0u);
        }
#pragma unroll
        for (int k = 0; k < kOrderBatch; k++)  // longest first
            bin[k] = kOrderBins - 1 - (int)min(r[k].y - r[k].x, (uint32_t)(kOrderBins - 1));
    };
    // up to kOrderBatch * nt tiles (8192 at 1024 threads) keep their bins in registers between the
    // histogram and the scatter; larger grids load their ranges again
    const bool one_round = T <= kOrderBatch * nt;
    int bin0[kOrderBatch];
    for (int base = 0; base < T; base += kOrderBatch * nt) {
        int bin[kOrderBatch];
        bins_of(base, bin);
#pragma unroll
        for (int k = 0; k < kOrderBatch; k++) {
            if (base + k * nt + tid < T) atomicAdd(&s_bin[bin[k]], 1u);
            bin0[k] = bin[k];
        }
    }
    __syncthreads();
    if (tid < 64) {  // exclusive scan of the bins by one wave, 16 bins per lane
        constexpr int per = kOrderBins / 64;
        uint32_t v[per], sum = 0;
#pragma unroll
        for (int k = 0; k < per; k++) { v[k] = s_bin[tid * per + k]; sum += v[k]; }
        uint32_t incl = sum;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const uint32_t o = __shfl_up(incl, off);
            if (tid >= off) incl += o;
        }
        uint32_t run = incl - sum;
#pragma unroll
        for (int k = 0; k < per; k++) { s_bin[tid * per + k] = run; run += v[k]; }
    }
    __syncthreads();
    for (int base = 0; base < T; base += kOrderBatch * nt) {
        int bin[kOrderBatch];
        if (one_round) {
#pragma unroll
            for (int k = 0; k < kOrderBatch; k++) bin[k] = bin0[k];
        } else {
            bins_of(base, bin);
        }
#pragma unroll
        for (int k = 0; k < kOrderBatch; k++) {
            const int t = base + k * nt + tid;
            if (t < T) order[atomicAdd(&s_bin[bin[k]], 1u)] = (uint32_t)t;
        }
    }
}

__global__ __launch_bounds__(1024) void tile_order_kernel(const uint2 *__restrict__ ranges, int T,
                                                          uint32_t *__restrict__ order) {
    __shared__ uint32_t s_bin[kOrderBins];
    order_tiles(ranges, T, order, s_bin);
}

// Tiles with more than kWaveSortMax instances (shorter runs are sorted in registers by the render
// forward): one workgroup each (workgroup t + 1 for tile t).  Up to 2048: wave sorts + merge path
// (merge_sort_run); longer: runs of kSortCap in LDS merged by the bitonic network's global steps.  Workgroup 0
// orders the tiles (order_tiles), so one launch does both (a launch costs ~4 us of the timeline).
__global__ __launch_bounds__(256) void tile_sort_kernel(const uint2 *__restrict__ ranges, int T,
                                                        uint32_t *__restrict__ order,
                                                        const uint32_t *__restrict__ gid_by_e,
                                                        const float *__restrict__ depths, uint32_t *__restrict__ upos,
                                                        uint32_t *__restrict__ tkey_hi, uint32_t *__restrict__ tkey_lo) {
    // 32 KiB of LDS, five workgroups per CU: the merge path's two 2048-key buffers, or a long tile's
    // 2048-key run (TileSortLds, 24 KiB).  (A 48 KiB layout for 4096-key LDS runs held three per CU; this
    // kernel is latency-bound per workgroup -- dependent key gathers, binary searches, barriers -- so the
    // runs of 257..2048 that dominate a training scene want the occupancy.)
    __shared__ uint64_t s_mem[2 * kSortCap];
    TileSortLds &s = *reinterpret_cast<TileSortLds *>(s_mem);
    if (blockIdx.x == 0) {
        order_tiles(ranges, T, order, reinterpret_cast<uint32_t *>(s_mem));
        return;
    }
    const uint2 r = ranges[blockIdx.x - 1];
    const int n = (int)(r.y - r.x);
    if (n <= kWaveSortMax) return;  // the render forward sorts these
    uint32_t *seg = upos + r.x;
    if (n <= kSortCap) {
        merge_sort_run(seg, n, gid_by_e, depths, s_mem);
        return;
    }
    // long tile: sort runs of kSortCap in LDS, then continue the network with its global steps
    // (stride >= kSortCap) on the segment's keys in tkey_hi/lo (free binning buffers) and its LDS
    // steps (stride < kSortCap) run by run.
    uint32_t *khi = tkey_hi + r.x, *klo = tkey_lo + r.x;
    int m = 1;
    while (m < n) m <<= 1;
    auto load_run = [&](int base, bool from_keys) {
        const int cnt = min(kSortCap, n - base);
        for (int i = threadIdx.x; i < cnt; i += blockDim.x) {
            const uint32_t e = seg[base + i];
            s.key[i] = from_keys ? (((uint64_t)khi[base + i] << 32) | klo[base + i]) : inst_key(e, gid_by_e, depths);
            s.val[i] = e;
        }
        __syncthreads();
        return cnt;
    };
    auto store_run = [&](int base, int cnt) {
        for (int i = threadIdx.x; i < cnt; i += blockDim.x) {
            seg[base + i] = s.val[i];
            khi[base + i] = (uint32_t)(s.key[i] >> 32);
            klo[base + i] = (uint32_t)s.key[i];
        }
        __syncthreads();
    };
    for (int base = 0; base < n; base += kSortCap) {
        const int cnt = load_run(base, false);
        lds_network(s, cnt, kSortCap, 2, kSortCap, 1);
        store_run(base, cnt);
    }
    for (int k = 2 * kSortCap; k <= m; k <<= 1) {
        for (int j = k >> 1; j >= kSortCap; j >>= 1) {
            const bool flip = j == (k >> 1);
            for (int p = threadIdx.x; p < (m >> 1); p += blockDim.x) {
                const int i = (p / j) * 2 * j + (p % j);
                const int q = flip ? (i ^ (k - 1)) : (i + j);
                if (i >= n || q >= n) continue;
                const uint64_t a = ((uint64_t)khi[i] << 32) | klo[i], b = ((uint64_t)khi[q] << 32) | klo[q];
                if (b < a) {
                    khi[i] = (uint32_t)(b >> 32); klo[i] = (uint32_t)b;
                    khi[q] = (uint32_t)(a >> 32); klo[q] = (uint32_t)a;
                    const uint32_t t = seg[i];
                    seg[i] = seg[q];
                    seg[q] = t;
                }
            }
            __syncthreads();
        }
        for (int base = 0; base < n; base += kSortCap) {
            const int cnt = load_run(base, true);
            lds_network(s, cnt, kSortCap, k, k, kSortCap >> 1);
            store_run(base, cnt);
        }
    }
}

hipError_t launch_binning(const Args &a, GeomState g, const int *radii, BinningState b, int L, ImageState img,
                          hipStream_t s) {
    const int T = a.gx * a.gy;
    if (L == 0) {
        hipError_t e = hipMemsetAsync(img.ranges, 0, sizeof(uint2) * (size_t)T, s);
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL(tile_order_kernel, dim3(1), dim3(1024), 0, s, img.ranges, T, img.order);
        return hipGetLastError();
    }
    uint32_t *look = b.scratch + bin_look_off();
    uint32_t *err = g.emit_chain + 1;
    if (b.count_items) {
        // counting binning: no digit histograms, the tile scan writes every range and uses (T + 63) / 64
        // look-back words
        hipLaunchKernelGGL(emit_instances_kernel, dim3((unsigned)nchunk_emit(L)), dim3(256), 0, s, a, g, radii, L, 0,
                           b.keys[0], b.gid_by_e, b.scratch, img.ranges, 0, look, (T + 63) / 64);
        if (b.count_items == 4) launch_counting<4>(b, L, T, img, look, err, s);
        else if (b.count_items == 8) launch_counting<8>(b, L, T, img, look, err, s);
        else launch_counting<16>(b, L, T, img, look, err, s);
    } else {
        const int npass = (b.key_bits + 7) / 8;
        const int nlook = npass * 256 * sort_nblk(L, kSortThreads * kItemsL);
        hipLaunchKernelGGL(emit_instances_kernel, dim3((unsigned)nchunk_emit(L)), dim3(256), 0, s, a, g, radii, L,
                           npass, b.keys[0], b.gid_by_e, b.scratch, img.ranges, T, look, nlook);
        const uint32_t *n_dev = b.scratch;  // L' <= L reached instances
        uint32_t *keys[2] = {b.keys[0], b.keys[1]};
        uint32_t *vals[2] = {b.vals[0], b.vals[1]};
        onesweep_sort<kSortThreads, kItemsL>(keys, vals, L, n_dev, b.key_bits, g.zero + geom_hist_off(a.P), look, err,
                                             s);
        hipLaunchKernelGGL(tile_ranges_kernel, dim3((L + 255) / 256), dim3(256), 0, s, b.sorted_keys, n_dev,
                           img.ranges);
    }
    hipLaunchKernelGGL(tile_sort_kernel, dim3(T + 1), dim3(256), 0, s, img.ranges, T, img.order, b.gid_by_e, g.depths,
                       b.upos, b.tmp_hi, b.tmp_lo);
    return hipGetLastError();
}

}  // namespace gs4d
