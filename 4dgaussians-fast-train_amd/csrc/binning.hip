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
//      splat actually reaches (half_reach, gs4d_internal.h) -- in one load-balanced stream
//      compaction pass: every workgroup takes a fixed number of candidates, whatever the splat sizes;
//   3. the emitted sequence is already depth-ordered, so a STABLE sort by tile id alone yields the
//      reference's (tile, depth, id) order: ceil(msb(T)/8) passes over u32 keys (2 at the metric
//      config instead of 6 over 12-byte pairs).
// Every pass is one launch.  Digit histograms are accumulated by the kernel that produces the keys
// (preprocess for depths, emission for tiles).  Scan, compaction and sort passes are single launches
// whose workgroups publish their chunk counts (one 32-bit status+count word per chunk and digit,
// agent-scope relaxed atomic stores and loads, so each word is its own flag) and sum the counts of
// all lower chunks directly (sum_published).
#include <algorithm>

#include "radix_sort.h"

namespace gs4d {

constexpr int kSortThreads = 1024;  // radix-sort workgroup: 16 waves rank one chunk together
constexpr int kItemsL = 8;     // keys per lane for the instance sort (8192 per workgroup)
constexpr int kItemsP = 4;     // keys per lane for the Gaussian depth sort (4096 per workgroup)
constexpr int kEmitPer = kEmitChunk / 256;  // candidates per lane in the emission pass

// ---------------------------------------------------------------------------------------------
// Zero-region layouts (u32 words).
static size_t nchunk_scan(int P) { return ((size_t)P + 255) / 256; }
static size_t nchunk_emit(int L) { return ((size_t)L + kEmitChunk - 1) / kEmitChunk; }
// geometry: counters | depth histograms | area-scan chain (+ err) | depth-sort look-back
__host__ __device__ static size_t geom_chain_off() { return kZeroHist + kHistWords; }
static size_t geom_look_off(int P) { return geom_chain_off() + nchunk_scan(P) + 64; }
// rounded to 256 B so that one fill kernel clears each region
size_t geom_zero_words(int P) { return align_up(geom_look_off(P) + (size_t)4 * 256 * sort_nblk(P, kSortThreads * kItemsP), 64); }
// binning: counters | tile histograms | emission chain (+ err) | instance-sort look-back
__host__ __device__ static size_t bin_chain_off() { return kZeroHist + kHistWords; }
static size_t bin_look_off(int L) { return bin_chain_off() + nchunk_emit(L) + 64; }
size_t binning_zero_words(int L) {
    return align_up(bin_look_off(L) + (size_t)kMaxPasses * 256 * sort_nblk(L, kSortThreads * kItemsL), 64);
}
size_t max_emit_chunks(int P, int T) {
    // L < 2^30 is enforced by the caller
    const size_t bound = ((size_t)P * (size_t)T + kEmitChunk - 1) / kEmitChunk;
    return std::min<size_t>(bound, ((size_t)1 << 30) / kEmitChunk) + 1;
}

// ---------------------------------------------------------------------------------------------
// Exclusive scan of the rect areas in depth-rank order: cand_off[r] = first candidate of rank r,
// cand_off[P] = num_rendered; and first_rank[j] = the rank owning candidate j * kEmitChunk.
// Rank-ordered splat records and the exclusive scan of the rect areas in depth-rank order:
// rank_geo[r] / rank_co[r] = the record of the Gaussian of depth rank r (gathered here with the whole
// chip's memory parallelism -- the sort's last pass runs on a few dozen workgroups only),
// cand_off[r] = its first candidate, cand_off[P] = num_rendered, first_rank[j] = the rank owning
// candidate j * kEmitChunk.  One rank per thread; chunk prefixes from the published counts.
__global__ __launch_bounds__(256) void rank_records_kernel(GeomState g, const int *__restrict__ radii, int n,
                                                           uint32_t jmax, uint32_t *__restrict__ chain) {
    __shared__ uint32_t s_w[4], s_tmp[4];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const uint32_t b = blockIdx.x;
    const int r = (int)b * 256 + tid;
    uint32_t v = 0;
    if (r < n) {
        const uint32_t gid = g.dvals[0][r];
        v = g.tiles_touched[gid];
        const float2 p = g.xy[gid];
        g.rank_geo[r] = make_float4(p.x, p.y, __int_as_float(radii[gid]), __uint_as_float(gid));
        g.rank_co[r] = g.conic_opacity[gid];
    }
    uint32_t x = v;
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
    const uint32_t prefix = block_prefix(chain + 64, b, total, chain + 1, s_tmp);
    const uint32_t run = prefix + before + x - v;
    if (r < n) {
        g.cand_off[r] = run;
        // chunk starts inside this rank's candidates
        for (uint32_t j = (run + kEmitChunk - 1) / kEmitChunk; j * (uint32_t)kEmitChunk < run + v && j < jmax; j++)
            g.first_rank[j] = (uint32_t)r;
        if (r == n - 1) g.cand_off[n] = run + v;
    }
}

hipError_t launch_depth_order(const Args &a, GeomState g, const int *radii, hipStream_t s) {
    // dkeys[0] = depth bits (unbinned: ~0u, last); afterwards dvals[0] = Gaussian id by depth rank
    uint32_t *keys[2] = {g.dkeys[0], g.dkeys[1]};
    uint32_t *vals[2] = {g.dvals[0], g.dvals[1]};
    uint32_t *chain = g.zero + geom_chain_off();
    onesweep_sort<kSortThreads, kItemsP>(keys, vals, a.P, nullptr, 32, g.zero + kZeroHist,
                                      g.zero + geom_look_off(a.P), chain + 1, s);
    hipLaunchKernelGGL(rank_records_kernel, dim3((unsigned)nchunk_scan(a.P)), dim3(256), 0, s, g, radii, a.P,
                       (uint32_t)max_emit_chunks(a.P, a.gx * a.gy), chain);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// K3: load-balanced emission.  Workgroup j takes candidates [j*2048, +2048) of the depth-ordered
// candidate sequence; lane t owns 8 consecutive ones.  Their owning ranks come from a load-balancing
// search in LDS: each rank starting inside the chunk marks its first slot, and a max-scan spreads the
// marks.  Each candidate is tested with half_reach; the reached ones are compacted in candidate
// order: keys[e] = tile, gid_by_e[e] = Gaussian | reach bits.  Emission offsets are chained by look-back; the last
// chunk stores L'.  Also accumulated: n_inst[g] (integer atomics), the tile-sort digit histograms,
// and (first T threads of the grid) zeroed tile ranges.
__global__ __launch_bounds__(256) void emit_instances_kernel(Args a, GeomState g, int L, int npass,
                                                             uint32_t *__restrict__ keys,
                                                             uint32_t *__restrict__ gid_by_e,
                                                             uint32_t *__restrict__ zero, uint2 *__restrict__ ranges) {
    __shared__ uint32_t s_own[kEmitChunk];
    __shared__ uint32_t s_off[kEmitChunk + 2];
    __shared__ uint32_t s_n[kEmitChunk + 1];
    __shared__ uint32_t s_hist[kMaxPasses][256];
    __shared__ uint32_t s_w[4], s_tmp[4];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    {
        const int gt = blockIdx.x * 256 + tid;
        if (gt < a.gx * a.gy) ranges[gt] = make_uint2(0u, 0u);
    }
    const uint32_t b = blockIdx.x;
    const uint32_t c0 = b * kEmitChunk;
    if (c0 >= (uint32_t)L) return;  // grid padding for the range zeroing
    const uint32_t c1 = min((uint32_t)L, c0 + kEmitChunk);
    const int rlo = (int)g.first_rank[b];
    const int nr = min(a.P - rlo, kEmitChunk + 1);  // ranks starting at or after c1 are ignored
    for (int i = tid; i < kEmitChunk; i += 256) s_own[i] = 0;
    for (int i = tid; i < kMaxPasses * 256; i += 256) (&s_hist[0][0])[i] = 0;
    __syncthreads();
    for (int i = tid; i < nr; i += 256) {
        const uint32_t st = g.cand_off[rlo + i];
        s_off[i] = st;
        s_n[i] = 0;
        if (st > c0 && st < c1) s_own[st - c0] = (uint32_t)i;
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
        uint32_t x = mx;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const uint32_t y = __shfl_up(x, off);
            if (lane >= off) x = max(x, y);
        }
        if (lane == 63) s_w[w] = x;
        __syncthreads();
        uint32_t carry = __shfl_up(x, 1);
        if (lane == 0) carry = 0;
        for (int q = 0; q < w; q++) carry = max(carry, s_w[q]);
#pragma unroll
        for (int k = 0; k < kEmitPer; k++) own[k] = max(own[k], carry);
    }
    // test the candidates (every gather issued before the first test)
    float4 geo[kEmitPer], co[kEmitPer];
#pragma unroll
    for (int k = 0; k < kEmitPer; k++) {
        const int r = rlo + (int)own[k];
        geo[k] = g.rank_geo[r];
        co[k] = g.rank_co[r];
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
            getRect(geo[k].x, geo[k].y, __float_as_int(geo[k].z), a.gx, a.gy, x0, y0, x1, y1);
            const uint32_t local = c - s_off[i], wdt = (uint32_t)(x1 - x0);
            const int ty = y0 + (int)(local / wdt), tx = x0 + (int)(local % wdt);
            reach[k] = half_reach(geo[k].x, geo[k].y, co[k], tx, ty, a.W, a.H);
            if (reach[k] != 0) {
                keep |= 1u << k;
                tile[k] = (uint32_t)(ty * a.gx + tx);
                atomicAdd(&s_n[i], 1u);
                for (int p = 0; p < npass; p++) atomicAdd(&s_hist[p][(tile[k] >> (8 * p)) & 0xFFu], 1u);
            }
        }
    }
    // compaction offsets: exclusive scan of the per-lane counts, chunk total chained by look-back
    const uint32_t cnt = __popc(keep);
    uint32_t x = cnt;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t y = __shfl_up(x, off);
        if (lane >= off) x += y;
    }
    __syncthreads();
    if (lane == 63) s_w[w] = x;
    __syncthreads();
    uint32_t before = 0, total = 0;
#pragma unroll
    for (int q = 0; q < 4; q++) {
        before += q < w ? s_w[q] : 0u;
        total += s_w[q];
    }
    uint32_t *chain = zero + bin_chain_off();
    const uint32_t prefix = block_prefix(chain + 64, b, total, chain + 1, s_tmp);
    if (tid == 0 && c1 == (uint32_t)L) zero[0] = prefix + total;  // L'
    uint32_t e = prefix + before + x - cnt;
#pragma unroll
    for (int k = 0; k < kEmitPer; k++) {
        if ((keep >> k) & 1u) {
            keys[e] = tile[k];
            gid_by_e[e] = __float_as_uint(geo[k].w) | (reach[k] << kReachShift);
            e++;
        }
    }
    for (int i = tid; i < nr; i += 256)
        if (s_n[i]) atomicAdd(&g.n_inst[__float_as_uint(g.rank_geo[rlo + i].w)], s_n[i]);
    uint32_t *hist = zero + kZeroHist + (b % kHistShards) * (kMaxPasses * 256);
    for (int p = 0; p < npass; p++)
        if (s_hist[p][tid]) atomicAdd(&hist[p * 256 + tid], s_hist[p][tid]);
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
    (void)radii;
    const int T = a.gx * a.gy;
    hipError_t e = hipMemsetAsync(b.scratch, 0, 4 * binning_zero_words(L), s);
    if (e != hipSuccess) return e;
    if (L == 0) return hipMemsetAsync(img.ranges, 0, sizeof(uint2) * (size_t)T, s);
    const int npass = (b.key_bits + 7) / 8;
    const int nblk = std::max<int>((int)nchunk_emit(L), (T + 255) / 256);
    hipLaunchKernelGGL(emit_instances_kernel, dim3(nblk), dim3(256), 0, s, a, g, L, npass, b.keys[0], b.gid_by_e,
                       b.scratch, img.ranges);
    const uint32_t *n_dev = b.scratch;  // L' <= L reached instances
    uint32_t *keys[2] = {b.keys[0], b.keys[1]};
    uint32_t *vals[2] = {b.vals[0], b.vals[1]};
    onesweep_sort<kSortThreads, kItemsL>(keys, vals, L, n_dev, b.key_bits, b.scratch + kZeroHist,
                                         b.scratch + bin_look_off(L), b.scratch + bin_chain_off() + 1, s);
    hipLaunchKernelGGL(tile_ranges_kernel, dim3((L + 255) / 256), dim3(256), 0, s, b.sorted_keys, n_dev, img.ranges);
    return hipGetLastError();
}

}  // namespace gs4d
