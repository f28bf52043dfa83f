// render.hip -- per-tile front-to-back alpha blending (K6) and its reverse walk (K7).
//
// Reference: cuda_rasterizer/forward.cu:261-379 (renderCUDA forward) and backward.cu:399-557
// (renderCUDA backward).
//
// MI355X mapping (not the reference's): ONE wave64 per 16x16 tile; each lane owns a column of 4
// pixels (rows r, r+4, r+8, r+12 with r = lane/16), processed as two pairs with packed-f32 VALU
// (v_pk_fma/mul/add_f32: two pixels per instruction).  A tile's sorted splats are fetched 64 at a
// time, one per lane (the next batch is prefetched while the current one is blended), converted to
// blend-ready constants and staged in LDS; the blend loop reads each splat with wave-uniform
// (broadcast) ds_read_b128.  The Gaussian falloff is evaluated in base 2 (log2(e) folded into the
// conic once per splat) so each pixel costs one v_exp_f32.  Which pixels a splat touches is kept in
// 64-bit lane masks (scalar unit); pixels are retired by a mask, and termination (T < 1e-4, rare)
// takes a wave-uniform side path, so the common path is branch- and select-light.
//
// Backward: per pixel the reference keeps accum_rec[3] and last_color[3] only to form
// dL/dalpha = sum_c (c_c - accum_rec_c) * dL/dpix_c; since dL/dpix is constant per pixel this is
// carried as one scalar A = accum_rec . dL/dpix, updated eagerly after each contributing splat
// (A = alpha CD + (1 - alpha) A, the same recurrence as backward.cu:515-517).  The 9 gradient terms of
// a splat (backward.cu:523,545-554) are linear in 6 per-pixel moments (sum u, sum u dx, sum u dy,
// sum u dx^2, sum u dx dy, sum u dy^2 with u = G dL/dalpha) and 3 colour sums; these 9 values are
// reduced over the wave with two v_permlane swaps and a 16-lane DPP tree (reduce-scatter), staged in
// LDS, and stored once per (tile, splat) instance at its emission slot (coalesced 48-byte records,
// no float atomics).  The per-Gaussian pass (preprocess_backward.hip) sums a Gaussian's records in
// a fixed order and applies the moment -> gradient map once (bitwise reproducible).
#include <type_traits>

#include "gs4d_internal.h"

namespace gs4d {

typedef float f2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f2 fma2(f2 a, f2 b, f2 c) { return __builtin_elementwise_fma(a, b, c); }
__device__ __forceinline__ f2 bc2(float x) { return f2{x, x}; }
// x + y of a pixel pair as one v_add_f32 (the backend would form a v_pk_add_f32 with op_sel, 4 issue
// cycles against ~2.5 for the plain add when other waves share the SIMD: tools/bench/valu_rates.hip)
__device__ __forceinline__ float hsum(f2 v) {
    float r;
    asm("v_add_f32 %0, %1, %2" : "=v"(r) : "v"(v.x), "v"(v.y));
    return r;
}


// Blend-ready splat constants.  geo = (x, y - yc, -a/2 log2e, -b log2e), opc = (-c/2 log2e, lo, 1/o, m),
// col = (r, g, b, depth): o G = m 2^(power2 + lo) with m = 1, lo = log2 o for a positive-definite conic (the
// opacity folded into the exponent: the common path has no o * G multiply) and m = o, lo = 0 otherwise.  power2 = log2(e) * power (forward.cu:340-342) at offset d = mean - pixel.
// Rows are measured from the tile's centre row yc = 16 ty + 7.5 (pixel row py = yc + yl, yl a
// half-integer in [-7.5, 7.5]): dy = (my - yc) - yl, the same two roundings in both kernels.
struct SplatLDS {
    float4 geo, opc, col;
};
struct SplatRegs {
    float4 geo, opc, col;
    uint32_t reach;  // bit h: the splat reaches some pixel centre of half tile h (rows 8h..8h+7)
};

// The alpha test of forward.cu:346-348 / backward.cu:486-490 is taken exactly as the reference states
// it: alpha = min(0.99, o G) >= 1/255, i.e. the rounded product o G >= 1/255 (the cap is above the
// threshold).  The splat record's 1/o (0 for o = 0) lets the backward accumulate its moments on
// o G dL/dalpha and divide by o once per splat record.
constexpr float kAlphaMin = 1.0f / 255.0f;

// A batch of 64 splats, each the Gaussian's packed 48-byte blend record (GeomState::splat, written by
// preprocess: s0 = (x, y, -a/2 log2e, -b log2e), s1 = (-c/2 log2e, o, 1/o, depth), s2 = (r, g, b, 0)),
// gathered straight into LDS by LDS-DMA loads (global_load_lds: per-lane global address, destination
// base + lane * 16): three 16-byte pieces of ONE contiguous record per splat, so the prefetch of the
// next batch spans the current batch's walk without holding registers.
struct RawLDS {
    float4 s0[64], s1[64], s2[64];
};
typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) const void gbl_void_t;
__device__ __forceinline__ void issue_raw_lds(RawLDS &r, bool valid, uint32_t gid, const float4 *__restrict__ splat) {
    if (valid) {
        const float4 *rec = splat + 3 * (size_t)gid;
        __builtin_amdgcn_global_load_lds((gbl_void_t *)rec, (lds_void_t *)r.s0, 16, 0, 0);
        __builtin_amdgcn_global_load_lds((gbl_void_t *)(rec + 1), (lds_void_t *)r.s1, 16, 0, 0);
        __builtin_amdgcn_global_load_lds((gbl_void_t *)(rec + 2), (lds_void_t *)r.s2, 16, 0, 0);
    }
}
// waits for this wave's LDS-DMA loads, then lane l reads its splat of the staged batch: blend constants
// with rows measured from the tile's centre row (geo.y = my - yc), zeros for lanes past the batch
// (opacity 0: the zero splat passes no pixel)
__device__ __forceinline__ void read_raw_lds(SplatRegs &s, const RawLDS &r, int lane, bool valid, float yc,
                                             bool block_barrier) {
    __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt(0): the LDS-DMA writes have landed (lgkm/exp counters not waited)
    if (block_barrier) __builtin_amdgcn_s_barrier();
    else __builtin_amdgcn_wave_barrier();
    if (valid) {
        const float4 s0 = r.s0[lane], s1 = r.s1[lane], s2 = r.s2[lane];
        s.geo = make_float4(s0.x, s0.y - yc, s0.z, s0.w);
        s.opc = make_float4(s1.x, s2.w, s1.z, s1.y);  // -c/2 log2e, exponent offset lo, 1/o, multiplier m
        // (the walks read c and lo as one 8-byte LDS load)
        s.col = make_float4(s2.x, s2.y, s2.z, s1.w);  // rgb, view depth
    } else {
        s.geo = s.opc = s.col = make_float4(0.f, 0.f, 0.f, 0.f);
    }
}

// Falloff of one splat at a pixel pair: exponent (base 2) and G = 2^power2.  Forward and backward use
// this one sequence, so they take identical blend decisions.
// alpha = min(0.99, o G) caps nothing for opacities at or below kCapFree: G = 2^power <= 1 wherever the
// power test passes (up to an ulp), so o G <= 0.98 (1 + ulp) < 0.99.
constexpr float kCapFree = 0.98f;
constexpr float kInvCapFree = 1.f / kCapFree;  // the record holds 1/o: o > kCapFree <=> 1/o < kInvCapFree
struct Falloff {
    f2 dy, pw, G, alpha;
};
// pa = geo.z dx^2 + lo (lane constant per splat: fmaf(geo.z dx, dx, lo)); FOLD: every splat of the walk has a
// positive-definite conic, so m = 1 and o G is the exponential itself
template <bool CAP = true, bool FOLD = false>
__device__ __forceinline__ Falloff falloff(const float4 &geo, const float4 &opc, float pa, float pb, f2 yl) {
    Falloff f;
    f.dy = bc2(geo.y) - yl;
    f.pw = fma2(f.dy, fma2(bc2(opc.x), f.dy, bc2(pb)), bc2(pa));
    f.G = f2{__builtin_amdgcn_exp2f(f.pw.x), __builtin_amdgcn_exp2f(f.pw.y)};
    const f2 al = FOLD ? f.G : bc2(opc.w) * f.G;
    // without CAP every splat of the batch has opacity <= kCapFree: min(0.99, o G) = o G
    f.alpha = CAP ? f2{fminf(0.99f, al.x), fminf(0.99f, al.y)} : al;
    return f;
}
__device__ __forceinline__ uint64_t ballot(bool p) { return __builtin_amdgcn_ballot_w64(p); }
// a wave-uniform 64-bit mask kept in scalar registers (the compiler's divergence analysis may otherwise move a
// loop-carried mask to VGPRs and turn its bit scans into vector code)
__device__ __forceinline__ uint64_t uniform64(uint64_t v) {
    return ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(v >> 32)) << 32) |
           __builtin_amdgcn_readfirstlane((uint32_t)v);
}
// this lane's bit of a wave mask, used directly as the select condition (no VALU shift)
__device__ __forceinline__ bool lane_bit(uint64_t m) { return __builtin_amdgcn_inverse_ballot_w64(m); }

// ---------------------------------------------------------------------------------------------
// A splat whose conic is positive definite has power <= 0 at every pixel (up to rounding at its
// centre), so the power test of forward.cu:341 is only evaluated in batches holding another splat.
// The same float operations, uncontracted, as preprocess.hip's choice of the record's opacity form.
__device__ __forceinline__ bool conic_pd(const float4 &geo, const float4 &opc) {
    // geo.z = -a/2 k, geo.w = -b k, opc.x = -c/2 k (k = log2 e > 0): a > 0 and ac - b^2 > 0
    return geo.z < 0.f && __fsub_rn(__fmul_rn(__fmul_rn(4.f, geo.z), opc.x), __fmul_rn(geo.w, geo.w)) > 0.f;
}

// ---------------------------------------------------------------------------------------------
// K4 for short tiles, fused into the forward: a run of up to 64*R instances is sorted by the key
// (depth bits << 32 | emission slot) by one wave in registers, lane l holding positions l, 64 + l, ..
// Inside a tile the emission slot increases with the Gaussian id (emission follows the visible
// Gaussians in id order), so this is the reference's (depth, id) order (rasterizer_impl.cu:94-105,
// 304-309) and the key carries its own value.  Bitonic network in its all-ascending ("flip") form,
// unrolled: every partner is a compile-time (register, lane-xor) pair, so cross-lane steps are
// shuffles and cross-register steps plain selects; a length that is not a power of two is padded
// with +inf keys.  The sorted slots are written back for the backward and returned in ev[].
template <int R>
__device__ __forceinline__ void sort_keys(uint64_t key[R], int lane) {
#pragma unroll
    for (int k = 2; k <= 64 * R; k <<= 1) {
#pragma unroll
        for (int j = k >> 1; j >= 1; j >>= 1) {
            const int mask = j == (k >> 1) ? k - 1 : j;  // flip, then half-cleaners
            const int lx = mask & 63, rx = mask >> 6;
            uint64_t pk[R];
#pragma unroll
            for (int r = 0; r < R; r++) {
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
            for (int r = 0; r < R; r++) {
                const bool lower = ((r * 64 + lane) & j) == 0;
                const uint64_t kr = key[r];
                key[r] = lower ? (pk[r] < kr ? pk[r] : kr) : (pk[r] > kr ? pk[r] : kr);
            }
        }
    }
}
// the sort keys of run positions base + r * 64 + lane (+inf past n)
template <int R>
__device__ __forceinline__ void load_keys(uint64_t key[R], const uint32_t *__restrict__ seg, int base, int n,
                                          const uint32_t *__restrict__ gid_by_e, const float *__restrict__ depths,
                                          int lane) {
#pragma unroll
    for (int r = 0; r < R; r++) {
        const int i = base + r * 64 + lane;
        const uint32_t e = i < n ? seg[i] : 0u;
        const uint32_t gid = i < n ? gid_by_e[e] & kGidMask : 0u;
        key[r] = i < n ? ((uint64_t)__float_as_uint(depths[gid]) << 32) | e : ~0ull;  // depths > 0.2
    }
}
template <int R>
__device__ __forceinline__ void sort_run(uint32_t *__restrict__ seg, int n, const uint32_t *__restrict__ gid_by_e,
                                         const float *__restrict__ depths, int lane, uint32_t ev[4]) {
    uint64_t key[R];
    load_keys<R>(key, seg, 0, n, gid_by_e, depths, lane);
    sort_keys<R>(key, lane);
#pragma unroll
    for (int r = 0; r < 4; r++) {
        const int i = r * 64 + lane;
        ev[r] = r < R ? (uint32_t)key[r < R ? r : 0] : 0u;
        if (r < R && i < n) seg[i] = ev[r];
    }
}

// TWO waves per tile: wave h blends half tile h (rows 8h .. 8h + 7; lane l holds the pixel pair at rows
// 8h + l/16 and 8h + l/16 + 4 of column l % 16), so a long tile's serial blend walk is split over two
// waves.  With one wave per tile every tile of the metric scene was resident at once and the kernel's end
// was set by the longest tiles walking alone on their SIMDs (a launch repeating every tile took only
// 0.67 of the first pass's time per extra pass).  The short run's sort is done once, by wave 0, and
// handed to wave 1 through LDS (the only cross-wave step, one barrier); each wave then stages and walks
// the splats that reach its half on its own (LDS-DMA gathers, no barriers), and retires when its half's
// pixels are all done.
__global__ __launch_bounds__(128) void render_forward_kernel(Args a, const uint2 *__restrict__ ranges,
                                                             const uint32_t *__restrict__ order,
                                                             uint32_t *__restrict__ upos,
                                                             const float *__restrict__ depths,
                                                             const uint32_t *__restrict__ gid_by_e,
                                                             const float4 *__restrict__ splat,
                                                             float *__restrict__ final_T,
                                                             uint32_t *__restrict__ n_contrib,
                                                             float *__restrict__ out_color,
                                                             float *__restrict__ out_depth) {
    __shared__ SplatLDS s_sp_all[2][64];
    __shared__ RawLDS s_raw_all[2];
    __shared__ uint32_t s_ev[kWaveSortMax];
    const int tile = (int)__builtin_amdgcn_readfirstlane(order[blockIdx.x]);  // longest runs first
    const int tx = tile % a.gx, ty = tile / a.gx;
    const int lane = threadIdx.x & 63;
    const int h = (int)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // this wave's half tile
    SplatLDS *s_sp = s_sp_all[h];
    RawLDS &s_raw = s_raw_all[h];
    const int px = tx * kBlockX + (lane & 15);
    const int py0 = ty * kBlockY + 8 * h + (lane >> 4);
    const float pfx = (float)px;
    const float yc = (float)(ty * kBlockY) + 7.5f;
    const float ylane = (float)(8 * h + (lane >> 4)) - 7.5f;
    const f2 yl = f2{ylane, ylane + 4.f};
    // live pixels (forward.cu:287-289: pixels outside the image never blend) as a per-lane alpha
    // threshold: 1/255 while the pixel blends, 2 (above any alpha) once it is outside or retired, so the
    // alpha test is one compare per pixel and needs no scalar mask
    f2 thr;
    thr.x = (px < a.W && py0 < a.H) ? kAlphaMin : 2.f;
    thr.y = (px < a.W && py0 + 4 < a.H) ? kAlphaMin : 2.f;
    f2 T = bc2(1.f), C0 = bc2(0.f), C1 = bc2(0.f), C2 = bc2(0.f), Dp = bc2(0.f);
    uint32_t stop[2] = {0, 0};  // list position of the terminating splat (retired pixels)
    uint2 range = ranges[tile];
    range.x = __builtin_amdgcn_readfirstlane(range.x);
    range.y = __builtin_amdgcn_readfirstlane(range.y);
    // short runs: sorted here (wave 0), their emission slots kept in registers (batch b in ev[0] after
    // b shifts)
    const int n_run = (int)(range.y - range.x);
    const bool in_regs = n_run <= kWaveSortMax;
    uint32_t ev[4] = {0u, 0u, 0u, 0u};
    if (in_regs && n_run > 128) {
        // 129..256: each wave sorts 128 keys in registers, then one merge-path step over the two sorted
        // halves (thread t emits positions 2t, 2t + 1, its start found by a binary search on its
        // diagonal) -- half the network depth of one wave sorting all 256 (the sort is the walk's
        // start-up latency).  The keys go through the splat staging area, unused until the walk.
        uint32_t *seg = upos + range.x;
        uint64_t *s_key = reinterpret_cast<uint64_t *>(&s_sp_all[0][0]);
        uint64_t key[2];
        load_keys<2>(key, seg, 128 * h, n_run, gid_by_e, depths, lane);
        sort_keys<2>(key, lane);
        s_key[128 * h + lane] = key[0];
        s_key[128 * h + 64 + lane] = key[1];
        __syncthreads();
        const int t = threadIdx.x, d = 2 * t;
        int lo = max(0, d - 128), hi = min(d, 128);
        while (lo < hi) {  // ties (the +inf padding only) go to the first half, as below
            const int mid = (lo + hi) >> 1;
            if (s_key[mid] > s_key[128 + d - 1 - mid]) hi = mid;
            else lo = mid + 1;
        }
        int i = lo, j = d - lo;
        uint64_t xk = i < 128 ? s_key[i] : ~0ull, yk = j < 128 ? s_key[128 + j] : ~0ull;
        uint32_t outv[2];
#pragma unroll
        for (int k = 0; k < 2; k++) {
            const bool first = xk <= yk;
            outv[k] = (uint32_t)(first ? xk : yk);
            if (first) {
                i++;
                xk = i < 128 ? s_key[i] : ~0ull;
            } else {
                j++;
                yk = j < 128 ? s_key[128 + j] : ~0ull;
            }
        }
#pragma unroll
        for (int k = 0; k < 2; k++) {
            s_ev[d + k] = outv[k];
            if (d + k < n_run) seg[d + k] = outv[k];
        }
        __syncthreads();
#pragma unroll
        for (int r = 0; r < 4; r++) ev[r] = s_ev[r * 64 + lane];
    } else if (in_regs) {
        if (h == 0) {
            if (n_run > 1) {
                uint32_t *seg = upos + range.x;
                if (n_run <= 64) sort_run<1>(seg, n_run, gid_by_e, depths, lane, ev);
                else sort_run<2>(seg, n_run, gid_by_e, depths, lane, ev);
            } else if (n_run == 1 && lane == 0) {
                ev[0] = upos[range.x];
            }
#pragma unroll
            for (int r = 0; r < 4; r++)
                if (r * 64 < n_run) s_ev[r * 64 + lane] = ev[r];
        }
        __syncthreads();
        if (h == 1) {
#pragma unroll
            for (int r = 0; r < 4; r++) ev[r] = r * 64 + lane < n_run ? s_ev[r * 64 + lane] : 0u;
        }
    }
    // gid_by_e of each batch's instances, 4 batches at a time (the short run's are all loaded here);
    // the next batch's attributes are issued before the current one is blended and only turned into
    // blend constants when it comes up, so their loads overlap the blend loop
    uint32_t ug[4];
    int ids_left = 0;
    auto refill = [&](uint32_t first) {  // list positions first + r*64 + lane
        if (!in_regs) {
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const uint32_t i = first + r * 64 + lane;
                ev[r] = i < range.y ? upos[i] : 0u;
            }
        }
#pragma unroll
        for (int r = 0; r < 4; r++) {
            const uint32_t i = first + r * 64 + lane;
            ug[r] = i < range.y ? gid_by_e[ev[r]] : 0u;
        }
        ids_left = 4;
    };
    // the next batch's attributes are gathered into this wave's LDS by LDS-DMA loads (as the backward
    // does), only its lanes' reach bits stay in a register
    uint32_t rnxt = 0;
    auto fetch = [&](uint32_t first) {
        if (ids_left == 0) refill(first);
        const uint32_t rge = ug[0];
        ev[0] = ev[1]; ev[1] = ev[2]; ev[2] = ev[3];
        ug[0] = ug[1]; ug[1] = ug[2]; ug[2] = ug[3];
        ids_left--;
        rnxt = rge >> kReachShift;
        issue_raw_lds(s_raw, first + lane < range.y, rge & kGidMask, splat);
    };
    if (range.x < range.y) fetch(range.x);
    for (uint32_t base = range.x; base < range.y; base += 64) {
        if (ballot(thr.x < 1.f || thr.y < 1.f) == 0) break;  // forward.cu:312-314 (this half)
        SplatRegs nxt;
        const bool valid = base + lane < range.y;
        read_raw_lds(nxt, s_raw, lane, valid, yc, false);  // this wave's own staging: no block barrier
        nxt.reach = valid ? rnxt : 0u;
        const uint64_t reach = ballot((nxt.reach >> h) & 1u);
        const uint64_t nonpd = ballot(!conic_pd(nxt.geo, nxt.opc));
        const bool cap = ballot(valid && nxt.opc.z < kInvCapFree) != 0;  // wave-uniform: a splat the 0.99 cap can bind
        // one wave writes and reads its own staging area: LDS operations of a wave complete in order
        __builtin_amdgcn_wave_barrier();
        s_sp[lane].geo = nxt.geo;
        s_sp[lane].opc = nxt.opc;
        s_sp[lane].col = nxt.col;
        __builtin_amdgcn_wave_barrier();
        if (base + 64 < range.y) fetch(base + 64);
        const uint32_t pos0 = base - range.x;
        // the batch's splats that reach this half, two at a time: both falloffs are independent, only
        // the blend updates chain (a lone last splat runs alone)
        auto blend = [&](const Falloff &f, const float4 &col, uint32_t j, auto pwc) {
            bool k0 = f.alpha.x >= thr.x, k1 = f.alpha.y >= thr.y;  // forward.cu:346-348 (live pixels)
            if (decltype(pwc)::value && ((nonpd >> j) & 1)) {  // forward.cu:341-342
                k0 = k0 && f.pw.x <= 0.0f;
                k1 = k1 && f.pw.y <= 0.0f;
            }
            f2 ae = f2{k0 ? f.alpha.x : 0.f, k1 ? f.alpha.y : 0.f};
            f2 tT = T * (bc2(1.f) - ae);  // forward.cu:349
            if (ballot(fminf(tT.x, tT.y) < 0.0001f) != 0) {
                // forward.cu:350-354: the splat that would drop T below 1e-4 is not blended; the pixel retires
                const bool t0 = tT.x < 0.0001f, t1 = tT.y < 0.0001f;
                ae = f2{t0 ? 0.f : ae.x, t1 ? 0.f : ae.y};
                tT = f2{t0 ? T.x : tT.x, t1 ? T.y : tT.y};
                stop[0] = t0 ? pos0 + j : stop[0];
                stop[1] = t1 ? pos0 + j : stop[1];
                thr = f2{t0 ? 2.f : thr.x, t1 ? 2.f : thr.y};
            }
            // every live pixel takes the update; pixels the splat does not touch have ae = 0
            const f2 w = ae * T;  // forward.cu:357-358
            C0 = fma2(bc2(col.x), w, C0);
            C1 = fma2(bc2(col.y), w, C1);
            C2 = fma2(bc2(col.z), w, C2);
            Dp = fma2(bc2(col.w), w, Dp);
            T = tT;
        };
        auto walk = [&](auto capc, auto pwc) {
            constexpr bool CAP = decltype(capc)::value, FOLD = !decltype(pwc)::value;
            for (uint64_t todo = reach; todo != 0;) {
                const uint32_t j0 = (uint32_t)__builtin_ctzll(todo);
                todo &= todo - 1;
                const bool two = todo != 0;
                const uint32_t j1 = two ? (uint32_t)__builtin_ctzll(todo) : j0;
                todo &= todo - (two ? 1 : 0);
                const float4 geo0 = s_sp[j0].geo, opc0 = s_sp[j0].opc, col0 = s_sp[j0].col;
                const float4 geo1 = s_sp[j1].geo, opc1 = s_sp[j1].opc, col1 = s_sp[j1].col;
                const float dx0 = geo0.x - pfx, dx1 = geo1.x - pfx;
                const Falloff f0 = falloff<CAP, FOLD>(geo0, opc0, fmaf(geo0.z * dx0, dx0, opc0.y), geo0.w * dx0, yl);
                const Falloff f1 = falloff<CAP, FOLD>(geo1, opc1, fmaf(geo1.z * dx1, dx1, opc1.y), geo1.w * dx1, yl);
                blend(f0, col0, j0, pwc);
                if (two) blend(f1, col1, j1, pwc);
            }
        };
        // the batch's walk without the 0.99 cap unless one of its splats has opacity > kCapFree, and
        // without the power test unless one has a conic that is not positive definite (cov3D_precomp)
        if (nonpd != 0) walk(std::true_type{}, std::true_type{});
        else if (cap) walk(std::true_type{}, std::false_type{});
        else walk(std::false_type{}, std::false_type{});
    }
    __builtin_amdgcn_s_waitcnt(0x0f70);  // an early exit may leave the next batch's LDS-DMA loads in flight
    const size_t HW = (size_t)a.W * a.H;
    const V3 bg = load_v3(a.bg);
#pragma unroll
    for (int k = 0; k < 2; k++) {
        const int py = py0 + 4 * k;
        if (px < a.W && py < a.H) {
            const float t = k ? T.y : T.x;
            const size_t pix = (size_t)py * a.W + px;
            final_T[pix] = t;
            // splats at positions >= n_contrib never blended into this pixel (the backward's bound):
            // the terminating splat's position, or the list length for pixels that never terminated
            n_contrib[pix] = (k ? thr.y : thr.x) < 1.f ? range.y - range.x : stop[k];
            out_color[pix] = (k ? C0.y : C0.x) + t * bg.x;
            out_color[HW + pix] = (k ? C1.y : C1.x) + t * bg.y;
            out_color[2 * HW + pix] = (k ? C2.y : C2.x) + t * bg.z;
            out_depth[pix] = k ? Dp.y : Dp.x;
        }
    }
}

hipError_t launch_render_forward(const Args &a, GeomState g, BinningState b, ImageState img, float *out_color,
                                 float *out_depth, hipStream_t s) {
    const int T = a.gx * a.gy;
    hipLaunchKernelGGL(render_forward_kernel, dim3(T), dim3(128), 0, s, a, img.ranges, img.order, b.upos, g.depths,
                       b.gid_by_e, g.splat, img.final_T, img.n_contrib, out_color, out_depth);
    return hipGetLastError();
}

// Diagnostic (test infrastructure's view of the blend arithmetic): o G and the base-2 exponent of given
// (Gaussian, pixel) pairs, by the exact sequence both blend kernels evaluate (read_raw_lds's row shift,
// falloff()), so the parity tests can measure how far the blend's alpha lies from the oracle's near the
// 1/255 threshold and size the near-threshold band from that measurement.
__global__ void pair_alpha_kernel(const float4 *__restrict__ splat, int n, const int *__restrict__ gid,
                                  const int *__restrict__ px, const int *__restrict__ py, float *__restrict__ og,
                                  float *__restrict__ pw) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float4 *rec = splat + 3 * (size_t)gid[i];
    const float4 s0 = rec[0], s1 = rec[1];
    const int ty = py[i] / kBlockY;
    const float yc = (float)(ty * kBlockY) + 7.5f;
    const float yl = (float)(py[i] - ty * kBlockY) - 7.5f;
    const float4 geo = make_float4(s0.x, s0.y - yc, s0.z, s0.w);
    const float4 opc = make_float4(s1.x, rec[2].w, s1.z, s1.y);
    const float dx = geo.x - (float)px[i];
    const Falloff f = falloff<false>(geo, opc, fmaf(geo.z * dx, dx, opc.y), geo.w * dx, f2{yl, yl});
    og[i] = f.alpha.x;
    pw[i] = f.pw.x;
}
hipError_t launch_pair_alpha(GeomState g, int n, const int *gid, const int *px, const int *py, float *og, float *pw,
                             hipStream_t s) {
    if (n > 0) hipLaunchKernelGGL(pair_alpha_kernel, dim3((n + 255) / 256), dim3(256), 0, s, g.splat, n, gid, px, py, og, pw);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// lanes 0-31 of the result hold a's half-wave sums, lanes 32-63 b's (v_permlane32_swap)
__device__ __forceinline__ float swap32_add(float a, float b) {
    auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(a), __float_as_uint(b), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
// rows (0,1,2,3) of the result hold (a rows 0+1, b rows 0+1, a rows 2+3, b rows 2+3) (v_permlane16_swap)
__device__ __forceinline__ float swap16_add(float a, float b) {
    auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(a), __float_as_uint(b), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// Per-lane partial sums of one splat of the reverse walk, its pixel pair already added: the moments
// of u = G dL/dalpha in the tile-centred row coordinate yl (sum u, sum u yl, sum u yl^2) and the
// colour sums (sum w dL/dpix_c, w = alpha T).
struct SplatPart {
    float u0, u1, u2, w0, w1, w2;
};

// Wave64 totals of two splats' partial sums, left in LDS as their 9 record values:
//   0 sum u, 1 sum dx u, 2 sum u yl, 3 sum dx^2 u, 4 sum dx u yl, 5 sum u yl^2, 6-8 colour sums
// (dx = mean.x - pixel x, per lane column).  v_permlane32_swap then v_permlane16_swap sum each value
// over the 4 lanes of a column (reduce-scatter: row r of x1 ends with (a.u0, a.u1, b.u0, b.u1)[r], of x2
// (a.u2, a.w0, b.u2, b.w0)[r], of x3 (a.w1, a.w2, b.w1, b.w2)[r]); the dx-weighted moments x4, x5 are
// formed on those column sums.  The 16 columns of each row are then reduce-scattered too, with DPP:
// pairs of registers halve at each of the four stages (column c with c ^ 8, the half-row mirror, c ^ 2,
// c ^ 1), so every lane ends with one finished total (15 DPP-stage instructions for the 5 registers
// instead of 20 for 5 butterflies) and writes it with ONE ds_write at a lane-constant offset `roff`
// (red_offset(); -1: nothing to write).
template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
// record float offset (from record j's start; record j + 1 follows at +12) of this lane's total
__device__ __forceinline__ int red_offset(int lane) {
    const int r = lane >> 4, c = lane & 15, splat = (r >> 1) * 12, odd = r & 1;
    switch (c) {
    case 0: return splat + (odd ? 2 : 0);   // x1: S u, S u yl
    case 4: return splat + (odd ? 8 : 7);   // x3: W1, W2
    case 8: return splat + (odd ? 6 : 5);   // x2: S u yl^2, W0
    case 12: return splat + (odd ? 4 : 1);  // x4: S dx u yl, S dx u
    case 2: return odd ? -1 : splat + 3;    // x5: S dx^2 u (odd rows hold nothing)
    default: return -1;
    }
}
__device__ __forceinline__ void wave_sum_pair_to_lds(const SplatPart &a, const SplatPart &b, float dxa, float dxb,
                                                     float *rec_pair, int lane, int roff) {
    const float h0 = swap32_add(a.u0, b.u0);  // lanes 0-31: a, 32-63: b
    const float h1 = swap32_add(a.u1, b.u1);
    const float h2 = swap32_add(a.u2, b.u2);
    const float h3 = swap32_add(a.w0, b.w0);
    const float h4 = swap32_add(a.w1, b.w1);
    const float h5 = swap32_add(a.w2, b.w2);
    const float x1 = swap16_add(h0, h1);
    const float x2 = swap16_add(h2, h3);
    const float x3 = swap16_add(h4, h5);
    const float dxs = lane < 32 ? dxa : dxb;  // rows 0-1 hold splat a, rows 2-3 splat b
    const float x4 = x1 * dxs;                 // (dx a.u0, dx a.u1, dx b.u0, dx b.u1)
    const float x5 = x4 * dxs;                 // (dx^2 a.u0, -, dx^2 b.u0, -)
    const bool c8 = (lane & 8) == 0, c4 = (lane & 4) == 0, c2 = (lane & 2) == 0;
    // stage A (c, c ^ 8): x1 | x2 -> z12, x3 | x4 -> z34, x5 -> z5
    const float z12 = (c8 ? x1 : x2) + dpp<0x128>(c8 ? x2 : x1);  // row_ror:8
    const float z34 = (c8 ? x3 : x4) + dpp<0x128>(c8 ? x4 : x3);
    const float z5 = x5 + dpp<0x128>(x5);
    // stage B (half-row mirror): z12 | z34 -> w
    const float w = (c4 ? z12 : z34) + dpp<0x141>(c4 ? z34 : z12);
    const float w5 = z5 + dpp<0x141>(z5);
    // stage C (c ^ 2): w | w5 -> v; stage D (c ^ 1)
    const float v = (c2 ? w : w5) + dpp<0x4E>(c2 ? w5 : w);  // quad_perm [2, 3, 0, 1]
    const float u = v + dpp<0xB1>(v);                         // quad_perm [1, 0, 3, 2]
    if (roff >= 0) rec_pair[roff] = u;
}

// Per-pixel state of the reverse walk (pairs): T (recovered backwards), A = accum_rec . dL/dpix and
// dL/dpix.  The background term of backward.cu:534, -T_final / (1 - alpha) (bg . dL/dpix), is the
// background taken as one more layer behind the last contributor (colour bg, alpha 1): A starts at
// bg . dL/dpix instead of 0, and T_final / (1 - alpha_i) = T_i prod_{i<j} (1 - alpha_j) follows from
// the walk's own T -- the same value up to rounding, without a per-pixel constant.
struct BwdPixels {
    f2 T[2], A[2], dp0[2], dp1[2], dp2[2];
};

// One half tile of one splat of the reverse walk: updates the half's pixel state and adds its
// per-lane partial sums (moments of u' = o G dL/dalpha in the tile-centred row coordinate yl -- the
// record divides them by o once -- and the colour sums) to U0..U2 / W0..W2.  The falloff is the
// forward's sequence (falloff()) on operand pairs: identical blend decisions.  Branch-free, so that the
// pair walk below is one basic block.
//   ALL: the splat lies below every pixel's n_contrib (the contributor test passes; pixels outside
//        the image have T = dL/dpix = 0 and contribute exact zeros).
//   GEN: the general splat: `chk` = its conic is not positive definite (power > 0 skips, forward.cu:341),
//        and the 0.99 cap applies; without GEN the opacity is <= kCapFree, so o * G never reaches the cap.
// The per-splat half of a step: falloff, the reference's skip decisions and alpha.
struct HalfAlpha {
    f2 ale, ae, om;  // o G with the skips applied, alpha, 1 - alpha
};
template <bool ALL, bool GEN>
__device__ __forceinline__ HalfAlpha half_alpha(const f2 Y2, const f2 C2, const f2 O2, const f2 pa2, const f2 pb2,
                                                f2 yl, bool chk, uint32_t contributor, uint32_t last0,
                                                uint32_t last1) {
    const f2 dy = Y2 - yl;  // Y2 = my - yc
    const f2 pw = fma2(dy, fma2(C2, dy, pb2), pa2);
    const f2 G = f2{__builtin_amdgcn_exp2f(pw.x), __builtin_amdgcn_exp2f(pw.y)};
    // o G: min(0.99, o G) >= 1/255 iff o G >= 1/255.  Without GEN every splat of the pair has a positive-
    // definite conic, whose record folds o into the exponent (O2 = m = 1)
    const f2 al = GEN ? O2 * G : G;
    // backward.cu:486-497: contributor test, alpha < 1/255 and power > 0 skip -- the forward's decisions
    bool k0 = al.x >= kAlphaMin, k1 = al.y >= kAlphaMin;
    if (!ALL) {
        k0 = k0 && contributor < last0;
        k1 = k1 && contributor < last1;
    }
    if (GEN) {
        k0 = k0 && (!chk || pw.x <= 0.0f);
        k1 = k1 && (!chk || pw.y <= 0.0f);
    }
    // the skip applied to o G: a skipped pixel has alpha 0 exactly
    HalfAlpha h;
    h.ale = f2{k0 ? al.x : 0.f, k1 ? al.y : 0.f};
    h.ae = GEN ? f2{fminf(0.99f, h.ale.x), fminf(0.99f, h.ale.y)} : h.ale;
    h.om = bc2(1.f) - h.ae;
    return h;
}
// The rest of a step once the splat's T (the transmittance in front of it, Tn) is known.
template <bool GEN>
__device__ __forceinline__ void half_accum(const HalfAlpha &h, const f2 Tn, f2 &A, const f2 dp0, const f2 dp1,
                                           const f2 dp2, const f2 R2, const f2 G2, const f2 B2, f2 yl, f2 yl2,
                                           f2 &U0, f2 &U1, f2 &U2, f2 &W0, f2 &W1, f2 &W2) {
    const f2 diff = fma2(B2, dp2, fma2(G2, dp1, fma2(R2, dp0, -A)));  // c . dL/dpix - accum_rec . dL/dpix
    A = fma2(h.ae, diff, A);                    // accum_rec for the next splat in front
    const f2 w = h.ae * Tn;                     // dchannel_dcolor (backward.cu:521)
    // u' = o G dL/dalpha = o G T diff (backward.cu:519-534, bg term in A's start value); without the
    // cap o G T = w
    const f2 u = (GEN ? h.ale * Tn : w) * diff;
    U0 += u;
    U1 = fma2(u, yl, U1);
    U2 = fma2(u, yl2, U2);
    W0 = fma2(w, dp0, W0);
    W1 = fma2(w, dp1, W1);
    W2 = fma2(w, dp2, W2);
}
// One half tile of one splat of the reverse walk: updates the half's pixel state and adds its
// per-lane partial sums (moments of u' = o G dL/dalpha in the tile-centred row coordinate yl -- the
// record divides them by o once -- and the colour sums) to U0..U2 / W0..W2.  The falloff is the
// forward's sequence (falloff()) on operand pairs: identical blend decisions.  Branch-free, so that the
// pair walk below is one basic block.
//   ALL: the splat lies below every pixel's n_contrib (the contributor test passes; pixels outside
//        the image have T = dL/dpix = 0 and contribute exact zeros).
//   GEN: the general splat: `chk` = its conic is not positive definite (power > 0 skips, forward.cu:341),
//        and the 0.99 cap applies; without GEN the opacity is <= kCapFree, so o * G never reaches the cap.
// Two splats walking the same half share one reciprocal (half_pair_step): T in front of the back splat
// a is T / (1 - alpha_a), in front of b T / ((1 - alpha_a)(1 - alpha_b)) -- one v_rcp_f32 of the
// product per pixel (8 issue cycles each) and two multiplies instead of two reciprocals.
struct SplatOps {
    f2 Y2, C2, O2, R2, G2, B2, pa2, pb2;
    bool chk;
    uint32_t contributor;
};
template <bool ALL, bool GEN>
__device__ __forceinline__ void half_step(f2 &T, f2 &A, const f2 dp0, const f2 dp1, const f2 dp2, const SplatOps &s,
                                          f2 yl, f2 yl2, uint32_t last0, uint32_t last1, f2 (&U)[6]) {
    const HalfAlpha h = half_alpha<ALL, GEN>(s.Y2, s.C2, s.O2, s.pa2, s.pb2, yl, s.chk, s.contributor, last0, last1);
    const f2 inv = f2{__builtin_amdgcn_rcpf(h.om.x), __builtin_amdgcn_rcpf(h.om.y)};
    const f2 Tn = T * inv;  // backward.cu:503
    T = Tn;
    half_accum<GEN>(h, Tn, A, dp0, dp1, dp2, s.R2, s.G2, s.B2, yl, yl2, U[0], U[1], U[2], U[3], U[4], U[5]);
}
template <bool ALL, bool GEN>
__device__ __forceinline__ void half_pair_step(f2 &T, f2 &A, const f2 dp0, const f2 dp1, const f2 dp2,
                                               const SplatOps &sa, const SplatOps &sb, f2 yl, f2 yl2, uint32_t last0,
                                               uint32_t last1, f2 (&Ua)[6], f2 (&Ub)[6]) {
    const HalfAlpha ha = half_alpha<ALL, GEN>(sa.Y2, sa.C2, sa.O2, sa.pa2, sa.pb2, yl, sa.chk, sa.contributor,
                                              last0, last1);
    const HalfAlpha hb = half_alpha<ALL, GEN>(sb.Y2, sb.C2, sb.O2, sb.pa2, sb.pb2, yl, sb.chk, sb.contributor,
                                              last0, last1);
    const f2 prod = ha.om * hb.om;
    const f2 r = f2{__builtin_amdgcn_rcpf(prod.x), __builtin_amdgcn_rcpf(prod.y)};
    const f2 Tb = T * r;         // backward.cu:503 twice: T / (1 - alpha_a) / (1 - alpha_b)
    const f2 Ta = Tb * hb.om;    // T / (1 - alpha_a)
    half_accum<GEN>(ha, Ta, A, dp0, dp1, dp2, sa.R2, sa.G2, sa.B2, yl, yl2, Ua[0], Ua[1], Ua[2], Ua[3], Ua[4], Ua[5]);
    half_accum<GEN>(hb, Tb, A, dp0, dp1, dp2, sb.R2, sb.G2, sb.B2, yl, yl2, Ub[0], Ub[1], Ub[2], Ub[3], Ub[4], Ub[5]);
    T = Tb;
}

// 4 waves per SIMD (<= 128 VGPRs, no spills): the reach-combo blocks hold at most the four falloff chains
// of one pair.
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(4, 4))) void render_backward_kernel(Args a, const uint2 *__restrict__ ranges, const uint32_t *__restrict__ order,
                            const uint32_t *__restrict__ gid_by_e,
                            const uint32_t *__restrict__ upos, const float4 *__restrict__ splat,
                            const float *__restrict__ final_Ts,
                            const uint32_t *__restrict__ n_contrib, const float *__restrict__ dL_dpixels,
                            float *__restrict__ contrib) {
    __shared__ SplatLDS s_sp[64];
    __shared__ float4 s_rec[64][3];  // reduced sums of the batch's splats
    const int tile = (int)__builtin_amdgcn_readfirstlane(order[blockIdx.x]);  // longest runs first
    const int tx = tile % a.gx, ty = tile / a.gx;
    const int lane = threadIdx.x;
    const int px = tx * kBlockX + (lane & 15);
    const int py0 = ty * kBlockY + (lane >> 4);
    const float pfx = (float)px;
    const size_t HW = (size_t)a.W * a.H;
    uint2 range = ranges[tile];
    range.x = __builtin_amdgcn_readfirstlane(range.x);
    range.y = __builtin_amdgcn_readfirstlane(range.y);
    if (range.y <= range.x) return;
    const V3 bg = load_v3(a.bg);
    // rows relative to the tile's centre row (ty*16 + 7.5): the y moments are accumulated in them
    const float ylane = (float)(lane >> 4) - 7.5f;
    const f2 yl[2] = {f2{ylane, ylane + 4.f}, f2{ylane + 8.f, ylane + 12.f}};
    const f2 yl2[2] = {yl[0] * yl[0], yl[1] * yl[1]};
    const float yc = (float)(ty * kBlockY) + 7.5f;
    const int roff = red_offset(lane);

    BwdPixels st;
    uint32_t lastc[4];
    uint64_t inside_m[4];
    uint32_t max_last = 0, min_last = 0xffffffffu;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int py = py0 + 4 * k;
        const bool inside = px < a.W && py < a.H;
        const size_t pix = (size_t)py * a.W + px;
        const float tf = inside ? final_Ts[pix] : 0.f;
        const float d0 = inside ? dL_dpixels[pix] : 0.f;
        const float d1 = inside ? dL_dpixels[HW + pix] : 0.f;
        const float d2 = inside ? dL_dpixels[2 * HW + pix] : 0.f;
        lastc[k] = inside ? n_contrib[pix] : 0u;
        inside_m[k] = ballot(inside);
        const float a0 = bg.x * d0 + bg.y * d1 + bg.z * d2;  // the background layer behind the last splat
        const int h = k >> 1;
        if (k & 1) {
            st.T[h].y = tf; st.dp0[h].y = d0; st.dp1[h].y = d1; st.dp2[h].y = d2; st.A[h].y = a0;
        } else {
            st.T[h].x = tf; st.dp0[h].x = d0; st.dp1[h].x = d1; st.dp2[h].x = d2; st.A[h].x = a0;
        }
        max_last = max(max_last, lastc[k]);
        if (inside) min_last = min(min_last, lastc[k]);
    }
    // splats at list position >= every pixel's n_contrib never contribute: the walk starts there;
    // below every inside pixel's n_contrib the contributor test (backward.cu:486-488) always passes
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        max_last = max(max_last, (uint32_t)__shfl_xor((int)max_last, off));
        min_last = min(min_last, (uint32_t)__shfl_xor((int)min_last, off));
    }
    max_last = __builtin_amdgcn_readfirstlane(max_last);
    min_last = __builtin_amdgcn_readfirstlane(min_last);

    const uint32_t len = range.y - range.x;
    const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
    for (uint32_t p = max_last + lane; p < len; p += 64) {
        float4 *rec = reinterpret_cast<float4 *>(contrib + (size_t)upos[range.x + p] * kContribStride);
        rec[0] = z4;
        rec[1] = z4;
        rec[2] = z4;
    }
    // The walk's instances: emission slot e (where the gradient record goes) and gid_by_e[e] of list
    // position end-1-lane of each batch, loaded 2 batches at a time (independent loads, one wait per
    // refill).  The next batch's attributes are issued before the current batch is blended and only
    // turned into blend constants after it, so their loads are the only ones in flight across the
    // blend loop.
    constexpr int kRing = 2;
    uint32_t ue[kRing], ug[kRing];
    int ids_left = 0;
    auto refill = [&](int end) {
#pragma unroll
        for (int r = 0; r < kRing; r++) {
            const int pos = end - 1 - (r * 64 + lane);
            ue[r] = pos >= 0 ? upos[range.x + pos] : 0u;
        }
#pragma unroll
        for (int r = 0; r < kRing; r++) {
            const int pos = end - 1 - (r * 64 + lane);
            ug[r] = pos >= 0 ? gid_by_e[ue[r]] : 0u;
        }
        ids_left = kRing;
    };
    __shared__ RawLDS s_raw;
    uint32_t unxt = 0;  // where this lane's splat record goes (the instance's emission slot)
    uint32_t rnxt = 0;  // its half-reach bits
    auto fetch = [&](int end) {  // ids of the batch ending at `end`, then its attribute loads
        if (ids_left == 0) refill(end);
        unxt = ue[0];
        const uint32_t ge = ug[0];
        rnxt = ge >> kReachShift;
#pragma unroll
        for (int r = 0; r + 1 < kRing; r++) {
            ue[r] = ue[r + 1];
            ug[r] = ug[r + 1];
        }
        ids_left--;
        issue_raw_lds(s_raw, lane < min(64, end), ge & kGidMask, splat);
    };
    if (max_last > 0) fetch((int)max_last);
    for (int end = (int)max_last; end > 0; end -= 64) {
        const int n = min(64, end);
        const uint32_t ucur = unxt;
        const uint64_t reach[2] = {ballot(lane < n && (rnxt & 1u)), ballot(lane < n && (rnxt & 2u))};
        SplatRegs nxt;
        read_raw_lds(nxt, s_raw, lane, lane < n, yc, true);  // my - yc, as the forward stages it
        // per-splat wave masks (the staged zero splats past n are neither)
        const uint64_t nonpd = ballot(lane < n && !conic_pd(nxt.geo, nxt.opc));
        const uint64_t hiop = ballot(lane < n && nxt.opc.z < kInvCapFree);
        __syncthreads();
        s_sp[lane].geo = nxt.geo;
        s_sp[lane].opc = nxt.opc;
        s_sp[lane].col = nxt.col;
        __syncthreads();
        if (end - 64 > 0) fetch(end - 64);
        // Splats in pairs, each pair one branch-free block over the (splat, half) steps it needs: the
        // falloffs are independent and only the short T / A updates chain, which gives the scheduler up
        // to four chains to interleave.  M0 / M1 = the splats (bit 0: j, bit 1: j + 1) walked on half 0 /
        // half 1: the halves each splat reaches in the common case, all four otherwise (a half a splat
        // does not reach has alpha < 1/255 at every pixel, so walking it changes nothing).  An odd
        // batch's last splat pairs with the zero splat staged past it (opacity 0: an exact no-op).  The
        // two splats' sums share one reduce-scatter.
        auto walk_pair = [&](int j, auto all, auto gen, auto m0, auto m1) {
            constexpr bool ALL = decltype(all)::value, GEN = decltype(gen)::value;
            constexpr int M[2] = {decltype(m0)::value, decltype(m1)::value};
            SplatPart part[2];
            float dxs[2], pa[2], pb[2];
            float4 geo[2], opc[2], col[2];
#pragma unroll
            for (int i = 0; i < 2; i++) {
                geo[i] = s_sp[j + i].geo; opc[i] = s_sp[j + i].opc; col[i] = s_sp[j + i].col;
                dxs[i] = geo[i].x - pfx;
                pa[i] = fmaf(geo[i].z * dxs[i], dxs[i], opc[i].y);  // forward: fmaf(geo.z dx, dx, lo), geo.w dx
                pb[i] = geo[i].w * dxs[i];
            }
            f2 U[2][6];
#pragma unroll
            for (int i = 0; i < 2; i++)
#pragma unroll
                for (int k = 0; k < 6; k++) U[i][k] = bc2(0.f);
            SplatOps so[2];
#pragma unroll
            for (int i = 0; i < 2; i++)
                so[i] = SplatOps{bc2(geo[i].y), bc2(opc[i].x), bc2(opc[i].w), bc2(col[i].x), bc2(col[i].y),
                                 bc2(col[i].z), bc2(pa[i]), bc2(pb[i]), ((nonpd >> (j + i)) & 1) != 0,
                                 (uint32_t)(end - 1 - (j + i))};
#pragma unroll
            for (int h = 0; h < 2; h++) {
                if (M[h] == 3)
                    half_pair_step<ALL, GEN>(st.T[h], st.A[h], st.dp0[h], st.dp1[h], st.dp2[h], so[0], so[1], yl[h],
                                             yl2[h], lastc[2 * h], lastc[2 * h + 1], U[0], U[1]);
                else if (M[h] != 0)
                    half_step<ALL, GEN>(st.T[h], st.A[h], st.dp0[h], st.dp1[h], st.dp2[h], so[M[h] >> 1], yl[h],
                                        yl2[h], lastc[2 * h], lastc[2 * h + 1], U[M[h] >> 1]);
            }
#pragma unroll
            for (int i = 0; i < 2; i++)
                part[i] = SplatPart{hsum(U[i][0]), hsum(U[i][1]), hsum(U[i][2]), hsum(U[i][3]), hsum(U[i][4]),
                                    hsum(U[i][5])};
            wave_sum_pair_to_lds(part[0], part[1], dxs[0], dxs[1], reinterpret_cast<float *>(s_rec[j]), lane, roff);
        };
        using I3 = std::integral_constant<int, 3>;
        auto walk_batch = [&](auto all) {
            for (int j = 0; j < n; j += 2) {
                if (((nonpd | hiop) >> j) & 3) {
                    walk_pair(j, all, std::true_type{}, I3{}, I3{});
                } else {
                    const uint32_t combo = (uint32_t)((reach[0] >> j) & 3u) | (uint32_t)(((reach[1] >> j) & 3u) << 2);
                    auto go = [&](auto c) {
                        constexpr int C = decltype(c)::value;
                        walk_pair(j, all, std::false_type{}, std::integral_constant<int, C & 3>{},
                                  std::integral_constant<int, (C >> 2)>{});
                    };
                    switch (combo) {
                    case 1: go(std::integral_constant<int, 1>{}); break;
                    case 2: go(std::integral_constant<int, 2>{}); break;
                    case 3: go(std::integral_constant<int, 3>{}); break;
                    case 4: go(std::integral_constant<int, 4>{}); break;
                    case 5: go(std::integral_constant<int, 5>{}); break;
                    case 6: go(std::integral_constant<int, 6>{}); break;
                    case 7: go(std::integral_constant<int, 7>{}); break;
                    case 8: go(std::integral_constant<int, 8>{}); break;
                    case 9: go(std::integral_constant<int, 9>{}); break;
                    case 10: go(std::integral_constant<int, 10>{}); break;
                    case 11: go(std::integral_constant<int, 11>{}); break;
                    case 12: go(std::integral_constant<int, 12>{}); break;
                    case 13: go(std::integral_constant<int, 13>{}); break;
                    case 14: go(std::integral_constant<int, 14>{}); break;
                    default: go(std::integral_constant<int, 15>{}); break;
                    }
                }
            }
        };
        // batches wholly below every inside pixel's n_contrib: the contributor test passes everywhere
        if ((uint32_t)(end - 1) < min_last) walk_batch(std::true_type{});
        else walk_batch(std::false_type{});
        __syncthreads();
        if (lane < n) {
            // lane j writes splat j's record, its y moments moved from the tile centre to the splat's
            // centre row: dy = my_l - yl (backward.cu:545-551 moments of dy)
            const float4 r0 = s_rec[lane][0], r1 = s_rec[lane][1], r2 = s_rec[lane][2];
            const float my_l = s_sp[lane].geo.y;  // this lane's splat, my - yc
            const float io = s_sp[lane].opc.z;    // 1 / o: the moments were taken on u' = o u
            // r0 = (S u, S dx u, S u yl, S dx^2 u), r1 = (S dx u yl, S u yl^2, W0, W1), r2 = (W2, -, -, -)
            const float s_u = r0.x, s_uyl = r0.z;
            const float v2 = my_l * s_u - s_uyl;                 // S u dy
            const float v4 = my_l * r0.y - r1.x;                 // S dx u dy
            const float v5 = my_l * v2 - (my_l * s_uyl - r1.y);  // S u dy^2
            float4 *rec = reinterpret_cast<float4 *>(contrib + (size_t)ucur * kContribStride);
            rec[0] = make_float4(s_u * io, r0.y * io, v2 * io, r0.w * io);
            rec[1] = make_float4(v4 * io, v5 * io, r1.z, r1.w);
            rec[2] = r2;
        }
    }
}

hipError_t launch_render_backward(const Args &a, GeomState g, const uint32_t *gid_by_e, const uint32_t *upos,
                                  ImageState img, const float *colors, const float *dL_dpix, float *contrib,
                                  hipStream_t s) {
    const int T = a.gx * a.gy;
    (void)colors;  // the splat records hold the colours the forward blended (colors_precomp or SH)
    hipLaunchKernelGGL(render_backward_kernel, dim3(T), dim3(64), 0, s, a, img.ranges, img.order, gid_by_e, upos,
                       g.splat, img.final_T, img.n_contrib, dL_dpix, contrib);
    return hipGetLastError();
}

}  // namespace gs4d
