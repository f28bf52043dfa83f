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
//   - grid gradients are summed per workgroup, then across workgroups, in exact integer arithmetic: every
//     (point, tap, feature) term is rounded once to 64-bit fixed point at its plane's power-of-two scale
//     and added into an LDS window over the plane's anchor box (ds_add_u64), whose nonzero cells go to the
//     packed gradient's 64-bit accumulators by one no-return integer atomic each.  Integer sums are
//     exact, so no schedule changes a bit: the backward is deterministic by construction (there is no
//     float-atomic mode).  The per-plane scale bounds every cell's sum: point i's terms are at most m_i =
//     max_f |dfeat_{i,l,f}| times the product of the other five planes' max|param| (each bilinear sample is a
//     convex combination of its plane's parameters), a cell takes at most one tap per point, so |sum| <=
//     sum_i m_i prod_q max|param_q| < 2^61 at the chosen scale (hex_plane_scale; details at
//     hexplane_backward_kernel).  One launch unpacks the accumulators to floats in the (1, F, H, W) layout.
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

// Backward, deterministic by construction.  A workgroup serves NPW consecutive points of the Morton order
// (hex_points_per_wg: 2048 / F, at least one chunk of 256 / (F/4) points, at most 128), so they cover a small
// box of the field.  Per level:
//   1. each point's reverse pass (F/4 lanes) writes its 6 plane gradients dv (F floats each), its bilinear
//      anchor cell (x0, y0) and unnormalised coordinates (ix, iy) to LDS, and reduces its coordinate
//      gradient with shuffles;
//   2. per plane: the anchors' box; every (point, tap, feature) term w * dv (make_tap's weights) is rounded
//      ONCE to a 64-bit fixed-point integer at the plane's power-of-two scale (hex_plane_scale) and added into
//      an LDS window over the box's cells with ds_add_u64; the window's nonzero sums then go to the packed
//      gradient's 64-bit accumulators with one no-return integer atomic each, and hex_fix_to_float_kernel
//      turns them into floats.  Integer sums are exact, so neither the order of the LDS adds nor that of the
//      workgroups' atomics changes a bit: the gradients are bitwise reproducible with no ordering work at all.
//      A box too large for the window at F features is covered in feature slices (F/2, F/4 per pass); beyond
//      that its terms go straight to the global accumulators (still exact).
// Measured on this chip (tools/bench/lds_atomics.hip, global_atomics.hip): ds_add_u64 ~7.4 lane-ops per clock
// per CU, as fast as a plain LDS read-modify-write (ds_add_f32: 0.33); global u64 atomics as fast as f32 ones
// (2x faster on 4096 hot addresses).  The previous design counting-sorted each plane's taps by cell in LDS
// and gathered them (float atomics across workgroups; a fixed-point mode that ranked taps by ballots was
// ~300 us against 225).
constexpr int kHexDvFloats = 2048;   // NPW * F
constexpr int kHexLdsWords = 20480;  // 80 KiB: two workgroups per CU, as the registers allow
// scale words: [0] max|dfeat|, [1 + p] max|param| of plane p, [32 + p] the scale of plane p (written by the
// backward's workgroup 0 for the conversion launches), [63] non-finite flag; then kHexHistWords words: per
// level, the histogram of the points' m_i = max_f |dfeat_{i,l,f}| by binary exponent (bin e counts the m_i
// in (2^(e-128), 2^(e-127)]: an upper bound of sum_i m_i that integer atomics build the same in every run)
constexpr int kHexNanWord = 63, kHexScaleWord = 32, kHexMxWords = 64;
constexpr int kHexHistBins = 256, kHexHistWords = GS4D_HEXPLANE_MAX_LEVELS * kHexHistBins;

__host__ __device__ __forceinline__ int hex_points_per_wg(int F) {
    const int ppc = kHexThreads / (F / 4);
    const int fit = kHexDvFloats / F;
    const int want = fit < 128 ? fit : 128;
    return ppc > want ? ppc : want;  // a whole number of chunks
}
// LDS words of the backward's fixed arrays (s_dv, s_anc, s_ixy, boxes); the rest of kHexLdsWords is the
// 64-bit window
__host__ __device__ __forceinline__ int hex_bwd_fixed_words(int F) {
    const int npw = hex_points_per_wg(F);
    // (+ 2 GS4D_HEXPLANE_MAX_LEVELS words: the per-level bound sums, doubles just below the window)
    return (6 * npw * F + 6 * npw * 3 + 6 * 4 + 4 * 6 * 4 + 8 + 1 + 2 * GS4D_HEXPLANE_MAX_LEVELS) & ~1;
}
__host__ __device__ __forceinline__ int hex_bwd_window(int F) { return (kHexLdsWords - hex_bwd_fixed_words(F)) / 2; }

// The fixed-point scale of plane p (of level l): 2^e with e chosen so that the largest possible cell sum fits
// 2^61.  A term is w dv with w <= 1 and dv = dfeat * the product of the level's 5 other plane values, each a
// convex combination of its plane's parameters, and a cell takes at most one tap per point, so
//   |sum| <= sum_i m_i prod_{q != p} max|param_q|,   m_i = max_f |dfeat_{i,l,f}|
// with sum_i m_i bounded from above by msum = sum_e hist[l][e] 2^(e-127) (each m_i rounded up to a power of
// two; computed in double: no overflow).  Round 5 used N max|dfeat| in its place: with heavy-tailed dfeat
// (a few points' gradients far above the rest) that wasted up to log2(max/mean) bits of every cell's
// resolution.  A zero bound (every term is 0) takes 1; a bound beyond the float exponent range clamps e to its
// minimum, -126 (the largest term is a float, < 2^128, so N of them scaled by 2^-126 still fit); non-finite
// inputs are flagged separately (kHexNanWord).
__device__ __forceinline__ float hex_plane_scale(double msum, const uint32_t *mx, int l, int p) {
    double b = msum;
    for (int q = 0; q < 6; q++)
        if (q != p) b *= (double)__uint_as_float(mx[1 + 6 * l + q]);
    if (!(b > 0.0)) return 1.f;
    int ex;
    (void)frexp(b, &ex);  // b < 2^ex
    return ldexpf(1.f, max(-126, min(127, 61 - ex)));
}
// the scale of plane pg as the backward's workgroup 0 stored it (the conversion launches run after it)
__device__ __forceinline__ float hex_stored_scale(const uint32_t *mx, int pg) { return __uint_as_float(mx[kHexScaleWord + pg]); }
__device__ __forceinline__ unsigned long long hex_fix(float v, float scale) {
    return (unsigned long long)__float2ll_rn(v * scale);  // scale is a power of two: v * scale is exact
}
// Maxima of |x| for the scales: blockIdx.y = r selects range r of `rg` (n_r floats at x_r) and its word
// mx[w_r]; a non-finite element sets mx[kHexNanWord] (fmaxf would skip a NaN).  Float bits of a
// non-negative value order like unsigned integers.
struct HexMaxRanges {
    const float *x[1 + 6 * GS4D_HEXPLANE_MAX_LEVELS];
    int64_t n[1 + 6 * GS4D_HEXPLANE_MAX_LEVELS];
    int first[2 + 6 * GS4D_HEXPLANE_MAX_LEVELS];  // first block of each range (blocks in proportion to its size)
    int nr;
    int N, levels, F;  // range 0 is dfeat, (N, levels F)
};
// Range 0 (dfeat): one (point, level) row of F floats per thread item: its m_i = max_f |dfeat| goes to the
// level's exponent histogram (LDS, then one global integer add per nonzero bin) and to the maximum.
__device__ __forceinline__ void hex_dfeat_pass(const HexMaxRanges &rg, int b, int nb, uint32_t *__restrict__ mx,
                                               float &m, bool &bad) {
    __shared__ uint32_t s_hist[GS4D_HEXPLANE_MAX_LEVELS][kHexHistBins];
    for (int e = threadIdx.x; e < rg.levels * kHexHistBins; e += 256) (&s_hist[0][0])[e] = 0u;
    __syncthreads();
    const int G = rg.F / 4;
    const float4 *x = reinterpret_cast<const float4 *>(rg.x[0]);
    const int64_t rows = (int64_t)rg.N * rg.levels;
    for (int64_t i = (int64_t)b * 256 + threadIdx.x; i < rows; i += (int64_t)nb * 256) {
        float a = 0.f;
        for (int k = 0; k < G; k++) {
            const float4 v = x[i * G + k];
            const float t = fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w)));
            bad |= !(t <= 3.4028235e38f) || v.x != v.x || v.y != v.y || v.z != v.z || v.w != v.w;
            a = fmaxf(a, t);
        }
        m = fmaxf(m, a);
        if (a > 0.f && a <= 3.4028235e38f) {
            // bin: the smallest e with a <= 2^(e-127) (denormals in bin 1: 2^-126)
            const uint32_t u = __float_as_uint(a), ex = u >> 23;
            const uint32_t e = ex == 0u ? 1u : ex + ((u & 0x7FFFFFu) != 0u ? 1u : 0u);
            atomicAdd(&s_hist[(int)(i % rg.levels)][min(e, (uint32_t)kHexHistBins - 1u)], 1u);
        }
    }
    __syncthreads();
    uint32_t *hist = mx + kHexMxWords;
    for (int e = threadIdx.x; e < rg.levels * kHexHistBins; e += 256) {
        const uint32_t c = (&s_hist[0][0])[e];
        if (c) atomicAdd(hist + e, c);
    }
}
__global__ __launch_bounds__(256) void hex_max_kernel(HexMaxRanges rg, uint32_t *__restrict__ mx) {
    int r = 0;
    while (r + 1 < rg.nr && (int)blockIdx.x >= rg.first[r + 1]) r++;
    const float4 *x = reinterpret_cast<const float4 *>(rg.x[r]);  // every range is float4-aligned, n % 4 == 0
    const int64_t n = r == 0 ? 0 : rg.n[r] / 4;
    const int b = (int)blockIdx.x - rg.first[r], nb = rg.first[r + 1] - rg.first[r];
    float m = 0.f;
    bool bad = false;
    if (r == 0) hex_dfeat_pass(rg, b, nb, mx, m, bad);  // uniform over the block
    // sixteen 16-byte loads in flight per thread per round (the range is split over few blocks: each block's
    // maximum is one atomicMax on the range's word, and those serialise; so the rounds must be few and wide)
    constexpr int kU = 16;
    for (int64_t i0 = (int64_t)b * (256 * kU) + threadIdx.x; i0 < n; i0 += (int64_t)nb * (256 * kU)) {
        float4 v[kU];
#pragma unroll
        for (int u = 0; u < kU; u++) v[u] = i0 + u * 256 < n ? x[i0 + u * 256] : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int u = 0; u < kU; u++) {
            const float a = fmaxf(fmaxf(fabsf(v[u].x), fabsf(v[u].y)), fmaxf(fabsf(v[u].z), fabsf(v[u].w)));
            bad |= !(a <= 3.4028235e38f) || v[u].x != v[u].x || v[u].y != v[u].y || v[u].z != v[u].z ||
                   v[u].w != v[u].w;
            m = fmaxf(m, a);
        }
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) m = fmaxf(m, __shfl_xor(m, off));
    const bool any_bad = __builtin_amdgcn_ballot_w64(bad) != 0;
    __shared__ float s_m[4];
    __shared__ int s_bad[4];
    if ((threadIdx.x & 63) == 0) {
        s_m[threadIdx.x >> 6] = m;
        s_bad[threadIdx.x >> 6] = any_bad;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        m = fmaxf(fmaxf(s_m[0], s_m[1]), fmaxf(s_m[2], s_m[3]));
        if (m > 0.f) atomicMax(mx + r, __float_as_uint(m));
        if (s_bad[0] | s_bad[1] | s_bad[2] | s_bad[3]) atomicOr(mx + kHexNanWord, 1u);
    }
}
// the fixed-point sums to floats in the packed layout, plane by plane (blockIdx.y), for callers that want the
// packed buffer (the glue writes the planes directly: the unpack's FIX load)
__global__ __launch_bounds__(256) void hex_fix_to_packed_kernel(gs4d_hexplane_layout lay, int N,
                                                                const uint32_t *__restrict__ mx,
                                                                const long long *__restrict__ acc,
                                                                float *__restrict__ out) {
    const int pg = blockIdx.y, l = pg / 6, p = pg - 6 * l;
    const gs4d_hexplane_plane pl = lay.plane[pg];
    const int64_t n = (int64_t)pl.W * pl.H * lay.F;
    (void)l, (void)p, (void)N;
    const float inv = 1.f / hex_stored_scale(mx, pg);
    const bool nan = mx[kHexNanWord] != 0;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
        out[pl.offset + i] = nan ? __builtin_nanf("") : (float)acc[pl.offset + i] * inv;
}

__global__ __launch_bounds__(kHexThreads) void hexplane_backward_kernel(int N, const float *__restrict__ pts,
                                                                        const uint32_t *__restrict__ order,
                                                                        gs4d_hexplane_layout lay,
                                                                        const float *__restrict__ packed,
                                                                        const float *__restrict__ dfeat,
                                                                        uint32_t *__restrict__ mx,
                                                                        unsigned long long *__restrict__ dfix,
                                                                        float *__restrict__ dpts) {
    __shared__ unsigned long long smem64[kHexLdsWords / 2];
    float *const smem = reinterpret_cast<float *>(smem64);
    const int F = lay.F, G = F / 4, ppc = kHexThreads / G;
    const int npw = hex_points_per_wg(F), cpw = npw / ppc;
    const int fixed = hex_bwd_fixed_words(F), wcap = hex_bwd_window(F);
    float *s_dv = smem;                                            // [6][npw][F]
    int *s_anc = (int *)(s_dv + 6 * npw * F);                      // [6][npw]: y0 << 16 | x0, -1: none
    float2 *s_ixy = (float2 *)(s_anc + 6 * npw);                   // [6][npw]
    int *s_box = (int *)(s_ixy + 6 * npw);                         // [6][4]: ax0, ay0, aw, ah
    int *s_wbox = s_box + 24;                                      // [waves][6][4]
    unsigned long long *s_win = smem64 + fixed / 2;                // [wcap]: the fixed-point window
    const int q = threadIdx.x % G, slot = threadIdx.x / G;
    const int lane = threadIdx.x & 63, wv = (int)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int64_t first = (int64_t)blockIdx.x * npw;
    // per level: msum = sum_e hist[l][e] 2^(e-127) (hex_plane_scale), the same fixed-order sum in every
    // workgroup (thread t takes bin t; the wave tree; the waves in order).  The waves' partials use the
    // window's first words before it is zeroed; the sums stay in the fixed region, just below the window.
    double *const s_msum = reinterpret_cast<double *>(s_win) - GS4D_HEXPLANE_MAX_LEVELS;
    {
        double *s_part = reinterpret_cast<double *>(s_win);  // [level][wave]
        const uint32_t *hist = mx + kHexMxWords;
        for (int l = 0; l < lay.levels; l++) {
            double v = ldexp((double)hist[l * kHexHistBins + threadIdx.x], (int)threadIdx.x - 127);
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
            if (lane == 0) s_part[l * (kHexThreads / 64) + wv] = v;
        }
        __syncthreads();
        if ((int)threadIdx.x < lay.levels) {
            double t = 0.0;
            for (int w = 0; w < kHexThreads / 64; w++) t += s_part[threadIdx.x * (kHexThreads / 64) + w];
            s_msum[threadIdx.x] = t;
        }
        __syncthreads();
        if (blockIdx.x == 0 && (int)threadIdx.x < 6 * lay.levels)  // for the conversion launches after this one
            mx[kHexScaleWord + threadIdx.x] = __float_as_uint(hex_plane_scale(s_msum[threadIdx.x / 6], mx,
                                                                              threadIdx.x / 6, threadIdx.x % 6));
    }
    for (int e = threadIdx.x; e < wcap; e += kHexThreads) s_win[e] = 0ull;  // flushes leave it zeroed
    __syncthreads();
    for (int l = 0; l < lay.levels; l++) {
        // 1. reverse passes
        for (int c = 0; c < cpw; c++) {
            const int j = c * ppc + slot;
            const int64_t i = first + j;
            const int n = i < N ? (order ? (int)order[i] : (int)i) : -1;
            if (n < 0) {
                if (q == 0)
                    for (int p = 0; p < 6; p++) s_anc[p * npw + j] = -1;
                continue;
            }
            const float4 p4 = reinterpret_cast<const float4 *>(pts)[n];
            const float pc[4] = {p4.x, p4.y, p4.z, p4.w};
            float gpt[4] = {0.f, 0.f, 0.f, 0.f};
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
                const gs4d_hexplane_plane pl = lay.plane[6 * l + p];
                const Tap t = make_tap(pc[kPairC0[p]], pc[kPairC1[p]], pl.W, pl.H);
                const TapVals r = load_taps(packed + pl.offset, t, F, q);
                float gix = 0.f, giy = 0.f;
                const float x1 = (float)(t.x0 + 1), y1 = (float)(t.y0 + 1), x0 = (float)t.x0, y0 = (float)t.y0;
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    const float go = dv[k];
                    // grid_sampler_2d_backward (bilinear): input gradient and coordinate gradient
                    gix -= sel(r.v00, k) * (y1 - t.iy) * go;
                    giy -= sel(r.v00, k) * (x1 - t.ix) * go;
                    gix += sel(r.v10, k) * (y1 - t.iy) * go;
                    giy -= sel(r.v10, k) * (t.ix - x0) * go;
                    gix -= sel(r.v01, k) * (t.iy - y0) * go;
                    giy += sel(r.v01, k) * (x1 - t.ix) * go;
                    gix += sel(r.v11, k) * (t.iy - y0) * go;
                    giy += sel(r.v11, k) * (t.ix - x0) * go;
                }
                *reinterpret_cast<float4 *>(s_dv + (p * npw + j) * F + 4 * q) = make_float4(dv[0], dv[1], dv[2], dv[3]);
                if (q == 0) {
                    const bool ok = t.x0 >= 0 && t.x0 < pl.W && t.y0 >= 0 && t.y0 < pl.H;  // false for NaN
                    s_anc[p * npw + j] = ok ? (t.y0 << 16) | t.x0 : -1;
                    s_ixy[p * npw + j] = make_float2(t.ix, t.iy);
                }
                gpt[kPairC0[p]] += t.gxm * gix;
                gpt[kPairC1[p]] += t.gym * giy;
            }
            // sum the coordinate gradient over the point's lanes; levels accumulate in dpts
#pragma unroll
            for (int k = 0; k < 4; k++)
                for (int off = 1; off < G; off <<= 1) gpt[k] += __shfl_xor(gpt[k], off, G);
            if (q == 0) {
                float4 *o = reinterpret_cast<float4 *>(dpts) + n;
                float4 acc = l == 0 ? make_float4(0.f, 0.f, 0.f, 0.f) : *o;
                acc.x += gpt[0]; acc.y += gpt[1]; acc.z += gpt[2]; acc.w += gpt[3];
                *o = acc;
            }
        }
        __syncthreads();
        // 2a. the anchors' boxes of the 6 planes (wave min/max, then over the waves)
        {
            int bx[6][4];
#pragma unroll
            for (int p = 0; p < 6; p++) {
                const int a = threadIdx.x < npw ? s_anc[p * npw + threadIdx.x] : -1;
                const bool ok = a >= 0;
                bx[p][0] = ok ? (a & 0xFFFF) : INT_MAX;
                bx[p][1] = ok ? (a >> 16) : INT_MAX;
                bx[p][2] = ok ? (a & 0xFFFF) : INT_MIN;
                bx[p][3] = ok ? (a >> 16) : INT_MIN;
            }
#pragma unroll
            for (int o = 32; o >= 1; o >>= 1)
#pragma unroll
                for (int p = 0; p < 6; p++) {
                    bx[p][0] = min(bx[p][0], __shfl_xor(bx[p][0], o, 64));
                    bx[p][1] = min(bx[p][1], __shfl_xor(bx[p][1], o, 64));
                    bx[p][2] = max(bx[p][2], __shfl_xor(bx[p][2], o, 64));
                    bx[p][3] = max(bx[p][3], __shfl_xor(bx[p][3], o, 64));
                }
            if (lane == 0)
#pragma unroll
                for (int p = 0; p < 6; p++)
#pragma unroll
                    for (int k = 0; k < 4; k++) s_wbox[(wv * 6 + p) * 4 + k] = bx[p][k];
        }
        __syncthreads();
        if (threadIdx.x < 6) {
            const int p = threadIdx.x;
            int x0 = INT_MAX, y0 = INT_MAX, x1 = INT_MIN, y1 = INT_MIN;
            for (int w = 0; w < kHexThreads / 64; w++) {
                x0 = min(x0, s_wbox[(w * 6 + p) * 4 + 0]);
                y0 = min(y0, s_wbox[(w * 6 + p) * 4 + 1]);
                x1 = max(x1, s_wbox[(w * 6 + p) * 4 + 2]);
                y1 = max(y1, s_wbox[(w * 6 + p) * 4 + 3]);
            }
            s_box[p * 4 + 0] = x0;
            s_box[p * 4 + 1] = y0;
            s_box[p * 4 + 2] = x1 >= x0 ? x1 - x0 + 1 : 0;
            s_box[p * 4 + 3] = y1 >= y0 ? y1 - y0 + 1 : 0;
        }
        __syncthreads();
        // 2b. per plane: fixed-point terms into the LDS window over the box's cells, then to HBM
        for (int p = 0; p < 6; p++) {
            const gs4d_hexplane_plane pl = lay.plane[6 * l + p];
            const int ax0 = s_box[p * 4 + 0], ay0 = s_box[p * 4 + 1], aw = s_box[p * 4 + 2], ah = s_box[p * 4 + 3];
            if (aw * ah == 0) continue;  // uniform
            const float scale = hex_plane_scale(s_msum[l], mx, l, p);
            const float *dvp = s_dv + p * npw * F;
            const int *ancp = s_anc + p * npw;
            const float2 *ixyp = s_ixy + p * npw;
            unsigned long long *dpl = dfix + pl.offset;
            // the touched cells: the anchors' box and its +1 neighbours inside the plane
            const int cw = min(ax0 + aw, pl.W - 1) - ax0 + 1, ch = min(ay0 + ah, pl.H - 1) - ay0 + 1;
            const int nc = cw * ch;
            int fp = F;  // features per pass (uniform)
            while (nc * fp > wcap && fp > 4) fp >>= 1;
            if (nc * fp > wcap) {
                // uniform: a box too large even at 4 features per pass -- terms straight to the accumulators
                for (int e = threadIdx.x; e < npw * F; e += kHexThreads) {
                    const int j = e / F, f = e - j * F;
                    const int a = ancp[j];
                    if (a < 0) continue;
                    const int x0 = a & 0xFFFF, y0 = a >> 16;
                    const float2 ixy = ixyp[j];
                    const float d = dvp[j * F + f];
                    const float xa = (float)(x0 + 1) - ixy.x, xb = ixy.x - (float)x0;
                    const float ya = (float)(y0 + 1) - ixy.y, yb = ixy.y - (float)y0;
                    const bool in_x1 = x0 + 1 < pl.W, in_y1 = y0 + 1 < pl.H;
                    unsigned long long *b0 = dpl + ((size_t)y0 * pl.W + x0) * F + f;
                    atomicAdd(b0, hex_fix((xa * ya) * d, scale));
                    if (in_x1) atomicAdd(b0 + F, hex_fix((xb * ya) * d, scale));
                    if (in_y1) atomicAdd(b0 + (size_t)pl.W * F, hex_fix((xa * yb) * d, scale));
                    if (in_x1 && in_y1) atomicAdd(b0 + (size_t)(pl.W + 1) * F, hex_fix((xb * yb) * d, scale));
                }
                // every wave is done reading this plane's s_dv / s_anc / s_ixy before any starts the next
                // level's step 1, which overwrites them (the branch is uniform: the barrier is reached by all)
                __syncthreads();
                continue;
            }
            const int gp = fp / 4, lg = __builtin_ctz(gp), lf = __builtin_ctz(fp);  // powers of two
            const float inv_cw = 1.f / (float)cw;
            for (int f0 = 0; f0 < F; f0 += fp) {
                // items (point j, tap t, group b): consecutive lanes take a tap's consecutive feature groups
                for (int e = threadIdx.x; e < npw * 4 * gp; e += kHexThreads) {
                    const int b = e & (gp - 1), t = (e >> lg) & 3, j = e >> (lg + 2);
                    const int a = ancp[j];
                    if (a < 0) continue;
                    const int x0 = a & 0xFFFF, y0 = a >> 16, tx = t & 1, ty = t >> 1;
                    if ((tx && x0 + 1 >= pl.W) || (ty && y0 + 1 >= pl.H)) continue;
                    const float2 ixy = ixyp[j];
                    // make_tap's weights: w00 = xa ya, w10 = xb ya, w01 = xa yb, w11 = xb yb
                    const float wx = tx ? ixy.x - (float)x0 : (float)(x0 + 1) - ixy.x;
                    const float wy = ty ? ixy.y - (float)y0 : (float)(y0 + 1) - ixy.y;
                    const float w = wx * wy;
                    const float4 d = *reinterpret_cast<const float4 *>(dvp + j * F + f0 + 4 * b);
                    unsigned long long *c = s_win + ((y0 + ty - ay0) * cw + (x0 + tx - ax0)) * fp + 4 * b;
                    atomicAdd(c + 0, hex_fix(w * d.x, scale));
                    atomicAdd(c + 1, hex_fix(w * d.y, scale));
                    atomicAdd(c + 2, hex_fix(w * d.z, scale));
                    atomicAdd(c + 3, hex_fix(w * d.w, scale));
                }
                __syncthreads();
                // flush the nonzero sums (and leave the window zeroed for the next pass)
                for (int e = threadIdx.x; e < nc * fp; e += kHexThreads) {
                    const unsigned long long v = s_win[e];
                    if (v == 0ull) continue;
                    s_win[e] = 0ull;
                    const int cell = e >> lf, f = e & (fp - 1);
                    // cell / cw by a float reciprocal: (cell + 0.5) / cw lies >= 0.5 / cw >= 2^-11 from an
                    // integer, far beyond the float quotient's error (cell < 2^16)
                    const int ry = (int)(((float)cell + 0.5f) * inv_cw), rx = cell - ry * cw;
                    atomicAdd(dpl + ((size_t)(ay0 + ry) * pl.W + ax0 + rx) * F + f0 + f, v);
                }
                __syncthreads();
            }
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
constexpr int kHexSortThreads = 1024, kHexSortItems = 4;
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
// FIX (unpack only): the source is the backward's 64-bit fixed-point sums `fix` (same layout), turned into
// floats at the plane's scale on the way (NaN everywhere when an input was not finite: a float sum would
// have propagated it)
template <bool PACK, int FC, bool FIX = false>  // FC: the feature count when known at compile time (all loads in flight), else 0
__global__ __launch_bounds__(kRepackThreads) void hexplane_repack_kernel(gs4d_hexplane_layout lay,
                                                                         float *__restrict__ packed,
                                                                         const long long *__restrict__ fix = nullptr,
                                                                         const uint32_t *__restrict__ mx = nullptr,
                                                                         int N = 0) {
    extern __shared__ float s_tile[];  // F x (TC + 1)
    int64_t tile = blockIdx.x;
    const int p = repack_plane(lay, tile);
    if (p >= 6 * lay.levels) return;
    const gs4d_hexplane_plane pl = lay.plane[p];
    float inv = 1.f;
    bool nan = false;
    if (FIX) {
        (void)N;
        inv = 1.f / hex_stored_scale(mx, p);
        nan = mx[kHexNanWord] != 0;
    }
    auto src = [&](int64_t i) -> float {  // element i of the plane's packed block
        if (!FIX) return packed[pl.offset + i];
        return nan ? __builtin_nanf("") : (float)fix[pl.offset + i] * inv;
    };
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
                v[j] = k < nc * FC ? src(c0 * F + k) : 0.f;
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
        for (int k = t; k < nc * F; k += kRepackThreads) s_tile[(k % F) * TS + k / F] = src(c0 * F + k);
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

// backward scratch: the scale words and the 64-bit fixed-point accumulators of the packed buffer
size_t gs4d_hexplane_backward_scratch_bytes(int N, const gs4d_hexplane_layout *lay) {
    (void)N;
    if (!lay) return 256;
    return 4 * (size_t)(kHexMxWords + kHexHistWords) + 8 * (size_t)lay->total + 256;
}

int gs4d_hexplane_backward(int N, const float *pts, const uint32_t *order, const gs4d_hexplane_layout *lay,
                           const float *packed, const float *dfeat, float *dpacked, float *dpts, void *scratch,
                           int deterministic, void *stream) {
    (void)deterministic;  // always deterministic (fixed-point sums); kept for the ABI
    if (N < 0 || !lay || (N > 0 && (!pts || !packed || !dfeat || !dpts || !scratch))) return 1;
    if (((size_t)pts & 15) || ((size_t)packed & 15) || ((size_t)dfeat & 15) || ((size_t)dpts & 15)) return 1;
    if (lay->levels < 1 || lay->levels > GS4D_HEXPLANE_MAX_LEVELS) return 1;
    hipStream_t s = (hipStream_t)stream;
    if (N == 0) {
        bool direct = true;
        for (int p = 0; p < 6 * lay->levels; p++) direct = direct && lay->plane[p].grad;
        if (direct) {
            for (int p = 0; p < 6 * lay->levels; p++)
                if (hipMemsetAsync(lay->plane[p].grad, 0, 4 * (size_t)lay->plane[p].W * lay->plane[p].H * lay->F, s) !=
                    hipSuccess)
                    return 3;
            return 0;
        }
        return dpacked && hipMemsetAsync(dpacked, 0, 4 * (size_t)lay->total, s) == hipSuccess ? 0 : 3;
    }
    const int64_t per_wg = hex_points_per_wg(lay->F);
    const int64_t nwg = ((int64_t)N + per_wg - 1) / per_wg;
    if (hex_bwd_window(lay->F) < 4 * 4) return 1;
    const int np = 6 * lay->levels;
    uint32_t *mx = (uint32_t *)align_up((size_t)scratch, 256);
    unsigned long long *dfix = (unsigned long long *)(mx + kHexMxWords + kHexHistWords);
    if (hipMemsetAsync(mx, 0, 4 * (size_t)(kHexMxWords + kHexHistWords) + 8 * (size_t)lay->total, s) != hipSuccess)
        return 3;
    HexMaxRanges rg;
    rg.nr = 1 + np;
    rg.N = N, rg.levels = lay->levels, rg.F = lay->F;
    rg.x[0] = dfeat;
    rg.n[0] = (int64_t)N * lay->levels * lay->F;
    for (int p = 0; p < np; p++) {
        rg.x[1 + p] = packed + lay->plane[p].offset;
        rg.n[1 + p] = (int64_t)lay->plane[p].W * lay->plane[p].H * lay->F;
    }
    rg.first[0] = 0;
    for (int r = 0; r < rg.nr; r++)  // >= 16 float4 per thread, at most 128 blocks per range
        rg.first[r + 1] = rg.first[r] + (int)std::min<int64_t>(128, std::max<int64_t>(1, (rg.n[r] + 16383) / 16384));
    static_assert(kHexScaleWord + 6 * GS4D_HEXPLANE_MAX_LEVELS <= kHexNanWord, "scale words overlap the flag");
    hipLaunchKernelGGL(hex_max_kernel, dim3(rg.first[rg.nr]), dim3(256), 0, s, rg, mx);
    hipLaunchKernelGGL(hexplane_backward_kernel, dim3((unsigned)nwg), dim3(kHexThreads), 0, s, N, pts, order, *lay,
                       packed, dfeat, mx, dfix, dpts);
    // the fixed-point sums to floats: straight into the (1, F, H, W) gradients when the caller set them (the
    // unpack transpose with the conversion on its load), else into the packed buffer
    bool direct = true;
    for (int p = 0; p < np; p++) direct = direct && lay->plane[p].grad;
    const dim3 grid((unsigned)repack_tiles(*lay));
    const size_t lds = 4 * (size_t)lay->F * (repack_cells(lay->F) + 1);
    const long long *fx = (const long long *)dfix;
    if (direct) {
        if (lay->F == 16)
            hipLaunchKernelGGL((hexplane_repack_kernel<false, 16, true>), grid, dim3(kRepackThreads), lds, s, *lay,
                               nullptr, fx, mx, N);
        else if (lay->F == 32)
            hipLaunchKernelGGL((hexplane_repack_kernel<false, 32, true>), grid, dim3(kRepackThreads), lds, s, *lay,
                               nullptr, fx, mx, N);
        else
            hipLaunchKernelGGL((hexplane_repack_kernel<false, 0, true>), grid, dim3(kRepackThreads), lds, s, *lay,
                               nullptr, fx, mx, N);
    } else {
        if (!dpacked) return 1;
        hipLaunchKernelGGL(hex_fix_to_packed_kernel, dim3(64, np), dim3(256), 0, s, *lay, N, mx, fx, dpacked);
    }
    return hipGetLastError() == hipSuccess ? 0 : 3;
}

}  // extern "C"
