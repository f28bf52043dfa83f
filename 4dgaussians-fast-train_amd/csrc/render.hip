// render.hip -- per-tile front-to-back alpha blending (K6) and its reverse walk (K7).
//
// Reference: cuda_rasterizer/forward.cu:261-379 (renderCUDA forward) and backward.cu:399-557
// (renderCUDA backward).
//
// MI355X mapping (not the reference's): ONE wave64 per 16x16 tile; each lane owns a column of 4
// pixels (rows r, r+4, r+8, r+12 with r = lane/16), so a splat's dx and the dx-only part of the
// Gaussian falloff are computed once per lane.  A tile's sorted splats are fetched 64 at a time,
// one per lane (the next batch is prefetched while the current one is blended), and broadcast to
// the wave with v_readlane into scalar registers: no LDS, no workgroup barriers.  The per-pixel
// body is branch-free (predicated with lane masks); a splat that reaches no pixel of the tile is
// skipped with one wave-uniform branch.  Terminated pixels are marked by a negative transmittance.
//
// Backward: per pixel the reference keeps accum_rec[3] and last_color[3] only to form
// dL/dalpha = sum_c (c_c - accum_rec_c) * dL/dpix_c; since dL/dpix is constant per pixel this is
// carried as one scalar (accum_rec . dL/dpix), which is algebraically identical.  The 9 gradient
// terms of a splat (backward.cu:523,545-554) are rewritten as uniform combinations of 6 per-lane
// moments (sum u, sum u dx, sum u dy, sum u dx^2, sum u dx dy, sum u dy^2 with u = G dL/dalpha)
// plus the 3 colour terms; these 9 values are reduced over the wave with two v_permlane swaps and
// a 16-lane DPP tree (reduce-scatter), and the splat's record is stored once per (tile, splat)
// instance at its sorted position (coalesced 48-byte records, no float atomics); a per-Gaussian
// pass sums a Gaussian's records in a fixed order (bitwise reproducible).
#include "gs4d_internal.h"

namespace gs4d {

constexpr int kPix = 4;  // pixels per lane

__device__ __forceinline__ float rl(float v, int l) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}

struct SplatRegs {
    float2 xy;
    float4 co;
    float4 cd;
};

__device__ __forceinline__ void load_splat(SplatRegs &r, bool valid, uint32_t gid, const float2 *__restrict__ xy,
                                           const float4 *__restrict__ conic_opacity, const float4 *__restrict__ rgbd) {
    if (valid) {
        r.xy = xy[gid];
        r.co = conic_opacity[gid];
        r.cd = rgbd[gid];
    } else {
        r.xy = make_float2(0.f, 0.f);
        r.co = make_float4(0.f, 0.f, 0.f, 0.f);
        r.cd = make_float4(0.f, 0.f, 0.f, 0.f);
    }
}

// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(64) void render_forward_kernel(Args a, const uint2 *__restrict__ ranges,
                                                            const uint32_t *__restrict__ point_list,
                                                            const float2 *__restrict__ xy,
                                                            const float4 *__restrict__ conic_opacity,
                                                            const float4 *__restrict__ rgbd,
                                                            float *__restrict__ final_T,
                                                            uint32_t *__restrict__ n_contrib,
                                                            float *__restrict__ out_color,
                                                            float *__restrict__ out_depth) {
    const int tile = blockIdx.x;
    const int tx = tile % a.gx, ty = tile / a.gx;
    const int lane = threadIdx.x;
    const int px = tx * kBlockX + (lane & 15);
    const int py0 = ty * kBlockY + (lane >> 4);
    const float pfx = (float)px;
    float pfy[kPix], T[kPix], C0[kPix], C1[kPix], C2[kPix], Dp[kPix];
    uint32_t last[kPix];
#pragma unroll
    for (int k = 0; k < kPix; k++) {
        pfy[k] = (float)(py0 + 4 * k);
        // outside pixels never blend (forward.cu:287-289): they start "terminated" (T < 0)
        T[k] = (px < a.W && py0 + 4 * k < a.H) ? 1.0f : -1.0f;
        C0[k] = C1[k] = C2[k] = Dp[k] = 0.f;
        last[k] = 0;
    }
    uint2 range = ranges[tile];
    range.x = __builtin_amdgcn_readfirstlane(range.x);
    range.y = __builtin_amdgcn_readfirstlane(range.y);
    SplatRegs cur, nxt;
    if (range.x < range.y) {
        const bool v = range.x + lane < range.y;
        load_splat(cur, v, v ? point_list[range.x + lane] : 0u, xy, conic_opacity, rgbd);
    }
    for (uint32_t base = range.x; base < range.y; base += 64) {
        bool live = false;
#pragma unroll
        for (int k = 0; k < kPix; k++) live |= T[k] > 0.f;
        if (!__any(live)) break;  // every pixel of the tile is done (forward.cu:312-314)
        const uint32_t n = min(64u, range.y - base);
        {
            const uint32_t nb = base + 64;
            const bool v = nb + lane < range.y;
            if (nb < range.y) load_splat(nxt, v, v ? point_list[nb + lane] : 0u, xy, conic_opacity, rgbd);
        }
        for (uint32_t j = 0; j < n; j++) {
            const float sx = rl(cur.xy.x, j), sy = rl(cur.xy.y, j);
            const float ca = rl(cur.co.x, j), cb = rl(cur.co.y, j), cc = rl(cur.co.z, j), op = rl(cur.co.w, j);
            const float dx = sx - pfx;
            const float pa = -0.5f * ca * dx * dx, pb = -cb * dx, pc = -0.5f * cc;
            float alpha[kPix];
            bool valid[kPix];
            uint64_t any = 0;
#pragma unroll
            for (int k = 0; k < kPix; k++) {
                const float dy = sy - pfy[k];
                const float power = pa + dy * (pb + pc * dy);  // = -0.5(a dx^2 + c dy^2) - b dx dy
                alpha[k] = fminf(0.99f, op * __expf(power));
                valid[k] = (power <= 0.0f) && (alpha[k] >= 1.0f / 255.0f) && (T[k] > 0.f);
                any |= __ballot(valid[k]);
            }
            if (any == 0) continue;  // this splat reaches no pixel of the wave
            const float cr = rl(cur.cd.x, j), cg = rl(cur.cd.y, j), cbl = rl(cur.cd.z, j), dep = rl(cur.cd.w, j);
            const uint32_t contributor = base - range.x + j + 1;
#pragma unroll
            for (int k = 0; k < kPix; k++) {
                const float test_T = T[k] * (1 - alpha[k]);
                const bool term = valid[k] && (test_T < 0.0001f);   // forward.cu:349-354
                const bool blend = valid[k] && !term;
                const float w = blend ? alpha[k] * T[k] : 0.f;
                C0[k] += cr * w;
                C1[k] += cg * w;
                C2[k] += cbl * w;
                Dp[k] += dep * w;
                T[k] = blend ? test_T : (term ? -T[k] : T[k]);
                last[k] = blend ? contributor : last[k];
            }
        }
        cur = nxt;
    }
    const size_t HW = (size_t)a.W * a.H;
    const V3 bg = load_v3(a.bg);
#pragma unroll
    for (int k = 0; k < kPix; k++) {
        const int py = py0 + 4 * k;
        if (px < a.W && py < a.H) {
            const float t = fabsf(T[k]);
            const size_t pix = (size_t)py * a.W + px;
            final_T[pix] = t;
            n_contrib[pix] = last[k];
            out_color[pix] = C0[k] + t * bg.x;
            out_color[HW + pix] = C1[k] + t * bg.y;
            out_color[2 * HW + pix] = C2[k] + t * bg.z;
            out_depth[pix] = Dp[k];
        }
    }
}

hipError_t launch_render_forward(const Args &a, GeomState g, BinningState b, ImageState img, float *out_color,
                                 float *out_depth, hipStream_t s) {
    const int T = a.gx * a.gy;
    hipLaunchKernelGGL(render_forward_kernel, dim3(T), dim3(64), 0, s, a, img.ranges, b.point_list, g.xy,
                       g.conic_opacity, g.rgbd, img.final_T, img.n_contrib, out_color, out_depth);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// 16-lane DPP row sum: every lane of each row ends with its row's total.
template <int CTRL>
__device__ __forceinline__ float dpp_add(float v) {
    return v + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float row_sum(float v) {
    v = dpp_add<0xB1>(v);   // quad_perm [1,0,3,2]
    v = dpp_add<0x4E>(v);   // quad_perm [2,3,0,1]
    v = dpp_add<0x141>(v);  // row_half_mirror
    v = dpp_add<0x140>(v);  // row_mirror
    return v;
}
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

// Wave64 totals of 9 per-lane values, returned as wave-uniform scalars.
__device__ __forceinline__ void wave_sum9(const float v[9], float out[9]) {
    const float h0 = swap32_add(v[0], v[1]);  // lo: v0, hi: v1
    const float h1 = swap32_add(v[2], v[3]);  // lo: v2, hi: v3
    const float h2 = swap32_add(v[4], v[5]);
    const float h3 = swap32_add(v[6], v[7]);
    const float h4 = swap32_add(v[8], 0.f);   // lo: v8, hi: 0
    const float q0 = row_sum(swap16_add(h0, h1));  // rows: v0, v2, v1, v3
    const float q1 = row_sum(swap16_add(h2, h3));  // rows: v4, v6, v5, v7
    const float q2 = row_sum(swap16_add(h4, 0.f)); // rows: v8, 0, 0, 0
    out[0] = rl(q0, 0);
    out[2] = rl(q0, 16);
    out[1] = rl(q0, 32);
    out[3] = rl(q0, 48);
    out[4] = rl(q1, 0);
    out[6] = rl(q1, 16);
    out[5] = rl(q1, 32);
    out[7] = rl(q1, 48);
    out[8] = rl(q2, 0);
}

__global__ __launch_bounds__(64) void render_backward_kernel(Args a, const uint2 *__restrict__ ranges,
                                                             const uint32_t *__restrict__ point_list,
                                                             const uint32_t *__restrict__ upos,
                                                             const float2 *__restrict__ xy,
                                                             const float4 *__restrict__ conic_opacity,
                                                             const float4 *__restrict__ rgbd,
                                                             const float *__restrict__ colors,
                                                             const float *__restrict__ final_Ts,
                                                             const uint32_t *__restrict__ n_contrib,
                                                             const float *__restrict__ dL_dpixels,
                                                             float *__restrict__ contrib) {
    const int tile = blockIdx.x;
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

    // per-pixel state: T (recovered backwards), A = accum_rec . dL/dpix, LCD = last_color . dL/dpix
    float pfy[kPix], T[kPix], Tf[kPix], dp0[kPix], dp1[kPix], dp2[kPix], bgdot[kPix], A[kPix], LCD[kPix], la[kPix];
    uint32_t lastc[kPix];
    uint32_t max_last = 0;
#pragma unroll
    for (int k = 0; k < kPix; k++) {
        const int py = py0 + 4 * k;
        pfy[k] = (float)py;
        const bool inside = px < a.W && py < a.H;
        const size_t pix = (size_t)py * a.W + px;
        Tf[k] = inside ? final_Ts[pix] : 0.f;
        T[k] = Tf[k];
        lastc[k] = inside ? n_contrib[pix] : 0u;
        dp0[k] = inside ? dL_dpixels[pix] : 0.f;
        dp1[k] = inside ? dL_dpixels[HW + pix] : 0.f;
        dp2[k] = inside ? dL_dpixels[2 * HW + pix] : 0.f;
        bgdot[k] = bg.x * dp0[k] + bg.y * dp1[k] + bg.z * dp2[k];
        A[k] = 0.f;
        LCD[k] = 0.f;
        la[k] = 0.f;
        max_last = max(max_last, lastc[k]);
    }
    // splats at list position >= every pixel's n_contrib never contribute: the walk starts there
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) max_last = max(max_last, (uint32_t)__shfl_xor((int)max_last, off));
    const float hw = 0.5f * a.W, hh = 0.5f * a.H;  // ddelx_dx, ddely_dy (backward.cu:460-461)

    const uint32_t len = range.y - range.x;
    const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
    for (uint32_t p = max_last + lane; p < len; p += 64) {
        float4 *rec = reinterpret_cast<float4 *>(contrib + (size_t)upos[range.x + p] * kContribStride);
        rec[0] = z4;
        rec[1] = z4;
        rec[2] = z4;
    }
    SplatRegs cur, nxt;
    float4 ccur, cnxt;  // colour operand (colors_precomp or the forward's rgb)
    uint32_t ucur = 0, unxt = 0;  // where this lane's splat record goes (unsorted instance position)
    auto fetch = [&](SplatRegs &r, float4 &c, uint32_t &u, int end) {
        const int n = min(64, end);
        const bool v = lane < n;
        const uint32_t gid = v ? point_list[range.x + end - 1 - lane] : 0u;
        u = v ? upos[range.x + end - 1 - lane] : 0u;
        load_splat(r, v, gid, xy, conic_opacity, rgbd);
        c = r.cd;
        if (colors && v) c = make_float4(colors[3 * gid], colors[3 * gid + 1], colors[3 * gid + 2], 0.f);
    };
    if (max_last > 0) fetch(cur, ccur, ucur, (int)max_last);
    for (int end = (int)max_last; end > 0; end -= 64) {
        const int n = min(64, end);
        if (end - 64 > 0) fetch(nxt, cnxt, unxt, end - 64);
        float acc[9];
#pragma unroll
        for (int q = 0; q < 9; q++) acc[q] = 0.f;
        for (int j = 0; j < n; j++) {
            const uint32_t contributor = (uint32_t)(end - 1 - j);
            const float sx = rl(cur.xy.x, j), sy = rl(cur.xy.y, j);
            const float ca = rl(cur.co.x, j), cb = rl(cur.co.y, j), cc = rl(cur.co.z, j), op = rl(cur.co.w, j);
            const float dx = sx - pfx;
            const float pa = -0.5f * ca * dx * dx, pb = -cb * dx, pc = -0.5f * cc;
            float G[kPix], alpha[kPix], dy[kPix];
            bool valid[kPix];
            uint64_t any = 0;
#pragma unroll
            for (int k = 0; k < kPix; k++) {
                dy[k] = sy - pfy[k];
                const float power = pa + dy[k] * (pb + pc * dy[k]);
                G[k] = __expf(power);
                alpha[k] = fminf(0.99f, op * G[k]);
                valid[k] = (contributor < lastc[k]) && (power <= 0.0f) && (alpha[k] >= 1.0f / 255.0f);
                any |= __ballot(valid[k]);
            }
            if (any == 0) continue;
            const float cr = rl(ccur.x, j), cg = rl(ccur.y, j), cbl = rl(ccur.z, j);
            float U0 = 0.f, U1 = 0.f, U2 = 0.f, W0 = 0.f, W1 = 0.f, W2 = 0.f;
#pragma unroll
            for (int k = 0; k < kPix; k++) {
                const float inv = __builtin_amdgcn_rcpf(1.f - alpha[k]);
                const float Tn = T[k] * inv;                                  // backward.cu:503
                const float CD = cr * dp0[k] + cg * dp1[k] + cbl * dp2[k];
                const float An = la[k] * LCD[k] + (1.f - la[k]) * A[k];       // backward.cu:515 dotted
                const float dLda = (CD - An) * Tn + (-Tf[k] * inv) * bgdot[k];  // :519,525,534
                const float u = valid[k] ? G[k] * dLda : 0.f;
                const float w = valid[k] ? alpha[k] * Tn : 0.f;               // dchannel_dcolor
                T[k] = valid[k] ? Tn : T[k];
                A[k] = valid[k] ? An : A[k];
                LCD[k] = valid[k] ? CD : LCD[k];
                la[k] = valid[k] ? alpha[k] : la[k];
                U0 += u;
                U1 += u * dy[k];
                U2 += u * dy[k] * dy[k];
                W0 += w * dp0[k];
                W1 += w * dp1[k];
                W2 += w * dp2[k];
            }
            const float v[9] = {U0, dx * U0, U1, dx * dx * U0, dx * U1, U2, W0, W1, W2};
            float R[9];
            wave_sum9(v, R);
            // backward.cu:545-554 in terms of the moments (dL_dG = op * dL_dalpha)
            const float g[9] = {hw * op * (-ca * R[1] - cb * R[2]),
                                hh * op * (-cc * R[2] - cb * R[1]),
                                -0.5f * op * R[3],
                                -0.5f * op * R[4],
                                -0.5f * op * R[5],
                                R[0],
                                R[6],
                                R[7],
                                R[8]};
#pragma unroll
            for (int q = 0; q < 9; q++) acc[q] = (lane == j) ? g[q] : acc[q];
        }
        if (lane < n) {
            float4 *rec = reinterpret_cast<float4 *>(contrib + (size_t)ucur * kContribStride);
            rec[0] = make_float4(acc[0], acc[1], acc[2], acc[3]);
            rec[1] = make_float4(acc[4], acc[5], acc[6], acc[7]);
            rec[2] = make_float4(acc[8], 0.f, 0.f, 0.f);
        }
        cur = nxt;
        ccur = cnxt;
        ucur = unxt;
    }
}

hipError_t launch_render_backward(const Args &a, GeomState g, const uint32_t *point_list, const uint32_t *upos,
                                  ImageState img, const float *colors, const float *dL_dpix, float *contrib,
                                  hipStream_t s) {
    const int T = a.gx * a.gy;
    hipLaunchKernelGGL(render_backward_kernel, dim3(T), dim3(64), 0, s, a, img.ranges, point_list, upos, g.xy,
                       g.conic_opacity, g.rgbd, colors, img.final_T, img.n_contrib, dL_dpix, contrib);
    return hipGetLastError();
}

}  // namespace gs4d
