// render.hip -- per-tile front-to-back alpha blending (K6) and its reverse walk (K7).
//
// Reference: cuda_rasterizer/forward.cu:261-379 (renderCUDA forward) and backward.cu:399-557
// (renderCUDA backward).
//
// MI355X mapping (not the reference's): ONE wave64 per 16x16 tile, each lane owns a column of 4
// pixels (rows r, r+4, r+8, r+12 with r = lane/16).  A tile's sorted splats are fetched 64 at a
// time, one per lane, into registers, then broadcast to the whole wave with v_readlane (scalar
// registers) -- no LDS and no workgroup barriers.  The 4 pixels of a lane share the splat's dx,
// so part of the Gaussian falloff is computed once per lane.  In the backward pass the 9 gradient
// terms of each splat are first summed over the lane's 4 pixels in registers, then over the wave
// with DPP row operations, and stored once per (tile, splat) instance with a plain store; a
// per-Gaussian pass later sums a Gaussian's instances in a fixed order (no float atomics, so the
// result is bitwise reproducible).
#include "gs4d_internal.h"

namespace gs4d {

constexpr int kPix = 4;  // pixels per lane

__device__ __forceinline__ float readlane_f(float v, int l) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
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
    const V3 bg = load_v3(a.bg);
    float T[kPix], C[kPix][3], Dp[kPix];
    uint32_t last[kPix];
    bool done[kPix];
#pragma unroll
    for (int k = 0; k < kPix; k++) {
        T[k] = 1.0f;
        C[k][0] = C[k][1] = C[k][2] = 0.f;
        Dp[k] = 0.f;
        last[k] = 0;
        done[k] = !(px < a.W && py0 + 4 * k < a.H);  // outside pixels never blend (forward.cu:287-289)
    }
    const uint2 range = ranges[tile];
    for (uint32_t base = range.x; base < range.y; base += 64) {
        bool any_live = false;
#pragma unroll
        for (int k = 0; k < kPix; k++) any_live |= !done[k];
        if (!__any(any_live)) break;   // forward.cu:312-314
        const uint32_t n = min(64u, range.y - base);
        float2 m_xy = make_float2(0.f, 0.f);
        float4 m_co = make_float4(0.f, 0.f, 0.f, 0.f), m_cd = make_float4(0.f, 0.f, 0.f, 0.f);
        if ((uint32_t)lane < n) {
            const uint32_t gid = point_list[base + lane];
            m_xy = xy[gid];
            m_co = conic_opacity[gid];
            m_cd = rgbd[gid];
        }
        for (uint32_t j = 0; j < n; j++) {
            const float sx = readlane_f(m_xy.x, j), sy = readlane_f(m_xy.y, j);
            const float ca = readlane_f(m_co.x, j), cb = readlane_f(m_co.y, j), cc = readlane_f(m_co.z, j);
            const float op = readlane_f(m_co.w, j);
            const float cr = readlane_f(m_cd.x, j), cg = readlane_f(m_cd.y, j), cbl = readlane_f(m_cd.z, j);
            const float dep = readlane_f(m_cd.w, j);
            const uint32_t contributor = base - range.x + j + 1;
            const float dx = sx - pfx;
#pragma unroll
            for (int k = 0; k < kPix; k++) {
                if (done[k]) continue;
                const float dy = sy - (float)(py0 + 4 * k);
                const float power = -0.5f * (ca * dx * dx + cc * dy * dy) - cb * dx * dy;
                if (power > 0.0f) continue;
                const float alpha = fminf(0.99f, op * __expf(power));
                if (alpha < 1.0f / 255.0f) continue;
                const float test_T = T[k] * (1 - alpha);
                if (test_T < 0.0001f) {
                    done[k] = true;
                    continue;
                }
                C[k][0] += cr * alpha * T[k];
                C[k][1] += cg * alpha * T[k];
                C[k][2] += cbl * alpha * T[k];
                Dp[k] += dep * alpha * T[k];
                T[k] = test_T;
                last[k] = contributor;
            }
        }
    }
    const size_t HW = (size_t)a.W * a.H;
#pragma unroll
    for (int k = 0; k < kPix; k++) {
        const int py = py0 + 4 * k;
        if (px < a.W && py < a.H) {
            const size_t pix = (size_t)py * a.W + px;
            final_T[pix] = T[k];
            n_contrib[pix] = last[k];
            out_color[pix] = C[k][0] + T[k] * bg.x;
            out_color[HW + pix] = C[k][1] + T[k] * bg.y;
            out_color[2 * HW + pix] = C[k][2] + T[k] * bg.z;
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
// Wave64 sum into lane 63 with DPP row operations (quad_perm, row_half_mirror, row_mirror,
// row_bcast15/31): six v_add_f32 with DPP source modifiers, no LDS.
template <int CTRL, int ROW_MASK>
__device__ __forceinline__ float dpp_add(float v) {
    const int moved = __builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, ROW_MASK, 0xF, false);
    return v + __int_as_float(moved);
}
__device__ __forceinline__ float wave_sum_lane63(float v) {
    v = dpp_add<0xB1, 0xF>(v);   // quad_perm [1,0,3,2]
    v = dpp_add<0x4E, 0xF>(v);   // quad_perm [2,3,0,1]
    v = dpp_add<0x141, 0xF>(v);  // row_half_mirror
    v = dpp_add<0x140, 0xF>(v);  // row_mirror
    v = dpp_add<0x142, 0xA>(v);  // row_bcast15 into rows 1,3
    v = dpp_add<0x143, 0xC>(v);  // row_bcast31 into rows 2,3
    return v;
}

__global__ __launch_bounds__(64) void render_backward_kernel(Args a, const uint2 *__restrict__ ranges,
                                                             const uint32_t *__restrict__ point_list,
                                                             const uint32_t *__restrict__ sorted_upos,
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
    const uint2 range = ranges[tile];
    if (range.y <= range.x) return;
    const float bgc[3] = {a.bg[0], a.bg[1], a.bg[2]};

    float T[kPix], T_final[kPix], dpix[kPix][3], accum[kPix][3], last_color[kPix][3], last_alpha[kPix], bgdot[kPix];
    uint32_t last_contrib[kPix];
#pragma unroll
    for (int k = 0; k < kPix; k++) {
        const int py = py0 + 4 * k;
        const bool inside = px < a.W && py < a.H;
        const size_t pix = (size_t)py * a.W + px;
        T_final[k] = inside ? final_Ts[pix] : 0.f;
        T[k] = T_final[k];
        last_contrib[k] = inside ? n_contrib[pix] : 0;
#pragma unroll
        for (int c = 0; c < 3; c++) {
            dpix[k][c] = inside ? dL_dpixels[c * HW + pix] : 0.f;
            accum[k][c] = 0.f;
            last_color[k][c] = 0.f;
        }
        last_alpha[k] = 0.f;
        bgdot[k] = 0.f;
#pragma unroll
        for (int c = 0; c < 3; c++) bgdot[k] += bgc[c] * dpix[k][c];
    }
    uint32_t max_last = 0;
#pragma unroll
    for (int k = 0; k < kPix; k++) max_last = max(max_last, last_contrib[k]);
    // splats at list position >= every pixel's n_contrib never contribute: start the walk there
    for (int off = 32; off > 0; off >>= 1) max_last = max(max_last, (uint32_t)__shfl_xor((int)max_last, off));
    const float ddelx_dx = 0.5f * a.W, ddely_dy = 0.5f * a.H;

    const uint32_t len = range.y - range.x;
    // instances past max_last get zero gradient terms
    for (uint32_t p = max_last + lane; p < len; p += 64) {
        const uint32_t u = sorted_upos[range.x + p];
#pragma unroll
        for (int q = 0; q < kContribStride; q++) contrib[(size_t)u * kContribStride + q] = 0.f;
    }
    // walk positions max_last-1 ... 0 in batches of 64 (back to front)
    for (int end = (int)max_last; end > 0; end -= 64) {
        const int n = min(64, end);
        // lane l holds the splat at position end-1-l
        float2 m_xy = make_float2(0.f, 0.f);
        float4 m_co = make_float4(0.f, 0.f, 0.f, 0.f);
        float3 m_c = make_float3(0.f, 0.f, 0.f);
        uint32_t m_upos = 0;
        if (lane < n) {
            const uint32_t si = range.x + end - 1 - lane;
            const uint32_t gid = point_list[si];
            m_upos = sorted_upos[si];
            m_xy = xy[gid];
            m_co = conic_opacity[gid];
            if (colors) {
                m_c = make_float3(colors[3 * gid], colors[3 * gid + 1], colors[3 * gid + 2]);
            } else {
                float4 t4 = rgbd[gid];
                m_c = make_float3(t4.x, t4.y, t4.z);
            }
        }
        float acc[kContribStride];
#pragma unroll
        for (int q = 0; q < kContribStride; q++) acc[q] = 0.f;
        for (int j = 0; j < n; j++) {
            const uint32_t contributor = (uint32_t)(end - 1 - j);
            const float sx = readlane_f(m_xy.x, j), sy = readlane_f(m_xy.y, j);
            const float ca = readlane_f(m_co.x, j), cb = readlane_f(m_co.y, j), cc = readlane_f(m_co.z, j);
            const float op = readlane_f(m_co.w, j);
            const float col[3] = {readlane_f(m_c.x, j), readlane_f(m_c.y, j), readlane_f(m_c.z, j)};
            const float dx = sx - pfx;
            float g[kContribStride];
#pragma unroll
            for (int q = 0; q < kContribStride; q++) g[q] = 0.f;
            bool any = false;
#pragma unroll
            for (int k = 0; k < kPix; k++) {
                if (contributor >= last_contrib[k]) continue;
                const float dy = sy - (float)(py0 + 4 * k);
                const float power = -0.5f * (ca * dx * dx + cc * dy * dy) - cb * dx * dy;
                if (power > 0.0f) continue;
                const float G = __expf(power);
                const float alpha = fminf(0.99f, op * G);
                if (alpha < 1.0f / 255.0f) continue;
                any = true;
                T[k] = T[k] / (1.f - alpha);
                const float dchannel_dcolor = alpha * T[k];
                float dL_dalpha = 0.0f;
#pragma unroll
                for (int c = 0; c < 3; c++) {
                    accum[k][c] = last_alpha[k] * last_color[k][c] + (1.f - last_alpha[k]) * accum[k][c];
                    last_color[k][c] = col[c];
                    dL_dalpha += (col[c] - accum[k][c]) * dpix[k][c];
                    g[6 + c] += dchannel_dcolor * dpix[k][c];
                }
                dL_dalpha *= T[k];
                last_alpha[k] = alpha;
                dL_dalpha += (-T_final[k] / (1.f - alpha)) * bgdot[k];
                const float dL_dG = op * dL_dalpha;
                const float gdx = G * dx, gdy = G * dy;
                const float dG_ddelx = -gdx * ca - gdy * cb;
                const float dG_ddely = -gdy * cc - gdx * cb;
                g[0] += dL_dG * dG_ddelx * ddelx_dx;
                g[1] += dL_dG * dG_ddely * ddely_dy;
                g[2] += -0.5f * gdx * dx * dL_dG;
                g[3] += -0.5f * gdx * dy * dL_dG;
                g[4] += -0.5f * gdy * dy * dL_dG;
                g[5] += G * dL_dalpha;
            }
            if (__any(any)) {
#pragma unroll
                for (int q = 0; q < kContribStride; q++) {
                    const float s = readlane_f(wave_sum_lane63(g[q]), 63);
                    acc[q] = (lane == j) ? s : acc[q];
                }
            }
        }
        if (lane < n) {
#pragma unroll
            for (int q = 0; q < kContribStride; q++) contrib[(size_t)m_upos * kContribStride + q] = acc[q];
        }
    }
}

hipError_t launch_render_backward(const Args &a, GeomState g, const uint32_t *point_list, const uint32_t *sorted_upos,
                                  ImageState img, const float *colors, const float *dL_dpix, float *contrib,
                                  hipStream_t s) {
    const int T = a.gx * a.gy;
    hipLaunchKernelGGL(render_backward_kernel, dim3(T), dim3(64), 0, s, a, img.ranges, point_list, sorted_upos, g.xy,
                       g.conic_opacity, g.rgbd, colors, img.final_T, img.n_contrib, dL_dpix, contrib);
    return hipGetLastError();
}

}  // namespace gs4d
