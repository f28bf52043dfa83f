// preprocess_backward.hip -- per-Gaussian backward: instance-gradient reduction, then
// computeCov2DCUDA (K8) + preprocessCUDA backward (K9) fused into one pass.
//
// Reference: cuda_rasterizer/backward.cu:144-274 (computeCov2DCUDA), :346-396 (preprocessCUDA),
// :20-139 (SH backward), :278-341 (cov3D backward); rasterize_points.cu:153-161 (zeroed outputs).
//
// 1. contrib_reduce: each Gaussian sums the per-(tile, Gaussian) records the render backward stored
//    at its emission slots -- consecutive, in tile-rect order -- with a fixed-order segmented
//    reduction, which replaces the reference's float atomics (backward.cu:523,545-554): bitwise
//    deterministic, and balanced (one lane per record, whatever the splat sizes).
// 2. gaussian_backward: the sums of the Gaussians whose records span waves, then K8 + K9 per
//    Gaussian except K9's SH part, which sh_backward runs after it with the block's coefficient
//    rows staged through LDS (coalesced loads and stores).  Every output element is written (zeros for culled Gaussians and for
//    SH coefficients >= (D+1)^2), so no zero-fill pass is needed.
#include <algorithm>

#include "gs4d_internal.h"

namespace gs4d {

// Render-level gradients of Gaussian g from its summed moments R (render.hip): backward.cu:545-554
// with dL/dG = opacity dL/dalpha, ddelx_dx = W/2, ddely_dy = H/2.  Returned as dL_dmeans2D (.z stays
// 0), dL_dcolors, dL_dopacity; the conic gradient uses the reference's float4 slots .x .y .w
// (backward.cu:549-551, read at :165).
struct GradOut {
    float *mean2D;
    float4 *conic;
    float *opacity;
    float *color;
    const float4 *conic_opacity;
    float hw, hh;
};
__device__ __forceinline__ void write_grads(const GradOut &o, uint32_t g, const float *R) {
    const float4 co = o.conic_opacity[g];
    const float op = co.w;
    o.mean2D[3 * g + 0] = o.hw * op * (-co.x * R[1] - co.y * R[2]);
    o.mean2D[3 * g + 1] = o.hh * op * (-co.z * R[2] - co.y * R[1]);
    o.mean2D[3 * g + 2] = 0.f;
    o.conic[g] = make_float4(-0.5f * op * R[3], -0.5f * op * R[4], 0.f, -0.5f * op * R[5]);
    o.opacity[g] = R[0];
    o.color[3 * g + 0] = R[6];
    o.color[3 * g + 1] = R[7];
    o.color[3 * g + 2] = R[8];
}
__device__ __forceinline__ void write_zero_grads(const GradOut &o, uint32_t g) {
    o.mean2D[3 * g + 0] = 0.f;
    o.mean2D[3 * g + 1] = 0.f;
    o.mean2D[3 * g + 2] = 0.f;
    o.conic[g] = make_float4(0.f, 0.f, 0.f, 0.f);
    o.opacity[g] = 0.f;
    o.color[3 * g + 0] = 0.f;
    o.color[3 * g + 1] = 0.f;
    o.color[3 * g + 2] = 0.f;
}
__device__ __forceinline__ void store9(float4 *p, const float *acc) {
    p[0] = make_float4(acc[0], acc[1], acc[2], acc[3]);
    p[1] = make_float4(acc[4], acc[5], acc[6], acc[7]);
    p[2] = make_float4(acc[8], 0.f, 0.f, 0.f);
}
__device__ __forceinline__ void add9(float *acc, const float4 *p) {
    const float4 a = p[0], b = p[1], c = p[2];
    acc[0] += a.x; acc[1] += a.y; acc[2] += a.z; acc[3] += a.w;
    acc[4] += b.x; acc[5] += b.y; acc[6] += b.z; acc[7] += b.w;
    acc[8] += c.x;
}

// One step of the wave's segmented inclusive scan by DPP moves (no LDS): lane l takes the (sums, flag) of
// the lane CTRL names (row_shr:n inside rows of 16, row_bcast:15 / :31 across rows, only the rows RM
// enables; lanes without a source read zeros, the identity) and adds its sums unless a segment head
// lies between them.
template <int CTRL, int RM>
__device__ __forceinline__ void seg_scan_step(float acc[9], bool &f) {
    const bool fu = __builtin_amdgcn_update_dpp(0, (int)f, CTRL, RM, 0xF, false) != 0;
    float up[9];
#pragma unroll
    for (int q = 0; q < 9; q++)
        up[q] = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(acc[q]), CTRL, RM, 0xF, false));
    if (!f) {
#pragma unroll
        for (int q = 0; q < 9; q++) acc[q] += up[q];
    }
    f = f || fu;
}

// Pass 1: one lane per emission slot, one wave per 64 slots.  A Gaussian's records occupy consecutive
// slots, so a segmented inclusive scan (fixed shuffle tree) sums each Gaussian's piece of the wave.
// Pieces that are a whole Gaussian are written out; a piece continuing from the previous wave goes
// to part[w][0], a piece that starts a Gaussian and continues into the next wave to part[w][1];
// e_first[g] = the Gaussian's first slot.
__global__ __launch_bounds__(256) void contrib_segments_kernel(const uint32_t *__restrict__ n_dev,
                                                               const uint32_t *__restrict__ gid_by_e,
                                                               const float4 *__restrict__ rec, GradOut o,
                                                               float4 *__restrict__ part,
                                                               uint32_t *__restrict__ e_first) {
    const int n = (int)__builtin_amdgcn_readfirstlane(*n_dev);
    const int lane = threadIdx.x & 63;
    const int w = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (w * 64 >= n) return;
    const int e = w * 64 + lane;
    const bool valid = e < n;
    const uint32_t key = valid ? gid_by_e[e] & kGidMask : 0xFFFFFFFFu;
    float acc[9];
    {
        float4 a = make_float4(0.f, 0.f, 0.f, 0.f), b = a, c = a;
        if (valid) {
            a = rec[3 * (size_t)e];
            b = rec[3 * (size_t)e + 1];
            c = rec[3 * (size_t)e + 2];
        }
        acc[0] = a.x; acc[1] = a.y; acc[2] = a.z; acc[3] = a.w;
        acc[4] = b.x; acc[5] = b.y; acc[6] = b.z; acc[7] = b.w;
        acc[8] = c.x;
    }
    uint32_t kp = __shfl_up(key, 1), kn = __shfl_down(key, 1);
    if (lane == 0) kp = e > 0 ? gid_by_e[e - 1] & kGidMask : 0xFFFFFFFFu;
    if (lane == 63) kn = e + 1 < n ? gid_by_e[e + 1] & kGidMask : 0xFFFFFFFFu;
    const bool head = valid && key != kp;  // first slot of its Gaussian
    const bool tail = valid && key != kn;  // last slot of its Gaussian
    if (head) e_first[key] = (uint32_t)e;  // locates the pieces of a Gaussian spanning waves
    bool f = head || lane == 0;
    seg_scan_step<0x111, 0xF>(acc, f);  // row_shr:1
    seg_scan_step<0x112, 0xF>(acc, f);  // row_shr:2
    seg_scan_step<0x114, 0xF>(acc, f);  // row_shr:4
    seg_scan_step<0x118, 0xF>(acc, f);  // row_shr:8
    seg_scan_step<0x142, 0xA>(acc, f);  // row_bcast:15 -> rows 1, 3
    seg_scan_step<0x143, 0xC>(acc, f);  // row_bcast:31 -> rows 2, 3
    const uint64_t endm = __ballot(valid && (tail || lane == 63));
    const int fe = __ffsll((unsigned long long)endm) - 1;  // end lane of the first piece
    const bool head0 = __ballot(head) & 1ull;
    if (valid && (tail || lane == 63)) {
        const bool starts = lane != fe || head0;  // the piece starts at its Gaussian's first slot
        if (starts && tail) write_grads(o, key, acc);
        else if (!starts) store9(part + ((size_t)w * 2) * 3, acc);
        else store9(part + ((size_t)w * 2 + 1) * 3, acc);
    }
}

// Pass 2 (at the start of gaussian_backward, one thread per Gaussian): a Gaussian whose slots span
// several waves sums its pieces in wave order -- part[w0][1] (its head piece) then part[w][0] of each
// following wave up to the one holding its last slot -- and a Gaussian without instances gets zeros.
// Then K8 + K9 without the SH part: dL/dcov3D, dL/dscale, dL/drot stored; dL/dmean3D's covariance +
// projection terms returned (the caller adds the SH term, backward.cu:390, and stores it).
__device__ __forceinline__ V3 gaussian_grads(
    int idx, const Args &a, const GeomState &g, const int *__restrict__ radii, const float *__restrict__ means3D,
    const float *__restrict__ scales, const float *__restrict__ rotations, const float *__restrict__ cov3Ds,
    const float *dL_dmean2D, const float4 *dL_dconic, float *__restrict__ dL_dcov3D, float *__restrict__ dL_dscale,
    float *__restrict__ dL_drot, const uint32_t *__restrict__ e_first, const float4 *__restrict__ part,
    const GradOut &o) {
    {
        const uint32_t ni = g.n_inst[idx];
        if (ni == 0) {
            write_zero_grads(o, (uint32_t)idx);
        } else {
            const uint32_t e0 = e_first[idx], w0 = e0 >> 6, w1 = (e0 + ni - 1) >> 6;
            if (w0 != w1) {
                float acc[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
                add9(acc, part + ((size_t)w0 * 2 + 1) * 3);
                for (uint32_t w = w0 + 1; w <= w1; w++) add9(acc, part + ((size_t)w * 2) * 3);
                write_grads(o, (uint32_t)idx, acc);
            }
        }
    }
    float dcov[6] = {0, 0, 0, 0, 0, 0};
    V3 dmean = v3(0, 0, 0);
    V3 dscale = v3(0, 0, 0);
    float4 drot = make_float4(0, 0, 0, 0);
    if (radii[idx] > 0) {
        const Mat4 view = load_mat4(a.viewmatrix, a.view_transposed), projm = load_mat4(a.projmatrix);
        const V3 m = v3(means3D[3 * idx], means3D[3 * idx + 1], means3D[3 * idx + 2]);
        float cov3D[6];
#pragma unroll
        for (int i = 0; i < 6; i++) cov3D[i] = cov3Ds[6 * (size_t)idx + i];
        const float4 dc = dL_dconic[idx];
        // K8 (backward.cu:144-274): the covariance part of dL/dmean (assigned, :273)
        dmean = cov2D_backward(m, a.focal_x, a.focal_y, a.tan_fovx, a.tan_fovy, cov3D, view,
                               make_float3(dc.x, dc.y, dc.w), dcov);
        // K9 (backward.cu:370-387): projection part
        const float *proj = projm.m;
        const float g2x = dL_dmean2D[3 * idx], g2y = dL_dmean2D[3 * idx + 1];
        float4 m_hom = transformPoint4x4(m, projm);
        float m_w = 1.0f / (m_hom.w + 0.0000001f);
        float mul1 = (proj[0] * m.x + proj[4] * m.y + proj[8] * m.z + proj[12]) * m_w * m_w;
        float mul2 = (proj[1] * m.x + proj[5] * m.y + proj[9] * m.z + proj[13]) * m_w * m_w;
        V3 dm2;
        dm2.x = (proj[0] * m_w - proj[3] * mul1) * g2x + (proj[1] * m_w - proj[3] * mul2) * g2y;
        dm2.y = (proj[4] * m_w - proj[7] * mul1) * g2x + (proj[5] * m_w - proj[7] * mul2) * g2y;
        dm2.z = (proj[8] * m_w - proj[11] * mul1) * g2x + (proj[9] * m_w - proj[11] * mul2) * g2y;
        dmean = dmean + dm2;
        // SH part (backward.cu:390-391): added by the caller
        // cov3D part (backward.cu:394-395)
        if (scales) {
            V3 sc = v3(scales[3 * idx], scales[3 * idx + 1], scales[3 * idx + 2]);
            float4 rot = reinterpret_cast<const float4 *>(rotations)[idx];
            cov3D_backward(sc, a.scale_modifier, rot, dcov, dscale, drot);
        }
    }
#pragma unroll
    for (int i = 0; i < 6; i++) dL_dcov3D[6 * (size_t)idx + i] = dcov[i];
    dL_dscale[3 * idx + 0] = dscale.x;
    dL_dscale[3 * idx + 1] = dscale.y;
    dL_dscale[3 * idx + 2] = dscale.z;
    reinterpret_cast<float4 *>(dL_drot)[idx] = drot;
    return dmean;
}

// Without SH coefficients (colours precomputed): one thread per Gaussian, dL/dmean3D = the two terms.
__global__ __launch_bounds__(256) void gaussian_backward_kernel(
    Args a, GeomState g, const int *__restrict__ radii, const float *__restrict__ means3D,
    const float *__restrict__ scales, const float *__restrict__ rotations, const float *__restrict__ cov3Ds,
    const float *dL_dmean2D, const float4 *dL_dconic, float *__restrict__ dL_dmean3D,
    float *__restrict__ dL_dcov3D, float *__restrict__ dL_dscale, float *__restrict__ dL_drot,
    const uint32_t *__restrict__ e_first, const float4 *__restrict__ part, GradOut o) {
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= a.P) return;
    const V3 dmean = gaussian_grads(idx, a, g, radii, means3D, scales, rotations, cov3Ds, dL_dmean2D, dL_dconic,
                                    dL_dcov3D, dL_dscale, dL_drot, e_first, part, o);
    dL_dmean3D[3 * idx + 0] = dmean.x;
    dL_dmean3D[3 * idx + 1] = dmean.y;
    dL_dmean3D[3 * idx + 2] = dmean.z;
}

// With SH coefficients: the same per-Gaussian work and K9's SH part (backward.cu:390-391 -> computeColorFromSH
// backward, :20-139) in one launch, one thread per Gaussian.  The block's coefficient rows are staged through
// LDS: the block reads its 128 rows of 3M floats (one contiguous span, float4 when M = 16 and aligned) into a
// 49-float-stride tile (odd stride: a wave's rows hit distinct banks), each thread takes its row into
// registers, writes its gradients back into the same row (zeros past (D + 1)^2 and for culled Gaussians), and
// the block stores the tile as one contiguous span.  dL/dmean3D = (covariance + projection terms) + the
// view-direction term, the reference's order (:390).  A thread per Gaussian straight from global memory
// (192-byte strided rows) took 12.6 us of the old gaussian_backward's 26 at P = 100k; two launches (this
// work split at the SH part) cost one launch more.
constexpr int kShThreads = 128, kShRow = 49;

template <bool kVec4>
__global__ __launch_bounds__(kShThreads) void gaussian_sh_backward_kernel(
    Args a, GeomState g, const int *__restrict__ radii, const float *__restrict__ means3D,
    const float *__restrict__ scales, const float *__restrict__ rotations, const float *__restrict__ cov3Ds,
    const float *dL_dmean2D, const float4 *dL_dconic, float *__restrict__ dL_dmean3D,
    float *__restrict__ dL_dcov3D, float *__restrict__ dL_dscale, float *__restrict__ dL_drot,
    const uint32_t *__restrict__ e_first, const float4 *__restrict__ part, GradOut o, const float *__restrict__ shs,
    const uint8_t *__restrict__ clamped, const float *dL_dcolor, float *__restrict__ dL_dsh) {
    __shared__ float tile[kShThreads * kShRow];
    const int g0 = blockIdx.x * kShThreads;
    // rows of M > 16 coefficients: only the first 16 can be used (D <= 3); the rest get zeros
    const int n = min(kShThreads, a.P - g0), row = 3 * a.M, rowl = min(row, 48);
    const size_t base = (size_t)g0 * row;
    const int total = n * row;
    if (kVec4) {  // row = 48 = 12 float4
        const float4 *s4 = reinterpret_cast<const float4 *>(shs + base);
        for (int i = threadIdx.x; i < total / 4; i += kShThreads) {
            const int r = i / 12, c = (i - r * 12) * 4;
            const float4 v = s4[i];
            float *t = tile + r * kShRow + c;
            t[0] = v.x, t[1] = v.y, t[2] = v.z, t[3] = v.w;
        }
    } else {
        for (int i = threadIdx.x; i < total; i += kShThreads) {
            const int r = i / row, c = i - r * row;
            if (c < 48) tile[r * kShRow + c] = shs[base + i];
        }
    }
    V3 dmean = v3(0, 0, 0);
    const int idx = g0 + threadIdx.x;
    if ((int)threadIdx.x < n)  // pass 2 writes this Gaussian's dL/dcolor (when it spans waves) before it is read
        dmean = gaussian_grads(idx, a, g, radii, means3D, scales, rotations, cov3Ds, dL_dmean2D, dL_dconic, dL_dcov3D,
                               dL_dscale, dL_drot, e_first, part, o);
    __syncthreads();
    if ((int)threadIdx.x < n) {
        float *trow = tile + threadIdx.x * kShRow;
        float shl[48];
#pragma unroll
        for (int k = 0; k < 48; k++) {
            shl[k] = k < rowl ? trow[k] : 0.f;
            if (k < rowl) trow[k] = 0.f;
        }
        if (radii[idx] > 0) {
            const uint8_t cl = clamped[idx];
            const V3 dRGB = v3(dL_dcolor[3 * idx] * ((cl & 1) ? 0.f : 1.f),
                               dL_dcolor[3 * idx + 1] * ((cl & 2) ? 0.f : 1.f),
                               dL_dcolor[3 * idx + 2] * ((cl & 4) ? 0.f : 1.f));
            const V3 m = v3(means3D[3 * idx], means3D[3 * idx + 1], means3D[3 * idx + 2]);
            const V3 dm = sh_backward(a.D, shl, m - load_v3(a.campos), dRGB, trow);
            dmean = dmean + dm;
        }
        dL_dmean3D[3 * idx + 0] = dmean.x;
        dL_dmean3D[3 * idx + 1] = dmean.y;
        dL_dmean3D[3 * idx + 2] = dmean.z;
    }
    __syncthreads();
    if (kVec4) {
        float4 *d4 = reinterpret_cast<float4 *>(dL_dsh + base);
        for (int i = threadIdx.x; i < total / 4; i += kShThreads) {
            const int r = i / 12, c = (i - r * 12) * 4;
            const float *t = tile + r * kShRow + c;
            d4[i] = make_float4(t[0], t[1], t[2], t[3]);
        }
    } else {
        for (int i = threadIdx.x; i < total; i += kShThreads) {
            const int r = i / row, c = i - r * row;
            dL_dsh[base + i] = c < 48 ? tile[r * kShRow + c] : 0.f;
        }
    }
}

size_t contrib_scratch_bytes(int R, int P) {
    const size_t nw = ((size_t)R + 63) / 64;
    return align_up(nw * 2 * 3 * sizeof(float4), 256) + align_up(4 * (size_t)P, 256) + 256;
}

static GradOut grad_out(const Args &a, GeomState g, float *dL_dmean2D, float4 *dL_dconic, float *dL_dopacity,
                        float *dL_dcolor) {
    return GradOut{dL_dmean2D, dL_dconic, dL_dopacity, dL_dcolor, g.conic_opacity, 0.5f * a.W, 0.5f * a.H};
}
static float4 *scratch_part(char *scratch) { return (float4 *)scratch; }
static uint32_t *scratch_e_first(char *scratch, int R) {
    const size_t nw = ((size_t)R + 63) / 64;
    return (uint32_t *)(scratch + align_up(nw * 2 * 3 * sizeof(float4), 256));
}

hipError_t launch_contrib_reduce(const Args &a, GeomState g, BinningState b, int R, const float *contrib,
                                 char *scratch, float *dL_dmean2D, float4 *dL_dconic, float *dL_dopacity,
                                 float *dL_dcolor, hipStream_t s) {
    if (R == 0) return hipSuccess;  // every Gaussian has n_inst = 0: gaussian_backward writes the zeros
    const size_t nw = ((size_t)R + 63) / 64;
    const uint32_t *n_dev = b.scratch;  // L' (binning.hip)
    hipLaunchKernelGGL(contrib_segments_kernel, dim3((unsigned)((nw + 3) / 4)), dim3(256), 0, s, n_dev, b.gid_by_e,
                       reinterpret_cast<const float4 *>(contrib), grad_out(a, g, dL_dmean2D, dL_dconic, dL_dopacity,
                                                                          dL_dcolor),
                       scratch_part(scratch), scratch_e_first(scratch, R));
    return hipGetLastError();
}

hipError_t launch_gaussian_backward(const Args &a, GeomState g, int R, char *scratch, const int *radii,
                                    const float *means3D, const float *shs, const float *scales, const float *rotations,
                                    const float *cov3D, float *dL_dmean2D, float4 *dL_dconic, float *dL_dopacity,
                                    float *dL_dcolor, float *dL_dmean3D, float *dL_dcov3D, float *dL_dsh,
                                    float *dL_dscale, float *dL_drot, hipStream_t s) {
    const GradOut o = grad_out(a, g, dL_dmean2D, dL_dconic, dL_dopacity, dL_dcolor);
    if (shs) {
        const bool vec4 = a.M == 16 && (((size_t)shs | (size_t)dL_dsh) & 15) == 0;
        hipLaunchKernelGGL(vec4 ? gaussian_sh_backward_kernel<true> : gaussian_sh_backward_kernel<false>,
                           dim3((a.P + kShThreads - 1) / kShThreads), dim3(kShThreads), 0, s, a, g, radii, means3D,
                           scales, rotations, cov3D, dL_dmean2D, dL_dconic, dL_dmean3D, dL_dcov3D, dL_dscale, dL_drot,
                           scratch_e_first(scratch, R), scratch_part(scratch), o, shs, g.clamped, dL_dcolor, dL_dsh);
    } else {
        hipLaunchKernelGGL(gaussian_backward_kernel, dim3((a.P + 255) / 256), dim3(256), 0, s, a, g, radii, means3D,
                           scales, rotations, cov3D, dL_dmean2D, dL_dconic, dL_dmean3D, dL_dcov3D,
                           dL_dscale, dL_drot, scratch_e_first(scratch, R), scratch_part(scratch), o);
    }
    return hipGetLastError();
}

}  // namespace gs4d
