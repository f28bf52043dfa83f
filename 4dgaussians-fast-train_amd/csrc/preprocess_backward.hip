// preprocess_backward.hip -- per-Gaussian backward: instance-gradient reduction, then
// computeCov2DCUDA (K8) + preprocessCUDA backward (K9) fused into one pass.
//
// Reference: cuda_rasterizer/backward.cu:144-274 (computeCov2DCUDA), :346-396 (preprocessCUDA),
// :20-139 (SH backward), :278-341 (cov3D backward); rasterize_points.cu:153-161 (zeroed outputs).
//
// 1. contrib_reduce: each Gaussian sums the per-(tile, Gaussian) records the render backward stored
//    at its unsorted instance positions [point_offsets[g], +n_inst[g]) -- in tile-rect order,
//    which replaces the reference's float atomics (backward.cu:523,545-554) by a fixed-order sum.
//    A workgroup's 256 Gaussians own one contiguous record range, streamed through LDS in chunks
//    with coalesced 16-byte loads.
// 2. gaussian_backward: K8 + K9 per Gaussian.  Every output element is written (zeros for culled
//    Gaussians and for SH coefficients >= (D+1)^2), so no zero-fill pass is needed.
#include "gs4d_internal.h"

namespace gs4d {

constexpr int kReduceChunk = 1024;  // records per LDS chunk (48 KB)

__global__ __launch_bounds__(256) void contrib_reduce_kernel(int P, GeomState g, const float *__restrict__ contrib,
                                                             float *__restrict__ dL_dmean2D,
                                                             float4 *__restrict__ dL_dconic,
                                                             float *__restrict__ dL_dopacity,
                                                             float *__restrict__ dL_dcolor) {
    __shared__ float4 s_rec[kReduceChunk * 3];
    const int tid = threadIdx.x;
    const int idx = blockIdx.x * 256 + tid;
    // the workgroup's record range (block_sums holds exclusive per-workgroup offsets, [nblk] = L)
    const uint32_t R0 = g.block_sums[blockIdx.x], R1 = g.block_sums[blockIdx.x + 1];
    uint32_t lo = 0, hi = 0;
    if (idx < P) {
        lo = g.point_offsets[idx];
        hi = lo + g.n_inst[idx];
    }
    float acc[9];
#pragma unroll
    for (int q = 0; q < 9; q++) acc[q] = 0.f;
    const float4 *src = reinterpret_cast<const float4 *>(contrib);
    for (uint32_t cs = R0; cs < R1; cs += kReduceChunk) {
        const uint32_t ce = min(R1, cs + kReduceChunk);
        const uint32_t nq = (ce - cs) * 3;
        __syncthreads();
        for (uint32_t q = tid; q < nq; q += 256) s_rec[q] = src[(size_t)cs * 3 + q];
        __syncthreads();
        const uint32_t a = max(lo, cs), b = min(hi, ce);
        for (uint32_t r = a; r < b; r++) {
            const float4 r0 = s_rec[(r - cs) * 3], r1 = s_rec[(r - cs) * 3 + 1], r2 = s_rec[(r - cs) * 3 + 2];
            acc[0] += r0.x; acc[1] += r0.y; acc[2] += r0.z; acc[3] += r0.w;
            acc[4] += r1.x; acc[5] += r1.y; acc[6] += r1.z; acc[7] += r1.w;
            acc[8] += r2.x;
        }
    }
    if (idx >= P) return;
    // render-level gradients, returned as dL_dmeans2D (.z stays 0), dL_dcolors, dL_dopacity; the conic
    // gradient uses the reference's float4 slots .x .y .w (backward.cu:549-551, read at :165)
    dL_dmean2D[3 * idx + 0] = acc[0];
    dL_dmean2D[3 * idx + 1] = acc[1];
    dL_dmean2D[3 * idx + 2] = 0.f;
    dL_dconic[idx] = make_float4(acc[2], acc[3], 0.f, acc[4]);
    dL_dopacity[idx] = acc[5];
    dL_dcolor[3 * idx + 0] = acc[6];
    dL_dcolor[3 * idx + 1] = acc[7];
    dL_dcolor[3 * idx + 2] = acc[8];
}

__global__ __launch_bounds__(256) void gaussian_backward_kernel(
    Args a, GeomState g, const int *__restrict__ radii, const float *__restrict__ means3D,
    const float *__restrict__ shs, const float *__restrict__ scales, const float *__restrict__ rotations,
    const float *__restrict__ cov3Ds, const float *__restrict__ dL_dmean2D, const float4 *__restrict__ dL_dconic,
    const float *__restrict__ dL_dcolor, float *__restrict__ dL_dmean3D, float *__restrict__ dL_dcov3D,
    float *__restrict__ dL_dsh, float *__restrict__ dL_dscale, float *__restrict__ dL_drot) {
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= a.P) return;
    float dcov[6] = {0, 0, 0, 0, 0, 0};
    V3 dmean = v3(0, 0, 0);
    V3 dscale = v3(0, 0, 0);
    float4 drot = make_float4(0, 0, 0, 0);
    float *dsh = shs ? dL_dsh + (size_t)idx * a.M * 3 : nullptr;
    int nsh_written = 0;
    if (radii[idx] > 0) {
        const Mat4 view = load_mat4(a.viewmatrix), projm = load_mat4(a.projmatrix);
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
        // SH part (backward.cu:390-391)
        if (shs) {
            const float *sh = shs + (size_t)idx * a.M * 3;
            const uint8_t cl = g.clamped[idx];
            V3 dRGB = v3(dL_dcolor[3 * idx] * ((cl & 1) ? 0.f : 1.f), dL_dcolor[3 * idx + 1] * ((cl & 2) ? 0.f : 1.f),
                         dL_dcolor[3 * idx + 2] * ((cl & 4) ? 0.f : 1.f));
            V3 dir_orig = m - load_v3(a.campos);
            dmean = dmean + sh_backward(a.D, sh, dir_orig, dRGB, dsh);
            nsh_written = (a.D + 1) * (a.D + 1);
        }
        // cov3D part (backward.cu:394-395)
        if (scales) {
            V3 sc = v3(scales[3 * idx], scales[3 * idx + 1], scales[3 * idx + 2]);
            float4 rot = reinterpret_cast<const float4 *>(rotations)[idx];
            cov3D_backward(sc, a.scale_modifier, rot, dcov, dscale, drot);
        }
    }
    if (dsh) {
        for (int k = nsh_written; k < a.M; k++) {
            dsh[3 * k + 0] = 0.f;
            dsh[3 * k + 1] = 0.f;
            dsh[3 * k + 2] = 0.f;
        }
    }
    dL_dmean3D[3 * idx + 0] = dmean.x;
    dL_dmean3D[3 * idx + 1] = dmean.y;
    dL_dmean3D[3 * idx + 2] = dmean.z;
#pragma unroll
    for (int i = 0; i < 6; i++) dL_dcov3D[6 * (size_t)idx + i] = dcov[i];
    dL_dscale[3 * idx + 0] = dscale.x;
    dL_dscale[3 * idx + 1] = dscale.y;
    dL_dscale[3 * idx + 2] = dscale.z;
    reinterpret_cast<float4 *>(dL_drot)[idx] = drot;
}

hipError_t launch_contrib_reduce(const Args &a, GeomState g, const float *contrib, float *dL_dmean2D,
                                 float4 *dL_dconic, float *dL_dopacity, float *dL_dcolor, hipStream_t s) {
    hipLaunchKernelGGL(contrib_reduce_kernel, dim3((a.P + 255) / 256), dim3(256), 0, s, a.P, g, contrib, dL_dmean2D,
                       dL_dconic, dL_dopacity, dL_dcolor);
    return hipGetLastError();
}

hipError_t launch_gaussian_backward(const Args &a, GeomState g, const int *radii, const float *means3D,
                                    const float *shs, const float *scales, const float *rotations, const float *cov3D,
                                    const float *dL_dmean2D, const float4 *dL_dconic, const float *dL_dcolor,
                                    float *dL_dmean3D, float *dL_dcov3D, float *dL_dsh, float *dL_dscale,
                                    float *dL_drot, hipStream_t s) {
    hipLaunchKernelGGL(gaussian_backward_kernel, dim3((a.P + 255) / 256), dim3(256), 0, s, a, g, radii, means3D, shs,
                       scales, rotations, cov3D, dL_dmean2D, dL_dconic, dL_dcolor, dL_dmean3D, dL_dcov3D, dL_dsh,
                       dL_dscale, dL_drot);
    return hipGetLastError();
}

}  // namespace gs4d
