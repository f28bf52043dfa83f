// preprocess_backward.hip -- per-Gaussian backward: instance-gradient reduction + computeCov2DCUDA (K8)
// + preprocessCUDA backward (K9), fused into one pass.
//
// Reference: cuda_rasterizer/backward.cu:144-274 (computeCov2DCUDA), :346-396 (preprocessCUDA),
// :20-139 (SH backward), :278-341 (cov3D backward); rasterize_points.cu:153-161 (zeroed outputs).
//
// Each Gaussian first sums the per-(tile, Gaussian) gradient terms that the render backward stored
// for its instances (contiguous by unsorted position, summed in tile order), which replaces the
// reference's float atomics (backward.cu:523,545-554).  Every output element is written (zeros for
// culled Gaussians and for SH coefficients >= (D+1)^2), so no zero-fill pass is needed.
#include "gs4d_internal.h"

namespace gs4d {

__global__ __launch_bounds__(256) void preprocess_backward_kernel(
    Args a, GeomState g, const int *__restrict__ radii, const float *__restrict__ contrib,
    const float *__restrict__ means3D, const float *__restrict__ shs, const float *__restrict__ scales,
    const float *__restrict__ rotations, const float *__restrict__ cov3Ds, float *__restrict__ dL_dmean2D,
    float *__restrict__ dL_dconic, float *__restrict__ dL_dopacity, float *__restrict__ dL_dcolor,
    float *__restrict__ dL_dmean3D, float *__restrict__ dL_dcov3D, float *__restrict__ dL_dsh,
    float *__restrict__ dL_dscale, float *__restrict__ dL_drot) {
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= a.P) return;
    const Mat4 view = load_mat4(a.viewmatrix), projm = load_mat4(a.projmatrix);
    const bool vis = radii[idx] > 0;
    float acc[kContribStride];
#pragma unroll
    for (int q = 0; q < kContribStride; q++) acc[q] = 0.f;
    // Instances exist only where the forward's tiles_touched > 0 (which implies its internal radius > 0).
    const uint32_t n = g.tiles_touched[idx];
    if (n > 0) {
        const float *c = contrib + (size_t)g.point_offsets[idx] * kContribStride;
        for (uint32_t u = 0; u < n; u++) {
#pragma unroll
            for (int q = 0; q < kContribStride; q++) acc[q] += c[(size_t)u * kContribStride + q];
        }
    }
    // render-level gradients (returned as dL_dmeans2D, dL_dcolors, dL_dopacity)
    dL_dmean2D[3 * idx + 0] = acc[0];
    dL_dmean2D[3 * idx + 1] = acc[1];
    dL_dmean2D[3 * idx + 2] = 0.f;
    if (dL_dconic) {
        dL_dconic[4 * idx + 0] = acc[2];
        dL_dconic[4 * idx + 1] = acc[3];
        dL_dconic[4 * idx + 2] = 0.f;
        dL_dconic[4 * idx + 3] = acc[4];
    }
    dL_dopacity[idx] = acc[5];
    dL_dcolor[3 * idx + 0] = acc[6];
    dL_dcolor[3 * idx + 1] = acc[7];
    dL_dcolor[3 * idx + 2] = acc[8];

    float dcov[6] = {0, 0, 0, 0, 0, 0};
    V3 dmean = v3(0, 0, 0);
    V3 dscale = v3(0, 0, 0);
    float4 drot = make_float4(0, 0, 0, 0);
    float *dsh = shs ? dL_dsh + (size_t)idx * a.M * 3 : nullptr;
    int nsh_written = 0;
    if (vis) {
        const V3 m = v3(means3D[3 * idx], means3D[3 * idx + 1], means3D[3 * idx + 2]);
        float cov3D[6];
#pragma unroll
        for (int i = 0; i < 6; i++) cov3D[i] = cov3Ds[6 * (size_t)idx + i];
        // K8 (backward.cu:144-274): assigns the covariance part of dL/dmean
        dmean = cov2D_backward(m, a.focal_x, a.focal_y, a.tan_fovx, a.tan_fovy, cov3D, view,
                               make_float3(acc[2], acc[3], acc[4]), dcov);
        // K9 (backward.cu:370-387): projection part
        const float *proj = projm.m;
        float4 m_hom = transformPoint4x4(m, projm);
        float m_w = 1.0f / (m_hom.w + 0.0000001f);
        float mul1 = (proj[0] * m.x + proj[4] * m.y + proj[8] * m.z + proj[12]) * m_w * m_w;
        float mul2 = (proj[1] * m.x + proj[5] * m.y + proj[9] * m.z + proj[13]) * m_w * m_w;
        V3 dm2;
        dm2.x = (proj[0] * m_w - proj[3] * mul1) * acc[0] + (proj[1] * m_w - proj[3] * mul2) * acc[1];
        dm2.y = (proj[4] * m_w - proj[7] * mul1) * acc[0] + (proj[5] * m_w - proj[7] * mul2) * acc[1];
        dm2.z = (proj[8] * m_w - proj[11] * mul1) * acc[0] + (proj[9] * m_w - proj[11] * mul2) * acc[1];
        dmean = dmean + dm2;
        // SH part (backward.cu:390-391)
        if (shs) {
            const float *sh = shs + (size_t)idx * a.M * 3;
            const uint8_t cl = g.clamped[idx];
            V3 dRGB = v3(acc[6] * ((cl & 1) ? 0.f : 1.f), acc[7] * ((cl & 2) ? 0.f : 1.f),
                         acc[8] * ((cl & 4) ? 0.f : 1.f));
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

hipError_t launch_preprocess_backward(const Args &a, GeomState g, const int *radii, const float *contrib,
                                      const float *means3D, const float *shs, const float *scales,
                                      const float *rotations, const float *cov3D, float *dL_dmean2D,
                                      float *dL_dconic, float *dL_dopacity, float *dL_dcolor, float *dL_dmean3D,
                                      float *dL_dcov3D, float *dL_dsh, float *dL_dscale, float *dL_drot,
                                      hipStream_t s) {
    hipLaunchKernelGGL(preprocess_backward_kernel, dim3((a.P + 255) / 256), dim3(256), 0, s, a, g, radii, contrib,
                       means3D, shs, scales, rotations, cov3D, dL_dmean2D, dL_dconic, dL_dopacity, dL_dcolor,
                       dL_dmean3D, dL_dcov3D, dL_dsh, dL_dscale, dL_drot);
    return hipGetLastError();
}

}  // namespace gs4d
