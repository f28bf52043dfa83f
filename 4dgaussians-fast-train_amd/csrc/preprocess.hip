// preprocess.hip -- per-Gaussian forward preprocess (K1), markVisible (K10) and the block-offset scan
// that replaces cub::DeviceScan::InclusiveSum (K2).
//
// Reference: cuda_rasterizer/forward.cu:155-256 (preprocessCUDA), auxiliary.h:139-164 (in_frustum),
// rasterizer_impl.cu:54-66 (checkFrustum), rasterizer_impl.cu:278-282 (scan + num_rendered).
#include "gs4d_internal.h"

namespace gs4d {

// One thread per Gaussian.  Besides the reference's outputs it produces num_rendered (the sum of
// tiles_touched, added per workgroup into 8 sharded u64 counters: only the total is ever needed).
__global__ __launch_bounds__(kPreprocessBlock) void preprocess_kernel(
    Args a, const float *__restrict__ means3D, const float *__restrict__ scales, const float *__restrict__ rotations,
    const float *__restrict__ opacities, const float *__restrict__ shs, const float *__restrict__ cov3D_precomp,
    const float *__restrict__ colors_precomp, int *__restrict__ radii, GeomState g, int *__restrict__ err_flag) {
    __shared__ uint32_t s_wave[kPreprocessBlock / 64];
    const int idx = blockIdx.x * kPreprocessBlock + threadIdx.x;
    const Mat4 view = load_mat4(a.viewmatrix, a.view_transposed), proj = load_mat4(a.projmatrix);
    uint32_t touched = 0;
    if (idx < a.P) {
        int my_r = 0;
        V3 p_orig = v3(means3D[3 * idx], means3D[3 * idx + 1], means3D[3 * idx + 2]);
        // in_frustum (auxiliary.h:146-154): only the near plane culls
        V3 p_view = transformPoint4x3(p_orig, view);
        bool ok = !(p_view.z <= 0.2f);
        if (!ok && a.prefiltered) atomicOr(err_flag, 1);
        float cov3[6];
        float3 cov;
        float det = 0.f;
        if (ok) {
            float4 p_hom = transformPoint4x4(p_orig, proj);
            float p_w = 1.0f / (p_hom.w + 0.0000001f);
            float p_proj_x = p_hom.x * p_w, p_proj_y = p_hom.y * p_w;
            if (cov3D_precomp != nullptr) {
#pragma unroll
                for (int i = 0; i < 6; i++) cov3[i] = cov3D_precomp[6 * (size_t)idx + i];
            } else {
                V3 sc = v3(scales[3 * idx], scales[3 * idx + 1], scales[3 * idx + 2]);
                float4 rot = reinterpret_cast<const float4 *>(rotations)[idx];
                computeCov3D(sc, a.scale_modifier, rot, cov3);
#pragma unroll
                for (int i = 0; i < 6; i++) g.cov3D[6 * (size_t)idx + i] = cov3[i];
            }
            cov = computeCov2D(p_orig, a.focal_x, a.focal_y, a.tan_fovx, a.tan_fovy, cov3, view);
            det = (cov.x * cov.z - cov.y * cov.y);
            ok = det != 0.0f;
            if (ok) {
                float det_inv = 1.f / det;
                float3 conic = make_float3(cov.z * det_inv, -cov.y * det_inv, cov.x * det_inv);
                float mid = 0.5f * (cov.x + cov.z);
                float lambda1 = mid + sqrtf(fmaxf(0.1f, mid * mid - det));
                float lambda2 = mid - sqrtf(fmaxf(0.1f, mid * mid - det));
                float my_radius = ceilf(3.f * sqrtf(fmaxf(lambda1, lambda2)));
                float2 point_image = make_float2(ndc2Pix(p_proj_x, a.W), ndc2Pix(p_proj_y, a.H));
                int x0, y0, x1, y1;
                getRect(point_image.x, point_image.y, (int)my_radius, a.gx, a.gy, x0, y0, x1, y1);
                uint32_t area = (uint32_t)((y1 - y0) * (x1 - x0));
                if (area != 0) {
                    float3 rgb;
                    uint8_t cl = 0;
                    if (colors_precomp == nullptr) {
                        const float *sh = shs + (size_t)idx * a.M * 3;
                        V3 dir = p_orig - load_v3(a.campos);
                        float len = sqrtf(dot(dir, dir));
                        dir = v3(dir.x / len, dir.y / len, dir.z / len);
                        V3 res;
                        if (a.M == 16 && ((size_t)shs & 15) == 0) {
                            // degree-3 layout: 12 float4 loads instead of 48 scalar loads strided 192 B
                            float shl[48];
                            const float4 *s4 = reinterpret_cast<const float4 *>(sh);
#pragma unroll
                            for (int q = 0; q < 12; q++) {
                                const float4 v = s4[q];
                                shl[4 * q] = v.x, shl[4 * q + 1] = v.y, shl[4 * q + 2] = v.z, shl[4 * q + 3] = v.w;
                            }
                            res = sh_eval(a.D, shl, dir);
                        } else {
                            res = sh_eval(a.D, sh, dir);
                        }
                        cl = (uint8_t)((res.x < 0) | ((res.y < 0) << 1) | ((res.z < 0) << 2));
                        rgb = make_float3(fmaxf(res.x, 0.0f), fmaxf(res.y, 0.0f), fmaxf(res.z, 0.0f));
                    } else {
                        rgb = make_float3(colors_precomp[3 * idx], colors_precomp[3 * idx + 1],
                                          colors_precomp[3 * idx + 2]);
                    }
                    const float4 co = make_float4(conic.x, conic.y, conic.z, opacities[idx]);
                    g.clamped[idx] = cl;
                    g.depths[idx] = p_view.z;
                    g.xy[idx] = point_image;
                    g.conic_opacity[idx] = co;
                    // the blend kernels' packed record: log2(e) folded into the conic (forward.cu:340-342 in
                    // base 2), 1/o for the backward's per-record division, colour and view depth.  For a
                    // positive-definite conic (the blend kernels' conic_pd on these same stored values) the
                    // opacity is folded into the exponent too: o G = 2^(power2 + log2 o), the record's
                    // multiplier is 1 and the blend's common path skips the o * G multiply; any other conic
                    // keeps multiplier o and exponent offset 0 (its power test needs the bare exponent).
                    float4 *rec = g.splat + 3 * (size_t)idx;
                    const float ga = (-0.5f * co.x) * kLog2e, gb = (-co.y) * kLog2e, gc = (-0.5f * co.z) * kLog2e;
                    const bool pd = ga < 0.f && 4.f * ga * gc - gb * gb > 0.f;
                    rec[0] = make_float4(point_image.x, point_image.y, ga, gb);
                    rec[1] = make_float4(gc, pd ? 1.f : co.w, co.w > 0.f ? 1.0f / co.w : 0.f, p_view.z);
                    rec[2] = make_float4(rgb.x, rgb.y, rgb.z, pd ? log2f(co.w) : 0.f);
                    my_r = (int)my_radius;
                    touched = area;
                }
            }
        }
        radii[idx] = my_r;
        g.tiles_touched[idx] = touched;
        g.n_inst[idx] = 0;
    }
    // workgroup sum of tiles_touched
    uint32_t v = touched;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    if ((threadIdx.x & 63) == 0) s_wave[threadIdx.x >> 6] = v;
    __syncthreads();
    const int shard = blockIdx.x % kHistShards;
    if (threadIdx.x == 0) {
        uint32_t t = 0;
#pragma unroll
        for (int w = 0; w < kPreprocessBlock / 64; w++) t += s_wave[w];
        if (t) atomicAdd(reinterpret_cast<unsigned long long *>(g.zero + kZeroL) + shard, (unsigned long long)t);
    }
}

hipError_t launch_preprocess(const Args &a, const float *means3D, const float *scales, const float *rotations,
                             const float *opacities, const float *shs, const float *cov3D_precomp,
                             const float *colors_precomp, int *radii, GeomState g, int *err_flag, hipStream_t s) {
    const int nblk = (a.P + kPreprocessBlock - 1) / kPreprocessBlock;
    hipLaunchKernelGGL(preprocess_kernel, dim3(nblk), dim3(kPreprocessBlock), 0, s, a, means3D, scales, rotations,
                       opacities, shs, cov3D_precomp, colors_precomp, radii, g, err_flag);
    return hipGetLastError();
}

// rasterizer_impl.cu:54-66 checkFrustum
__global__ void mark_visible_kernel(int P, const float *__restrict__ means3D, const float *__restrict__ viewmatrix,
                                    int view_transposed,
                                    uint8_t *__restrict__ present) {
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= P) return;
    const Mat4 view = load_mat4(viewmatrix, view_transposed);
    V3 p = v3(means3D[3 * idx], means3D[3 * idx + 1], means3D[3 * idx + 2]);
    V3 pv = transformPoint4x3(p, view);
    present[idx] = !(pv.z <= 0.2f);
}

hipError_t launch_mark_visible(int P, const float *means3D, const float *viewmatrix, int view_transposed,
                               uint8_t *present, hipStream_t s) {
    hipLaunchKernelGGL(mark_visible_kernel, dim3((P + 255) / 256), dim3(256), 0, s, P, means3D, viewmatrix,
                       view_transposed, present);
    return hipGetLastError();
}

}  // namespace gs4d
