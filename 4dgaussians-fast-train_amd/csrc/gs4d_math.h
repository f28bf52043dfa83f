// gs4d_math.h -- per-Gaussian device math of the rasterizer (gfx950).
//
// Restates the arithmetic of the reference kernels (paths relative to
// submodules/depth-diff-gaussian-rasterization/cuda_rasterizer/):
//   auxiliary.h:22-164   SH constants, ndc2Pix, getRect, transforms, dnormvdv, in_frustum
//   forward.cu:20-152    computeColorFromSH, computeCov2D, computeCov3D
//   backward.cu:20-341   SH backward, cov2D backward, cov3D backward
// glm 0.9.9 column-major semantics are kept literally (Mat3::m[col][row], products summed in glm's
// order, type_mat3x3.inl:486-519) so that the float results track the reference op for op.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gs4d {

constexpr int kBlockX = 16;  // config.h:16
constexpr int kBlockY = 16;  // config.h:17
constexpr int kChannels = 3; // config.h:15

constexpr float kSH_C0 = 0.28209479177387814f;
constexpr float kSH_C1 = 0.4886025119029199f;
constexpr float kSH_C2_0 = 1.0925484305920792f, kSH_C2_1 = -1.0925484305920792f, kSH_C2_2 = 0.31539156525252005f,
                kSH_C2_3 = -1.0925484305920792f, kSH_C2_4 = 0.5462742152960396f;
constexpr float kSH_C3_0 = -0.5900435899266435f, kSH_C3_1 = 2.890611442640554f, kSH_C3_2 = -0.4570457994644658f,
                kSH_C3_3 = 0.3731763325901154f, kSH_C3_4 = -0.4570457994644658f, kSH_C3_5 = 1.445305721320277f,
                kSH_C3_6 = -0.5900435899266435f;

struct V3 {
    float x, y, z;
};
__device__ __forceinline__ V3 v3(float x, float y, float z) { return V3{x, y, z}; }
__device__ __forceinline__ V3 operator+(V3 a, V3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ V3 operator-(V3 a, V3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ V3 operator*(float s, V3 a) { return v3(s * a.x, s * a.y, s * a.z); }
__device__ __forceinline__ V3 operator*(V3 a, float s) { return v3(a.x * s, a.y * s, a.z * s); }
__device__ __forceinline__ V3 mulv(V3 a, V3 b) { return v3(a.x * b.x, a.y * b.y, a.z * b.z); }
__device__ __forceinline__ float dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }

// glm::mat3, m[col][row]
struct Mat3 {
    float m[3][3];
};
__device__ __forceinline__ Mat3 mat3_cols(float a0, float a1, float a2, float a3, float a4, float a5, float a6,
                                          float a7, float a8) {
    Mat3 r;
    r.m[0][0] = a0; r.m[0][1] = a1; r.m[0][2] = a2;
    r.m[1][0] = a3; r.m[1][1] = a4; r.m[1][2] = a5;
    r.m[2][0] = a6; r.m[2][1] = a7; r.m[2][2] = a8;
    return r;
}
__device__ __forceinline__ Mat3 operator*(const Mat3 &A, const Mat3 &B) {
    Mat3 R;
#pragma unroll
    for (int c = 0; c < 3; c++)
#pragma unroll
        for (int r = 0; r < 3; r++)
            R.m[c][r] = A.m[0][r] * B.m[c][0] + A.m[1][r] * B.m[c][1] + A.m[2][r] * B.m[c][2];
    return R;
}
__device__ __forceinline__ Mat3 transpose(const Mat3 &A) {
    Mat3 R;
#pragma unroll
    for (int c = 0; c < 3; c++)
#pragma unroll
        for (int r = 0; r < 3; r++) R.m[c][r] = A.m[r][c];
    return R;
}
__device__ __forceinline__ V3 col(const Mat3 &A, int c) { return v3(A.m[c][0], A.m[c][1], A.m[c][2]); }

// auxiliary.h:41-44 (double literals: evaluated in double, rounded once)
__device__ __forceinline__ float ndc2Pix(float v, int S) { return (float)((((double)v + 1.0) * S - 1.0) * 0.5); }

// auxiliary.h:46-56
__device__ __forceinline__ void getRect(float px, float py, int max_radius, int gx, int gy, int &x0, int &y0,
                                        int &x1, int &y1) {
    x0 = min(gx, max(0, (int)((px - (float)max_radius) / kBlockX)));
    y0 = min(gy, max(0, (int)((py - (float)max_radius) / kBlockY)));
    x1 = min(gx, max(0, (int)((px + (float)max_radius + kBlockX - 1) / kBlockX)));
    y1 = min(gy, max(0, (int)((py + (float)max_radius + kBlockY - 1) / kBlockY)));
}

// auxiliary.h:58-97.  The 16 matrix entries live in kernel arguments (SGPRs).
struct Mat4 {
    float m[16];
};
__device__ __forceinline__ V3 transformPoint4x3(V3 p, const Mat4 &M) {
    const float *m = M.m;
    return v3(m[0] * p.x + m[4] * p.y + m[8] * p.z + m[12], m[1] * p.x + m[5] * p.y + m[9] * p.z + m[13],
              m[2] * p.x + m[6] * p.y + m[10] * p.z + m[14]);
}
__device__ __forceinline__ float4 transformPoint4x4(V3 p, const Mat4 &M) {
    const float *m = M.m;
    return make_float4(m[0] * p.x + m[4] * p.y + m[8] * p.z + m[12], m[1] * p.x + m[5] * p.y + m[9] * p.z + m[13],
                       m[2] * p.x + m[6] * p.y + m[10] * p.z + m[14], m[3] * p.x + m[7] * p.y + m[11] * p.z + m[15]);
}
__device__ __forceinline__ V3 transformVec4x3Transpose(V3 p, const Mat4 &M) {
    const float *m = M.m;
    return v3(m[0] * p.x + m[1] * p.y + m[2] * p.z, m[4] * p.x + m[5] * p.y + m[6] * p.z,
              m[8] * p.x + m[9] * p.y + m[10] * p.z);
}
// auxiliary.h:107-117
__device__ __forceinline__ V3 dnormvdv(V3 v, V3 dv) {
    float sum2 = v.x * v.x + v.y * v.y + v.z * v.z;
    float invsum32 = 1.0f / sqrtf(sum2 * sum2 * sum2);
    V3 r;
    r.x = ((+sum2 - v.x * v.x) * dv.x - v.y * v.x * dv.y - v.z * v.x * dv.z) * invsum32;
    r.y = (-v.x * v.y * dv.x + (sum2 - v.y * v.y) * dv.y - v.z * v.y * dv.z) * invsum32;
    r.z = (-v.x * v.z * dv.x - v.y * v.z * dv.y + (sum2 - v.z * v.z) * dv.z) * invsum32;
    return r;
}

// Rotation matrix of the UN-normalised quaternion (r,x,y,z) as glm::mat3 columns (forward.cu:127-138)
__device__ __forceinline__ Mat3 quat_mat(float r, float x, float y, float z) {
    return mat3_cols(1.f - 2.f * (y * y + z * z), 2.f * (x * y - r * z), 2.f * (x * z + r * y), 2.f * (x * y + r * z),
                     1.f - 2.f * (x * x + z * z), 2.f * (y * z - r * x), 2.f * (x * z - r * y), 2.f * (y * z + r * x),
                     1.f - 2.f * (x * x + y * y));
}

// forward.cu:118-152 -> upper triangle [00,01,02,11,12,22]
__device__ __forceinline__ void computeCov3D(V3 scale, float mod, float4 rot, float cov[6]) {
    Mat3 S = mat3_cols(1, 0, 0, 0, 1, 0, 0, 0, 1);
    S.m[0][0] = mod * scale.x;
    S.m[1][1] = mod * scale.y;
    S.m[2][2] = mod * scale.z;
    Mat3 R = quat_mat(rot.x, rot.y, rot.z, rot.w);
    Mat3 M = S * R;
    Mat3 Sigma = transpose(M) * M;
    cov[0] = Sigma.m[0][0]; cov[1] = Sigma.m[0][1]; cov[2] = Sigma.m[0][2];
    cov[3] = Sigma.m[1][1]; cov[4] = Sigma.m[1][2]; cov[5] = Sigma.m[2][2];
}

// forward.cu:74-113 -> (a, b, c) of the 2x2 screen-space covariance incl. the +0.3 low-pass
__device__ __forceinline__ float3 computeCov2D(V3 mean, float focal_x, float focal_y, float tan_fovx, float tan_fovy,
                                               const float cov3D[6], const Mat4 &view) {
    V3 t = transformPoint4x3(mean, view);
    const float limx = 1.3f * tan_fovx, limy = 1.3f * tan_fovy;
    const float txtz = t.x / t.z, tytz = t.y / t.z;
    t.x = fminf(limx, fmaxf(-limx, txtz)) * t.z;
    t.y = fminf(limy, fmaxf(-limy, tytz)) * t.z;
    Mat3 J = mat3_cols(focal_x / t.z, 0.0f, -(focal_x * t.x) / (t.z * t.z), 0.0f, focal_y / t.z,
                       -(focal_y * t.y) / (t.z * t.z), 0, 0, 0);
    const float *v = view.m;
    Mat3 W = mat3_cols(v[0], v[4], v[8], v[1], v[5], v[9], v[2], v[6], v[10]);
    Mat3 T = W * J;
    Mat3 Vrk = mat3_cols(cov3D[0], cov3D[1], cov3D[2], cov3D[1], cov3D[3], cov3D[4], cov3D[2], cov3D[4], cov3D[5]);
    Mat3 cov = transpose(T) * transpose(Vrk) * T;
    cov.m[0][0] += 0.3f;
    cov.m[1][1] += 0.3f;
    return make_float3(cov.m[0][0], cov.m[0][1], cov.m[1][1]);
}

// SH coefficient k of channel c for a Gaussian whose coefficients start at `sh` (layout (M,3))
#define GS4D_SH(k) v3(sh[3 * (k) + 0], sh[3 * (k) + 1], sh[3 * (k) + 2])

// forward.cu:20-71: returns the unclamped value; caller clamps at 0 and records the flags
__device__ __forceinline__ V3 sh_eval(int deg, const float *sh, V3 dir) {
    V3 result = kSH_C0 * GS4D_SH(0);
    if (deg > 0) {
        float x = dir.x, y = dir.y, z = dir.z;
        result = result - kSH_C1 * y * GS4D_SH(1) + kSH_C1 * z * GS4D_SH(2) - kSH_C1 * x * GS4D_SH(3);
        if (deg > 1) {
            float xx = x * x, yy = y * y, zz = z * z;
            float xy = x * y, yz = y * z, xz = x * z;
            result = result + kSH_C2_0 * xy * GS4D_SH(4) + kSH_C2_1 * yz * GS4D_SH(5) +
                     kSH_C2_2 * (2.0f * zz - xx - yy) * GS4D_SH(6) + kSH_C2_3 * xz * GS4D_SH(7) +
                     kSH_C2_4 * (xx - yy) * GS4D_SH(8);
            if (deg > 2) {
                result = result + kSH_C3_0 * y * (3.0f * xx - yy) * GS4D_SH(9) + kSH_C3_1 * xy * z * GS4D_SH(10) +
                         kSH_C3_2 * y * (4.0f * zz - xx - yy) * GS4D_SH(11) +
                         kSH_C3_3 * z * (2.0f * zz - 3.0f * xx - 3.0f * yy) * GS4D_SH(12) +
                         kSH_C3_4 * x * (4.0f * zz - xx - yy) * GS4D_SH(13) + kSH_C3_5 * z * (xx - yy) * GS4D_SH(14) +
                         kSH_C3_6 * x * (xx - 3.0f * yy) * GS4D_SH(15);
            }
        }
    }
    result = result + v3(0.5f, 0.5f, 0.5f);
    return result;
}

// backward.cu:20-139.  dL_dRGB already masked by the clamp flags.  Writes the (D+1)^2 used SH
// gradients to dsh (layout (M,3)) and returns the view-direction part of dL/dmean.
__device__ __forceinline__ V3 sh_backward(int deg, const float *sh, V3 dir_orig, V3 dL_dRGB, float *dsh) {
    const float len = sqrtf(dot(dir_orig, dir_orig));
    V3 dir = v3(dir_orig.x / len, dir_orig.y / len, dir_orig.z / len);
    V3 dRGBdx = v3(0, 0, 0), dRGBdy = v3(0, 0, 0), dRGBdz = v3(0, 0, 0);
    const float x = dir.x, y = dir.y, z = dir.z;
#define GS4D_DSH(k, val)                                                                                               \
    {                                                                                                                  \
        V3 g_ = (val) * dL_dRGB;                                                                                       \
        dsh[3 * (k) + 0] = g_.x;                                                                                       \
        dsh[3 * (k) + 1] = g_.y;                                                                                       \
        dsh[3 * (k) + 2] = g_.z;                                                                                       \
    }
    GS4D_DSH(0, kSH_C0);
    if (deg > 0) {
        GS4D_DSH(1, -kSH_C1 * y);
        GS4D_DSH(2, kSH_C1 * z);
        GS4D_DSH(3, -kSH_C1 * x);
        dRGBdx = -kSH_C1 * GS4D_SH(3);
        dRGBdy = -kSH_C1 * GS4D_SH(1);
        dRGBdz = kSH_C1 * GS4D_SH(2);
        if (deg > 1) {
            float xx = x * x, yy = y * y, zz = z * z;
            float xy = x * y, yz = y * z, xz = x * z;
            GS4D_DSH(4, kSH_C2_0 * xy);
            GS4D_DSH(5, kSH_C2_1 * yz);
            GS4D_DSH(6, kSH_C2_2 * (2.f * zz - xx - yy));
            GS4D_DSH(7, kSH_C2_3 * xz);
            GS4D_DSH(8, kSH_C2_4 * (xx - yy));
            dRGBdx = dRGBdx + kSH_C2_0 * y * GS4D_SH(4) + kSH_C2_2 * 2.f * -x * GS4D_SH(6) + kSH_C2_3 * z * GS4D_SH(7) +
                     kSH_C2_4 * 2.f * x * GS4D_SH(8);
            dRGBdy = dRGBdy + kSH_C2_0 * x * GS4D_SH(4) + kSH_C2_1 * z * GS4D_SH(5) + kSH_C2_2 * 2.f * -y * GS4D_SH(6) +
                     kSH_C2_4 * 2.f * -y * GS4D_SH(8);
            dRGBdz = dRGBdz + kSH_C2_1 * y * GS4D_SH(5) + kSH_C2_2 * 2.f * 2.f * z * GS4D_SH(6) +
                     kSH_C2_3 * x * GS4D_SH(7);
            if (deg > 2) {
                GS4D_DSH(9, kSH_C3_0 * y * (3.f * xx - yy));
                GS4D_DSH(10, kSH_C3_1 * xy * z);
                GS4D_DSH(11, kSH_C3_2 * y * (4.f * zz - xx - yy));
                GS4D_DSH(12, kSH_C3_3 * z * (2.f * zz - 3.f * xx - 3.f * yy));
                GS4D_DSH(13, kSH_C3_4 * x * (4.f * zz - xx - yy));
                GS4D_DSH(14, kSH_C3_5 * z * (xx - yy));
                GS4D_DSH(15, kSH_C3_6 * x * (xx - 3.f * yy));
                dRGBdx = dRGBdx + (kSH_C3_0 * GS4D_SH(9) * 3.f * 2.f * xy + kSH_C3_1 * GS4D_SH(10) * yz +
                                   kSH_C3_2 * GS4D_SH(11) * -2.f * xy + kSH_C3_3 * GS4D_SH(12) * -3.f * 2.f * xz +
                                   kSH_C3_4 * GS4D_SH(13) * (-3.f * xx + 4.f * zz - yy) +
                                   kSH_C3_5 * GS4D_SH(14) * 2.f * xz + kSH_C3_6 * GS4D_SH(15) * 3.f * (xx - yy));
                dRGBdy = dRGBdy + (kSH_C3_0 * GS4D_SH(9) * 3.f * (xx - yy) + kSH_C3_1 * GS4D_SH(10) * xz +
                                   kSH_C3_2 * GS4D_SH(11) * (-3.f * yy + 4.f * zz - xx) +
                                   kSH_C3_3 * GS4D_SH(12) * -3.f * 2.f * yz + kSH_C3_4 * GS4D_SH(13) * -2.f * xy +
                                   kSH_C3_5 * GS4D_SH(14) * -2.f * yz + kSH_C3_6 * GS4D_SH(15) * -3.f * 2.f * xy);
                dRGBdz = dRGBdz + (kSH_C3_1 * GS4D_SH(10) * xy + kSH_C3_2 * GS4D_SH(11) * 4.f * 2.f * yz +
                                   kSH_C3_3 * GS4D_SH(12) * 3.f * (2.f * zz - xx - yy) +
                                   kSH_C3_4 * GS4D_SH(13) * 4.f * 2.f * xz + kSH_C3_5 * GS4D_SH(14) * (xx - yy));
            }
        }
    }
#undef GS4D_DSH
    V3 dL_ddir = v3(dot(dRGBdx, dL_dRGB), dot(dRGBdy, dL_dRGB), dot(dRGBdz, dL_dRGB));
    return dnormvdv(dir_orig, dL_ddir);
}
#undef GS4D_SH

// backward.cu:278-341: gradients w.r.t. the scale (NOT multiplied by mod, Q26) and the quaternion used as-is
__device__ __forceinline__ void cov3D_backward(V3 scale, float mod, float4 rot, const float dc[6], V3 &dL_dscale,
                                               float4 &dL_drot) {
    const float r = rot.x, x = rot.y, y = rot.z, z = rot.w;
    Mat3 R = quat_mat(r, x, y, z);
    Mat3 S = mat3_cols(1, 0, 0, 0, 1, 0, 0, 0, 1);
    V3 s = mod * scale;
    S.m[0][0] = s.x;
    S.m[1][1] = s.y;
    S.m[2][2] = s.z;
    Mat3 M = S * R;
    Mat3 dL_dSigma = mat3_cols(dc[0], 0.5f * dc[1], 0.5f * dc[2], 0.5f * dc[1], dc[3], 0.5f * dc[4], 0.5f * dc[2],
                               0.5f * dc[4], dc[5]);
    Mat3 M2;
#pragma unroll
    for (int c = 0; c < 3; c++)
#pragma unroll
        for (int q = 0; q < 3; q++) M2.m[c][q] = 2.0f * M.m[c][q];
    Mat3 dL_dM = M2 * dL_dSigma;
    Mat3 Rt = transpose(R);
    Mat3 dMt = transpose(dL_dM);
    dL_dscale.x = dot(col(Rt, 0), col(dMt, 0));
    dL_dscale.y = dot(col(Rt, 1), col(dMt, 1));
    dL_dscale.z = dot(col(Rt, 2), col(dMt, 2));
#pragma unroll
    for (int q = 0; q < 3; q++) {
        dMt.m[0][q] *= s.x;
        dMt.m[1][q] *= s.y;
        dMt.m[2][q] *= s.z;
    }
    const float(*d)[3] = dMt.m;
    dL_drot.x = 2 * z * (d[0][1] - d[1][0]) + 2 * y * (d[2][0] - d[0][2]) + 2 * x * (d[1][2] - d[2][1]);
    dL_drot.y = 2 * y * (d[1][0] + d[0][1]) + 2 * z * (d[2][0] + d[0][2]) + 2 * r * (d[1][2] - d[2][1]) -
                4 * x * (d[2][2] + d[1][1]);
    dL_drot.z = 2 * x * (d[1][0] + d[0][1]) + 2 * r * (d[2][0] - d[0][2]) + 2 * z * (d[1][2] + d[2][1]) -
                4 * y * (d[2][2] + d[0][0]);
    dL_drot.w = 2 * r * (d[0][1] - d[1][0]) + 2 * x * (d[2][0] + d[0][2]) + 2 * y * (d[1][2] + d[2][1]) -
                4 * z * (d[1][1] + d[0][0]);
}

// backward.cu:144-274 for one Gaussian: dL/dconic (a, b, c slots) -> dL/dcov3D (6) and the cov part of dL/dmean
__device__ __forceinline__ V3 cov2D_backward(V3 mean, float h_x, float h_y, float tan_fovx, float tan_fovy,
                                             const float cov3D[6], const Mat4 &view, float3 dL_dconic,
                                             float dL_dcov[6]) {
    V3 t = transformPoint4x3(mean, view);
    const float limx = 1.3f * tan_fovx, limy = 1.3f * tan_fovy;
    const float txtz = t.x / t.z, tytz = t.y / t.z;
    t.x = fminf(limx, fmaxf(-limx, txtz)) * t.z;
    t.y = fminf(limy, fmaxf(-limy, tytz)) * t.z;
    const float x_grad_mul = txtz < -limx || txtz > limx ? 0 : 1;
    const float y_grad_mul = tytz < -limy || tytz > limy ? 0 : 1;
    Mat3 J = mat3_cols(h_x / t.z, 0.0f, -(h_x * t.x) / (t.z * t.z), 0.0f, h_y / t.z, -(h_y * t.y) / (t.z * t.z), 0, 0,
                       0);
    const float *v = view.m;
    Mat3 W = mat3_cols(v[0], v[4], v[8], v[1], v[5], v[9], v[2], v[6], v[10]);
    Mat3 Vrk = mat3_cols(cov3D[0], cov3D[1], cov3D[2], cov3D[1], cov3D[3], cov3D[4], cov3D[2], cov3D[4], cov3D[5]);
    Mat3 T = W * J;
    Mat3 cov2D = transpose(T) * transpose(Vrk) * T;
    float a = cov2D.m[0][0] += 0.3f;
    float b = cov2D.m[0][1];
    float c = cov2D.m[1][1] += 0.3f;
    float denom = a * c - b * b;
    float dL_da = 0, dL_db = 0, dL_dc = 0;
    float denom2inv = 1.0f / ((denom * denom) + 0.0000001f);
    const float(*Tq)[3] = T.m;
    if (denom2inv != 0) {
        dL_da = denom2inv * (-c * c * dL_dconic.x + 2 * b * c * dL_dconic.y + (denom - a * c) * dL_dconic.z);
        dL_dc = denom2inv * (-a * a * dL_dconic.z + 2 * a * b * dL_dconic.y + (denom - a * c) * dL_dconic.x);
        dL_db = denom2inv * 2 * (b * c * dL_dconic.x - (denom + 2 * b * b) * dL_dconic.y + a * b * dL_dconic.z);
        dL_dcov[0] = (Tq[0][0] * Tq[0][0] * dL_da + Tq[0][0] * Tq[1][0] * dL_db + Tq[1][0] * Tq[1][0] * dL_dc);
        dL_dcov[3] = (Tq[0][1] * Tq[0][1] * dL_da + Tq[0][1] * Tq[1][1] * dL_db + Tq[1][1] * Tq[1][1] * dL_dc);
        dL_dcov[5] = (Tq[0][2] * Tq[0][2] * dL_da + Tq[0][2] * Tq[1][2] * dL_db + Tq[1][2] * Tq[1][2] * dL_dc);
        dL_dcov[1] = 2 * Tq[0][0] * Tq[0][1] * dL_da + (Tq[0][0] * Tq[1][1] + Tq[0][1] * Tq[1][0]) * dL_db +
                     2 * Tq[1][0] * Tq[1][1] * dL_dc;
        dL_dcov[2] = 2 * Tq[0][0] * Tq[0][2] * dL_da + (Tq[0][0] * Tq[1][2] + Tq[0][2] * Tq[1][0]) * dL_db +
                     2 * Tq[1][0] * Tq[1][2] * dL_dc;
        dL_dcov[4] = 2 * Tq[0][2] * Tq[0][1] * dL_da + (Tq[0][1] * Tq[1][2] + Tq[0][2] * Tq[1][1]) * dL_db +
                     2 * Tq[1][1] * Tq[1][2] * dL_dc;
    } else {
#pragma unroll
        for (int i = 0; i < 6; i++) dL_dcov[i] = 0;
    }
    const float(*Vq)[3] = Vrk.m;
    float dL_dT00 = 2 * (Tq[0][0] * Vq[0][0] + Tq[0][1] * Vq[0][1] + Tq[0][2] * Vq[0][2]) * dL_da +
                    (Tq[1][0] * Vq[0][0] + Tq[1][1] * Vq[0][1] + Tq[1][2] * Vq[0][2]) * dL_db;
    float dL_dT01 = 2 * (Tq[0][0] * Vq[1][0] + Tq[0][1] * Vq[1][1] + Tq[0][2] * Vq[1][2]) * dL_da +
                    (Tq[1][0] * Vq[1][0] + Tq[1][1] * Vq[1][1] + Tq[1][2] * Vq[1][2]) * dL_db;
    float dL_dT02 = 2 * (Tq[0][0] * Vq[2][0] + Tq[0][1] * Vq[2][1] + Tq[0][2] * Vq[2][2]) * dL_da +
                    (Tq[1][0] * Vq[2][0] + Tq[1][1] * Vq[2][1] + Tq[1][2] * Vq[2][2]) * dL_db;
    float dL_dT10 = 2 * (Tq[1][0] * Vq[0][0] + Tq[1][1] * Vq[0][1] + Tq[1][2] * Vq[0][2]) * dL_dc +
                    (Tq[0][0] * Vq[0][0] + Tq[0][1] * Vq[0][1] + Tq[0][2] * Vq[0][2]) * dL_db;
    float dL_dT11 = 2 * (Tq[1][0] * Vq[1][0] + Tq[1][1] * Vq[1][1] + Tq[1][2] * Vq[1][2]) * dL_dc +
                    (Tq[0][0] * Vq[1][0] + Tq[0][1] * Vq[1][1] + Tq[0][2] * Vq[1][2]) * dL_db;
    float dL_dT12 = 2 * (Tq[1][0] * Vq[2][0] + Tq[1][1] * Vq[2][1] + Tq[1][2] * Vq[2][2]) * dL_dc +
                    (Tq[0][0] * Vq[2][0] + Tq[0][1] * Vq[2][1] + Tq[0][2] * Vq[2][2]) * dL_db;
    const float(*Wq)[3] = W.m;
    float dL_dJ00 = Wq[0][0] * dL_dT00 + Wq[0][1] * dL_dT01 + Wq[0][2] * dL_dT02;
    float dL_dJ02 = Wq[2][0] * dL_dT00 + Wq[2][1] * dL_dT01 + Wq[2][2] * dL_dT02;
    float dL_dJ11 = Wq[1][0] * dL_dT10 + Wq[1][1] * dL_dT11 + Wq[1][2] * dL_dT12;
    float dL_dJ12 = Wq[2][0] * dL_dT10 + Wq[2][1] * dL_dT11 + Wq[2][2] * dL_dT12;
    float tz = 1.f / t.z;
    float tz2 = tz * tz;
    float tz3 = tz2 * tz;
    float dL_dtx = x_grad_mul * -h_x * tz2 * dL_dJ02;
    float dL_dty = y_grad_mul * -h_y * tz2 * dL_dJ12;
    float dL_dtz = -h_x * tz2 * dL_dJ00 - h_y * tz2 * dL_dJ11 + (2 * h_x * t.x) * tz3 * dL_dJ02 +
                   (2 * h_y * t.y) * tz3 * dL_dJ12;
    return transformVec4x3Transpose(v3(dL_dtx, dL_dty, dL_dtz), view);
}

}  // namespace gs4d
