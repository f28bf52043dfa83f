/*
 * gs4d_oracle.c -- CPU restatement of the reference differentiable Gaussian rasterizer.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the parity oracle for the MI355X HIP path and the timed
 * CPU baseline of bench.py.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
 * may load it; the product library (libgs4d.so / diff_gaussian_rasterization._C) never links it.
 *
 * It restates, function by function, the algorithm of
 *   submodules/depth-diff-gaussian-rasterization/cuda_rasterizer/{forward.cu,backward.cu,
 *   rasterizer_impl.cu,auxiliary.h,config.h}
 * (paths relative to the reference root).  glm 0.9.9 column-major semantics are followed
 * literally: a glm::mat3 is stored here as m[col][row] and products are summed in glm's order
 * (third_party/glm/glm/detail/type_mat3x3.inl:486-519).
 *
 * Deliberate, documented differences from the CUDA reference (none changes a result beyond the
 * stated tolerances):
 *   - The reference's K7 accumulates per-Gaussian gradients with float atomicAdd in an unspecified
 *     order (backward.cu:523,545-554).  The oracle sums the same per-(tile, Gaussian) terms in
 *     double precision, in sorted-list order, then rounds once: a deterministic, order-free value.
 *   - CUB's stable radix sort (rasterizer_impl.cu:304-309) is restated as a comparison sort on
 *     (key, unsorted position), which yields the identical permutation.
 *   - nvcc contracts a*b+c into FMA by default; this file is compiled with -ffp-contract=off,
 *     so individual results may differ from the CUDA build in the last ulp.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define BLOCK_X 16 /* config.h:16 */
#define BLOCK_Y 16 /* config.h:17 */
#define BLOCK_SIZE (BLOCK_X * BLOCK_Y) /* auxiliary.h:18 */
#define NCH 3                          /* config.h:15 NUM_CHANNELS */

/* auxiliary.h:22-39 */
static const float SH_C0 = 0.28209479177387814f;
static const float SH_C1 = 0.4886025119029199f;
static const float SH_C2[5] = {1.0925484305920792f, -1.0925484305920792f, 0.31539156525252005f,
                               -1.0925484305920792f, 0.5462742152960396f};
static const float SH_C3[7] = {-0.5900435899266435f, 2.890611442640554f, -0.4570457994644658f,
                               0.3731763325901154f, -0.4570457994644658f, 1.445305721320277f,
                               -0.5900435899266435f};

typedef struct { float x, y, z; } f3;
typedef struct { float x, y, z, w; } f4;
typedef struct { float m[3][3]; } mat3; /* m[col][row], glm convention */

static inline float fminf_(float a, float b) { return a < b ? a : b; }
static inline float fmaxf_(float a, float b) { return a > b ? a : b; }

/* The alpha test's near-threshold band at one (pixel, splat) pair.  Two float evaluations of
 * power = -0.5 (a dx^2 + c dy^2) - b dx dy (forward.cu:336-338) in different operation orders (the blend
 * kernels: base 2, pre-scaled conic, FMA) differ by a few roundings of the terms' magnitudes, and alpha = o
 * exp(power) inherits that absolute difference as a relative one.  So the band scales with
 * 1 + 0.5 (|a| dx^2 + |c| dy^2) + |b dx dy|: band_alpha is the allowance per unit of it (set from the
 * measured differences, oracle/parity.py). */
static inline int near_alpha(float alpha, const float *co, float dx, float dy, float band_alpha) {
    const float mag = 1.0f + 0.5f * (fabsf(co[0]) * dx * dx + fabsf(co[2]) * dy * dy) + fabsf(co[1] * dx * dy);
    return fabsf(alpha * 255.0f - 1.0f) <= band_alpha * mag;
}

/* glm::mat3(a0..a8): columns (a0,a1,a2), (a3,a4,a5), (a6,a7,a8) */
static inline mat3 mat3_cols(float a0, float a1, float a2, float a3, float a4, float a5, float a6,
                             float a7, float a8) {
    mat3 r;
    r.m[0][0] = a0; r.m[0][1] = a1; r.m[0][2] = a2;
    r.m[1][0] = a3; r.m[1][1] = a4; r.m[1][2] = a5;
    r.m[2][0] = a6; r.m[2][1] = a7; r.m[2][2] = a8;
    return r;
}
/* type_mat3x3.inl:486-519: R[c][r] = A[0][r]*B[c][0] + A[1][r]*B[c][1] + A[2][r]*B[c][2] */
static inline mat3 mat3_mul(const mat3 *A, const mat3 *B) {
    mat3 R;
    for (int c = 0; c < 3; c++)
        for (int r = 0; r < 3; r++)
            R.m[c][r] = A->m[0][r] * B->m[c][0] + A->m[1][r] * B->m[c][1] + A->m[2][r] * B->m[c][2];
    return R;
}
static inline mat3 mat3_T(const mat3 *A) {
    mat3 R;
    for (int c = 0; c < 3; c++)
        for (int r = 0; r < 3; r++) R.m[c][r] = A->m[r][c];
    return R;
}
/* glm::dot (func_geometric.inl compute_dot): (x*x' + y*y') + z*z' */
static inline float dot3(const float *a, const float *b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }

/* auxiliary.h:41-44 -- note the double literals: the arithmetic is done in double */
static inline float ndc2Pix(float v, int S) { return (float)((((double)v + 1.0) * S - 1.0) * 0.5); }

/* auxiliary.h:46-56 */
static inline void getRect(float px, float py, int max_radius, int gx, int gy, int *rmin_x, int *rmin_y,
                           int *rmax_x, int *rmax_y) {
    int a;
    a = (int)((px - (float)max_radius) / BLOCK_X); a = a > 0 ? a : 0; *rmin_x = a < gx ? a : gx;
    a = (int)((py - (float)max_radius) / BLOCK_Y); a = a > 0 ? a : 0; *rmin_y = a < gy ? a : gy;
    a = (int)((px + (float)max_radius + BLOCK_X - 1) / BLOCK_X); a = a > 0 ? a : 0; *rmax_x = a < gx ? a : gx;
    a = (int)((py + (float)max_radius + BLOCK_Y - 1) / BLOCK_Y); a = a > 0 ? a : 0; *rmax_y = a < gy ? a : gy;
}

/* auxiliary.h:58-66 */
static inline f3 transformPoint4x3(f3 p, const float *m) {
    f3 t = {m[0] * p.x + m[4] * p.y + m[8] * p.z + m[12], m[1] * p.x + m[5] * p.y + m[9] * p.z + m[13],
            m[2] * p.x + m[6] * p.y + m[10] * p.z + m[14]};
    return t;
}
/* auxiliary.h:68-77 */
static inline f4 transformPoint4x4(f3 p, const float *m) {
    f4 t = {m[0] * p.x + m[4] * p.y + m[8] * p.z + m[12], m[1] * p.x + m[5] * p.y + m[9] * p.z + m[13],
            m[2] * p.x + m[6] * p.y + m[10] * p.z + m[14], m[3] * p.x + m[7] * p.y + m[11] * p.z + m[15]};
    return t;
}
/* auxiliary.h:89-97 */
static inline f3 transformVec4x3Transpose(f3 p, const float *m) {
    f3 t = {m[0] * p.x + m[1] * p.y + m[2] * p.z, m[4] * p.x + m[5] * p.y + m[6] * p.z,
            m[8] * p.x + m[9] * p.y + m[10] * p.z};
    return t;
}
/* auxiliary.h:107-117 */
static inline f3 dnormvdv(f3 v, f3 dv) {
    float sum2 = v.x * v.x + v.y * v.y + v.z * v.z;
    float invsum32 = 1.0f / sqrtf(sum2 * sum2 * sum2);
    f3 r;
    r.x = ((+sum2 - v.x * v.x) * dv.x - v.y * v.x * dv.y - v.z * v.x * dv.z) * invsum32;
    r.y = (-v.x * v.y * dv.x + (sum2 - v.y * v.y) * dv.y - v.z * v.y * dv.z) * invsum32;
    r.z = (-v.x * v.z * dv.x - v.y * v.z * dv.y + (sum2 - v.z * v.z) * dv.z) * invsum32;
    return r;
}
/* auxiliary.h:139-164 (returns 1 when visible; prefiltered violations are reported, not trapped) */
static inline int in_frustum(int idx, const float *pts, const float *view, const float *proj, f3 *p_view) {
    f3 p = {pts[3 * idx], pts[3 * idx + 1], pts[3 * idx + 2]};
    (void)proj; /* p_proj is computed but only used by the commented-out xy test (auxiliary.h:149-154) */
    *p_view = transformPoint4x3(p, view);
    return !(p_view->z <= 0.2f);
}

/* forward.cu:20-71 */
static void sh_forward(int idx, int deg, int max_coeffs, const float *means, const float *campos, const float *shs,
                       uint8_t *clamped, float *rgb_out) {
    f3 pos = {means[3 * idx], means[3 * idx + 1], means[3 * idx + 2]};
    float dir[3] = {pos.x - campos[0], pos.y - campos[1], pos.z - campos[2]};
    float len = sqrtf(dot3(dir, dir));
    dir[0] = dir[0] / len; dir[1] = dir[1] / len; dir[2] = dir[2] / len;
    const float *sh = shs + (size_t)idx * max_coeffs * 3;
    float res[3];
    for (int c = 0; c < 3; c++) res[c] = SH_C0 * sh[c];
    if (deg > 0) {
        float x = dir[0], y = dir[1], z = dir[2];
        for (int c = 0; c < 3; c++)
            res[c] = res[c] - SH_C1 * y * sh[3 + c] + SH_C1 * z * sh[6 + c] - SH_C1 * x * sh[9 + c];
        if (deg > 1) {
            float xx = x * x, yy = y * y, zz = z * z;
            float xy = x * y, yz = y * z, xz = x * z;
            for (int c = 0; c < 3; c++)
                res[c] = res[c] + SH_C2[0] * xy * sh[12 + c] + SH_C2[1] * yz * sh[15 + c] +
                         SH_C2[2] * (2.0f * zz - xx - yy) * sh[18 + c] + SH_C2[3] * xz * sh[21 + c] +
                         SH_C2[4] * (xx - yy) * sh[24 + c];
            if (deg > 2) {
                for (int c = 0; c < 3; c++)
                    res[c] = res[c] + SH_C3[0] * y * (3.0f * xx - yy) * sh[27 + c] + SH_C3[1] * xy * z * sh[30 + c] +
                             SH_C3[2] * y * (4.0f * zz - xx - yy) * sh[33 + c] +
                             SH_C3[3] * z * (2.0f * zz - 3.0f * xx - 3.0f * yy) * sh[36 + c] +
                             SH_C3[4] * x * (4.0f * zz - xx - yy) * sh[39 + c] +
                             SH_C3[5] * z * (xx - yy) * sh[42 + c] + SH_C3[6] * x * (xx - 3.0f * yy) * sh[45 + c];
            }
        }
    }
    uint8_t cl = 0;
    for (int c = 0; c < 3; c++) {
        res[c] += 0.5f;
        if (res[c] < 0) cl |= (uint8_t)(1u << c);
        rgb_out[c] = fmaxf_(res[c], 0.0f);
    }
    clamped[idx] = cl;
}

/* forward.cu:118-152 */
static void cov3d_forward(const float *scale, float mod, const float *rot, float *cov3D) {
    mat3 S = mat3_cols(1, 0, 0, 0, 1, 0, 0, 0, 1);
    S.m[0][0] = mod * scale[0];
    S.m[1][1] = mod * scale[1];
    S.m[2][2] = mod * scale[2];
    float r = rot[0], x = rot[1], y = rot[2], z = rot[3]; /* not normalised (forward.cu:127) */
    mat3 R = mat3_cols(1.f - 2.f * (y * y + z * z), 2.f * (x * y - r * z), 2.f * (x * z + r * y),
                       2.f * (x * y + r * z), 1.f - 2.f * (x * x + z * z), 2.f * (y * z - r * x),
                       2.f * (x * z - r * y), 2.f * (y * z + r * x), 1.f - 2.f * (x * x + y * y));
    mat3 M = mat3_mul(&S, &R);
    mat3 Mt = mat3_T(&M);
    mat3 Sigma = mat3_mul(&Mt, &M);
    cov3D[0] = Sigma.m[0][0]; cov3D[1] = Sigma.m[0][1]; cov3D[2] = Sigma.m[0][2];
    cov3D[3] = Sigma.m[1][1]; cov3D[4] = Sigma.m[1][2]; cov3D[5] = Sigma.m[2][2];
}

/* forward.cu:74-113 */
static void cov2d_forward(f3 mean, float focal_x, float focal_y, float tan_fovx, float tan_fovy, const float *cov3D,
                          const float *view, float *out3) {
    f3 t = transformPoint4x3(mean, view);
    const float limx = 1.3f * tan_fovx, limy = 1.3f * tan_fovy;
    const float txtz = t.x / t.z, tytz = t.y / t.z;
    t.x = fminf_(limx, fmaxf_(-limx, txtz)) * t.z;
    t.y = fminf_(limy, fmaxf_(-limy, tytz)) * t.z;
    mat3 J = mat3_cols(focal_x / t.z, 0.0f, -(focal_x * t.x) / (t.z * t.z), 0.0f, focal_y / t.z,
                       -(focal_y * t.y) / (t.z * t.z), 0, 0, 0);
    mat3 W = mat3_cols(view[0], view[4], view[8], view[1], view[5], view[9], view[2], view[6], view[10]);
    mat3 T = mat3_mul(&W, &J);
    mat3 Vrk = mat3_cols(cov3D[0], cov3D[1], cov3D[2], cov3D[1], cov3D[3], cov3D[4], cov3D[2], cov3D[4], cov3D[5]);
    mat3 Tt = mat3_T(&T), Vt = mat3_T(&Vrk);
    mat3 A = mat3_mul(&Tt, &Vt);
    mat3 cov = mat3_mul(&A, &T);
    cov.m[0][0] += 0.3f;
    cov.m[1][1] += 0.3f;
    out3[0] = cov.m[0][0]; out3[1] = cov.m[0][1]; out3[2] = cov.m[1][1];
}

/* ---------------------------------------------------------------------------------------------- */
/* Forward state, the oracle's analogue of GeometryState / BinningState / ImageState
 * (rasterizer_impl.h:31-67).                                                                    */
typedef struct {
    int P, D, M, W, H, gx, gy, L;
    /* geometry (per Gaussian) */
    float *depths, *means2D, *cov3D, *conic_opacity, *rgb;
    uint8_t *clamped;
    int *radii;
    uint32_t *tiles_touched, *point_offsets;
    /* binning (per instance) */
    uint64_t *keys;      /* sorted */
    uint32_t *point_list;  /* sorted Gaussian ids */
    uint32_t *sorted_upos; /* unsorted position of each sorted instance */
    /* image */
    uint32_t *ranges; /* 2 per tile */
    float *final_T;
    uint32_t *n_contrib;
} gs4d_oracle_state;

void gs4d_oracle_set_threads(int n) {
#ifdef _OPENMP
    if (n > 0) omp_set_num_threads(n);
#else
    (void)n;
#endif
}
int gs4d_oracle_get_threads(void) {
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}

void gs4d_oracle_free(gs4d_oracle_state *s) {
    if (!s) return;
    free(s->depths); free(s->means2D); free(s->cov3D); free(s->conic_opacity); free(s->rgb);
    free(s->clamped); free(s->radii); free(s->tiles_touched); free(s->point_offsets);
    free(s->keys); free(s->point_list); free(s->sorted_upos);
    free(s->ranges); free(s->final_T); free(s->n_contrib);
    free(s);
}

/* rasterizer_impl.cu:35-50 */
static uint32_t getHigherMsb(uint32_t n) {
    uint32_t msb = sizeof(n) * 4;
    uint32_t step = msb;
    while (step > 1) {
        step /= 2;
        if (n >> msb) msb += step; else msb -= step;
    }
    if (n >> msb) msb++;
    return msb;
}

typedef struct { uint64_t key; uint32_t upos; uint32_t val; } kv_t;
static int kv_cmp(const void *a, const void *b) {
    const kv_t *x = (const kv_t *)a, *y = (const kv_t *)b;
    if (x->key != y->key) return x->key < y->key ? -1 : 1;
    return x->upos < y->upos ? -1 : (x->upos > y->upos);
}

/* ---------------------------------------------------------------------------------------------- */
/* Rasterizer::markVisible (rasterizer_impl.cu:54-66,141-153) */
void gs4d_oracle_mark_visible(int P, const float *means3D, const float *view, const float *proj, uint8_t *present) {
#pragma omp parallel for schedule(static)
    for (int i = 0; i < P; i++) {
        f3 pv;
        present[i] = (uint8_t)in_frustum(i, means3D, view, proj, &pv);
    }
}

/* Rasterizer::forward (rasterizer_impl.cu:198-339).  Returns the state (owned by the caller, free
 * with gs4d_oracle_free) and writes out_color (3,H,W), out_depth (1,H,W), radii (P).  *status is
 * 0 on success, 1 on a prefiltered-contract violation (auxiliary.h:156-160). */
gs4d_oracle_state *gs4d_oracle_forward(int P, int D, int M, const float *background, int width, int height,
                                       const float *means3D, const float *shs, const float *colors_precomp,
                                       const float *opacities, const float *scales, float scale_modifier,
                                       const float *rotations, const float *cov3D_precomp, const float *viewmatrix,
                                       const float *projmatrix, const float *cam_pos, float tan_fovx,
                                       float tan_fovy, int prefiltered, float *out_color, float *out_depth,
                                       int *radii_out, int *num_rendered, int *status) {
    gs4d_oracle_state *s = (gs4d_oracle_state *)calloc(1, sizeof(gs4d_oracle_state));
    const int W = width, H = height;
    s->P = P; s->D = D; s->M = M; s->W = W; s->H = H;
    s->gx = (W + BLOCK_X - 1) / BLOCK_X;
    s->gy = (H + BLOCK_Y - 1) / BLOCK_Y;
    const int gx = s->gx, gy = s->gy, T = gx * gy;
    const float focal_y = height / (2.0f * tan_fovy); /* rasterizer_impl.cu:223-224 */
    const float focal_x = width / (2.0f * tan_fovx);
    *status = 0;

    size_t Pz = (size_t)(P > 0 ? P : 1);
    s->depths = (float *)calloc(Pz, 4);
    s->means2D = (float *)calloc(Pz * 2, 4);
    s->cov3D = (float *)calloc(Pz * 6, 4);
    s->conic_opacity = (float *)calloc(Pz * 4, 4);
    s->rgb = (float *)calloc(Pz * 3, 4);
    s->clamped = (uint8_t *)calloc(Pz, 1);
    s->radii = (int *)calloc(Pz, 4);
    s->tiles_touched = (uint32_t *)calloc(Pz, 4);
    s->point_offsets = (uint32_t *)calloc(Pz, 4);
    s->ranges = (uint32_t *)calloc((size_t)T * 2, 4);
    s->final_T = (float *)calloc((size_t)W * H, 4);
    s->n_contrib = (uint32_t *)calloc((size_t)W * H, 4);

    int violation = 0;
    /* K1: preprocessCUDA (forward.cu:155-256) */
#pragma omp parallel for schedule(static) reduction(| : violation)
    for (int idx = 0; idx < P; idx++) {
        s->radii[idx] = 0;
        s->tiles_touched[idx] = 0;
        f3 p_view;
        if (!in_frustum(idx, means3D, viewmatrix, projmatrix, &p_view)) {
            if (prefiltered) violation = 1;
            continue;
        }
        f3 p_orig = {means3D[3 * idx], means3D[3 * idx + 1], means3D[3 * idx + 2]};
        f4 p_hom = transformPoint4x4(p_orig, projmatrix);
        float p_w = 1.0f / (p_hom.w + 0.0000001f);
        float p_proj_x = p_hom.x * p_w, p_proj_y = p_hom.y * p_w;
        const float *cov3D;
        if (cov3D_precomp) {
            cov3D = cov3D_precomp + (size_t)idx * 6;
        } else {
            cov3d_forward(scales + (size_t)idx * 3, scale_modifier, rotations + (size_t)idx * 4, s->cov3D + (size_t)idx * 6);
            cov3D = s->cov3D + (size_t)idx * 6;
        }
        float cov[3];
        cov2d_forward(p_orig, focal_x, focal_y, tan_fovx, tan_fovy, cov3D, viewmatrix, cov);
        float det = (cov[0] * cov[2] - cov[1] * cov[1]);
        if (det == 0.0f) continue;
        float det_inv = 1.f / det;
        float conic[3] = {cov[2] * det_inv, -cov[1] * det_inv, cov[0] * det_inv};
        float mid = 0.5f * (cov[0] + cov[2]);
        float lambda1 = mid + sqrtf(fmaxf_(0.1f, mid * mid - det));
        float lambda2 = mid - sqrtf(fmaxf_(0.1f, mid * mid - det));
        float my_radius = ceilf(3.f * sqrtf(fmaxf_(lambda1, lambda2)));
        float px = ndc2Pix(p_proj_x, W), py = ndc2Pix(p_proj_y, H);
        int r0x, r0y, r1x, r1y;
        getRect(px, py, (int)my_radius, gx, gy, &r0x, &r0y, &r1x, &r1y);
        if ((r1x - r0x) * (r1y - r0y) == 0) continue;
        if (!colors_precomp) sh_forward(idx, D, M, means3D, cam_pos, shs, s->clamped, s->rgb + (size_t)idx * 3);
        s->depths[idx] = p_view.z;
        s->radii[idx] = (int)my_radius;
        s->means2D[2 * idx] = px;
        s->means2D[2 * idx + 1] = py;
        s->conic_opacity[4 * idx + 0] = conic[0];
        s->conic_opacity[4 * idx + 1] = conic[1];
        s->conic_opacity[4 * idx + 2] = conic[2];
        s->conic_opacity[4 * idx + 3] = opacities[idx];
        s->tiles_touched[idx] = (uint32_t)((r1y - r0y) * (r1x - r0x));
    }
    if (violation) *status = 1;

    /* K2: InclusiveSum (rasterizer_impl.cu:278); H1 (:282) */
    uint32_t acc = 0;
    for (int i = 0; i < P; i++) { acc += s->tiles_touched[i]; s->point_offsets[i] = acc; }
    const int L = P > 0 ? (int)acc : 0;
    s->L = L;
    *num_rendered = L;

    /* K3: duplicateWithKeys (rasterizer_impl.cu:70-111) */
    kv_t *kv = (kv_t *)malloc(sizeof(kv_t) * (size_t)(L > 0 ? L : 1));
#pragma omp parallel for schedule(dynamic, 256)
    for (int idx = 0; idx < P; idx++) {
        if (s->radii[idx] > 0) {
            uint32_t off = idx == 0 ? 0 : s->point_offsets[idx - 1];
            int r0x, r0y, r1x, r1y;
            getRect(s->means2D[2 * idx], s->means2D[2 * idx + 1], s->radii[idx], gx, gy, &r0x, &r0y, &r1x, &r1y);
            uint32_t dbits;
            memcpy(&dbits, &s->depths[idx], 4);
            for (int y = r0y; y < r1y; y++)
                for (int x = r0x; x < r1x; x++) {
                    uint64_t key = (uint64_t)(uint32_t)(y * gx + x);
                    key <<= 32;
                    key |= dbits;
                    kv[off].key = key;
                    kv[off].upos = off;
                    kv[off].val = (uint32_t)idx;
                    off++;
                }
        }
    }
    /* K4: stable radix sort on bits [0, 32+msb(T)) (rasterizer_impl.cu:301-309).  All keys are
     * below 2^(32+msb(T)), so sorting the full key is the same permutation. */
    (void)getHigherMsb;
    qsort(kv, (size_t)L, sizeof(kv_t), kv_cmp);
    s->keys = (uint64_t *)malloc(8 * (size_t)(L > 0 ? L : 1));
    s->point_list = (uint32_t *)malloc(4 * (size_t)(L > 0 ? L : 1));
    s->sorted_upos = (uint32_t *)malloc(4 * (size_t)(L > 0 ? L : 1));
    for (int i = 0; i < L; i++) { s->keys[i] = kv[i].key; s->point_list[i] = kv[i].val; s->sorted_upos[i] = kv[i].upos; }
    free(kv);

    /* H2 + K5: identifyTileRanges (rasterizer_impl.cu:116-138,311-318) */
    for (int idx = 0; idx < L; idx++) {
        uint32_t cur = (uint32_t)(s->keys[idx] >> 32);
        if (idx == 0) s->ranges[2 * cur] = 0;
        else {
            uint32_t prev = (uint32_t)(s->keys[idx - 1] >> 32);
            if (cur != prev) { s->ranges[2 * prev + 1] = (uint32_t)idx; s->ranges[2 * cur] = (uint32_t)idx; }
        }
        if (idx == L - 1) s->ranges[2 * cur + 1] = (uint32_t)L;
    }

    /* K6: renderCUDA forward (forward.cu:261-379) */
    const float *features = colors_precomp ? colors_precomp : s->rgb;
#pragma omp parallel for schedule(dynamic, 1)
    for (int tile = 0; tile < T; tile++) {
        const int bx = tile % gx, by = tile / gx;
        const uint32_t rs = s->ranges[2 * tile], re = s->ranges[2 * tile + 1];
        for (int ty = 0; ty < BLOCK_Y; ty++)
            for (int tx = 0; tx < BLOCK_X; tx++) {
                const int pxi = bx * BLOCK_X + tx, pyi = by * BLOCK_Y + ty;
                if (!(pxi < W && pyi < H)) continue;
                const float pfx = (float)pxi, pfy = (float)pyi;
                float Tr = 1.0f, C[NCH] = {0, 0, 0}, Dp = 0;
                uint32_t contributor = 0, last_contributor = 0;
                for (uint32_t k = rs; k < re; k++) {
                    contributor++;
                    const uint32_t g = s->point_list[k];
                    const float dx = s->means2D[2 * g] - pfx, dy = s->means2D[2 * g + 1] - pfy;
                    const float *co = s->conic_opacity + 4 * (size_t)g;
                    float power = -0.5f * (co[0] * dx * dx + co[2] * dy * dy) - co[1] * dx * dy;
                    if (power > 0.0f) continue;
                    float alpha = fminf_(0.99f, co[3] * expf(power));
                    if (alpha < 1.0f / 255.0f) continue;
                    float test_T = Tr * (1 - alpha);
                    if (test_T < 0.0001f) break; /* done = true: no later Gaussian is considered */
                    for (int ch = 0; ch < NCH; ch++) C[ch] += features[(size_t)g * NCH + ch] * alpha * Tr;
                    Dp += s->depths[g] * alpha * Tr;
                    Tr = test_T;
                    last_contributor = contributor;
                }
                const size_t pix = (size_t)W * pyi + pxi;
                s->final_T[pix] = Tr;
                s->n_contrib[pix] = last_contributor;
                for (int ch = 0; ch < NCH; ch++) out_color[(size_t)ch * H * W + pix] = C[ch] + Tr * background[ch];
                out_depth[pix] = Dp;
            }
    }
    if (radii_out) memcpy(radii_out, s->radii, sizeof(int) * (size_t)P);
    return s;
}

/* Near-threshold flags for the parity tests.  The blend's two discrete decisions, alpha >= 1/255
 * (forward.cu:346-348, backward.cu:486-490) and T(1 - alpha) >= 1e-4 (forward.cu:350-354), flip
 * between two correct float implementations when their operand lies within rounding of the
 * threshold.  This replays the K6 walk of every pixel and flags:
 *   pix_flag bit 0   some splat before the pixel's termination has |255 alpha - 1| within its near_alpha band
 *   pix_flag bit 1   some blended splat has |test_T / 1e-4 - 1| <= band_T (termination may flip)
 *   gauss_flag bit 0 the Gaussian is such a near-1/255 splat at some pixel
 *   gauss_flag bit 1 the Gaussian is such a near-termination splat at some pixel
 * A flip moves the flipping splat's own term of that pixel by O(1) of the term; every other splat of
 * the pixel moves by at most alpha_flip * T_flip (<= 1/255 resp. ~1e-2) of one pixel's term, far below
 * the gradient tolerance, and an implementation that walks past a flipped termination adds terms of
 * T < 1e-4.  Every element outside the flagged sets must agree to the north star's tolerance; the flagged ones
 * are bounded by the size a single flip can have.  Returns the number of flagged pixels. */
int gs4d_oracle_flip_flags(const gs4d_oracle_state *s, float band_alpha, float band_T, uint8_t *pix_flag,
                           uint8_t *gauss_flag) {
    const int W = s->W, H = s->H, gx = s->gx, T = s->gx * s->gy;
    const float a_thr = 1.0f / 255.0f;
    int nflag = 0;
    memset(gauss_flag, 0, (size_t)(s->P > 0 ? s->P : 0));
#pragma omp parallel for schedule(dynamic, 1) reduction(+ : nflag)
    for (int tile = 0; tile < T; tile++) {
        const int bx = tile % gx, by = tile / gx;
        const uint32_t rs = s->ranges[2 * tile], re = s->ranges[2 * tile + 1];
        for (int ty = 0; ty < BLOCK_Y; ty++)
            for (int tx = 0; tx < BLOCK_X; tx++) {
                const int pxi = bx * BLOCK_X + tx, pyi = by * BLOCK_Y + ty;
                if (!(pxi < W && pyi < H)) continue;
                const float pfx = (float)pxi, pfy = (float)pyi;
                float Tr = 1.0f;
                int done = 0;
                uint8_t f = 0;
                for (uint32_t k = rs; k < re && !done; k++) {
                    const uint32_t g = s->point_list[k];
                    const float dx = s->means2D[2 * g] - pfx, dy = s->means2D[2 * g + 1] - pfy;
                    const float *co = s->conic_opacity + 4 * (size_t)g;
                    float power = -0.5f * (co[0] * dx * dx + co[2] * dy * dy) - co[1] * dx * dy;
                    if (power > 0.0f) continue;
                    float alpha = fminf_(0.99f, co[3] * expf(power));
                    if (near_alpha(alpha, co, dx, dy, band_alpha)) {
                        f |= 1;
                        __atomic_fetch_or(&gauss_flag[g], (uint8_t)1, __ATOMIC_RELAXED);
                    }
                    if (alpha < a_thr) continue;
                    float test_T = Tr * (1 - alpha);
                    if (fabsf(test_T * 1e4f - 1.0f) <= band_T) {
                        f |= 2;
                        __atomic_fetch_or(&gauss_flag[g], (uint8_t)2, __ATOMIC_RELAXED);
                    }
                    if (test_T < 0.0001f) done = 1;
                    else Tr = test_T;
                }
                pix_flag[(size_t)W * pyi + pxi] = f;
                nflag += f != 0;
            }
    }
    return nflag;
}

/* ---------------------------------------------------------------------------------------------- */
/* backward.cu:20-139 */
static void sh_backward(int idx, int deg, int max_coeffs, const float *means, const float *campos, const float *shs,
                        const uint8_t *clamped, const float *dL_dcolor, float *dL_dmeans, float *dL_dshs) {
    float pos[3] = {means[3 * idx], means[3 * idx + 1], means[3 * idx + 2]};
    float dir_orig[3] = {pos[0] - campos[0], pos[1] - campos[1], pos[2] - campos[2]};
    float len = sqrtf(dot3(dir_orig, dir_orig));
    float dir[3] = {dir_orig[0] / len, dir_orig[1] / len, dir_orig[2] / len};
    const float *sh = shs + (size_t)idx * max_coeffs * 3;
    float dRGB[3];
    for (int c = 0; c < 3; c++) dRGB[c] = dL_dcolor[3 * idx + c] * (((clamped[idx] >> c) & 1) ? 0.f : 1.f);
    float dx[3] = {0, 0, 0}, dy[3] = {0, 0, 0}, dz[3] = {0, 0, 0};
    float x = dir[0], y = dir[1], z = dir[2];
    float *dsh = dL_dshs + (size_t)idx * max_coeffs * 3;
#define SH(i, c) sh[3 * (i) + (c)]
#define DSH(i, val) for (int c = 0; c < 3; c++) dsh[3 * (i) + c] = (val) * dRGB[c]
    DSH(0, SH_C0);
    if (deg > 0) {
        float d1 = -SH_C1 * y, d2 = SH_C1 * z, d3 = -SH_C1 * x;
        DSH(1, d1); DSH(2, d2); DSH(3, d3);
        for (int c = 0; c < 3; c++) {
            dx[c] = -SH_C1 * SH(3, c);
            dy[c] = -SH_C1 * SH(1, c);
            dz[c] = SH_C1 * SH(2, c);
        }
        if (deg > 1) {
            float xx = x * x, yy = y * y, zz = z * z;
            float xy = x * y, yz = y * z, xz = x * z;
            float d4 = SH_C2[0] * xy, d5 = SH_C2[1] * yz, d6 = SH_C2[2] * (2.f * zz - xx - yy), d7 = SH_C2[3] * xz,
                  d8 = SH_C2[4] * (xx - yy);
            DSH(4, d4); DSH(5, d5); DSH(6, d6); DSH(7, d7); DSH(8, d8);
            for (int c = 0; c < 3; c++) {
                dx[c] += SH_C2[0] * y * SH(4, c) + SH_C2[2] * 2.f * -x * SH(6, c) + SH_C2[3] * z * SH(7, c) +
                         SH_C2[4] * 2.f * x * SH(8, c);
                dy[c] += SH_C2[0] * x * SH(4, c) + SH_C2[1] * z * SH(5, c) + SH_C2[2] * 2.f * -y * SH(6, c) +
                         SH_C2[4] * 2.f * -y * SH(8, c);
                dz[c] += SH_C2[1] * y * SH(5, c) + SH_C2[2] * 2.f * 2.f * z * SH(6, c) + SH_C2[3] * x * SH(7, c);
            }
            if (deg > 2) {
                float d9 = SH_C3[0] * y * (3.f * xx - yy), d10 = SH_C3[1] * xy * z,
                      d11 = SH_C3[2] * y * (4.f * zz - xx - yy), d12 = SH_C3[3] * z * (2.f * zz - 3.f * xx - 3.f * yy),
                      d13 = SH_C3[4] * x * (4.f * zz - xx - yy), d14 = SH_C3[5] * z * (xx - yy),
                      d15 = SH_C3[6] * x * (xx - 3.f * yy);
                DSH(9, d9); DSH(10, d10); DSH(11, d11); DSH(12, d12); DSH(13, d13); DSH(14, d14); DSH(15, d15);
                for (int c = 0; c < 3; c++) {
                    dx[c] += (SH_C3[0] * SH(9, c) * 3.f * 2.f * xy + SH_C3[1] * SH(10, c) * yz +
                              SH_C3[2] * SH(11, c) * -2.f * xy + SH_C3[3] * SH(12, c) * -3.f * 2.f * xz +
                              SH_C3[4] * SH(13, c) * (-3.f * xx + 4.f * zz - yy) + SH_C3[5] * SH(14, c) * 2.f * xz +
                              SH_C3[6] * SH(15, c) * 3.f * (xx - yy));
                    dy[c] += (SH_C3[0] * SH(9, c) * 3.f * (xx - yy) + SH_C3[1] * SH(10, c) * xz +
                              SH_C3[2] * SH(11, c) * (-3.f * yy + 4.f * zz - xx) +
                              SH_C3[3] * SH(12, c) * -3.f * 2.f * yz + SH_C3[4] * SH(13, c) * -2.f * xy +
                              SH_C3[5] * SH(14, c) * -2.f * yz + SH_C3[6] * SH(15, c) * -3.f * 2.f * xy);
                    dz[c] += (SH_C3[1] * SH(10, c) * xy + SH_C3[2] * SH(11, c) * 4.f * 2.f * yz +
                              SH_C3[3] * SH(12, c) * 3.f * (2.f * zz - xx - yy) + SH_C3[4] * SH(13, c) * 4.f * 2.f * xz +
                              SH_C3[5] * SH(14, c) * (xx - yy));
                }
            }
        }
    }
#undef SH
#undef DSH
    f3 dL_ddir = {dot3(dx, dRGB), dot3(dy, dRGB), dot3(dz, dRGB)};
    f3 v = {dir_orig[0], dir_orig[1], dir_orig[2]};
    f3 dm = dnormvdv(v, dL_ddir);
    dL_dmeans[3 * idx + 0] += dm.x;
    dL_dmeans[3 * idx + 1] += dm.y;
    dL_dmeans[3 * idx + 2] += dm.z;
}

/* backward.cu:278-341 */
static void cov3d_backward(int idx, const float *scale, float mod, const float *rot, const float *dL_dcov3Ds,
                           float *dL_dscales, float *dL_drots) {
    float r = rot[0], x = rot[1], y = rot[2], z = rot[3];
    mat3 R = mat3_cols(1.f - 2.f * (y * y + z * z), 2.f * (x * y - r * z), 2.f * (x * z + r * y),
                       2.f * (x * y + r * z), 1.f - 2.f * (x * x + z * z), 2.f * (y * z - r * x),
                       2.f * (x * z - r * y), 2.f * (y * z + r * x), 1.f - 2.f * (x * x + y * y));
    mat3 S = mat3_cols(1, 0, 0, 0, 1, 0, 0, 0, 1);
    float s[3] = {mod * scale[0], mod * scale[1], mod * scale[2]};
    S.m[0][0] = s[0]; S.m[1][1] = s[1]; S.m[2][2] = s[2];
    mat3 M = mat3_mul(&S, &R);
    const float *dc = dL_dcov3Ds + 6 * (size_t)idx;
    mat3 dSigma = mat3_cols(dc[0], 0.5f * dc[1], 0.5f * dc[2], 0.5f * dc[1], dc[3], 0.5f * dc[4], 0.5f * dc[2],
                            0.5f * dc[4], dc[5]);
    mat3 M2;
    for (int c = 0; c < 3; c++)
        for (int rr = 0; rr < 3; rr++) M2.m[c][rr] = 2.0f * M.m[c][rr];
    mat3 dM = mat3_mul(&M2, &dSigma);
    mat3 Rt = mat3_T(&R), dMt = mat3_T(&dM);
    dL_dscales[3 * idx + 0] = dot3(Rt.m[0], dMt.m[0]);
    dL_dscales[3 * idx + 1] = dot3(Rt.m[1], dMt.m[1]);
    dL_dscales[3 * idx + 2] = dot3(Rt.m[2], dMt.m[2]);
    for (int i = 0; i < 3; i++) { dMt.m[0][i] *= s[0]; dMt.m[1][i] *= s[1]; dMt.m[2][i] *= s[2]; }
    float (*d)[3] = dMt.m;
    float q0 = 2 * z * (d[0][1] - d[1][0]) + 2 * y * (d[2][0] - d[0][2]) + 2 * x * (d[1][2] - d[2][1]);
    float q1 = 2 * y * (d[1][0] + d[0][1]) + 2 * z * (d[2][0] + d[0][2]) + 2 * r * (d[1][2] - d[2][1]) -
               4 * x * (d[2][2] + d[1][1]);
    float q2 = 2 * x * (d[1][0] + d[0][1]) + 2 * r * (d[2][0] - d[0][2]) + 2 * z * (d[1][2] + d[2][1]) -
               4 * y * (d[2][2] + d[0][0]);
    float q3 = 2 * r * (d[0][1] - d[1][0]) + 2 * x * (d[2][0] + d[0][2]) + 2 * y * (d[1][2] + d[2][1]) -
               4 * z * (d[1][1] + d[0][0]);
    dL_drots[4 * idx + 0] = q0; dL_drots[4 * idx + 1] = q1; dL_drots[4 * idx + 2] = q2; dL_drots[4 * idx + 3] = q3;
}

/* One pixel of K7 (renderCUDA backward, backward.cu:399-557): the reverse walk over the tile list
 * [rs, re) from T_final / last_contributor, adding each pair's 9 terms (dL_dmean2D x/y, dL_dconic
 * x/y/w, dL_dopacity, dL_dcolor rgb) in double to cb[(k - cb_off) * 9 + q].  flip_kind 1 inverts the
 * alpha test (backward.cu:486-490) of list position flip_k: the walk the near-threshold bounds replay
 * for a blend that took the other side of 1/255 (termination is not tested by the backward; its flip
 * enters through T_final and last_contributor). */
#define NO_FLIP 0xffffffffu
static void pixel_backward(const gs4d_oracle_state *s, const float *color_ptr, const float *background,
                           const float *dL_dpixel, uint32_t rs, uint32_t re, float pfx, float pfy, float T_final,
                           uint32_t last_contributor, uint32_t flip_k, int flip_kind, double *cb_base, uint32_t cb_off) {
    const float ddelx_dx = 0.5f * s->W, ddely_dy = 0.5f * s->H; /* backward.cu:460-461 (0.5 * W is exact) */
    float Tr = T_final;
    float accum_rec[NCH] = {0, 0, 0}, last_color[NCH] = {0, 0, 0};
    float last_alpha = 0;
    float bg_dot_dpixel = 0;
    for (int i = 0; i < NCH; i++) bg_dot_dpixel += background[i] * dL_dpixel[i];
    for (uint32_t k = re; k-- > rs;) {
        const uint32_t contributor = k - rs; /* 0-based position in the tile list */
        if (contributor >= last_contributor) continue;
        const uint32_t g = s->point_list[k];
        const float dx = s->means2D[2 * g] - pfx, dy = s->means2D[2 * g + 1] - pfy;
        const float *co = s->conic_opacity + 4 * (size_t)g;
        const float power = -0.5f * (co[0] * dx * dx + co[2] * dy * dy) - co[1] * dx * dy;
        if (power > 0.0f) continue;
        const float G = expf(power);
        const float alpha = fminf_(0.99f, co[3] * G);
        int pass = alpha >= 1.0f / 255.0f;
        if (k == flip_k && flip_kind == 1) pass = !pass;
        if (!pass) continue;
        Tr = Tr / (1.f - alpha);
        const float dchannel_dcolor = alpha * Tr;
        float dL_dalpha = 0.0f;
        double *cb = cb_base + (size_t)(k - cb_off) * 9;
        for (int ch = 0; ch < NCH; ch++) {
            const float c = color_ptr[(size_t)g * NCH + ch];
            accum_rec[ch] = last_alpha * last_color[ch] + (1.f - last_alpha) * accum_rec[ch];
            last_color[ch] = c;
            const float dL_dchannel = dL_dpixel[ch];
            dL_dalpha += (c - accum_rec[ch]) * dL_dchannel;
            cb[6 + ch] += (double)(dchannel_dcolor * dL_dchannel);
        }
        dL_dalpha *= Tr;
        last_alpha = alpha;
        dL_dalpha += (-T_final / (1.f - alpha)) * bg_dot_dpixel;
        const float dL_dG = co[3] * dL_dalpha;
        const float gdx = G * dx, gdy = G * dy;
        const float dG_ddelx = -gdx * co[0] - gdy * co[1];
        const float dG_ddely = -gdy * co[2] - gdx * co[1];
        cb[0] += (double)(dL_dG * dG_ddelx * ddelx_dx);
        cb[1] += (double)(dL_dG * dG_ddely * ddely_dy);
        cb[2] += (double)(-0.5f * gdx * dx * dL_dG);
        cb[3] += (double)(-0.5f * gdx * dy * dL_dG);
        cb[4] += (double)(-0.5f * gdy * dy * dL_dG);
        cb[5] += (double)(G * dL_dalpha);
    }
}

void gs4d_oracle_backward_tail(const gs4d_oracle_state *s, const float *means3D, const float *shs, const float *scales,
                               float scale_modifier, const float *rotations, const float *cov3D_precomp,
                               const float *viewmatrix, const float *projmatrix, const float *campos, float tan_fovx,
                               float tan_fovy, const int *radii_in, const float *dL_dmean2D, const float *dL_dconic,
                               const float *dL_dcolor, float *dL_dmean3D, float *dL_dcov3D, float *dL_dsh,
                               float *dL_dscale, float *dL_drot);

/* Rasterizer::backward (rasterizer_impl.cu:343-437).  Output arrays must be zero-initialised by
 * the caller, exactly like RasterizeGaussiansBackwardCUDA (rasterize_points.cu:153-161).
 * Layouts: dL_dmean2D (P,3), dL_dconic (P,4), dL_dopacity (P), dL_dcolor (P,3), dL_dmean3D (P,3),
 * dL_dcov3D (P,6), dL_dsh (P,M,3), dL_dscale (P,3), dL_drot (P,4). */
void gs4d_oracle_backward(const gs4d_oracle_state *s, const float *background, const float *means3D,
                          const float *shs, const float *colors_precomp, const float *scales, float scale_modifier,
                          const float *rotations, const float *cov3D_precomp, const float *viewmatrix,
                          const float *projmatrix, const float *campos, float tan_fovx, float tan_fovy,
                          const int *radii_in, const float *dL_dpix, float *dL_dmean2D, float *dL_dconic,
                          float *dL_dopacity, float *dL_dcolor, float *dL_dmean3D, float *dL_dcov3D, float *dL_dsh,
                          float *dL_dscale, float *dL_drot) {
    const int P = s->P, W = s->W, H = s->H, gx = s->gx, gy = s->gy, L = s->L;
    const int T = gx * gy;
    const float *color_ptr = colors_precomp ? colors_precomp : s->rgb;

    /* K7: renderCUDA backward (backward.cu:399-557).  Each (tile, Gaussian) pair's contributions
     * are summed per tile in double, stored per sorted instance, then reduced per Gaussian. */
    enum { NG = 9 };
    double *contrib = (double *)calloc((size_t)(L > 0 ? L : 1) * NG, sizeof(double));
#pragma omp parallel for schedule(dynamic, 1)
    for (int tile = 0; tile < T; tile++) {
        const int bx = tile % gx, by = tile / gx;
        const uint32_t rs = s->ranges[2 * tile], re = s->ranges[2 * tile + 1];
        if (re <= rs) continue;
        for (int ty = 0; ty < BLOCK_Y; ty++)
            for (int tx = 0; tx < BLOCK_X; tx++) {
                const int pxi = bx * BLOCK_X + tx, pyi = by * BLOCK_Y + ty;
                if (!(pxi < W && pyi < H)) continue;
                const size_t pix = (size_t)W * pyi + pxi;
                float dL_dpixel[NCH];
                for (int i = 0; i < NCH; i++) dL_dpixel[i] = dL_dpix[(size_t)i * H * W + pix];
                pixel_backward(s, color_ptr, background, dL_dpixel, rs, re, (float)pxi, (float)pyi, s->final_T[pix],
                               s->n_contrib[pix], NO_FLIP, 0, contrib, 0);
            }
    }
    /* per-Gaussian reduction in unsorted-instance order (deterministic) */
    uint32_t *inv = (uint32_t *)malloc(4 * (size_t)(L > 0 ? L : 1));
    for (int k = 0; k < L; k++) inv[s->sorted_upos[k]] = (uint32_t)k;
#pragma omp parallel for schedule(static)
    for (int g = 0; g < P; g++) {
        if (!(s->radii[g] > 0)) continue;
        uint32_t b = g == 0 ? 0 : s->point_offsets[g - 1], e = s->point_offsets[g];
        double acc[NG] = {0};
        for (uint32_t u = b; u < e; u++) {
            const double *cb = contrib + (size_t)inv[u] * NG;
            for (int q = 0; q < NG; q++) acc[q] += cb[q];
        }
        dL_dmean2D[3 * g + 0] = (float)acc[0];
        dL_dmean2D[3 * g + 1] = (float)acc[1];
        dL_dconic[4 * g + 0] = (float)acc[2];
        dL_dconic[4 * g + 1] = (float)acc[3];
        dL_dconic[4 * g + 3] = (float)acc[4];
        dL_dopacity[g] = (float)acc[5];
        for (int ch = 0; ch < NCH; ch++) dL_dcolor[3 * g + ch] = (float)acc[6 + ch];
    }
    free(inv);
    free(contrib);

    gs4d_oracle_backward_tail(s, means3D, shs, scales, scale_modifier, rotations, cov3D_precomp, viewmatrix,
                              projmatrix, campos, tan_fovx, tan_fovy, radii_in, dL_dmean2D, dL_dconic, dL_dcolor,
                              dL_dmean3D, dL_dcov3D, dL_dsh, dL_dscale, dL_drot);
}

/* K8 (computeCov2DCUDA, backward.cu:144-274) + K9 (preprocessCUDA backward, backward.cu:346-396) of every
 * Gaussian from its K7 totals dL_dmean2D (P,3), dL_dconic (P,4) and dL_dcolor (P,3) (dL_dopacity is final
 * after K7).  Outputs as gs4d_oracle_backward's, zero-initialised by the caller.  Linear in the K7 totals
 * for a fixed forward state, which the near-threshold bounds use to carry the K7 terms' intervals to the
 * final gradients. */
void gs4d_oracle_backward_tail(const gs4d_oracle_state *s, const float *means3D, const float *shs, const float *scales,
                               float scale_modifier, const float *rotations, const float *cov3D_precomp,
                               const float *viewmatrix, const float *projmatrix, const float *campos, float tan_fovx,
                               float tan_fovy, const int *radii_in, const float *dL_dmean2D, const float *dL_dconic,
                               const float *dL_dcolor, float *dL_dmean3D, float *dL_dcov3D, float *dL_dsh,
                               float *dL_dscale, float *dL_drot) {
    const int P = s->P, D = s->D, M = s->M, W = s->W, H = s->H;
    const int *radii = radii_in ? radii_in : s->radii;
    const float focal_y = H / (2.0f * tan_fovy);
    const float focal_x = W / (2.0f * tan_fovx);
    const float *cov3Ds = cov3D_precomp ? cov3D_precomp : s->cov3D;
    /* K8: computeCov2DCUDA (backward.cu:144-274) */
#pragma omp parallel for schedule(static)
    for (int idx = 0; idx < P; idx++) {
        if (!(radii[idx] > 0)) continue;
        const float *cov3D = cov3Ds + 6 * (size_t)idx;
        f3 mean = {means3D[3 * idx], means3D[3 * idx + 1], means3D[3 * idx + 2]};
        float dcx = dL_dconic[4 * idx], dcy = dL_dconic[4 * idx + 1], dcz = dL_dconic[4 * idx + 3];
        f3 t = transformPoint4x3(mean, viewmatrix);
        const float limx = 1.3f * tan_fovx, limy = 1.3f * tan_fovy;
        const float txtz = t.x / t.z, tytz = t.y / t.z;
        t.x = fminf_(limx, fmaxf_(-limx, txtz)) * t.z;
        t.y = fminf_(limy, fmaxf_(-limy, tytz)) * t.z;
        const float x_grad_mul = txtz < -limx || txtz > limx ? 0 : 1;
        const float y_grad_mul = tytz < -limy || tytz > limy ? 0 : 1;
        const float h_x = focal_x, h_y = focal_y;
        mat3 J = mat3_cols(h_x / t.z, 0.0f, -(h_x * t.x) / (t.z * t.z), 0.0f, h_y / t.z, -(h_y * t.y) / (t.z * t.z),
                           0, 0, 0);
        const float *v = viewmatrix;
        mat3 Wm = mat3_cols(v[0], v[4], v[8], v[1], v[5], v[9], v[2], v[6], v[10]);
        mat3 Vrk = mat3_cols(cov3D[0], cov3D[1], cov3D[2], cov3D[1], cov3D[3], cov3D[4], cov3D[2], cov3D[4], cov3D[5]);
        mat3 Tm = mat3_mul(&Wm, &J);
        mat3 Tt = mat3_T(&Tm), Vt = mat3_T(&Vrk);
        mat3 A = mat3_mul(&Tt, &Vt);
        mat3 cov2D = mat3_mul(&A, &Tm);
        float a = cov2D.m[0][0] += 0.3f;
        float b = cov2D.m[0][1];
        float c = cov2D.m[1][1] += 0.3f;
        float denom = a * c - b * b;
        float dL_da = 0, dL_db = 0, dL_dc = 0;
        float denom2inv = 1.0f / ((denom * denom) + 0.0000001f);
        float (*Tq)[3] = Tm.m;
        float *dcov = dL_dcov3D + 6 * (size_t)idx;
        if (denom2inv != 0) {
            dL_da = denom2inv * (-c * c * dcx + 2 * b * c * dcy + (denom - a * c) * dcz);
            dL_dc = denom2inv * (-a * a * dcz + 2 * a * b * dcy + (denom - a * c) * dcx);
            dL_db = denom2inv * 2 * (b * c * dcx - (denom + 2 * b * b) * dcy + a * b * dcz);
            dcov[0] = (Tq[0][0] * Tq[0][0] * dL_da + Tq[0][0] * Tq[1][0] * dL_db + Tq[1][0] * Tq[1][0] * dL_dc);
            dcov[3] = (Tq[0][1] * Tq[0][1] * dL_da + Tq[0][1] * Tq[1][1] * dL_db + Tq[1][1] * Tq[1][1] * dL_dc);
            dcov[5] = (Tq[0][2] * Tq[0][2] * dL_da + Tq[0][2] * Tq[1][2] * dL_db + Tq[1][2] * Tq[1][2] * dL_dc);
            dcov[1] = 2 * Tq[0][0] * Tq[0][1] * dL_da + (Tq[0][0] * Tq[1][1] + Tq[0][1] * Tq[1][0]) * dL_db +
                      2 * Tq[1][0] * Tq[1][1] * dL_dc;
            dcov[2] = 2 * Tq[0][0] * Tq[0][2] * dL_da + (Tq[0][0] * Tq[1][2] + Tq[0][2] * Tq[1][0]) * dL_db +
                      2 * Tq[1][0] * Tq[1][2] * dL_dc;
            dcov[4] = 2 * Tq[0][2] * Tq[0][1] * dL_da + (Tq[0][1] * Tq[1][2] + Tq[0][2] * Tq[1][1]) * dL_db +
                      2 * Tq[1][1] * Tq[1][2] * dL_dc;
        } else {
            for (int i = 0; i < 6; i++) dcov[i] = 0;
        }
        float (*Vq)[3] = Vrk.m;
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
        float (*Wq)[3] = Wm.m;
        float dL_dJ00 = Wq[0][0] * dL_dT00 + Wq[0][1] * dL_dT01 + Wq[0][2] * dL_dT02;
        float dL_dJ02 = Wq[2][0] * dL_dT00 + Wq[2][1] * dL_dT01 + Wq[2][2] * dL_dT02;
        float dL_dJ11 = Wq[1][0] * dL_dT10 + Wq[1][1] * dL_dT11 + Wq[1][2] * dL_dT12;
        float dL_dJ12 = Wq[2][0] * dL_dT10 + Wq[2][1] * dL_dT11 + Wq[2][2] * dL_dT12;
        float tz = 1.f / t.z, tz2 = tz * tz, tz3 = tz2 * tz;
        float dL_dtx = x_grad_mul * -h_x * tz2 * dL_dJ02;
        float dL_dty = y_grad_mul * -h_y * tz2 * dL_dJ12;
        float dL_dtz = -h_x * tz2 * dL_dJ00 - h_y * tz2 * dL_dJ11 + (2 * h_x * t.x) * tz3 * dL_dJ02 +
                       (2 * h_y * t.y) * tz3 * dL_dJ12;
        f3 dt = {dL_dtx, dL_dty, dL_dtz};
        f3 dm = transformVec4x3Transpose(dt, viewmatrix);
        dL_dmean3D[3 * idx + 0] = dm.x; /* assignment (backward.cu:273) */
        dL_dmean3D[3 * idx + 1] = dm.y;
        dL_dmean3D[3 * idx + 2] = dm.z;
    }

    /* K9: preprocessCUDA backward (backward.cu:346-396) */
#pragma omp parallel for schedule(static)
    for (int idx = 0; idx < P; idx++) {
        if (!(radii[idx] > 0)) continue;
        f3 m = {means3D[3 * idx], means3D[3 * idx + 1], means3D[3 * idx + 2]};
        const float *proj = projmatrix;
        f4 m_hom = transformPoint4x4(m, proj);
        float m_w = 1.0f / (m_hom.w + 0.0000001f);
        float mul1 = (proj[0] * m.x + proj[4] * m.y + proj[8] * m.z + proj[12]) * m_w * m_w;
        float mul2 = (proj[1] * m.x + proj[5] * m.y + proj[9] * m.z + proj[13]) * m_w * m_w;
        float g2x = dL_dmean2D[3 * idx], g2y = dL_dmean2D[3 * idx + 1];
        float dmx = (proj[0] * m_w - proj[3] * mul1) * g2x + (proj[1] * m_w - proj[3] * mul2) * g2y;
        float dmy = (proj[4] * m_w - proj[7] * mul1) * g2x + (proj[5] * m_w - proj[7] * mul2) * g2y;
        float dmz = (proj[8] * m_w - proj[11] * mul1) * g2x + (proj[9] * m_w - proj[11] * mul2) * g2y;
        dL_dmean3D[3 * idx + 0] += dmx;
        dL_dmean3D[3 * idx + 1] += dmy;
        dL_dmean3D[3 * idx + 2] += dmz;
        if (shs) sh_backward(idx, D, M, means3D, campos, shs, s->clamped, dL_dcolor, dL_dmean3D, dL_dsh);
        if (scales)
            cov3d_backward(idx, scales + 3 * (size_t)idx, scale_modifier, rotations + 4 * (size_t)idx, dL_dcov3D,
                           dL_dscale, dL_drot);
    }
}

/* Accessors for the Python test wrapper (ctypes) */
int gs4d_oracle_state_L(const gs4d_oracle_state *s) { return s->L; }
void gs4d_oracle_state_export(const gs4d_oracle_state *s, float *depths, float *means2D, float *conic_opacity,
                              float *rgb, uint8_t *clamped, uint32_t *tiles_touched, uint32_t *point_list,
                              uint32_t *ranges, float *final_T, uint32_t *n_contrib, float *cov3D) {
    const size_t P = (size_t)s->P, L = (size_t)s->L, N = (size_t)s->W * s->H, T = (size_t)s->gx * s->gy;
    if (depths) memcpy(depths, s->depths, 4 * P);
    if (means2D) memcpy(means2D, s->means2D, 8 * P);
    if (conic_opacity) memcpy(conic_opacity, s->conic_opacity, 16 * P);
    if (rgb) memcpy(rgb, s->rgb, 12 * P);
    if (clamped) memcpy(clamped, s->clamped, P);
    if (tiles_touched) memcpy(tiles_touched, s->tiles_touched, 4 * P);
    if (point_list) memcpy(point_list, s->point_list, 4 * L);
    if (ranges) memcpy(ranges, s->ranges, 8 * T);
    if (final_T) memcpy(final_T, s->final_T, 4 * N);
    if (n_contrib) memcpy(n_contrib, s->n_contrib, 4 * N);
    if (cov3D) memcpy(cov3D, s->cov3D, 24 * P);
}

/* Test entry: SH -> RGB of forward.cu:20-71 for every Gaussian (no culling), used to pin the
 * restatement against the reference's own utils/sh_utils.py:eval_sh. */
void gs4d_oracle_sh_forward(int P, int D, int M, const float *means, const float *campos, const float *shs,
                            float *rgb_out, uint8_t *clamped_out) {
    for (int i = 0; i < P; i++) sh_forward(i, D, M, means, campos, shs, clamped_out, rgb_out + 3 * (size_t)i);
}

/* ---------------------------------------------------------------------------------------------- */
/* Near-threshold bounds for the parity tests.
 *
 * The blend's two discrete decisions, alpha >= 1/255 (forward.cu:346-348, backward.cu:486-490) and
 * T(1 - alpha) >= 1e-4 (forward.cu:350-354), can go either way between two correct float
 * implementations when their operand lies within rounding of the threshold.  For every pixel this
 * replays the forward walk, finds those decisions (|255 alpha - 1| within near_alpha's band before the pixel's
 * termination; |T(1 - alpha) / 1e-4 - 1| <= band_T for a splat that passed the alpha test), and for EACH
 * of them replays the pixel's forward and backward with that one decision taken the other way.  The
 * differences bound what a flip can change:
 *   pix_rad[p]      sum over the pixel's near decisions of max_ch |colour(flipped) - colour(oracle)|
 *   depth_rad[p]    the same for the depth
 *   rad9[g * 9 + q] sum over all near decisions of all pixels of |term_q(flipped) - term_q(oracle)| of
 *                   Gaussian g's K7 totals (q: dL_dmean2D x/y, dL_dconic x/y/w, dL_dopacity, dL_dcolor
 *                   rgb), i.e. the flipping splat's own term and the T / accum_rec changes it causes in
 *                   every other splat of the pixel
 * pix_flag / gauss_flag: bit 0 = a near-1/255 decision (at the pixel / of the Gaussian), bit 1 = a
 * near-termination one.  Several near decisions of one pixel are bounded by the sum of their single
 * flips (their joint effect differs from that sum only at second order).  rad9 is linear-mapped to the
 * final gradients by the caller (gs4d_oracle_backward_tail is linear in the K7 totals).
 * Returns the number of flagged pixels. */
typedef struct {
    float T;
    uint32_t n_contrib;
    float C[NCH];
    float D;
} pixwalk_t;

/* forward.cu:309-367 for one pixel, with the decision of list position flip_k inverted (flip_kind 1:
 * the alpha test, 2: the termination test) */
static void pixel_forward(const gs4d_oracle_state *s, const float *features, uint32_t rs, uint32_t re, float pfx,
                          float pfy, uint32_t flip_k, int flip_kind, pixwalk_t *o) {
    float Tr = 1.0f, C[NCH] = {0, 0, 0}, Dp = 0;
    uint32_t contributor = 0, last_contributor = 0;
    for (uint32_t k = rs; k < re; k++) {
        contributor++;
        const uint32_t g = s->point_list[k];
        const float dx = s->means2D[2 * g] - pfx, dy = s->means2D[2 * g + 1] - pfy;
        const float *co = s->conic_opacity + 4 * (size_t)g;
        float power = -0.5f * (co[0] * dx * dx + co[2] * dy * dy) - co[1] * dx * dy;
        if (power > 0.0f) continue;
        float alpha = fminf_(0.99f, co[3] * expf(power));
        int pass = alpha >= 1.0f / 255.0f;
        if (k == flip_k && flip_kind == 1) pass = !pass;
        if (!pass) continue;
        float test_T = Tr * (1 - alpha);
        int term = test_T < 0.0001f;
        if (k == flip_k && flip_kind == 2) term = !term;
        if (term) break;
        for (int ch = 0; ch < NCH; ch++) C[ch] += features[(size_t)g * NCH + ch] * alpha * Tr;
        Dp += s->depths[g] * alpha * Tr;
        Tr = test_T;
        last_contributor = contributor;
    }
    o->T = Tr;
    o->n_contrib = last_contributor;
    for (int ch = 0; ch < NCH; ch++) o->C[ch] = C[ch];
    o->D = Dp;
}

int gs4d_oracle_flip_bounds(const gs4d_oracle_state *s, const float *background, const float *colors_precomp,
                            const float *dL_dpix, float band_alpha, float band_T, uint8_t *pix_flag,
                            uint8_t *gauss_flag, float *pix_rad, float *depth_rad, double *rad9) {
    const int W = s->W, H = s->H, gx = s->gx, T = s->gx * s->gy;
    const float *features = colors_precomp ? colors_precomp : s->rgb;
    const float a_thr = 1.0f / 255.0f;
    int nflag = 0;
    memset(gauss_flag, 0, (size_t)(s->P > 0 ? s->P : 0));
    memset(rad9, 0, sizeof(double) * 9 * (size_t)(s->P > 0 ? s->P : 0));
    memset(pix_rad, 0, sizeof(float) * (size_t)W * H);
    memset(depth_rad, 0, sizeof(float) * (size_t)W * H);
    memset(pix_flag, 0, (size_t)W * H);
#pragma omp parallel for schedule(dynamic, 1) reduction(+ : nflag)
    for (int tile = 0; tile < T; tile++) {
        const int bx = tile % gx, by = tile / gx;
        const uint32_t rs = s->ranges[2 * tile], re = s->ranges[2 * tile + 1];
        if (re <= rs) continue;
        const size_t n = re - rs;
        double *ref9 = NULL, *alt9 = NULL;
        uint32_t *near_k = NULL;
        uint8_t *near_kind = NULL;
        size_t near_cap = 0;
        for (int ty = 0; ty < BLOCK_Y; ty++)
            for (int tx = 0; tx < BLOCK_X; tx++) {
                const int pxi = bx * BLOCK_X + tx, pyi = by * BLOCK_Y + ty;
                if (!(pxi < W && pyi < H)) continue;
                const float pfx = (float)pxi, pfy = (float)pyi;
                const size_t pix = (size_t)W * pyi + pxi;
                /* the near decisions of the oracle's own walk (as gs4d_oracle_flip_flags finds them) */
                size_t nn = 0;
                float Tr = 1.0f;
                uint8_t f = 0;
                for (uint32_t k = rs; k < re; k++) {
                    const uint32_t g = s->point_list[k];
                    const float dx = s->means2D[2 * g] - pfx, dy = s->means2D[2 * g + 1] - pfy;
                    const float *co = s->conic_opacity + 4 * (size_t)g;
                    float power = -0.5f * (co[0] * dx * dx + co[2] * dy * dy) - co[1] * dx * dy;
                    if (power > 0.0f) continue;
                    float alpha = fminf_(0.99f, co[3] * expf(power));
                    int kinds = 0;
                    if (near_alpha(alpha, co, dx, dy, band_alpha)) kinds |= 1;
                    float test_T = Tr * (1 - alpha);
                    if (alpha >= a_thr && fabsf(test_T * 1e4f - 1.0f) <= band_T) kinds |= 2;
                    for (int kind = 1; kind <= 2; kind++) {
                        if (!(kinds & kind)) continue;
                        if (nn == near_cap) {
                            near_cap = near_cap ? 2 * near_cap : 16;
                            near_k = (uint32_t *)realloc(near_k, 4 * near_cap);
                            near_kind = (uint8_t *)realloc(near_kind, near_cap);
                        }
                        near_k[nn] = k;
                        near_kind[nn] = (uint8_t)kind;
                        nn++;
                        f |= (uint8_t)kind;
                        __atomic_fetch_or(&gauss_flag[g], (uint8_t)kind, __ATOMIC_RELAXED);
                    }
                    if (alpha < a_thr) continue;
                    if (test_T < 0.0001f) break;
                    Tr = test_T;
                }
                pix_flag[pix] = f;
                if (!nn) continue;
                nflag++;
                if (!ref9) {
                    ref9 = (double *)malloc(sizeof(double) * 9 * n);
                    alt9 = (double *)malloc(sizeof(double) * 9 * n);
                }
                float dL_dpixel[NCH];
                for (int i = 0; i < NCH; i++) dL_dpixel[i] = dL_dpix[(size_t)i * H * W + pix];
                pixwalk_t pr, pa;
                pixel_forward(s, features, rs, re, pfx, pfy, NO_FLIP, 0, &pr);
                memset(ref9, 0, sizeof(double) * 9 * n);
                pixel_backward(s, features, background, dL_dpixel, rs, re, pfx, pfy, pr.T, pr.n_contrib, NO_FLIP, 0,
                               ref9, rs);
                float prad = 0, drad = 0;
                for (size_t d = 0; d < nn; d++) {
                    pixel_forward(s, features, rs, re, pfx, pfy, near_k[d], near_kind[d], &pa);
                    memset(alt9, 0, sizeof(double) * 9 * n);
                    pixel_backward(s, features, background, dL_dpixel, rs, re, pfx, pfy, pa.T, pa.n_contrib, near_k[d],
                                   near_kind[d], alt9, rs);
                    float cmax = 0;
                    for (int ch = 0; ch < NCH; ch++) {
                        const float a = pa.C[ch] + pa.T * background[ch], b = pr.C[ch] + pr.T * background[ch];
                        cmax = fmaxf_(cmax, fabsf(a - b));
                    }
                    prad += cmax;
                    drad += fabsf(pa.D - pr.D);
                    for (size_t k = 0; k < n; k++) {
                        const double *x = alt9 + 9 * k, *y = ref9 + 9 * k;
                        const uint32_t g = s->point_list[rs + k];
                        for (int q = 0; q < 9; q++) {
                            const double dq = fabs(x[q] - y[q]);
                            if (dq != 0.0) {
#pragma omp atomic
                                rad9[9 * (size_t)g + q] += dq;
                            }
                        }
                    }
                }
                pix_rad[pix] = prad;
                depth_rad[pix] = drad;
            }
        free(ref9);
        free(alt9);
        free(near_k);
        free(near_kind);
    }
    return nflag;
}

/* The (Gaussian, pixel) pairs of the forward walks near one of the blend's thresholds: kind 1, alpha within
 * band of 1/255 (relative; before each pixel's termination); kind 2, a splat passing the alpha test whose
 * T(1 - alpha) lies within band of 1e-4 (relative).  gid / px / py, the oracle's o G = co[3] * expf(power)
 * (alpha before the 0.99 cap) and near_alpha's magnitude factor, for measuring the blend kernels' operands
 * against them.  Writes at most
 * max_n; returns the count found (which may exceed max_n). */
int gs4d_oracle_near_pairs(const gs4d_oracle_state *s, int kind, float band, int max_n, int *gid, int *px, int *py,
                           float *og, float *mag) {
    const int W = s->W, H = s->H, gx = s->gx, T = s->gx * s->gy;
    int count = 0;
#pragma omp parallel for schedule(dynamic, 1)
    for (int tile = 0; tile < T; tile++) {
        const int bx = tile % gx, by = tile / gx;
        const uint32_t rs = s->ranges[2 * tile], re = s->ranges[2 * tile + 1];
        for (int ty = 0; ty < BLOCK_Y; ty++)
            for (int tx = 0; tx < BLOCK_X; tx++) {
                const int pxi = bx * BLOCK_X + tx, pyi = by * BLOCK_Y + ty;
                if (!(pxi < W && pyi < H)) continue;
                const float pfx = (float)pxi, pfy = (float)pyi;
                float Tr = 1.0f;
                for (uint32_t k = rs; k < re; k++) {
                    const uint32_t g = s->point_list[k];
                    const float dx = s->means2D[2 * g] - pfx, dy = s->means2D[2 * g + 1] - pfy;
                    const float *co = s->conic_opacity + 4 * (size_t)g;
                    float power = -0.5f * (co[0] * dx * dx + co[2] * dy * dy) - co[1] * dx * dy;
                    if (power > 0.0f) continue;
                    const float o_g = co[3] * expf(power);
                    float alpha = fminf_(0.99f, o_g);
                    const float test_T = Tr * (1 - alpha);
                    const int near = kind == 1 ? near_alpha(alpha, co, dx, dy, band)
                                               : alpha >= 1.0f / 255.0f && fabsf(test_T * 1e4f - 1.0f) <= band;
                    if (near) {
                        int i;
#pragma omp atomic capture
                        i = count++;
                        if (i < max_n) {
                            gid[i] = (int)g;
                            px[i] = pxi;
                            py[i] = pyi;
                            og[i] = o_g;
                            mag[i] = 1.0f + 0.5f * (fabsf(co[0]) * dx * dx + fabsf(co[2]) * dy * dy) +
                                     fabsf(co[1] * dx * dy);
                        }
                    }
                    if (alpha < 1.0f / 255.0f) continue;
                    if (test_T < 0.0001f) break;
                    Tr = test_T;
                }
            }
    }
    return count;
}
