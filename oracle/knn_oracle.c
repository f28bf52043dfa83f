/*
 * knn_oracle.c -- CPU restatement of simple_knn's distCUDA2 (TEST INFRASTRUCTURE ONLY).
 *
 * Only tests/ may load it (through oracle.py); the product library never links it.  It follows
 * submodules/simple-knn/simple_knn.cu:47-223 step by step, in the reference's order:
 *   SimpleKNN::knn (:187-223): cub Reduce min/max of the points with init {0,0,0} (:193-202), so the
 *   box always contains the origin; coord2Morton (:56-72); stable SortPairs of (code, index)
 *   (:212-215, restated as a comparison sort on (code, index)); boxMinMax over blocks of BOX_SIZE
 *   sorted points (:80-119); boxMeanDist (:149-185) with distBoxPoint (:121-131) and
 *   updateKBest<3> (:133-147).
 * Arithmetic: compiled with -ffp-contract=off, distances as (dx*dx + dy*dy) + dz*dz; nvcc's default
 * FMA contraction may change the last ulp of the CUDA build.  The float -> uint32 conversion of a
 * NaN grid coordinate (degenerate axis, 0/0) is 0, as on the GPU.
 */
#include <float.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define KNN_BOX 1024 /* simple_knn.cu:12 BOX_SIZE */

static uint32_t prep_morton(uint32_t x) { /* simple_knn.cu:47-54 */
    x = (x | (x << 16)) & 0x030000FF;
    x = (x | (x << 8)) & 0x0300F00F;
    x = (x | (x << 4)) & 0x030C30C3;
    x = (x | (x << 2)) & 0x09249249;
    return x;
}
static uint32_t grid_coord(float c, float mn, float mx) {
    float v = ((c - mn) / (mx - mn)) * (float)((1 << 10) - 1);
    return v >= 0.f ? (uint32_t)v : 0u;
}
static float cmin(float a, float b) { return fminf(a, b); } /* CUDA min(float,float) */
static float cmax(float a, float b) { return fmaxf(a, b); }

typedef struct { uint32_t code, idx; } knn_kv;
static int knn_kv_cmp(const void *a, const void *b) {
    const knn_kv *x = (const knn_kv *)a, *y = (const knn_kv *)b;
    if (x->code != y->code) return x->code < y->code ? -1 : 1;
    return x->idx < y->idx ? -1 : (x->idx > y->idx);
}
static float sqd(const float *a, const float *b) {
    float dx = b[0] - a[0], dy = b[1] - a[1], dz = b[2] - a[2];
    return dx * dx + dy * dy + dz * dz;
}
static void update3(float *best, float d) { /* simple_knn.cu:133-147 */
    for (int j = 0; j < 3; j++)
        if (best[j] > d) { float t = best[j]; best[j] = d; d = t; }
}
static float box_dist(const float *mn, const float *mx, const float *p) { /* simple_knn.cu:121-131 */
    float d[3] = {0.f, 0.f, 0.f};
    for (int c = 0; c < 3; c++)
        if (p[c] < mn[c] || p[c] > mx[c]) d[c] = fminf(fabsf(p[c] - mn[c]), fabsf(p[c] - mx[c]));
    return d[0] * d[0] + d[1] * d[1] + d[2] * d[2];
}

void gs4d_oracle_knn(int P, const float *pts, float *mean_dists) {
    if (P <= 0) return;
    float mn[3] = {0.f, 0.f, 0.f}, mx[3] = {0.f, 0.f, 0.f}; /* init {0,0,0} */
    for (int i = 0; i < P; i++)
        for (int c = 0; c < 3; c++) {
            mn[c] = cmin(mn[c], pts[3 * i + c]);
            mx[c] = cmax(mx[c], pts[3 * i + c]);
        }
    knn_kv *kv = (knn_kv *)malloc(sizeof(knn_kv) * (size_t)P);
    for (int i = 0; i < P; i++) {
        uint32_t x = prep_morton(grid_coord(pts[3 * i], mn[0], mx[0]));
        uint32_t y = prep_morton(grid_coord(pts[3 * i + 1], mn[1], mx[1]));
        uint32_t z = prep_morton(grid_coord(pts[3 * i + 2], mn[2], mx[2]));
        kv[i].code = x | (y << 1) | (z << 2);
        kv[i].idx = (uint32_t)i;
    }
    qsort(kv, (size_t)P, sizeof(knn_kv), knn_kv_cmp);
    const int nbox = (P + KNN_BOX - 1) / KNN_BOX;
    float *bmn = (float *)malloc(sizeof(float) * 3 * (size_t)nbox), *bmx = (float *)malloc(sizeof(float) * 3 * (size_t)nbox);
    for (int b = 0; b < nbox; b++) { /* simple_knn.cu:80-119 */
        for (int c = 0; c < 3; c++) { bmn[3 * b + c] = FLT_MAX; bmx[3 * b + c] = -FLT_MAX; }
        for (int i = b * KNN_BOX; i < P && i < (b + 1) * KNN_BOX; i++)
            for (int c = 0; c < 3; c++) {
                bmn[3 * b + c] = cmin(bmn[3 * b + c], pts[3 * kv[i].idx + c]);
                bmx[3 * b + c] = cmax(bmx[3 * b + c], pts[3 * kv[i].idx + c]);
            }
    }
#pragma omp parallel for schedule(dynamic, 256)
    for (int idx = 0; idx < P; idx++) { /* simple_knn.cu:149-185 */
        const float *p = pts + 3 * kv[idx].idx;
        float best[3] = {FLT_MAX, FLT_MAX, FLT_MAX};
        int lo = idx - 3 > 0 ? idx - 3 : 0, hi = idx + 3 < P - 1 ? idx + 3 : P - 1;
        for (int i = lo; i <= hi; i++)
            if (i != idx) update3(best, sqd(p, pts + 3 * kv[i].idx));
        float reject = best[2];
        best[0] = best[1] = best[2] = FLT_MAX;
        for (int b = 0; b < nbox; b++) {
            float d = box_dist(bmn + 3 * b, bmx + 3 * b, p);
            if (d > reject || d > best[2]) continue;
            for (int i = b * KNN_BOX; i < P && i < (b + 1) * KNN_BOX; i++)
                if (i != idx) update3(best, sqd(p, pts + 3 * kv[i].idx));
        }
        mean_dists[kv[idx].idx] = (best[0] + best[1] + best[2]) / 3.0f;
    }
    free(bmn);
    free(bmx);
    free(kv);
}
