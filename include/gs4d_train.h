/*
 * gs4d_train.h -- C ABI of libgs4d's train-step kernels: the rows SURVEY.md §8f lists on either side
 * of the rasterizer (the HexPlane deformation field before it, the loss / densification statistics /
 * optimizer after it).  Each entry point replaces a PyTorch formulation of the reference; the
 * reference file:line it restates is given with it.  Same conventions as gs4d.h: device pointers,
 * fp32, C-contiguous, launches enqueued on `stream`, status 0 = OK, 1 = bad argument, 3 = HIP error.
 */
#ifndef GS4D_TRAIN_H_INCLUDED
#define GS4D_TRAIN_H_INCLUDED

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- L1 loss: utils/loss_utils.py:20-21 l1_loss(x, y) = |x - y|.mean(), and its autograd gradient.
 * forward: *loss = mean |x - y| (fp64 partial sums in a fixed order), sign[i] = sign(x[i] - y[i]);
 * scratch must hold gs4d_l1_scratch_bytes(n) bytes and be all zero on entry (the completion counters and
 * partial slots of the workgroup that finishes last: it sums the partials itself, no second launch); a call
 * leaves it zero again, so a caller zeroes its scratch once and keeps it (one scratch per stream: two calls
 * in flight at once must not share one).  backward: grad[i] = sign[i] * (*dloss) / n. */
size_t gs4d_l1_scratch_bytes(int64_t n);
int gs4d_l1_loss_forward(int64_t n, const float *x, const float *y, int8_t *sign, float *loss, void *scratch,
                         void *stream);
/* Value AND gradient in one pass, for an upstream gradient `dloss` known on the host (a training step's
 * loss.backward() with dloss = 1): grad = sign(x - y) * (dloss * (1 / n)), bitwise what
 * gs4d_l1_loss_forward + gs4d_l1_loss_backward give, without writing and re-reading the signs.  n % 4 == 0 and
 * 16-byte aligned x, y, grad (GS4D_ERR_ARG otherwise). */
int gs4d_l1_loss_grad(int64_t n, const float *x, const float *y, float dloss, float *loss, float *grad, void *scratch,
                      void *stream);
int gs4d_l1_loss_backward(int64_t n, const int8_t *sign, const float *dloss, float *grad, void *stream);

/* ---- the deformation's tail and the activations before the rasterizer, in one pass each way:
 * scene/deformation.py:140-146 (residual adds of the heads' outputs, features = cat(f_dc, f_rest),
 * scene/gaussian_model.py:116-118) and gaussian_renderer/__init__.py:97-99 (exp, normalize, sigmoid):
 *   means = xyz + dx, scales = exp(s + ds), rot = (r + dr) / max(|r + dr|, 1e-12), opac = sigmoid(o + do),
 *   shs[:, 0] = f_dc + dshs[:, 0:3], shs[:, 1:] = f_rest + dshs[:, 3:] (K = 1 + K_rest coefficients).
 * Any delta may be NULL (that head is off: zero).  xyz, s (P, 3), r (P, 4), o (P, 1), f_dc (P, 1, 3),
 * f_rest (P, K-1, 3), dshs (P, 3K).  backward: given the gradients of the five outputs (each may be
 * NULL: zero), writes d xyz, d s, d r, d o, d f_dc and d f_rest (the slices of d shs, whose flat
 * (P, 3K) form is also the gradient of dshs), and the same values again into the deltas' gradients
 * g_dx, g_ds, g_dr, g_do where those are not NULL (separate buffers: autograd hands them to other
 * functions while the bases' gradients may become leaf .grad tensors). */
int gs4d_deform_tail_forward(int P, int K, const float *xyz, const float *s, const float *r, const float *o,
                             const float *f_dc, const float *f_rest, const float *dx, const float *ds, const float *dr,
                             const float *d_o, const float *dshs, float *means, float *scales, float *rot,
                             float *opac, float *shs, void *stream);
int gs4d_deform_tail_backward(int P, int K, const float *scales, const float *r, const float *dr, const float *opac,
                              const float *g_means, const float *g_scales, const float *g_rot, const float *g_opac,
                              const float *g_shs, float *d_xyz, float *d_s, float *d_r, float *d_o, float *d_fdc,
                              float *d_frest, float *g_dx, float *g_ds, float *g_dr, float *g_do, void *stream);

/* ---- split-K partial sums: out[i] = sum over s = 0 .. S-1 (in that order) of parts[s * n + i].  The
 * deformation MLP's weight gradients dW = dY^T X over P ~ 1e5 rows are split-K GEMMs
 * (gs4d_train/deformation.py _splitk_dw) whose per-chunk results this adds in one pass. */
int gs4d_sum_slices(const float *parts, int S, int64_t n, float *out, void *stream);

/* ---- densification statistics: train.py:346-349 and scene/gaussian_model.py:521-523.
 * For every i with visible[i]: max_radii[i] = max(max_radii[i], radii[i]) (skipped when radii is
 * NULL), grad_accum[i] += |viewspace_grad[i, 0:2]|, denom[i] += 1.  viewspace_grad is (P, 3).  visible may
 * be NULL when radii is given: the mask is then radii[i] > 0, train.py:229-232's own definition of it. */
int gs4d_densify_stats(int P, const float *viewspace_grad, const uint8_t *visible, const int *radii, float *grad_accum,
                       float *denom, float *max_radii, void *stream);

/* ---- Adam: torch.optim.Adam(params, lr, betas=(0.9, 0.999), eps=1e-15) as built by
 * scene/gaussian_model.py:165-184, one launch for up to GS4D_ADAM_MAX_TENSORS tensors.  Per element:
 *   m = m + (1 - beta1) (g - m);  v = beta2 v + (1 - beta2) g^2;
 *   p = p + neg_step_size * m / (sqrt(v) / bias_correction2_sqrt + eps)
 * with neg_step_size = -lr / (1 - beta1^step) and bias_correction2_sqrt = sqrt(1 - beta2^step)
 * computed by the caller in double precision (as torch does).  first_chunk of tensor i must be the
 * sum of gs4d_adam_chunks(n) over tensors 0..i-1. */
#define GS4D_ADAM_MAX_TENSORS 48
typedef struct {
    float *param;
    const float *grad;
    float *exp_avg;
    float *exp_avg_sq;
    int64_t n;
    int64_t first_chunk;
    float neg_step_size;
    float bias_correction2_sqrt;
} gs4d_adam_tensor;
typedef struct {
    int count;
    float beta1, one_minus_beta1, beta2, one_minus_beta2, eps;
    gs4d_adam_tensor t[GS4D_ADAM_MAX_TENSORS];
} gs4d_adam_batch;
int64_t gs4d_adam_chunks(int64_t n);
int gs4d_adam_step(const gs4d_adam_batch *batch, void *stream);

/* ---- Row surgery of densification and pruning: scene/gaussian_model.py:316-506 (prune_points,
 * densification_postfix, densify_and_clone, densify_and_split, and the optimizer-state edits they make).
 * One call rebuilds every per-Gaussian tensor (parameters, their Adam moments, statistics, the deformation
 * table) by one ROW PLAN: output row r < K is old row keep[r]; the A appended rows K + j are, per tensor mode:
 * GATHER -- old row append[j] for j < A - given_rows, then given[j - (A - given_rows)] (rows the caller
 * computed, e.g. a split's children's positions); ZERO_NEW -- zero (the new rows' Adam moments).  ZERO makes
 * every output row zero (the statistics the reference resets after densifying; src unused).  A copy is a copy:
 * the result is bitwise the reference's cat / boolean-index sequence, in its row order.  Elements are 1 or 4
 * bytes; rows are `width` elements, contiguous. */
#define GS4D_ROWS_MAX_TENSORS 32
enum { GS4D_ROWS_GATHER = 0, GS4D_ROWS_ZERO_NEW = 1, GS4D_ROWS_ZERO = 2 };
typedef struct {
    const void *src;    /* (P, width) old rows */
    const void *given;  /* (given_rows, width): the last appended rows of a GATHER tensor */
    void *dst;          /* (K + A, width) */
    int64_t width;
    int64_t given_rows; /* 0 <= given_rows <= A */
    int esize;          /* 1 or 4 */
    int mode;
} gs4d_rows_tensor;
typedef struct {
    int count;
    int64_t K, A;
    const int32_t *keep;    /* K old row indices, in output order */
    const int32_t *append;  /* old row indices of the gathered appended rows (A - given_rows of them per tensor) */
    gs4d_rows_tensor t[GS4D_ROWS_MAX_TENSORS];
} gs4d_rows_batch;
int gs4d_rows_assemble(const gs4d_rows_batch *batch, void *stream);

/* ---- HexPlane field: scene/hexplane.py:75-110 interpolate_ms_features (concat_features=True) over the
 * planes of init_grid_param (:50-72), each sampled with F.grid_sample(align_corners=True, bilinear,
 * padding_mode="border") (:22-48).  pts: (N, 4) normalised (x, y, z, t), 16-byte aligned.
 * feat: (N, levels * F) = for each level the product over the 6 coordinate pairs (0,1) (0,2) (0,3)
 * (1,2) (1,3) (2,3) of the pair's bilinear sample.  Plane 6*l + p of level l is a (1, F, H, W)
 * parameter tensor with W = reso[c0], H = reso[c1]; the kernels read a packed channels-last copy
 * of all planes (gs4d_hexplane_pack); the backward writes the plane gradients (every element: no zero
 * fill needed) into a packed buffer that gs4d_hexplane_unpack writes back to (1, F, H, W) gradient
 * tensors.  dpts receives the gradient w.r.t. pts (all 4 columns).  The plane gradients are always bitwise
 * reproducible: every term is rounded once to a 64-bit fixed-point integer and the integer sums (LDS windows
 * per workgroup, integer atomics across workgroups) are exact; `deterministic` is accepted and ignored (the
 * round-4 ABI's float-atomic mode is gone).  scratch: gs4d_hexplane_backward_scratch_bytes, required.  When
 * every lay->plane[p].grad is set, the gradients are written straight to those (1, F, H, W) tensors and
 * dpacked may be NULL (no packed round trip, no unpack call); otherwise dpacked receives them. */
#define GS4D_HEXPLANE_MAX_LEVELS 4
typedef struct {
    int W, H;
    int64_t offset; /* first float of the plane in the packed buffer: (H, W, F) */
    const float *param; /* (1, F, H, W) parameter (pack source) */
    float *grad;        /* (1, F, H, W) gradient (unpack destination) */
} gs4d_hexplane_plane;
typedef struct {
    int levels, F; /* F: features per plane, a multiple of 4 with F / 4 a power of two */
    int64_t total; /* floats in the packed buffer */
    gs4d_hexplane_plane plane[6 * GS4D_HEXPLANE_MAX_LEVELS];
} gs4d_hexplane_layout;
/* Fills offsets/total from the per-plane sizes W[6*levels], H[6*levels]; param/grad pointers are set by the caller. */
int gs4d_hexplane_layout_init(gs4d_hexplane_layout *lay, int levels, int F, const int *W, const int *H);
int gs4d_hexplane_pack(const gs4d_hexplane_layout *lay, float *packed, void *stream);
int gs4d_hexplane_unpack(const gs4d_hexplane_layout *lay, const float *packed, void *stream);
/* Visiting order of the points (a 3-D Morton order of the normalised x, y, z; any permutation of 0..N-1
 * gives the same results up to float summation order, NULL = identity).  Morton-consecutive points touch
 * small boxes of cells, which the backward's per-workgroup tap sort and gather exploit. */
size_t gs4d_hexplane_order_scratch_bytes(int N);
int gs4d_hexplane_order(int N, const float *pts, uint32_t *order, void *scratch, void *stream);
int gs4d_hexplane_forward(int N, const float *pts, const uint32_t *order, const gs4d_hexplane_layout *lay,
                          const float *packed, float *feat, void *stream);
/* scratch of gs4d_hexplane_backward: the scale words and 64-bit accumulators for the packed buffer */
size_t gs4d_hexplane_backward_scratch_bytes(int N, const gs4d_hexplane_layout *lay);
int gs4d_hexplane_backward(int N, const float *pts, const uint32_t *order, const gs4d_hexplane_layout *lay,
                           const float *packed, const float *dfeat, float *dpacked, float *dpts, void *scratch,
                           int deterministic, void *stream);

/* ---- The field's input points, scene/hexplane.py:20-21 (normalize_aabb with aabb = (max corner, min corner))
 * + :166 (torch.cat((pts, timestamps), -1)) in one pass: pts (N, 4) = ((xyz - aabb[0]) * s - 1, t) with
 * s = (1 / (aabb[1] - aabb[0])) * 2, the reference's float operations; xyz rows ld_xyz floats apart, t rows
 * ld_t apart (ld_t 0: one time for every point), aabb (2, 3) on the device, pts 16-byte aligned.  backward: dxyz (N, 3) = dpts[:, :3] * s. */
int gs4d_hexplane_points(int N, const float *xyz, int64_t ld_xyz, const float *t, int64_t ld_t, const float *aabb,
                         float *pts, void *stream);
int gs4d_hexplane_points_backward(int N, const float *dpts, const float *aabb, float *dxyz, void *stream);
/* The same with add (nullable, (N, 3) contiguous): dxyz = add + the points' gradient -- xyz's other gradient
 * (the deformation tail's, xyz + dx) summed in by this pass instead of a separate add. */
int gs4d_hexplane_points_backward_add(int N, const float *dpts, const float *aabb, const float *add, float *dxyz,
                                      void *stream);

/* ---- HexPlane regularisers: scene/gaussian_model.py:538-577 (compute_regulation = plane_tv_weight *
 * _plane_regulation + time_smoothness_weight * _time_regulation + l1_time_planes * _l1_regulation) with
 * scene/regulation.py:22-28 compute_plane_smoothness.  For every plane t (1, C, H, W) of the batch:
 *   w_smooth * mean over (C, H-2, W) of ((t[y+2] - t[y+1]) - (t[y+1] - t[y]))^2  +  w_l1 * mean |1 - t|
 * (w_smooth: plane_tv_weight for the spatial planes, time_smoothness_weight for the time planes; w_l1:
 * l1_time_planes for the time planes, 0 otherwise).  H >= 3.  forward: *loss = the sum over the
 * batch (fp64 partials summed in a fixed order; scratch of gs4d_reg_scratch_bytes, all zero on entry and left
 * zero, as the L1 loss's above).  backward: grad
 * (1, C, H, W) of each plane = dloss * d(loss)/d(t), the gradient autograd derives from the
 * reference's graph: assigned, or with accumulate = 1 added to what grad holds (the plane's .grad after
 * the field's backward: the sum autograd would form, without its extra add per plane).  first_block of
 * plane i = the sum of gs4d_reg_blocks over planes 0..i-1. */
#define GS4D_REG_MAX_PLANES 24
typedef struct {
    const float *data;
    float *grad;
    int C, H, W;
    float w_smooth, w_l1;
    int64_t first_block;
} gs4d_reg_plane;
typedef struct {
    int count;
    int accumulate;
    gs4d_reg_plane p[GS4D_REG_MAX_PLANES];
} gs4d_reg_batch;
int64_t gs4d_reg_blocks(int C, int H, int W);
size_t gs4d_reg_scratch_bytes(const gs4d_reg_batch *batch);
int gs4d_hexplane_reg_forward(const gs4d_reg_batch *batch, float *loss, void *scratch, void *stream);
int gs4d_hexplane_reg_backward(const gs4d_reg_batch *batch, const float *dloss, void *stream);
/* The backward and the value in one pass over the planes: the gradient as gs4d_hexplane_reg_backward, and *loss
 * bitwise as gs4d_hexplane_reg_forward would give it (same partials, same order); scratch as for the forward.
 * base (nullable): *loss = *base + value instead (one fp32 add: the loss term the value joins). */
int gs4d_hexplane_reg_backward_value(const gs4d_reg_batch *batch, const float *dloss, float *loss, const float *base,
                                     void *scratch, void *stream);

/* ---- Linear-layer weight gradients over many rows: for each problem, dw (n, W) = dy^T x and db (n)
 * = column sums of dy (db may be NULL) -- the backward of F.linear as autograd forms it -- for dy (P, n)
 * and x (P, W) given with row strides ld_dy >= n and ld_x >= W (x may be a column block of a wider
 * matrix).  Up to 8 problems with the same P and W per call; n <= 16 or n = 48, n * W <= 8192,
 * W in {64, 128, 256}.  Replaces the weight/bias gradients of the deformation heads' second layers
 * (scene/deformation.py:73-78, 152-164).  fp32, partial sums reduced in a fixed order. */
typedef struct gs4d_dw_problem {
    const float *dy;
    const float *x;
    float *dw;
    float *db;
    int n, ld_dy, ld_x;
} gs4d_dw_problem;
size_t gs4d_linear_dw_scratch_bytes(int P, int W, int count, const int *n);
int gs4d_linear_dw(int P, int W, int count, const gs4d_dw_problem *problems, void *scratch, void *stream);

/* ---- The deformation heads' second layers, backward (scene/deformation.py:73-78, evaluated as one
 * block: a = relu(h W1^T + b1) of shape (P, kW), head i = a[:, iW:(i+1)W] W2_i^T + b2_i), in one pass
 * over a: da = (a > 0) * [g_0 W2_0 | ... | g_{k-1} W2_{k-1}] (P, kW), db1 = column sums of da, and for each
 * head dW2_i = g_i^T a_i (n_i, W), db2_i = column sums of g_i -- what autograd forms with k mm, one
 * threshold_backward, a sum and 2k weight/bias reductions.  W in {64, 128, 256}, k W <= 768, n_i <= 16
 * or n_i = 48 (then W <= 128); g_i (P, n_i) contiguous (16-byte aligned when n_i = 48), a and da (P, kW) contiguous,
 * W2_i (n_i, W).  fp32, partial sums
 * reduced in a fixed order. */
#define GS4D_HEADS_MAX 8
typedef struct gs4d_heads_bwd {
    int P, W, k;
    const float *a;
    float *da;
    float *db1;
    int n[GS4D_HEADS_MAX];
    const float *g[GS4D_HEADS_MAX];
    const float *w2[GS4D_HEADS_MAX];
    float *dw2[GS4D_HEADS_MAX];
    float *db2[GS4D_HEADS_MAX];
} gs4d_heads_bwd;
size_t gs4d_heads_backward_scratch_bytes(int P, int W, int k, const int *n);
int gs4d_heads_backward(const gs4d_heads_bwd *args, void *scratch, void *stream);
/* The same pass on the bf16 path: a and da bf16 (uint16 bits; da rounded once from the f32 products), the
 * sums and g, W2, dW2, db1, db2 fp32.  n_i <= 16, or n_i = 48 with W in {64, 128}.  Same scratch size. */
typedef struct gs4d_heads_bwd_bf16 {
    int P, W, k;
    const uint16_t *a;
    uint16_t *da;
    float *db1;
    int n[GS4D_HEADS_MAX];
    const float *g[GS4D_HEADS_MAX];
    const float *w2[GS4D_HEADS_MAX];
    float *dw2[GS4D_HEADS_MAX];
    float *db2[GS4D_HEADS_MAX];
} gs4d_heads_bwd_bf16;
int gs4d_heads_backward_bf16(const gs4d_heads_bwd_bf16 *args, void *scratch, void *stream);
/* The bf16 block's input gradient dh (P, W) fp32 = da (P, KW) bf16 @ W1 (KW, W), given W1^T (W, KW) bf16 (the block
 * forward's w1t); bf16 MFMA, fp32 accumulation.  KW a multiple of 64, W in {64, 128}, 16-byte aligned. */
int gs4d_mlp_dx_bf16(int P, int KW, int W, const uint16_t *da, const uint16_t *w1t, float *dh, void *stream);
/* Its weight gradient dW1 (KW, W) fp32 = da^T hb over the P rows (da (P, KW), hb (P, W) bf16; W = 128, KW a multiple
 * of W): per 1024-row chunk and head a bf16-MFMA block (LDS transpose reads), the chunks summed in order. */
size_t gs4d_mlp_dw_bf16_scratch_bytes(int P, int KW, int W);
int gs4d_mlp_dw_bf16(int P, int KW, int W, const uint16_t *da, const uint16_t *hb, float *dw, void *scratch,
                     void *stream);
/* The fp32 block's input gradient dh (P, W) = da (P, KW) @ W1 (KW, W), given W1^T (W, KW) (the block forward's
 * w1t), f32 MFMA with f32 products and sums in one fixed order: the same bits in every process
 * (scene/deformation.py:73-78's heads, the input gradient autograd forms by one GEMM).  KW a multiple of 64, W in
 * {64, 128}; rows 16-byte aligned. */
int gs4d_mlp_dx_f32(int P, int KW, int W, const float *da, const float *w1t, float *dh, void *stream);
/* Its weight gradient dW1 (KW, W) = da^T h over the P rows (da (P, KW), h (P, W) row-major): per row chunk and
 * 64-row block of dW1 an f32-MFMA block, its waves summed in a fixed order, the chunks summed in order (scratch:
 * gs4d_mlp_dw_f32_scratch_bytes). */
size_t gs4d_mlp_dw_f32_scratch_bytes(int P, int KW, int W);
int gs4d_mlp_dw_f32(int P, int KW, int W, const float *da, const float *h, float *dw, void *scratch, void *stream);

/* ---- The deformation field's first layer, backward, when feature_out is ONE Linear (defor_depth <= 1,
 * scene/deformation.py:51-55: hidden = x W^T + b) and every head begins with ReLU, so the heads read
 * h = relu(hidden).  Given g = dL/dh (P, Fout), h (P, Fout), x (P, Fin), W (Fout, Fin), one pass over the
 * rows (f32 MFMA, exact f32 products) writes what autograd forms with threshold_backward, two GEMMs and a
 * sum: dx = (g * (h > 0)) W (P, Fin), dW = (g * (h > 0))^T x (Fout, Fin), db = column sums of
 * g * (h > 0) (Fout); partial sums reduced in a fixed order.  (Fin, Fout) in {(32, 128), (64, 64),
 * (32, 64)}; contiguous; g, h, W 16-byte aligned; scratch of gs4d_feature_relu_backward_scratch_bytes. */
int gs4d_feature_relu_forward(int P, int Fin, int Fout, const float *x, const float *w, const float *b, float *h,
                              void *stream);  /* h = relu(x W^T + b), f32 MFMA; same shapes; x, W 16-byte aligned */
/* The same, also writing h rounded to bf16 into hb (uint16 bits, (ceil(P/16)*16, Fout); its padding rows hold row
 * P - 1's values), the input gs4d_heads_block_forward_bf16 takes when its h is NULL.  hb NULL: as above. */
int gs4d_feature_relu_forward_hb(int P, int Fin, int Fout, const float *x, const float *w, const float *b, float *h,
                                 uint16_t *hb, void *stream);
size_t gs4d_feature_relu_backward_scratch_bytes(int P, int Fin, int Fout);
int gs4d_feature_relu_backward(int P, int Fin, int Fout, const float *g, const float *h, const float *x,
                               const float *w, float *dx, float *dw, float *db, void *scratch, void *stream);

/* ---- The deformation heads' second layers, forward (scene/deformation.py:73-78 as one block): given
 * a = relu(h W1^T + b1) (P, kW), out_i = a[:, iW:(i+1)W] W2_i^T + b2_i (P, n_i) for every head in one pass
 * over a (f32 MFMA, exact f32 products), where torch runs k GEMMs on column slices.  W in {64, 128, 256},
 * 1 <= k <= 8, 1 <= n_i <= 64, the W2s (n_i, W) 16-byte aligned and at most 64 KiB together; a contiguous,
 * 16-byte aligned; out_i (P, n_i) contiguous. */
typedef struct gs4d_heads_fwd {
    int P, W, k;
    const float *a;
    int n[GS4D_HEADS_MAX];
    const float *w2[GS4D_HEADS_MAX];
    const float *b2[GS4D_HEADS_MAX];
    float *out[GS4D_HEADS_MAX];
} gs4d_heads_fwd;
int gs4d_heads_forward(const gs4d_heads_fwd *args, void *stream);

/* ---- The whole heads block, forward: a = relu(h W1^T + b1) (P, kW) AND out_i = a[:, iW:(i+1)W] W2_i^T + b2_i
 * (P, n_i) in one pass (f32 MFMA, exact f32 products); a is written for the backward and not read back.
 * Replaces the (P x W) @ (W x kW) first-layer GEMM plus gs4d_heads_forward.  W in {64, 128}, 1 <= k <= 8,
 * 1 <= n_i <= 64; h (P, W), W1 (kW, W) = the heads' first-layer weights stacked, b1 (kW), a (P, kW) contiguous
 * and 16-byte aligned WITH ROOM FOR ceil(P / 16) * 16 ROWS (the padding rows receive don't-care values: the
 * kernel stores whole 16-row blocks unconditionally), W2_i (n_i, W) 16-byte aligned, out_i (P, n_i) contiguous. */
typedef struct gs4d_heads_block_fwd {
    int P, W, k;
    const float *h;
    const float *w1;
    const float *b1;
    float *a;
    float *w1t;  /* nullable: W1^T (W, kW), written for the backward's input gradient (gs4d_mlp_dx_f32) */
    int n[GS4D_HEADS_MAX];
    const float *w2[GS4D_HEADS_MAX];
    const float *b2[GS4D_HEADS_MAX];
    float *out[GS4D_HEADS_MAX];
} gs4d_heads_block_fwd;
int gs4d_heads_block_forward(const gs4d_heads_block_fwd *args, void *stream);
/* The same block on bf16 operands (hyper.mlp_dtype = "bf16"): h, W1, W2 rounded to bf16, fp32 accumulation
 * (v_mfma_f32_16x16x32_bf16), a = relu(z + b1) stored as bf16 (uint16 bits, (ceil(P/16)*16, kW)), out_i fp32.
 * hb (nullable): h rounded to bf16, (ceil(P/16)*16, W), for the backward's weight-gradient GEMM; w1t (nullable):
 * W1^T rounded to bf16 (W, kW), for its input gradient (gs4d_mlp_dx_bf16).  h NULL: hb is an INPUT instead, h
 * already rounded to bf16 (gs4d_feature_relu_forward_hb): read as bf16, not converted per head, not written.
 * Returns 4 (GS4D_TRAIN_ERR_LDS) when the device cannot give the kernel its LDS (also for the fp32 form). */
#define GS4D_TRAIN_ERR_LDS 4
typedef struct gs4d_heads_block_fwd_bf16 {
    int P, W, k;
    const float *h;
    const float *w1;
    const float *b1;
    uint16_t *a;
    uint16_t *hb;
    uint16_t *w1t;
    int n[GS4D_HEADS_MAX];
    const float *w2[GS4D_HEADS_MAX];
    const float *b2[GS4D_HEADS_MAX];
    float *out[GS4D_HEADS_MAX];
} gs4d_heads_block_fwd_bf16;
int gs4d_heads_block_forward_bf16(const gs4d_heads_block_fwd_bf16 *args, void *stream);

#ifdef __cplusplus
}
#endif

#endif /* GS4D_TRAIN_H_INCLUDED */
