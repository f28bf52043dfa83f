// capi.hip -- the extern "C" boundary of libgs4d (include/gs4d.h) and the forward/backward
// orchestration that replaces CudaRasterizer::Rasterizer (rasterizer_impl.cu:141-437).
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <string>
#include <vector>

#include "../../include/gs4d.h"
#include "gs4d_internal.h"

namespace gs4d {

static thread_local std::string g_last_error;
static thread_local bool g_profiling = false;
// profiling level >= 2: the blend kernels (idempotent: pure functions of their inputs, the forward's
// in-place run sort included) are launched this many times back to back inside their stage, and the
// stage reports the per-launch average -- a kernel duration free of the event brackets' gaps, which is
// what rocprofv3's kernel trace measures (bench.py's roofline)
static thread_local int g_stage_repeats = 1;
static thread_local std::vector<std::pair<const char *, hipEvent_t>> g_marks;
static thread_local std::vector<int> g_mark_div;
static thread_local std::vector<std::pair<const char *, float>> g_timings;

static int fail(int code, const std::string &msg) {
    g_last_error = msg;
    return code;
}

#define GS4D_HIP(expr)                                                                                                  \
    do {                                                                                                               \
        hipError_t e_ = (expr);                                                                                        \
        if (e_ != hipSuccess)                                                                                          \
            return fail(GS4D_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_));                               \
    } while (0)

// Debug mode = the reference's CHECK_CUDA (auxiliary.h:166-173): synchronise after every stage.
#define GS4D_STAGE(name, expr)                                                                                          \
    do {                                                                                                               \
        GS4D_HIP(expr);                                                                                                \
        if (debug) {                                                                                                   \
            hipError_t e_ = hipStreamSynchronize(stream);                                                              \
            if (e_ != hipSuccess)                                                                                      \
                return fail(GS4D_ERR_HIP, std::string("[HIP ERROR] in stage ") + name + ": " + hipGetErrorString(e_)); \
        }                                                                                                              \
        mark(name, stream);                                                                                            \
    } while (0)

// A blend-kernel stage: under profiling level >= 2 its launch is preceded by a bracket of its own and
// repeated g_stage_repeats times, and the stage's time is the per-launch average.
#define GS4D_REPEATED_STAGE(name, expr)                                                                                 \
    do {                                                                                                               \
        const int reps_ = g_profiling ? g_stage_repeats : 1;                                                           \
        if (reps_ > 1) mark(name "_pre", stream);                                                                      \
        for (int r_ = 0; r_ < reps_; r_++) GS4D_HIP(expr);                                                             \
        if (debug) {                                                                                                   \
            hipError_t e_ = hipStreamSynchronize(stream);                                                              \
            if (e_ != hipSuccess)                                                                                      \
                return fail(GS4D_ERR_HIP, std::string("[HIP ERROR] in stage ") + name + ": " + hipGetErrorString(e_)); \
        }                                                                                                              \
        mark(name, stream, reps_);                                                                                     \
    } while (0)

static void mark(const char *name, hipStream_t s, int div = 1) {
    if (!g_profiling) return;
    hipEvent_t ev;
    if (hipEventCreate(&ev) != hipSuccess) return;
    (void)hipEventRecord(ev, s);
    g_marks.emplace_back(name, ev);
    g_mark_div.push_back(div);
}
static void begin_marks(hipStream_t s) {
    for (auto &m : g_marks) (void)hipEventDestroy(m.second);
    g_marks.clear();
    g_mark_div.clear();
    mark("begin", s);
}
static void end_marks() {
    if (!g_profiling || g_marks.empty()) return;
    (void)hipEventSynchronize(g_marks.back().second);
    g_timings.clear();
    for (size_t i = 1; i < g_marks.size(); i++) {
        float ms = 0.f;
        (void)hipEventElapsedTime(&ms, g_marks[i - 1].second, g_marks[i].second);
        g_timings.emplace_back(g_marks[i].first, ms / (float)g_mark_div[i]);
    }
    for (auto &m : g_marks) (void)hipEventDestroy(m.second);
    g_marks.clear();
    g_mark_div.clear();
}

static char *carve(char *&p, size_t bytes) {
    char *r = p;
    p += align_up(bytes, 256);
    return r;
}

// Sizes are computed by carving from a null base, so required() and carve() cannot disagree.
size_t GeomState::required(int P, int T) { return (size_t)carve(nullptr, P, T).zero + 4 * geom_zero_words(P) + 512; }
GeomState GeomState::carve(char *base, int P, int T) {
    char *p = (char *)align_up((size_t)base, 256);
    const size_t n = (size_t)P;
    GeomState g;
    g.depths = (float *)gs4d::carve(p, 4 * n);
    g.radii = (int *)gs4d::carve(p, 4 * n);
    g.xy = (float2 *)gs4d::carve(p, 8 * n);
    g.conic_opacity = (float4 *)gs4d::carve(p, 16 * n);
    g.splat = (float4 *)gs4d::carve(p, 48 * n);
    g.cov3D = (float *)gs4d::carve(p, 24 * n);
    g.clamped = (uint8_t *)gs4d::carve(p, n);
    g.tiles_touched = (uint32_t *)gs4d::carve(p, 4 * n);
    g.n_inst = (uint32_t *)gs4d::carve(p, 4 * n);
    g.vis_gid = (uint32_t *)gs4d::carve(p, 4 * n);
    g.cand_off = (uint32_t *)gs4d::carve(p, 4 * n + 4);
    g.first_vis = (uint32_t *)gs4d::carve(p, 4 * max_emit_chunks(P, T));
    g.emit_chain = (uint32_t *)gs4d::carve(p, 4 * (max_emit_chunks(P, T) + 64));
    g.zero = (uint32_t *)gs4d::carve(p, 4 * geom_zero_words(P));
    return g;
}

size_t ImageState::required(int W, int H) { return (size_t)carve(nullptr, W, H).order + 4 * (size_t)((W + 15) / 16) * ((H + 15) / 16) + 512; }
ImageState ImageState::carve(char *base, int W, int H) {
    char *p = (char *)align_up((size_t)base, 256);
    const size_t N = (size_t)W * H;
    const size_t T = (size_t)((W + kBlockX - 1) / kBlockX) * ((H + kBlockY - 1) / kBlockY);
    ImageState s;
    s.final_T = (float *)gs4d::carve(p, 4 * N);
    s.n_contrib = (uint32_t *)gs4d::carve(p, 4 * N);
    s.ranges = (uint2 *)gs4d::carve(p, 8 * T);
    s.order = (uint32_t *)gs4d::carve(p, 4 * T);
    return s;
}

// rasterizer_impl.cu:35-50
static uint32_t higher_msb(uint32_t n) {
    uint32_t msb = sizeof(n) * 4;
    uint32_t step = msb;
    while (step > 1) {
        step /= 2;
        if (n >> msb) msb += step; else msb -= step;
    }
    if (n >> msb) msb++;
    return msb;
}

}  // namespace gs4d

namespace gs4d {

// instances are sorted by tile id only; tile ids need msb(T) bits (rasterizer_impl.cu:301)
size_t BinningState::required(int L, int T) {
    BinningState b = carve(nullptr, L, T);
    return (size_t)b.scratch + 4 * binning_zero_words(L, T) + 512;
}
BinningState BinningState::carve(char *base, int L, int T) {
    char *p = (char *)align_up((size_t)base, 256);
    BinningState b;
    b.key_bits = (int)higher_msb((uint32_t)T);
    for (int i = 0; i < 2; i++) {
        b.keys[i] = (uint32_t *)gs4d::carve(p, 4 * (size_t)L);
        b.vals[i] = (uint32_t *)gs4d::carve(p, 4 * (size_t)L);
    }
    b.gid_by_e = (uint32_t *)gs4d::carve(p, 4 * (size_t)L);
    const int final_buf = ((b.key_bits + 7) / 8) & 1;  // each LSD pass swaps the ping-pong buffers
    b.upos = b.vals[final_buf];
    b.sorted_keys = b.keys[final_buf];
    b.tmp_hi = b.keys[final_buf ^ 1];
    b.tmp_lo = b.vals[final_buf ^ 1];
    b.count_items = gs4d::count_items(L, T);
    b.tile_hist = b.count_items ? (uint32_t *)gs4d::carve(p, 4 * tile_hist_words(L, T)) : nullptr;
    b.scratch = (uint32_t *)gs4d::carve(p, 4 * binning_zero_words(L, T));
    return b;
}

static Args make_args(int P, int D, int M, int W, int H, const float *bg, float scale_modifier, const float *view,
                      const float *proj, const float *campos, float tan_fovx, float tan_fovy, int prefiltered) {
    Args a;
    memset(&a, 0, sizeof(a));
    a.P = P; a.D = D; a.M = M; a.W = W; a.H = H;
    a.gx = (W + kBlockX - 1) / kBlockX;
    a.gy = (H + kBlockY - 1) / kBlockY;
    a.scale_modifier = scale_modifier;
    a.tan_fovx = tan_fovx;
    a.tan_fovy = tan_fovy;
    a.focal_y = H / (2.0f * tan_fovy);  // rasterizer_impl.cu:223-224
    a.focal_x = W / (2.0f * tan_fovx);
    a.viewmatrix = view;
    a.projmatrix = proj;
    a.campos = campos;
    a.bg = bg;
    a.prefiltered = prefiltered;
    return a;
}

}  // namespace gs4d

using namespace gs4d;

extern "C" {

const char *gs4d_last_error(void) { return g_last_error.c_str(); }
const char *gs4d_version(void) { return "gs4d 0.1.0 gfx950"; }
void gs4d_set_profiling(int enabled) {
    g_profiling = enabled != 0;
    g_stage_repeats = enabled >= 2 ? enabled : 1;
}
int gs4d_last_timings(const char **names, float *ms, int max_entries) {
    int n = (int)g_timings.size();
    for (int i = 0; i < n && i < max_entries; i++) {
        if (names) names[i] = g_timings[i].first;
        if (ms) ms[i] = g_timings[i].second;
    }
    return n;
}

int gs4d_debug_pair_alpha(int P, int width, int height, const char *geometry_buffer, int n, const int *gid,
                          const int *px, const int *py, float *og, float *pw, void *stream_) {
    if (P <= 0 || width <= 0 || height <= 0 || n < 0 || !geometry_buffer || (n > 0 && (!gid || !px || !py || !og || !pw)))
        return fail(GS4D_ERR_ARG, "debug_pair_alpha: bad args");
    const int T = ((width + kBlockX - 1) / kBlockX) * ((height + kBlockY - 1) / kBlockY);
    GeomState g = GeomState::carve(const_cast<char *>(geometry_buffer), P, T);
    GS4D_HIP(launch_pair_alpha(g, n, gid, px, py, og, pw, (hipStream_t)stream_));
    return GS4D_OK;
}
int gs4d_mark_visible_ex(int P, const float *means3D, const float *viewmatrix, const float *projmatrix,
                         uint8_t *present, void *stream_, int view_transposed) {
    hipStream_t stream = (hipStream_t)stream_;
    if (P < 0 || (P > 0 && (!means3D || !viewmatrix || !present))) return fail(GS4D_ERR_ARG, "mark_visible: bad args");
    if (P == 0) return GS4D_OK;
    GS4D_HIP(launch_mark_visible(P, means3D, viewmatrix, view_transposed ? 1 : 0, present, stream));
    return GS4D_OK;
}
int gs4d_mark_visible(int P, const float *means3D, const float *viewmatrix, const float *projmatrix,
                      uint8_t *present, void *stream) {
    return gs4d_mark_visible_ex(P, means3D, viewmatrix, projmatrix, present, stream, 0);
}

int gs4d_forward_ex(gs4d_alloc_fn geometry_alloc, void *geometry_ctx, gs4d_alloc_fn binning_alloc, void *binning_ctx,
                    gs4d_alloc_fn image_alloc, void *image_ctx, int P, int D, int M, const float *background,
                    int width, int height, const float *means3D, const float *shs, const float *colors_precomp,
                    const float *opacities, const float *scales, float scale_modifier, const float *rotations,
                    const float *cov3D_precomp, const float *viewmatrix, const float *projmatrix,
                    const float *cam_pos, float tan_fovx, float tan_fovy, int prefiltered, float *out_color,
                    float *out_depth, int *radii, int debug, void *stream_, int *num_rendered, int view_transposed) {
    hipStream_t stream = (hipStream_t)stream_;
    *num_rendered = 0;
    if (P < 0 || width <= 0 || height <= 0) return fail(GS4D_ERR_ARG, "forward: P must be >= 0 and the image non-empty");
    if (P == 0) return GS4D_OK;
    if (P >= (1 << 30)) return fail(GS4D_ERR_ARG, "forward: at most 2^30 Gaussians");
    if (!means3D || !opacities || !viewmatrix || !projmatrix || !background || !out_color || !out_depth)
        return fail(GS4D_ERR_ARG, "forward: missing required input");
    if (!colors_precomp && (!shs || !cam_pos))
        return fail(GS4D_ERR_ARG, "forward: provide either SHs (+campos) or precomputed colors");
    if (!colors_precomp && (D < 0 || D > 3 || (D + 1) * (D + 1) > M))
        return fail(GS4D_ERR_ARG, "forward: SH degree must be in [0,3] with (D+1)^2 <= M coefficients");
    if (!cov3D_precomp && (!scales || !rotations))
        return fail(GS4D_ERR_ARG, "forward: provide either scales+rotations or precomputed 3D covariances");
    if (((size_t)rotations & 15) != 0 && rotations) return fail(GS4D_ERR_ARG, "forward: rotations must be 16-byte aligned");

    Args a = make_args(P, D, M, width, height, background, scale_modifier, viewmatrix, projmatrix, cam_pos, tan_fovx,
                       tan_fovy, prefiltered);
    a.view_transposed = view_transposed ? 1 : 0;
    begin_marks(stream);

    if ((int64_t)a.gx * a.gy >= (int64_t)1 << 30) return fail(GS4D_ERR_ARG, "forward: at most 2^30 - 1 tiles");
    const int T = a.gx * a.gy;
    a.exact_div = T >= (1 << 20);  // the emission's float-reciprocal rect division is exact below 2^20 tiles
    char *gbuf = geometry_alloc(geometry_ctx, GeomState::required(P, T) + 16);
    if (!gbuf) return fail(GS4D_ERR_ALLOC, "forward: geometry buffer allocation failed");
    GeomState g = GeomState::carve(gbuf, P, T);
    char *ibuf = image_alloc(image_ctx, ImageState::required(width, height));
    if (!ibuf) return fail(GS4D_ERR_ALLOC, "forward: image buffer allocation failed");
    ImageState img = ImageState::carve(ibuf, width, height);
    int *radii_ptr = radii ? radii : g.radii;

    // one memset: prefiltered flag, num_rendered shards, depth-sort histograms and look-back words
    GS4D_HIP(hipMemsetAsync(g.zero, 0, 4 * geom_zero_words(P), stream));
    GS4D_STAGE("preprocess", launch_preprocess(a, means3D, scales, rotations, opacities, shs, cov3D_precomp,
                                               colors_precomp, radii_ptr, g, (int *)(g.zero + kZeroFlag), stream));

    // H1: the single device->host synchronisation of the forward (rasterizer_impl.cu:282).  The scan of
    // the visible Gaussians is enqueued before the host waits, so the GPU keeps working during the
    // round trip.
    // The staging word and its event belong to the device the stream runs on: a thread may call the
    // forward on several devices (the caller switches the current device per call).
    struct Readback {
        uint32_t *pinned = nullptr;
        hipEvent_t copied = nullptr;
    };
    static thread_local Readback readback[kMaxDevices];
    int dev = 0;
    GS4D_HIP(hipGetDevice(&dev));
    if (dev < 0 || dev >= kMaxDevices) return fail(GS4D_ERR_ARG, "forward: device index out of range");
    Readback &rb = readback[dev];
    if (!rb.pinned) GS4D_HIP(hipHostMalloc((void **)&rb.pinned, 128, hipHostMallocDefault));
    if (!rb.copied) GS4D_HIP(hipEventCreateWithFlags(&rb.copied, hipEventDisableTiming));
    uint32_t *pinned = rb.pinned;
    hipEvent_t copied = rb.copied;
    GS4D_HIP(hipMemcpyAsync(pinned, g.zero, 4 * (kZeroL + 16), hipMemcpyDeviceToHost, stream));
    GS4D_HIP(hipEventRecord(copied, stream));
    GS4D_STAGE("visible_scan", launch_visible_scan(a, g, stream));
    GS4D_HIP(hipEventSynchronize(copied));
    if (prefiltered && pinned[kZeroFlag] != 0)
        return fail(GS4D_ERR_PREFILTERED, "Point is filtered although prefiltered is set. This shouldn't happen!");
    // num_rendered keeps the reference's meaning (all 3-sigma rect instances, rasterizer_impl.cu:282)
    // and sizes the binning buffer; only the L' <= L instances that reach a pixel are materialised,
    // and L' stays on the device.
    uint64_t L64 = 0;
    for (int i = 0; i < kHistShards; i++) L64 += reinterpret_cast<const uint64_t *>(pinned + kZeroL)[i];
    if (L64 >= (1u << 30)) return fail(GS4D_ERR_ARG, "forward: more than 2^30 tile instances");
    const int L = (int)L64;
    *num_rendered = L;

    char *bbuf = binning_alloc(binning_ctx, BinningState::required(L, T));
    if (!bbuf) return fail(GS4D_ERR_ALLOC, "forward: binning buffer allocation failed");
    BinningState b = BinningState::carve(bbuf, L, T);
    GS4D_STAGE("binning", launch_binning(a, g, radii_ptr, b, L, img, stream));
    GS4D_REPEATED_STAGE("render", launch_render_forward(a, g, b, img, out_color, out_depth, stream));
    end_marks();
    return GS4D_OK;
}

int gs4d_backward_ex(int P, int D, int M, int R, const float *background, int width, int height,
                     const float *means3D, const float *shs, const float *colors_precomp, const float *scales,
                     float scale_modifier, const float *rotations, const float *cov3D_precomp,
                     const float *viewmatrix, const float *projmatrix, const float *campos, float tan_fovx,
                     float tan_fovy, const int *radii, char *geom_buffer, char *binning_buffer, char *image_buffer,
                     const float *dL_dpix, float *dL_dmean2D, float *dL_dconic, float *dL_dopacity,
                     float *dL_dcolor, float *dL_dmean3D, float *dL_dcov3D, float *dL_dsh, float *dL_dscale,
                     float *dL_drot, gs4d_alloc_fn scratch_alloc, void *scratch_ctx, int debug, void *stream_,
                     int view_transposed) {
    hipStream_t stream = (hipStream_t)stream_;
    if (P < 0 || R < 0) return fail(GS4D_ERR_ARG, "backward: bad sizes");
    if (P == 0) return GS4D_OK;
    if (!geom_buffer || !image_buffer || (R > 0 && !binning_buffer) || !dL_dpix || !means3D)
        return fail(GS4D_ERR_ARG, "backward: missing buffers");
    if (shs && (D < 0 || D > 3 || (D + 1) * (D + 1) > M))
        return fail(GS4D_ERR_ARG, "backward: SH degree must be in [0,3] with (D+1)^2 <= M coefficients");
    if (rotations && ((size_t)rotations & 15) != 0) return fail(GS4D_ERR_ARG, "backward: rotations must be 16-byte aligned");
    if (((size_t)dL_drot & 15) != 0) return fail(GS4D_ERR_ARG, "backward: dL_drot must be 16-byte aligned");
    if (!viewmatrix || !projmatrix || !background || (shs && !campos))
        return fail(GS4D_ERR_ARG, "backward: missing camera inputs");
    Args a = make_args(P, D, M, width, height, background, scale_modifier, viewmatrix, projmatrix, campos, tan_fovx,
                       tan_fovy, 0);
    a.view_transposed = view_transposed ? 1 : 0;
    begin_marks(stream);
    const int T = a.gx * a.gy;
    GeomState g = GeomState::carve(geom_buffer, P, T);
    ImageState img = ImageState::carve(image_buffer, width, height);
    const int *radii_ptr = radii ? radii : g.radii;
    // backward scratch: per-instance gradient records (R x 48 B) | per-Gaussian conic gradients |
    // segmented-reduction partials
    const size_t rec_bytes = align_up((size_t)R * kContribStride * sizeof(float), 256);
    const size_t dconic_bytes = align_up(16 * (size_t)P, 256);
    char *scratch = scratch_alloc(scratch_ctx, rec_bytes + dconic_bytes + contrib_scratch_bytes(R, P) + 256);
    if (!scratch) return fail(GS4D_ERR_ALLOC, "backward: scratch allocation failed");
    float *contrib = (float *)align_up((size_t)scratch, 256);
    char *reduce_scratch = (char *)contrib + rec_bytes + dconic_bytes;
    float4 *dconic = (dL_dconic && ((size_t)dL_dconic & 15) == 0) ? (float4 *)dL_dconic
                                                                   : (float4 *)((char *)contrib + rec_bytes);
    BinningState b = {};
    if (R > 0) {
        b = BinningState::carve(binning_buffer, R, T);
        const float *color_ptr = colors_precomp;  // NULL -> the forward's rgb (rasterizer_impl.cu:392)
        GS4D_REPEATED_STAGE("render_backward",
                            launch_render_backward(a, g, b.gid_by_e, b.upos, img, color_ptr, dL_dpix, contrib, stream));
    }
    GS4D_STAGE("contrib_reduce", launch_contrib_reduce(a, g, b, R, contrib, reduce_scratch, dL_dmean2D, dconic,
                                                       dL_dopacity, dL_dcolor, stream));
    const float *cov3D_ptr = cov3D_precomp ? cov3D_precomp : g.cov3D;  // rasterizer_impl.cu:414
    GS4D_STAGE("gaussian_backward",
               launch_gaussian_backward(a, g, R, reduce_scratch, radii_ptr, means3D, shs, scales, rotations, cov3D_ptr,
                                        dL_dmean2D, dconic, dL_dopacity, dL_dcolor, dL_dmean3D, dL_dcov3D, dL_dsh,
                                        dL_dscale, dL_drot, stream));
    if (dL_dconic && (float *)dconic != dL_dconic)
        GS4D_HIP(hipMemcpyAsync(dL_dconic, dconic, 16 * (size_t)P, hipMemcpyDeviceToDevice, stream));
    end_marks();
    return GS4D_OK;
}

int gs4d_forward(gs4d_alloc_fn geometry_alloc, void *geometry_ctx, gs4d_alloc_fn binning_alloc, void *binning_ctx,
                 gs4d_alloc_fn image_alloc, void *image_ctx, int P, int D, int M, const float *background, int width,
                 int height, const float *means3D, const float *shs, const float *colors_precomp,
                 const float *opacities, const float *scales, float scale_modifier, const float *rotations,
                 const float *cov3D_precomp, const float *viewmatrix, const float *projmatrix, const float *cam_pos,
                 float tan_fovx, float tan_fovy, int prefiltered, float *out_color, float *out_depth, int *radii,
                 int debug, void *stream, int *num_rendered) {
    return gs4d_forward_ex(geometry_alloc, geometry_ctx, binning_alloc, binning_ctx, image_alloc, image_ctx, P, D, M,
                           background, width, height, means3D, shs, colors_precomp, opacities, scales, scale_modifier,
                           rotations, cov3D_precomp, viewmatrix, projmatrix, cam_pos, tan_fovx, tan_fovy, prefiltered,
                           out_color, out_depth, radii, debug, stream, num_rendered, 0);
}

int gs4d_backward(int P, int D, int M, int R, const float *background, int width, int height, const float *means3D,
                  const float *shs, const float *colors_precomp, const float *scales, float scale_modifier,
                  const float *rotations, const float *cov3D_precomp, const float *viewmatrix,
                  const float *projmatrix, const float *campos, float tan_fovx, float tan_fovy, const int *radii,
                  char *geom_buffer, char *binning_buffer, char *image_buffer, const float *dL_dpix,
                  float *dL_dmean2D, float *dL_dconic, float *dL_dopacity, float *dL_dcolor, float *dL_dmean3D,
                  float *dL_dcov3D, float *dL_dsh, float *dL_dscale, float *dL_drot, gs4d_alloc_fn scratch_alloc,
                  void *scratch_ctx, int debug, void *stream) {
    return gs4d_backward_ex(P, D, M, R, background, width, height, means3D, shs, colors_precomp, scales,
                            scale_modifier, rotations, cov3D_precomp, viewmatrix, projmatrix, campos, tan_fovx,
                            tan_fovy, radii, geom_buffer, binning_buffer, image_buffer, dL_dpix, dL_dmean2D,
                            dL_dconic, dL_dopacity, dL_dcolor, dL_dmean3D, dL_dcov3D, dL_dsh, dL_dscale, dL_drot,
                            scratch_alloc, scratch_ctx, debug, stream, 0);
}

int gs4d_knn_mean_dist(int P, const float *points, float *mean_dists, gs4d_alloc_fn scratch_alloc, void *scratch_ctx,
                       void *stream_) {
    hipStream_t stream = (hipStream_t)stream_;
    if (P < 0 || P >= (1 << 30)) return fail(GS4D_ERR_ARG, "knn: P must be in [0, 2^30)");
    if (P == 0) return GS4D_OK;
    if (!points || !mean_dists || !scratch_alloc) return fail(GS4D_ERR_ARG, "knn: missing buffers");
    char *scratch = scratch_alloc(scratch_ctx, knn_scratch_bytes(P));
    if (!scratch) return fail(GS4D_ERR_ALLOC, "knn: scratch allocation failed");
    GS4D_HIP(launch_knn(P, points, mean_dists, scratch, stream));
    return GS4D_OK;
}

}  // extern "C"
