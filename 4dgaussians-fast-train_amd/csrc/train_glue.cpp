// train_glue.cpp -- the `gs4d_train._C` extension: PyTorch-ROCm tensors -> the train-step C ABI
// (include/gs4d_train.h).  Launches go to the current HIP stream; CPU tensors raise.
#include <ATen/ATen.h>
#include <c10/hip/HIPGuard.h>
#include <c10/hip/HIPStream.h>
#define ROCBLAS_BETA_FEATURES_API  // rocblas_gemm*_get_solutions: the candidates of the GEMM tuner
#include <rocblas/rocblas.h>

#include <cmath>
#include <limits>
#include <map>
#include <set>
#include <mutex>
#include <unordered_map>
#include <torch/extension.h>

#include <string>
#include <tuple>
#include <vector>

#include "../../include/gs4d.h"
#include "../../include/gs4d_train.h"

namespace {
void need(bool ok, const std::string &msg) {
    if (!ok) throw std::runtime_error(msg);
}
void check(int st, const char *what) {
    if (st != 0) throw std::runtime_error(std::string(what) + " failed (status " + std::to_string(st) + ")");
}
void gpu_f32(const torch::Tensor &t, const char *name) {
    need(t.is_cuda(), std::string(name) + " must be a HIP (GPU) tensor");
    need(t.scalar_type() == torch::kFloat32, std::string(name) + " must be float32");
    need(t.is_contiguous(), std::string(name) + " must be contiguous");
}
hipStream_t stream_of(const torch::Tensor &t) { return c10::hip::getCurrentHIPStream(t.device().index()).stream(); }

// Scratch for the last-workgroup totals (L1 loss, regulariser): its ticket word must be zero on entry and each
// call leaves it zero, so one buffer is kept per (device, stream, user) -- zeroed when made or grown -- instead of
// a fresh allocation (and a memset launch) per call.  Calls on one stream are ordered, so they may share it.
void *ticket_scratch(const torch::Tensor &like, size_t bytes, int user) {
    struct Key {
        int dev;
        hipStream_t s;
        int user;
        bool operator<(const Key &o) const {
            return std::tie(dev, s, user) < std::tie(o.dev, o.s, o.user);
        }
    };
    static std::mutex mu;
    static auto *bufs = new std::map<Key, torch::Tensor>();  // never destroyed: no device frees at process exit
    const Key k{(int)like.device().index(), stream_of(like), user};
    std::lock_guard<std::mutex> lk(mu);
    torch::Tensor &b = (*bufs)[k];
    if (!b.defined() || (size_t)b.numel() < bytes)
        b = torch::zeros({(int64_t)std::max<size_t>(bytes, 4096)}, like.options().dtype(torch::kUInt8));
    return b.data_ptr();
}
}  // namespace

// l1_loss forward: returns (loss (0-dim), sign (int8, x's shape))
std::tuple<torch::Tensor, torch::Tensor> l1_forward(const torch::Tensor &x_, const torch::Tensor &y_) {
    need(x_.sizes() == y_.sizes(), "l1_loss: shapes differ");
    need(x_.is_cuda() && y_.is_cuda(), "l1_loss: inputs must be HIP (GPU) tensors");
    c10::hip::HIPGuard guard(x_.device().index());
    torch::Tensor x = x_.to(torch::kFloat32).contiguous(), y = y_.to(torch::kFloat32).contiguous();
    const int64_t n = x.numel();
    torch::Tensor sign = torch::empty(x.sizes(), x.options().dtype(torch::kInt8));
    torch::Tensor loss = torch::empty({}, x.options());
    check(gs4d_l1_loss_forward(n, x.data_ptr<float>(), y.data_ptr<float>(), sign.data_ptr<int8_t>(),
                               loss.data_ptr<float>(), ticket_scratch(x, gs4d_l1_scratch_bytes(n), 0), stream_of(x)),
          "l1_loss forward");
    return {loss, sign};
}

// value and gradient in one pass (gs4d_l1_loss_grad); dloss = the upstream gradient (1 for loss.backward())
std::tuple<torch::Tensor, torch::Tensor> l1_loss_grad(const torch::Tensor &x_, const torch::Tensor &y_, double dloss) {
    need(x_.sizes() == y_.sizes(), "l1_loss: shapes differ");
    need(x_.is_cuda() && y_.is_cuda(), "l1_loss: inputs must be HIP (GPU) tensors");
    c10::hip::HIPGuard guard(x_.device().index());
    torch::Tensor x = x_.to(torch::kFloat32).contiguous(), y = y_.to(torch::kFloat32).contiguous();
    const int64_t n = x.numel();
    need(n % 4 == 0, "l1_loss_grad: numel must be a multiple of 4");
    torch::Tensor grad = torch::empty(x.sizes(), x.options());
    torch::Tensor loss = torch::empty({}, x.options());
    check(gs4d_l1_loss_grad(n, x.data_ptr<float>(), y.data_ptr<float>(), (float)dloss, loss.data_ptr<float>(),
                            grad.data_ptr<float>(), ticket_scratch(x, gs4d_l1_scratch_bytes(n), 0), stream_of(x)),
          "l1_loss_grad");
    return {loss, grad};
}

torch::Tensor l1_backward(const torch::Tensor &sign, const torch::Tensor &dloss_) {
    c10::hip::HIPGuard guard(sign.device().index());
    torch::Tensor dloss = dloss_.to(torch::kFloat32).contiguous();
    torch::Tensor grad = torch::empty(sign.sizes(), sign.options().dtype(torch::kFloat32));
    check(gs4d_l1_loss_backward(sign.numel(), sign.data_ptr<int8_t>(), dloss.data_ptr<float>(), grad.data_ptr<float>(),
                                stream_of(sign)),
          "l1_loss backward");
    return grad;
}

void densify_stats(const torch::Tensor &vs_grad, const torch::Tensor &visible, const torch::Tensor &radii,
                   torch::Tensor &grad_accum, torch::Tensor &denom, torch::Tensor &max_radii) {
    gpu_f32(vs_grad, "viewspace grad");
    gpu_f32(grad_accum, "xyz_gradient_accum");
    gpu_f32(denom, "denom");
    const int P = (int)vs_grad.size(0);
    need(vs_grad.dim() == 2 && vs_grad.size(1) == 3, "viewspace grad must be (P, 3)");
    // an empty visibility mask: radii > 0 filters (train.py's definition of the mask; radii required then)
    need(visible.numel() == 0 || (visible.scalar_type() == torch::kBool && visible.numel() == P && visible.is_cuda()),
         "visibility must be bool (P) or empty");
    need(visible.numel() || radii.numel(), "densify_stats: an empty visibility mask needs the radii");
    need(grad_accum.numel() == P && denom.numel() == P, "accumulators must have P elements");
    c10::hip::HIPGuard guard(vs_grad.device().index());
    torch::Tensor vis = visible.contiguous();
    torch::Tensor r;
    if (radii.numel()) {
        need(radii.numel() == P && radii.is_cuda(), "radii must have P elements");
        gpu_f32(max_radii, "max_radii2D");
        r = radii.to(torch::kInt32).contiguous();
    }
    check(gs4d_densify_stats(P, vs_grad.data_ptr<float>(),
                             vis.numel() ? reinterpret_cast<const uint8_t *>(vis.data_ptr<bool>()) : nullptr,
                             r.defined() ? r.data_ptr<int>() : nullptr, grad_accum.data_ptr<float>(),
                             denom.data_ptr<float>(), r.defined() ? max_radii.data_ptr<float>() : nullptr,
                             stream_of(vs_grad)),
          "densify_stats");
}

// One multi-tensor Adam step over lists of equally long (param, grad, exp_avg, exp_avg_sq) tensors;
// neg_step_sizes / bc2_sqrts hold the per-tensor scalars (torch computes them in double).
void adam_step(std::vector<torch::Tensor> params, std::vector<torch::Tensor> grads, std::vector<torch::Tensor> exp_avgs,
               std::vector<torch::Tensor> exp_avg_sqs, std::vector<double> neg_step_sizes, std::vector<double> bc2_sqrts,
               double beta1, double beta2, double eps) {
    const size_t n = params.size();
    need(grads.size() == n && exp_avgs.size() == n && exp_avg_sqs.size() == n && neg_step_sizes.size() == n &&
             bc2_sqrts.size() == n,
         "adam_step: list lengths differ");
    if (n == 0) return;
    c10::hip::HIPGuard guard(params[0].device().index());
    hipStream_t s = stream_of(params[0]);
    gs4d_adam_batch b;
    auto reset = [&]() {
        b.count = 0;
        b.beta1 = (float)beta1;
        b.one_minus_beta1 = (float)(1.0 - beta1);
        b.beta2 = (float)beta2;
        b.one_minus_beta2 = (float)(1.0 - beta2);
        b.eps = (float)eps;
    };
    reset();
    int64_t chunks = 0;
    for (size_t i = 0; i < n; i++) {
        need(grads[i].layout() == torch::kStrided, "FusedAdam does not support sparse gradients");
        if (!grads[i].is_contiguous()) grads[i] = grads[i].contiguous();  // kept alive by the vector until launch
        for (auto *t : {&params[i], &grads[i], &exp_avgs[i], &exp_avg_sqs[i]}) gpu_f32(*t, "adam tensor");
        need(params[i].device() == params[0].device(), "adam_step: tensors on several devices");
        need(grads[i].numel() == params[i].numel() && exp_avgs[i].numel() == params[i].numel() &&
                 exp_avg_sqs[i].numel() == params[i].numel(),
             "adam_step: tensor sizes differ");
        if (b.count == GS4D_ADAM_MAX_TENSORS) {
            check(gs4d_adam_step(&b, (void *)s), "adam_step");
            reset();
            chunks = 0;
        }
        gs4d_adam_tensor &d = b.t[b.count++];
        d.param = params[i].data_ptr<float>();
        d.grad = grads[i].data_ptr<float>();
        d.exp_avg = exp_avgs[i].data_ptr<float>();
        d.exp_avg_sq = exp_avg_sqs[i].data_ptr<float>();
        d.n = params[i].numel();
        d.first_chunk = chunks;
        d.neg_step_size = (float)neg_step_sizes[i];
        d.bias_correction2_sqrt = (float)bc2_sqrts[i];
        chunks += gs4d_adam_chunks(d.n);
    }
    check(gs4d_adam_step(&b, (void *)s), "adam_step");
}

// ---- HexPlane field -------------------------------------------------------------------------------
static gs4d_hexplane_layout hex_layout(const std::vector<torch::Tensor> &planes) {
    need(!planes.empty() && planes.size() % 6 == 0, "hexplane: expected 6 planes per level");
    const int levels = (int)(planes.size() / 6);
    const int F = (int)planes[0].size(1);
    std::vector<int> W, H;
    for (auto &p : planes) {
        gpu_f32(p, "hexplane plane");
        need(p.dim() == 4 && p.size(0) == 1 && p.size(1) == F, "hexplane planes must be (1, F, H, W) with one F");
        W.push_back((int)p.size(3));
        H.push_back((int)p.size(2));
    }
    gs4d_hexplane_layout lay;
    check(gs4d_hexplane_layout_init(&lay, levels, F, W.data(), H.data()), "hexplane layout");
    for (size_t i = 0; i < planes.size(); i++) lay.plane[i].param = planes[i].data_ptr<float>();
    return lay;
}

// returns (feat (N, levels*F), packed channels-last planes and the point order for the backward)
// order_in: a point order (N int32 indices) to reuse -- any permutation gives the same field; the
// Morton order only buys locality, so a caller may keep one across calls while N is unchanged
std::tuple<torch::Tensor, torch::Tensor, torch::Tensor> hexplane_forward(const torch::Tensor &pts_,
                                                                         std::vector<torch::Tensor> planes,
                                                                         c10::optional<torch::Tensor> order_in) {
    need(pts_.dim() == 2 && pts_.size(1) == 4 && pts_.is_cuda(), "hexplane: pts must be (N, 4) on the GPU");
    c10::hip::HIPGuard guard(pts_.device().index());
    torch::Tensor pts = pts_.to(torch::kFloat32).contiguous();
    gs4d_hexplane_layout lay = hex_layout(planes);
    const int N = (int)pts.size(0);
    torch::Tensor packed = torch::empty({lay.total}, pts.options());
    torch::Tensor feat = torch::empty({N, (int64_t)lay.levels * lay.F}, pts.options());
    hipStream_t s = stream_of(pts);
    check(gs4d_hexplane_pack(&lay, packed.data_ptr<float>(), (void *)s), "hexplane pack");
    torch::Tensor order;
    if (order_in.has_value() && order_in->defined() && order_in->numel() == N) {
        need(order_in->is_cuda() && order_in->scalar_type() == torch::kInt32 && order_in->is_contiguous() &&
                 order_in->device() == pts.device(),
             "hexplane: order must be a contiguous int32 GPU tensor of N indices");
        order = *order_in;
    } else {
        order = torch::empty({N}, pts.options().dtype(torch::kInt32));
        torch::Tensor scratch =
            torch::empty({(int64_t)gs4d_hexplane_order_scratch_bytes(N)}, pts.options().dtype(torch::kUInt8));
        check(gs4d_hexplane_order(N, pts.data_ptr<float>(), (uint32_t *)order.data_ptr<int>(), scratch.data_ptr(),
                                  (void *)s),
              "hexplane order");
    }
    check(gs4d_hexplane_forward(N, pts.data_ptr<float>(), (const uint32_t *)order.data_ptr<int>(), &lay,
                                packed.data_ptr<float>(), feat.data_ptr<float>(), (void *)s),
          "hexplane forward");
    return {feat, packed, order};
}

// returns (dpts (N, 4), plane gradients (1, F, H, W) each)
std::tuple<torch::Tensor, std::vector<torch::Tensor>> hexplane_backward(const torch::Tensor &pts_,
                                                                         std::vector<torch::Tensor> planes,
                                                                         const torch::Tensor &packed,
                                                                         const torch::Tensor &dfeat_,
                                                                         const torch::Tensor &order,
                                                                         bool deterministic) {
    c10::hip::HIPGuard guard(pts_.device().index());
    torch::Tensor pts = pts_.to(torch::kFloat32).contiguous(), dfeat = dfeat_.to(torch::kFloat32).contiguous();
    gs4d_hexplane_layout lay = hex_layout(planes);
    const int N = (int)pts.size(0);
    need(packed.numel() == lay.total, "hexplane backward: packed buffer size");
    need(dfeat.dim() == 2 && dfeat.size(0) == N && dfeat.size(1) == (int64_t)lay.levels * lay.F, "hexplane backward: dfeat shape");
    (void)deterministic;  // the backward is always deterministic (fixed-point sums)
    torch::Tensor scratch = torch::empty({(int64_t)gs4d_hexplane_backward_scratch_bytes(N, &lay)},
                                         pts.options().dtype(torch::kUInt8));
    torch::Tensor dpts = torch::empty({N, 4}, pts.options());
    std::vector<torch::Tensor> grads;
    for (size_t i = 0; i < planes.size(); i++) {
        grads.push_back(torch::empty_like(planes[i]));
        lay.plane[i].grad = grads.back().data_ptr<float>();
    }
    hipStream_t s = stream_of(pts);
    need(order.numel() == N && order.scalar_type() == torch::kInt32 && order.is_contiguous(), "hexplane backward: order");
    check(gs4d_hexplane_backward(N, pts.data_ptr<float>(), (const uint32_t *)order.data_ptr<int>(), &lay,
                                 packed.data_ptr<float>(), dfeat.data_ptr<float>(), nullptr,
                                 dpts.data_ptr<float>(), scratch.data_ptr(), 1, (void *)s),
          "hexplane backward");  // the plane gradients are written directly (grad pointers set)
    return {dpts, grads};
}


// ---- deformation tail + activations (gs4d_deform_tail_forward / _backward)
static const float *opt_f32(const c10::optional<torch::Tensor> &t, int64_t numel, const char *name) {
    if (!t.has_value() || !t->defined()) return nullptr;
    gpu_f32(*t, name);
    need(t->is_contiguous() && t->numel() == numel, "deform_tail: optional tensors must be contiguous with the right size");
    return t->data_ptr<float>();
}

std::vector<torch::Tensor> deform_tail_forward(const torch::Tensor &xyz, const torch::Tensor &s, const torch::Tensor &r,
                                               const torch::Tensor &o, const torch::Tensor &f_dc,
                                               const torch::Tensor &f_rest, const c10::optional<torch::Tensor> &dx,
                                               const c10::optional<torch::Tensor> &ds,
                                               const c10::optional<torch::Tensor> &dr,
                                               const c10::optional<torch::Tensor> &d_o,
                                               const c10::optional<torch::Tensor> &dshs) {
    const int64_t P = xyz.size(0);
    const int K = 1 + (int)f_rest.size(1);
    for (auto *t : {&xyz, &s, &r, &o, &f_dc, &f_rest}) {
        gpu_f32(*t, "deform_tail input");
        need(t->is_contiguous() && t->size(0) == P, "deform_tail: inputs must be contiguous with P rows");
    }
    need(xyz.numel() == 3 * P && s.numel() == 3 * P && r.numel() == 4 * P && o.numel() == P && f_dc.numel() == 3 * P &&
             f_rest.numel() == 3 * (K - 1) * P,
         "deform_tail: xyz / scales (P, 3), rotations (P, 4), opacity (P, 1), f_dc (P, 1, 3), f_rest (P, K-1, 3)");
    c10::hip::HIPGuard guard(xyz.device().index());
    auto means = torch::empty_like(xyz), scales = torch::empty_like(s), rot = torch::empty_like(r),
         opac = torch::empty_like(o), shs = torch::empty({P, K, 3}, xyz.options());
    check(gs4d_deform_tail_forward((int)P, K, xyz.data_ptr<float>(), s.data_ptr<float>(), r.data_ptr<float>(),
                                   o.data_ptr<float>(), f_dc.data_ptr<float>(), K > 1 ? f_rest.data_ptr<float>() : nullptr,
                                   opt_f32(dx, 3 * P, "dx"), opt_f32(ds, 3 * P, "ds"), opt_f32(dr, 4 * P, "dr"),
                                   opt_f32(d_o, P, "do"), opt_f32(dshs, 3 * K * P, "dshs"), means.data_ptr<float>(),
                                   scales.data_ptr<float>(), rot.data_ptr<float>(), opac.data_ptr<float>(),
                                   shs.data_ptr<float>(), (void *)stream_of(xyz)),
          "deform_tail forward");
    return {means, scales, rot, opac, shs};
}

std::vector<torch::Tensor> deform_tail_backward(const torch::Tensor &scales, const torch::Tensor &r,
                                                const c10::optional<torch::Tensor> &dr, const torch::Tensor &opac,
                                                const c10::optional<torch::Tensor> &g_means,
                                                const c10::optional<torch::Tensor> &g_scales,
                                                const c10::optional<torch::Tensor> &g_rot,
                                                const c10::optional<torch::Tensor> &g_opac,
                                                const c10::optional<torch::Tensor> &g_shs, int64_t K,
                                                std::vector<bool> has_delta) {
    need(has_delta.size() == 4, "deform_tail_backward: has_delta = (dx, ds, dr, do)");
    const int64_t P = scales.size(0);
    c10::hip::HIPGuard guard(scales.device().index());
    auto o3 = scales.options();
    auto d_xyz = torch::empty({P, 3}, o3), d_s = torch::empty({P, 3}, o3), d_r = torch::empty({P, 4}, o3),
         d_o = torch::empty({P, 1}, o3), d_fdc = torch::empty({P, 1, 3}, o3), d_frest = torch::empty({P, K - 1, 3}, o3);
    torch::Tensor gd[4];
    const int64_t w[4] = {3, 3, 4, 1};
    for (int i = 0; i < 4; i++) gd[i] = has_delta[i] ? torch::empty({P, w[i]}, o3) : torch::Tensor();
    auto ptr = [](torch::Tensor &t) { return t.defined() ? t.data_ptr<float>() : nullptr; };
    check(gs4d_deform_tail_backward((int)P, (int)K, scales.data_ptr<float>(), r.data_ptr<float>(),
                                    opt_f32(dr, 4 * P, "dr"), opac.data_ptr<float>(), opt_f32(g_means, 3 * P, "g_means"),
                                    opt_f32(g_scales, 3 * P, "g_scales"), opt_f32(g_rot, 4 * P, "g_rot"),
                                    opt_f32(g_opac, P, "g_opac"), opt_f32(g_shs, 3 * K * P, "g_shs"),
                                    d_xyz.data_ptr<float>(), d_s.data_ptr<float>(), d_r.data_ptr<float>(),
                                    d_o.data_ptr<float>(), d_fdc.data_ptr<float>(),
                                    K > 1 ? d_frest.data_ptr<float>() : nullptr, ptr(gd[0]), ptr(gd[1]), ptr(gd[2]),
                                    ptr(gd[3]), (void *)stream_of(scales)),
          "deform_tail backward");
    return {d_xyz, d_s, d_r, d_o, d_fdc, d_frest, gd[0], gd[1], gd[2], gd[3]};
}

// ---- HexPlane regularisers ------------------------------------------------------------------------
static gs4d_reg_batch reg_batch(const std::vector<torch::Tensor> &planes, const std::vector<double> &w_smooth,
                                const std::vector<double> &w_l1, const std::vector<torch::Tensor> *grads) {
    need(!planes.empty() && planes.size() <= GS4D_REG_MAX_PLANES, "hexplane_reg: 1..24 planes");
    need(w_smooth.size() == planes.size() && w_l1.size() == planes.size(), "hexplane_reg: one weight pair per plane");
    gs4d_reg_batch b;
    b.count = (int)planes.size();
    b.accumulate = 0;
    int64_t blocks = 0;
    for (size_t i = 0; i < planes.size(); i++) {
        const torch::Tensor &p = planes[i];
        gpu_f32(p, "hexplane_reg plane");
        need(p.dim() == 4 && p.size(0) == 1 && p.size(2) >= 3, "hexplane_reg planes must be (1, C, H >= 3, W)");
        gs4d_reg_plane &d = b.p[i];
        d.data = p.data_ptr<float>();
        d.grad = grads ? (*grads)[i].data_ptr<float>() : nullptr;
        d.C = (int)p.size(1);
        d.H = (int)p.size(2);
        d.W = (int)p.size(3);
        d.w_smooth = (float)w_smooth[i];
        d.w_l1 = (float)w_l1[i];
        d.first_block = blocks;
        blocks += gs4d_reg_blocks(d.C, d.H, d.W);
    }
    return b;
}

torch::Tensor hexplane_reg_forward(std::vector<torch::Tensor> planes, std::vector<double> w_smooth,
                                   std::vector<double> w_l1) {
    gs4d_reg_batch b = reg_batch(planes, w_smooth, w_l1, nullptr);
    c10::hip::HIPGuard guard(planes[0].device().index());
    hipStream_t s = stream_of(planes[0]);
    auto loss = torch::empty({}, planes[0].options());
    check(gs4d_hexplane_reg_forward(&b, loss.data_ptr<float>(), ticket_scratch(planes[0], gs4d_reg_scratch_bytes(&b), 1),
                                    (void *)s),
          "hexplane_reg forward");
    return loss;
}

std::vector<torch::Tensor> hexplane_reg_backward(std::vector<torch::Tensor> planes, std::vector<double> w_smooth,
                                                 std::vector<double> w_l1, const torch::Tensor &dloss_) {
    std::vector<torch::Tensor> grads;
    for (auto &p : planes) grads.push_back(torch::empty_like(p));
    gs4d_reg_batch b = reg_batch(planes, w_smooth, w_l1, &grads);
    c10::hip::HIPGuard guard(planes[0].device().index());
    auto dloss = dloss_.to(planes[0].device(), torch::kFloat32).contiguous();
    check(gs4d_hexplane_reg_backward(&b, dloss.data_ptr<float>(), (void *)stream_of(planes[0])), "hexplane_reg backward");
    return grads;
}

// the regulariser's gradient added in place to the planes' existing gradients (one launch for all); with_value:
// also its value (unscaled), from the same pass (a 0-dim tensor; else an undefined one)
torch::Tensor hexplane_reg_accumulate(std::vector<torch::Tensor> planes, std::vector<torch::Tensor> grads,
                                      std::vector<double> w_smooth, std::vector<double> w_l1, const torch::Tensor &dloss_,
                                      bool with_value, c10::optional<torch::Tensor> base) {
    need(grads.size() == planes.size(), "hexplane_reg_accumulate: one gradient per plane");
    for (size_t i = 0; i < planes.size(); i++) {
        gpu_f32(grads[i], "hexplane_reg gradient");
        need(grads[i].sizes() == planes[i].sizes() && grads[i].is_contiguous(),
             "hexplane_reg_accumulate: gradients must be contiguous and shaped like their planes");
    }
    gs4d_reg_batch b = reg_batch(planes, w_smooth, w_l1, &grads);
    b.accumulate = 1;
    c10::hip::HIPGuard guard(planes[0].device().index());
    auto dloss = dloss_.to(planes[0].device(), torch::kFloat32).contiguous();
    if (!with_value) {
        check(gs4d_hexplane_reg_backward(&b, dloss.data_ptr<float>(), (void *)stream_of(planes[0])),
              "hexplane_reg accumulate");
        return torch::Tensor();
    }
    auto loss = torch::empty({}, planes[0].options());
    const float *bp = nullptr;
    if (base && base->defined()) {
        gpu_f32(*base, "hexplane_reg base");
        need(base->numel() == 1 && base->device() == planes[0].device(), "hexplane_reg base: one value on the planes' device");
        bp = base->data_ptr<float>();
    }
    check(gs4d_hexplane_reg_backward_value(&b, dloss.data_ptr<float>(), loss.data_ptr<float>(), bp,
                                           ticket_scratch(planes[0], gs4d_reg_scratch_bytes(&b), 1),
                                           (void *)stream_of(planes[0])),
          "hexplane_reg accumulate");
    return loss;
}

// ---- Linear weight gradients: [(dw (n, W), db (n))] for pairs dy (P, n), x (P, W) (row strides kept)
std::vector<torch::Tensor> linear_dw(const std::vector<torch::Tensor> &dys, const std::vector<torch::Tensor> &xs) {
    need(!dys.empty() && dys.size() == xs.size() && dys.size() <= 8, "linear_dw: 1-8 (dy, x) pairs");
    const auto &d0 = dys[0];
    c10::hip::HIPGuard guard(d0.device().index());
    const int P = (int)d0.size(0), W = (int)xs[0].size(1), count = (int)dys.size();
    std::vector<gs4d_dw_problem> probs(count);
    std::vector<int> ns(count);
    std::vector<torch::Tensor> out;
    for (int i = 0; i < count; i++) {
        const auto &dy = dys[i], &x = xs[i];
        need(dy.is_cuda() && x.is_cuda() && dy.scalar_type() == torch::kFloat32 && x.scalar_type() == torch::kFloat32,
             "linear_dw: float32 GPU tensors");
        need(dy.dim() == 2 && x.dim() == 2 && dy.size(0) == P && x.size(0) == P && x.size(1) == W,
             "linear_dw: dy (P, n) and x (P, W), same P and W for every pair");
        need(dy.stride(1) == 1 && x.stride(1) == 1, "linear_dw: rows must be contiguous");
        auto dw = torch::empty({dy.size(1), W}, dy.options());
        auto db = torch::empty({dy.size(1)}, dy.options());
        ns[i] = (int)dy.size(1);
        probs[i] = gs4d_dw_problem{dy.data_ptr<float>(), x.data_ptr<float>(), dw.data_ptr<float>(), db.data_ptr<float>(),
                                   ns[i], (int)dy.stride(0), (int)x.stride(0)};
        out.push_back(dw);
        out.push_back(db);
    }
    const size_t sb = gs4d_linear_dw_scratch_bytes(P, W, count, ns.data());
    auto scratch = torch::empty({(int64_t)sb}, d0.options().dtype(torch::kUInt8));
    check(gs4d_linear_dw(P, W, count, probs.data(), scratch.data_ptr(), (void *)stream_of(d0)), "linear_dw");
    return out;
}

// ---- heads block backward: (da, db1, [dW2_i, db2_i]...) for a (P, kW), g_i (P, n_i), W2_i (n_i, W)
std::vector<torch::Tensor> heads_backward(const torch::Tensor &a, const std::vector<torch::Tensor> &gs,
                                          const std::vector<torch::Tensor> &w2s) {
    const int k = (int)gs.size();
    need(k >= 1 && k <= GS4D_HEADS_MAX && (int)w2s.size() == k, "heads_backward: 1-8 heads");
    const bool bf = a.scalar_type() == torch::kBFloat16;  // the bf16 path: a and da bf16, the rest fp32
    need(a.is_cuda() && (a.scalar_type() == torch::kFloat32 || bf) && a.dim() == 2 && a.is_contiguous(),
         "heads_backward: a contiguous float32 or bfloat16 (P, kW) GPU tensor");
    need(a.size(1) % k == 0, "heads_backward: a must be (P, kW)");
    c10::hip::HIPGuard guard(a.device().index());
    gs4d_heads_bwd b{};
    b.P = (int)a.size(0), b.k = k, b.W = (int)(a.size(1) / k);
    auto da = torch::empty_like(a);
    auto db1 = torch::empty({a.size(1)}, a.options().dtype(torch::kFloat32));
    b.a = (const float *)a.data_ptr(), b.da = (float *)da.data_ptr(), b.db1 = db1.data_ptr<float>();
    std::vector<torch::Tensor> out = {da, db1};
    std::vector<torch::Tensor> keep;
    for (int i = 0; i < k; i++) {
        auto g = gs[i].contiguous();
        const auto &w2 = w2s[i];
        need(g.is_cuda() && g.scalar_type() == torch::kFloat32 && g.dim() == 2 && g.size(0) == b.P,
             "heads_backward: g_i (P, n_i) float32");
        need(w2.is_cuda() && w2.scalar_type() == torch::kFloat32 && w2.dim() == 2 && w2.is_contiguous() &&
                 w2.size(0) == g.size(1) && w2.size(1) == b.W,
             "heads_backward: W2_i (n_i, W) contiguous float32");
        b.n[i] = (int)g.size(1);
        b.g[i] = g.data_ptr<float>();
        b.w2[i] = w2.data_ptr<float>();
        auto dw2 = torch::empty({g.size(1), b.W}, g.options());
        auto db2 = torch::empty({g.size(1)}, g.options());
        b.dw2[i] = dw2.data_ptr<float>(), b.db2[i] = db2.data_ptr<float>();
        out.push_back(dw2);
        out.push_back(db2);
        keep.push_back(g);
    }
    const size_t sb = gs4d_heads_backward_scratch_bytes(b.P, b.W, k, b.n);
    auto scratch = torch::empty({(int64_t)sb}, a.options().dtype(torch::kUInt8));
    if (bf) {
        // same field layout, a / da as bf16 bits
        gs4d_heads_bwd_bf16 bb{};
        bb.P = b.P, bb.W = b.W, bb.k = b.k, bb.db1 = b.db1;
        bb.a = (const uint16_t *)a.data_ptr(), bb.da = (uint16_t *)da.data_ptr();
        for (int i = 0; i < k; i++)
            bb.n[i] = b.n[i], bb.g[i] = b.g[i], bb.w2[i] = b.w2[i], bb.dw2[i] = b.dw2[i], bb.db2[i] = b.db2[i];
        check(gs4d_heads_backward_bf16(&bb, scratch.data_ptr(), (void *)stream_of(a)), "heads_backward_bf16");
    } else {
        check(gs4d_heads_backward(&b, scratch.data_ptr(), (void *)stream_of(a)), "heads_backward");
    }
    return out;
}

// ---- first deformation layer backward: (dx, dW, db) for g = dL/dh, h = relu(x W^T + b) (P, Fout), x (P, Fin)
std::vector<torch::Tensor> feature_relu_backward(const torch::Tensor &g_, const torch::Tensor &h, const torch::Tensor &x,
                                                 const torch::Tensor &w) {
    auto g = g_.contiguous();
    for (const torch::Tensor *t : std::initializer_list<const torch::Tensor *>{&g, &h, &x, &w})
        gpu_f32(*t, "feature_relu_backward operand");
    need(h.is_contiguous() && x.is_contiguous() && w.is_contiguous(), "feature_relu_backward: contiguous operands");
    need(g.dim() == 2 && h.sizes() == g.sizes() && x.dim() == 2 && x.size(0) == g.size(0) && w.dim() == 2 &&
             w.size(0) == g.size(1) && w.size(1) == x.size(1),
         "feature_relu_backward: g, h (P, Fout), x (P, Fin), W (Fout, Fin)");
    c10::hip::HIPGuard guard(g.device().index());
    const int P = (int)g.size(0), Fout = (int)g.size(1), Fin = (int)x.size(1);
    auto dx = torch::empty_like(x);
    auto dw = torch::empty_like(w);
    auto db = torch::empty({Fout}, w.options());
    auto scratch = torch::empty({(int64_t)gs4d_feature_relu_backward_scratch_bytes(P, Fin, Fout)},
                                g.options().dtype(torch::kUInt8));
    check(gs4d_feature_relu_backward(P, Fin, Fout, g.data_ptr<float>(), h.data_ptr<float>(), x.data_ptr<float>(),
                                     w.data_ptr<float>(), dx.data_ptr<float>(), dw.data_ptr<float>(),
                                     db.data_ptr<float>(), scratch.data_ptr(), (void *)stream_of(g)),
          "feature_relu_backward");
    return {dx, dw, db};
}

// ---- heads block forward: [out_i (P, n_i)] for a (P, kW), W2_i (n_i, W), b2_i (n_i)
std::vector<torch::Tensor> heads_forward(const torch::Tensor &a, const std::vector<torch::Tensor> &w2s,
                                         const std::vector<torch::Tensor> &b2s) {
    const int k = (int)w2s.size();
    need(k >= 1 && k <= GS4D_HEADS_MAX && (int)b2s.size() == k, "heads_forward: 1-8 heads");
    need(a.is_cuda() && a.scalar_type() == torch::kFloat32 && a.dim() == 2 && a.is_contiguous() && a.size(1) % k == 0,
         "heads_forward: a contiguous float32 (P, kW) GPU tensor");
    c10::hip::HIPGuard guard(a.device().index());
    gs4d_heads_fwd b{};
    b.P = (int)a.size(0), b.W = (int)(a.size(1) / k), b.k = k, b.a = a.data_ptr<float>();
    std::vector<torch::Tensor> out, keep;
    for (int i = 0; i < k; i++) {
        auto w2 = w2s[i].contiguous();
        auto b2 = b2s[i].contiguous();
        need(w2.is_cuda() && w2.scalar_type() == torch::kFloat32 && w2.dim() == 2 && w2.size(1) == b.W &&
                 b2.scalar_type() == torch::kFloat32 && b2.numel() == w2.size(0),
             "heads_forward: W2_i (n_i, W), b2_i (n_i) float32");
        b.n[i] = (int)w2.size(0);
        b.w2[i] = w2.data_ptr<float>();
        b.b2[i] = b2.data_ptr<float>();
        auto o = torch::empty({a.size(0), w2.size(0)}, a.options());
        b.out[i] = o.data_ptr<float>();
        out.push_back(o);
        keep.push_back(w2);
        keep.push_back(b2);
    }
    check(gs4d_heads_forward(&b, (void *)stream_of(a)), "heads_forward");
    return out;
}

// ---- heads block forward, both layers: (a, W1^T, [out_i]) for h (P, W), W1 (kW, W), b1 (kW), W2_i (n_i, W), b2_i (n_i)
std::vector<torch::Tensor> heads_block_forward(const torch::Tensor &h, const torch::Tensor &w1, const torch::Tensor &b1,
                                               const std::vector<torch::Tensor> &w2s,
                                               const std::vector<torch::Tensor> &b2s) {
    const int k = (int)w2s.size();
    need(k >= 1 && k <= GS4D_HEADS_MAX && (int)b2s.size() == k, "heads_block_forward: 1-8 heads");
    for (const torch::Tensor *t : std::initializer_list<const torch::Tensor *>{&h, &w1, &b1})
        gpu_f32(*t, "heads_block_forward operand");
    need(h.dim() == 2 && h.is_contiguous() && w1.dim() == 2 && w1.is_contiguous() && b1.is_contiguous() &&
             w1.size(1) == h.size(1) && w1.size(0) == k * h.size(1) && b1.numel() == w1.size(0),
         "heads_block_forward: h (P, W), W1 (kW, W), b1 (kW) contiguous");
    c10::hip::HIPGuard guard(h.device().index());
    gs4d_heads_block_fwd b{};
    b.P = (int)h.size(0), b.W = (int)h.size(1), b.k = k;
    // whole 16-row blocks are stored (the ABI's padding rows); the caller sees the first P rows
    auto a_pad = torch::empty({(h.size(0) + 15) / 16 * 16, w1.size(0)}, h.options());
    auto a = a_pad.narrow(0, 0, h.size(0));
    auto w1t = torch::empty({w1.size(1), w1.size(0)}, h.options());  // W1^T (W, kW), for the input gradient
    b.h = h.data_ptr<float>(), b.w1 = w1.data_ptr<float>(), b.b1 = b1.data_ptr<float>(), b.a = a_pad.data_ptr<float>();
    b.w1t = w1t.data_ptr<float>();
    std::vector<torch::Tensor> out{a, w1t}, keep;
    for (int i = 0; i < k; i++) {
        auto w2 = w2s[i].contiguous();
        auto b2 = b2s[i].contiguous();
        need(w2.is_cuda() && w2.scalar_type() == torch::kFloat32 && w2.dim() == 2 && w2.size(1) == b.W &&
                 b2.scalar_type() == torch::kFloat32 && b2.numel() == w2.size(0),
             "heads_block_forward: W2_i (n_i, W), b2_i (n_i) float32");
        b.n[i] = (int)w2.size(0);
        b.w2[i] = w2.data_ptr<float>();
        b.b2[i] = b2.data_ptr<float>();
        auto o = torch::empty({h.size(0), w2.size(0)}, h.options());
        b.out[i] = o.data_ptr<float>();
        out.push_back(o);
        keep.push_back(w2);
        keep.push_back(b2);
    }
    check(gs4d_heads_block_forward(&b, (void *)stream_of(h)), "heads_block_forward");
    return out;
}

// ---- heads block forward on bf16 operands: (a bf16, hb bf16, W1^T bf16, [out_i fp32]); same operands as above
// hb_in (optional): h already rounded to bf16 by feature_relu_forward(..., with_hb=True); the kernel then reads it
// instead of h and the returned hb is hb_in
std::vector<torch::Tensor> heads_block_forward_bf16(const torch::Tensor &h, const torch::Tensor &w1,
                                                    const torch::Tensor &b1, const std::vector<torch::Tensor> &w2s,
                                                    const std::vector<torch::Tensor> &b2s,
                                                    const c10::optional<torch::Tensor> &hb_in) {
    const int k = (int)w2s.size();
    need(k >= 1 && k <= GS4D_HEADS_MAX && (int)b2s.size() == k, "heads_block_forward_bf16: 1-8 heads");
    for (const torch::Tensor *t : std::initializer_list<const torch::Tensor *>{&h, &w1, &b1})
        gpu_f32(*t, "heads_block_forward_bf16 operand");
    need(h.dim() == 2 && h.is_contiguous() && w1.dim() == 2 && w1.is_contiguous() && b1.is_contiguous() &&
             w1.size(1) == h.size(1) && w1.size(0) == k * h.size(1) && b1.numel() == w1.size(0),
         "heads_block_forward_bf16: h (P, W), W1 (kW, W), b1 (kW) contiguous");
    c10::hip::HIPGuard guard(h.device().index());
    gs4d_heads_block_fwd_bf16 b{};
    b.P = (int)h.size(0), b.W = (int)h.size(1), b.k = k;
    const int64_t rows = (h.size(0) + 15) / 16 * 16;
    auto bopt = h.options().dtype(torch::kBFloat16);
    auto a_pad = torch::empty({rows, w1.size(0)}, bopt);
    auto w1t = torch::empty({w1.size(1), w1.size(0)}, bopt);  // W1^T (W, kW)
    b.w1 = w1.data_ptr<float>(), b.b1 = b1.data_ptr<float>();
    b.a = (uint16_t *)a_pad.data_ptr(), b.w1t = (uint16_t *)w1t.data_ptr();
    torch::Tensor hb_out;
    if (hb_in.has_value() && hb_in->defined()) {
        const torch::Tensor &hb = *hb_in;
        need(hb.is_cuda() && hb.scalar_type() == torch::kBFloat16 && hb.dim() == 2 && hb.size(0) == h.size(0) &&
                 hb.size(1) == h.size(1) && hb.stride(1) == 1 && hb.stride(0) == hb.size(1) &&
                 ((size_t)hb.data_ptr() & 15) == 0,
             "heads_block_forward_bf16: hb (P, W) bf16, contiguous rows, 16-byte aligned");
        b.h = nullptr;  // the kernel reads hb (only rows < P)
        b.hb = (uint16_t *)hb.data_ptr();
        hb_out = hb;
    } else {
        auto hb_pad = torch::empty({rows, h.size(1)}, bopt);
        b.h = h.data_ptr<float>();
        b.hb = (uint16_t *)hb_pad.data_ptr();
        hb_out = hb_pad.narrow(0, 0, h.size(0));
    }
    std::vector<torch::Tensor> out{a_pad.narrow(0, 0, h.size(0)), hb_out, w1t}, keep;
    for (int i = 0; i < k; i++) {
        auto w2 = w2s[i].contiguous();
        auto b2 = b2s[i].contiguous();
        need(w2.is_cuda() && w2.scalar_type() == torch::kFloat32 && w2.dim() == 2 && w2.size(1) == b.W &&
                 b2.scalar_type() == torch::kFloat32 && b2.numel() == w2.size(0),
             "heads_block_forward_bf16: W2_i (n_i, W), b2_i (n_i) float32");
        b.n[i] = (int)w2.size(0);
        b.w2[i] = w2.data_ptr<float>();
        b.b2[i] = b2.data_ptr<float>();
        auto o = torch::empty({h.size(0), w2.size(0)}, h.options());
        b.out[i] = o.data_ptr<float>();
        out.push_back(o);
        keep.push_back(w2);
        keep.push_back(b2);
    }
    check(gs4d_heads_block_forward_bf16(&b, (void *)stream_of(h)), "heads_block_forward_bf16");
    return out;
}

// ---- the bf16 block's input gradient: dh (P, W) fp32 = da (P, KW) bf16 @ W1 from W1^T (W, KW) bf16
torch::Tensor mlp_dx_bf16(const torch::Tensor &da, const torch::Tensor &w1t) {
    need(da.is_cuda() && w1t.is_cuda() && da.scalar_type() == torch::kBFloat16 && w1t.scalar_type() == torch::kBFloat16,
         "mlp_dx_bf16: bf16 GPU tensors");
    need(da.dim() == 2 && w1t.dim() == 2 && da.is_contiguous() && w1t.is_contiguous() && w1t.size(1) == da.size(1),
         "mlp_dx_bf16: da (P, KW), W1^T (W, KW), contiguous");
    c10::hip::HIPGuard guard(da.device().index());
    auto dh = torch::empty({da.size(0), w1t.size(0)}, da.options().dtype(torch::kFloat32));
    check(gs4d_mlp_dx_bf16((int)da.size(0), (int)da.size(1), (int)w1t.size(0), (const uint16_t *)da.data_ptr(),
                           (const uint16_t *)w1t.data_ptr(), dh.data_ptr<float>(), (void *)stream_of(da)),
          "mlp_dx_bf16");
    return dh;
}

// ---- the bf16 block's first-layer weight gradient: dW1 (KW, W) fp32 = da^T hb
torch::Tensor mlp_dw_bf16(const torch::Tensor &da, const torch::Tensor &hb) {
    need(da.is_cuda() && hb.is_cuda() && da.scalar_type() == torch::kBFloat16 && hb.scalar_type() == torch::kBFloat16,
         "mlp_dw_bf16: bf16 GPU tensors");
    need(da.dim() == 2 && hb.dim() == 2 && da.size(0) == hb.size(0) && da.stride(1) == 1 && hb.stride(1) == 1 &&
             da.stride(0) == da.size(1) && hb.stride(0) == hb.size(1),
         "mlp_dw_bf16: da (P, KW), hb (P, W), rows contiguous");
    c10::hip::HIPGuard guard(da.device().index());
    const int P = (int)da.size(0), KW = (int)da.size(1), W = (int)hb.size(1);
    auto dw = torch::empty({KW, W}, da.options().dtype(torch::kFloat32));
    auto scratch = torch::empty({(int64_t)gs4d_mlp_dw_bf16_scratch_bytes(P, KW, W)}, da.options().dtype(torch::kUInt8));
    check(gs4d_mlp_dw_bf16(P, KW, W, (const uint16_t *)da.data_ptr(), (const uint16_t *)hb.data_ptr(),
                           dw.data_ptr<float>(), scratch.data_ptr(), (void *)stream_of(da)),
          "mlp_dw_bf16");
    return dw;
}

// ---- row surgery (gs4d_rows_assemble): every tensor rebuilt by one row plan in one launch.  srcs: the old (P, ...)
// tensors (a ZERO tensor's gives only its shape and dtype); givens[i]: the last appended rows of a GATHER tensor
// (or None); keep: (K) int32 old row indices; append: int32 old row indices of the gathered appended rows (empty
// when none).  Returns the new (K + A, ...) tensors.
std::vector<torch::Tensor> rows_assemble(const std::vector<torch::Tensor> &srcs,
                                         const std::vector<c10::optional<torch::Tensor>> &givens,
                                         const std::vector<int64_t> &modes, const torch::Tensor &keep,
                                         const torch::Tensor &append, int64_t A) {
    const int n = (int)srcs.size();
    need(n >= 1 && n <= GS4D_ROWS_MAX_TENSORS && (int)givens.size() == n && (int)modes.size() == n,
         "rows_assemble: 1-32 tensors, one given and one mode each");
    need(keep.is_cuda() && keep.scalar_type() == torch::kInt32 && keep.dim() == 1 && keep.is_contiguous(),
         "rows_assemble: keep must be a contiguous int32 GPU vector");
    need(A >= 0, "rows_assemble: A >= 0");
    const int64_t K = keep.size(0);
    const bool has_append = append.defined() && append.numel() > 0;
    if (has_append)
        need(append.is_cuda() && append.scalar_type() == torch::kInt32 && append.dim() == 1 && append.is_contiguous() &&
                 append.size(0) <= A,
             "rows_assemble: append must be a contiguous int32 GPU vector of at most A indices");
    c10::hip::HIPGuard guard(keep.device().index());
    gs4d_rows_batch b{};
    b.count = 0, b.K = K, b.A = A;
    b.keep = keep.data_ptr<int32_t>();
    b.append = has_append ? append.data_ptr<int32_t>() : nullptr;
    std::vector<torch::Tensor> out, keepalive;
    for (int i = 0; i < n; i++) {
        const torch::Tensor &s = srcs[i];
        need(s.is_cuda() && s.device() == keep.device() && s.dim() >= 1 && s.is_contiguous(),
             "rows_assemble: sources are contiguous GPU tensors on keep's device");
        const int es = (int)s.element_size();
        need(es == 1 || es == 4, "rows_assemble: 1- or 4-byte elements");
        const int64_t mode = modes[i];
        need(mode >= GS4D_ROWS_GATHER && mode <= GS4D_ROWS_ZERO, "rows_assemble: mode");
        std::vector<int64_t> shape(s.sizes().begin(), s.sizes().end());
        int64_t width = 1;
        for (size_t d = 1; d < shape.size(); d++) width *= shape[d];
        shape[0] = K + A;
        auto d = torch::empty(shape, s.options());
        out.push_back(d);
        if (width == 0) continue;  // rows without elements (e.g. SH rest at degree 0): nothing to copy
        gs4d_rows_tensor &t = b.t[b.count++];
        t.src = s.data_ptr(), t.dst = d.data_ptr(), t.width = width, t.esize = es, t.mode = (int)mode;
        t.given_rows = 0;
        if (mode == GS4D_ROWS_GATHER && givens[i].has_value() && givens[i]->defined()) {
            auto g = givens[i]->to(s.scalar_type()).contiguous();
            need(g.is_cuda() && g.device() == s.device() && g.dim() >= 1 && g.size(0) <= A && g.numel() == g.size(0) * width,
                 "rows_assemble: given rows (<= A, ...) with the source's row width");
            t.given = g.data_ptr();
            t.given_rows = g.size(0);
            keepalive.push_back(g);
        }
        if (mode == GS4D_ROWS_GATHER)
            need(A - t.given_rows <= (has_append ? append.size(0) : 0), "rows_assemble: too few append indices");
    }
    if (K + A > 0) check(gs4d_rows_assemble(&b, (void *)stream_of(keep)), "rows_assemble");
    return out;
}

// ---- the fp32 block's input gradient: dh (P, W) = da (P, KW) @ W1 from W1^T (W, KW), f32 MFMA, fixed order
torch::Tensor mlp_dx_f32(const torch::Tensor &da, const torch::Tensor &w1t) {
    gpu_f32(da, "mlp_dx_f32: da");
    gpu_f32(w1t, "mlp_dx_f32: W1^T");
    need(da.dim() == 2 && w1t.dim() == 2 && w1t.size(1) == da.size(1), "mlp_dx_f32: da (P, KW), W1^T (W, KW)");
    c10::hip::HIPGuard guard(da.device().index());
    auto dh = torch::empty({da.size(0), w1t.size(0)}, da.options());
    check(gs4d_mlp_dx_f32((int)da.size(0), (int)da.size(1), (int)w1t.size(0), da.data_ptr<float>(), w1t.data_ptr<float>(),
                          dh.data_ptr<float>(), (void *)stream_of(da)),
          "mlp_dx_f32");
    return dh;
}

// ---- the fp32 block's first-layer weight gradient: dW1 (KW, W) = da^T h, f32 MFMA, fixed order
torch::Tensor mlp_dw_f32(const torch::Tensor &da, const torch::Tensor &h) {
    gpu_f32(da, "mlp_dw_f32: da");
    gpu_f32(h, "mlp_dw_f32: h");
    need(da.dim() == 2 && h.dim() == 2 && da.size(0) == h.size(0), "mlp_dw_f32: da (P, KW), h (P, W)");
    c10::hip::HIPGuard guard(da.device().index());
    const int P = (int)da.size(0), KW = (int)da.size(1), W = (int)h.size(1);
    auto dw = torch::empty({KW, W}, da.options());
    auto scratch = torch::empty({(int64_t)gs4d_mlp_dw_f32_scratch_bytes(P, KW, W)}, da.options().dtype(torch::kUInt8));
    check(gs4d_mlp_dw_f32(P, KW, W, da.data_ptr<float>(), h.data_ptr<float>(), dw.data_ptr<float>(), scratch.data_ptr(),
                          (void *)stream_of(da)),
          "mlp_dw_f32");
    return dw;
}

// ---- first deformation layer forward: h = relu(x W^T + b)
// with_hb: also h rounded to bf16 ((P, W) view of a (ceil(P/16)*16, W) buffer) for the bf16 heads block
std::vector<torch::Tensor> feature_relu_forward(const torch::Tensor &x, const torch::Tensor &w, const torch::Tensor &b,
                                                bool with_hb) {
    for (const torch::Tensor *t : std::initializer_list<const torch::Tensor *>{&x, &w, &b})
        gpu_f32(*t, "feature_relu_forward operand");
    need(x.is_contiguous() && w.is_contiguous() && b.is_contiguous() && x.dim() == 2 && w.dim() == 2 &&
             w.size(1) == x.size(1) && b.numel() == w.size(0),
         "feature_relu_forward: x (P, Fin), W (Fout, Fin), b (Fout), contiguous");
    c10::hip::HIPGuard guard(x.device().index());
    auto h = torch::empty({x.size(0), w.size(0)}, x.options());
    torch::Tensor hb;
    if (with_hb) hb = torch::empty({(x.size(0) + 15) / 16 * 16, w.size(0)}, x.options().dtype(torch::kBFloat16));
    check(gs4d_feature_relu_forward_hb((int)x.size(0), (int)x.size(1), (int)w.size(0), x.data_ptr<float>(),
                                       w.data_ptr<float>(), b.data_ptr<float>(), h.data_ptr<float>(),
                                       with_hb ? (uint16_t *)hb.data_ptr() : nullptr, (void *)stream_of(x)),
          "feature_relu_forward");
    if (with_hb) return {h, hb.narrow(0, 0, x.size(0))};
    return {h};
}

// ---- the field's input points: (pts (N, 4)) from xyz (N, 3+), t (N, 1+), aabb (2, 3); backward dxyz
torch::Tensor hexplane_points(const torch::Tensor &xyz, const torch::Tensor &t, const torch::Tensor &aabb_) {
    gpu_f32(xyz, "xyz");
    // t: (N, 1) float32 on the device, rows ld_t apart -- contiguous, or one value broadcast (stride 0)
    need(t.is_cuda() && t.scalar_type() == torch::kFloat32 && (t.is_contiguous() || t.stride(0) == 0),
         "hexplane_points: timestamps must be a float32 GPU tensor, contiguous or broadcast");
    need(xyz.dim() == 2 && xyz.size(1) >= 3 && xyz.stride(1) == 1 && t.dim() == 2 && t.size(0) == xyz.size(0),
         "hexplane_points: xyz (N, 3) with unit column stride, t (N, 1)");
    c10::hip::HIPGuard guard(xyz.device().index());
    auto aabb = aabb_.to(xyz.device(), torch::kFloat32).contiguous();
    need(aabb.numel() == 6, "hexplane_points: aabb (2, 3)");
    auto pts = torch::empty({xyz.size(0), 4}, xyz.options());
    check(gs4d_hexplane_points((int)xyz.size(0), xyz.data_ptr<float>(), xyz.stride(0), t.data_ptr<float>(), t.stride(0),
                               aabb.data_ptr<float>(), pts.data_ptr<float>(), (void *)stream_of(xyz)),
          "hexplane_points");
    return pts;
}
// add (optional): another (N, 3) gradient of xyz, summed in by the same pass
torch::Tensor hexplane_points_backward(const torch::Tensor &dpts_, const torch::Tensor &aabb_,
                                       const c10::optional<torch::Tensor> &add_) {
    auto dpts = dpts_.contiguous();
    gpu_f32(dpts, "dpts");
    need(dpts.dim() == 2 && dpts.size(1) == 4, "hexplane_points_backward: dpts (N, 4)");
    c10::hip::HIPGuard guard(dpts.device().index());
    auto aabb = aabb_.to(dpts.device(), torch::kFloat32).contiguous();
    torch::Tensor add;
    if (add_.has_value() && add_->defined()) {
        add = add_->to(torch::kFloat32).contiguous();
        need(add.is_cuda() && add.device() == dpts.device() && add.dim() == 2 && add.size(0) == dpts.size(0) &&
                 add.size(1) == 3,
             "hexplane_points_backward: add (N, 3) on dpts' device");
    }
    auto dxyz = torch::empty({dpts.size(0), 3}, dpts.options());
    check(gs4d_hexplane_points_backward_add((int)dpts.size(0), dpts.data_ptr<float>(), aabb.data_ptr<float>(),
                                            add.defined() ? add.data_ptr<float>() : nullptr, dxyz.data_ptr<float>(),
                                            (void *)stream_of(dpts)),
          "hexplane_points_backward");
    return dxyz;
}

// ---- plain f32 GEMMs of the deformation MLP on rocBLAS with a tuned kernel ------------------------------
// torch dispatches these f32 GEMMs to hipBLASLt, whose heuristic pick for the MLP's shapes runs at
// 100-125 TF/s of the 157 TF/s f32 peak; some rocBLAS (Tensile) kernels are 20-40 % faster on them
// (tools/tunableop_probe.sh, profiles/r03_tunableop_results.csv).  Which kernels exist, and their solution
// indices, depend on the rocBLAS build, so nothing is hard-coded: on the first call for a shape class,
// gemm_f32 asks rocBLAS for every solution that serves the problem (rocblas_gemm_ex_get_solutions /
// rocblas_gemm_strided_batched_ex_get_solutions), times each on the caller's stream (hipEvents; the library's
// own pick included as solution 0) and keeps the fastest for that class.  A class is the shape with its one
// large dimension (the point count, which densification changes every few hundred steps) rounded up to a
// 1/8-octave bucket, so a new point count reuses its bucket's kernel instead of re-tuning.  A cached kernel
// rocBLAS rejects for an exact shape is re-tuned for it.  Each choice is logged once (stderr) and readable
// through gemm_tuned().
// Column-major semantics: C (m x n) [+ i * sC] = op(A) op(B) for batch i, f32 inputs, f32 accumulation.
// One handle per (host thread, device, stream): the forward and the autograd engine's backward thread may both
// call in (rocblas_set_stream on a shared handle would race), GEMMs queued on two streams must not share a
// handle's workspace, and a default stream is the null handle on every device, so the device is part of the
// key.  Handles live for the process (a handful: one per thread and stream that ever ran a GEMM).
namespace {
struct HandleKey {
    int dev;
    hipStream_t st;
    bool operator==(const HandleKey &o) const { return dev == o.dev && st == o.st; }
};
struct HandleKeyHash {
    size_t operator()(const HandleKey &k) const {
        return std::hash<const void *>()((const void *)k.st) * 31u + (size_t)k.dev;
    }
};
rocblas_handle rocblas_for(const torch::Tensor &t) {
    static thread_local std::unordered_map<HandleKey, rocblas_handle, HandleKeyHash> handles;
    const int dev = t.device().index();
    const hipStream_t st = stream_of(t);
    const HandleKey key{dev, st};
    auto it = handles.find(key);
    if (it != handles.end()) return it->second;
    rocblas_handle h = nullptr;
    TORCH_CHECK(rocblas_create_handle(&h) == rocblas_status_success, "rocblas_create_handle");
    TORCH_CHECK(rocblas_set_stream(h, st) == rocblas_status_success, "rocblas_set_stream");
    // no kernel that sums split-K partials with atomics: the train step stays bitwise reproducible whichever
    // solution the tuner picks (rocBLAS leaves such kernels out of the candidates and its own choice)
    TORCH_CHECK(rocblas_set_atomics_mode(h, rocblas_atomics_not_allowed) == rocblas_status_success,
                "rocblas_set_atomics_mode");
    handles.emplace(key, h);
    return h;
}
// 1/8-octave bucket of a dimension: its upper end (so every size in a bucket maps to the same class)
int64_t dim_bucket(int64_t v) {
    if (v <= 64) return v;
    int e = 63 - __builtin_clzll((unsigned long long)v);  // 2^e <= v < 2^(e+1)
    const int64_t step = (int64_t)1 << (e - 3);
    return (v + step - 1) / step * step;
}
struct TunedGemm {
    int32_t solution = 0;  // 0: rocBLAS's own pick
    double us = 0, default_us = 0;
    int candidates = 0;
};
std::mutex g_tune_mu;
std::map<std::string, TunedGemm> g_tuned;  // class key -> choice (and exact keys of re-tuned shapes)
std::set<std::string> g_verified;          // exact shapes whose kernel's product was checked
}  // namespace

std::vector<std::tuple<std::string, int64_t, double, double, int64_t>> gemm_tuned() {
    std::lock_guard<std::mutex> lk(g_tune_mu);
    std::vector<std::tuple<std::string, int64_t, double, double, int64_t>> out;
    for (const auto &kv : g_tuned)
        out.emplace_back(kv.first, kv.second.solution, kv.second.us, kv.second.default_us, kv.second.candidates);
    return out;
}

// A and B may instead both be bf16 (the bf16 MLP path): bf16 products, f32 accumulation, f32 C.
// tune: true = the tuned kernel for the shape's class (first call of a class tunes it), false = rocBLAS's
// own pick.  Returns the solution index that ran (0 = rocBLAS's own pick).  The handles disallow atomics, so
// every candidate is deterministic.
int64_t gemm_f32(torch::Tensor A, torch::Tensor B, torch::Tensor C, bool ta, bool tb, int64_t m, int64_t n, int64_t k,
                 int64_t lda, int64_t ldb, int64_t ldc, int64_t batch, int64_t sA, int64_t sB, int64_t sC, bool tune) {
    const bool bf = A.scalar_type() == torch::kBFloat16;
    const auto ab_type = bf ? torch::kBFloat16 : torch::kFloat32;
    TORCH_CHECK(A.is_cuda() && B.is_cuda() && C.is_cuda() && A.scalar_type() == ab_type && B.scalar_type() == ab_type &&
                    C.scalar_type() == torch::kFloat32,
                "gemm_f32: A, B both f32 or both bf16, C f32 device tensors");
    const rocblas_datatype abt = bf ? rocblas_datatype_bf16_r : rocblas_datatype_f32_r;
    TORCH_CHECK(m > 0 && n > 0 && k > 0 && batch > 0 && m < INT32_MAX && n < INT32_MAX && k < INT32_MAX,
                "gemm_f32: sizes");
    // every element the call touches lies inside the tensors' storage
    auto span = [](const torch::Tensor &t, int64_t rows, int64_t cols, int64_t ld, int64_t stride, int64_t nb) {
        const int64_t last = (nb - 1) * stride + (cols - 1) * ld + rows;  // elements from data_ptr
        return t.storage_offset() + last <= (int64_t)(t.storage().nbytes() / t.element_size());
    };
    TORCH_CHECK(lda >= (ta ? k : m) && ldb >= (tb ? n : k) && ldc >= m, "gemm_f32: leading dimensions");
    TORCH_CHECK(span(A, ta ? k : m, ta ? m : k, lda, sA, batch) && span(B, tb ? n : k, tb ? k : n, ldb, sB, batch) &&
                    span(C, m, n, ldc, sC, batch),
                "gemm_f32: operands exceed their tensors");
    const c10::hip::HIPGuard guard(A.device().index());
    rocblas_handle h = rocblas_for(A);
    const hipStream_t stream = stream_of(A);
    const float one = 1.f, zero = 0.f;
    const rocblas_operation oa = ta ? rocblas_operation_transpose : rocblas_operation_none;
    const rocblas_operation ob = tb ? rocblas_operation_transpose : rocblas_operation_none;
    // no flags: rocblas_gemm_flags_check_solution_index would make the call only validate the index and return
    // without computing (an earlier tuner passed it and timed kernels that never ran)
    const uint32_t flags = rocblas_gemm_flags_none;
    auto run = [&](int32_t sol) {
        const rocblas_gemm_algo algo = sol ? rocblas_gemm_algo_solution_index : rocblas_gemm_algo_standard;
        if (batch == 1)
            return rocblas_gemm_ex(h, oa, ob, (int)m, (int)n, (int)k, &one, A.data_ptr(), abt, (int)lda, B.data_ptr(),
                                   abt, (int)ldb, &zero, C.data_ptr<float>(), rocblas_datatype_f32_r, (int)ldc,
                                   C.data_ptr<float>(), rocblas_datatype_f32_r, (int)ldc, rocblas_datatype_f32_r, algo,
                                   sol, sol ? flags : 0);
        return rocblas_gemm_strided_batched_ex(h, oa, ob, (int)m, (int)n, (int)k, &one, A.data_ptr(), abt, (int)lda,
                                               sA, B.data_ptr(), abt, (int)ldb, sB, &zero, C.data_ptr<float>(),
                                               rocblas_datatype_f32_r, (int)ldc, sC, C.data_ptr<float>(),
                                               rocblas_datatype_f32_r, (int)ldc, sC, (int)batch, rocblas_datatype_f32_r,
                                               algo, sol, sol ? flags : 0);
    };
    auto run_default = [&]() {
        const rocblas_status st = run(0);
        TORCH_CHECK(st == rocblas_status_success, "gemm_f32: rocBLAS status ", (int)st);
        return (int64_t)0;
    };
    if (!tune) return run_default();

    // the shape class: the large dimension (> 4096: the point count) bucketed, the others exact
    auto key_of = [&](bool exact) {
        auto d = [&](int64_t v) { return exact || v <= 4096 ? v : dim_bucket(v); };
        std::string key = std::string(bf ? "bf16" : "f32") + (ta ? " t" : " n") + (tb ? "t" : "n") + " m=" +
                          std::to_string(d(m)) + " n=" + std::to_string(d(n)) + " k=" + std::to_string(d(k)) +
                          " lda=" + std::to_string(d(lda)) + " ldb=" + std::to_string(d(ldb)) + " ldc=" +
                          std::to_string(d(ldc)) + " batch=" + std::to_string(batch) + " dev=" +
                          std::to_string(A.device().index());
        return exact ? key + " (exact)" : key;
    };
    const std::string ckey = key_of(false), xkey = key_of(true);
    {
        int32_t sol = -1;
        bool verified = false;
        {
            std::lock_guard<std::mutex> lk(g_tune_mu);
            auto it = g_tuned.find(xkey);
            if (it == g_tuned.end()) it = g_tuned.find(ckey);
            if (it != g_tuned.end()) {
                sol = it->second.solution;
                verified = g_verified.count(xkey) != 0;
            }
        }
        if (sol == 0) return run_default();
        if (sol != -1) {
            if (verified) {
                if (run(sol) == rocblas_status_success) return sol;
            } else {
                // the class's kernel on a shape it was not tuned on: checked once against rocBLAS's own pick
                run_default();
                const torch::Tensor ref = torch::from_blob(C.data_ptr<float>(), {batch, n, m},
                                                           {batch > 1 ? sC : 0, ldc, 1}, C.options()).clone();
                if (run(sol) == rocblas_status_success) {
                    const torch::Tensor got =
                        torch::from_blob(C.data_ptr<float>(), {batch, n, m}, {batch > 1 ? sC : 0, ldc, 1}, C.options());
                    const float err = (got - ref).abs().max().item<float>();
                    if (std::isfinite(err) && err <= 1e-4f * ref.abs().max().item<float>()) {
                        std::lock_guard<std::mutex> lk(g_tune_mu);
                        g_verified.insert(xkey);
                        return sol;
                    }
                }
            }
            // rejected or wrong for this exact shape: tune it below under its exact key
        }
    }
    // the candidates: every solution rocBLAS has for this exact problem
    std::vector<rocblas_int> sols;
    rocblas_int count = 0;
    auto list = [&](rocblas_int *arr, rocblas_int *sz) {
        if (batch == 1)
            return rocblas_gemm_ex_get_solutions(h, oa, ob, (int)m, (int)n, (int)k, &one, A.data_ptr(), abt, (int)lda,
                                                 B.data_ptr(), abt, (int)ldb, &zero, C.data_ptr<float>(),
                                                 rocblas_datatype_f32_r, (int)ldc, C.data_ptr<float>(),
                                                 rocblas_datatype_f32_r, (int)ldc, rocblas_datatype_f32_r,
                                                 rocblas_gemm_algo_solution_index, flags, arr, sz);
        return rocblas_gemm_strided_batched_ex_get_solutions(
            h, oa, ob, (int)m, (int)n, (int)k, &one, A.data_ptr(), abt, (int)lda, sA, B.data_ptr(), abt, (int)ldb, sB,
            &zero, C.data_ptr<float>(), rocblas_datatype_f32_r, (int)ldc, sC, C.data_ptr<float>(),
            rocblas_datatype_f32_r, (int)ldc, sC, (int)batch, rocblas_datatype_f32_r, rocblas_gemm_algo_solution_index,
            flags, arr, sz);
    };
    if (list(nullptr, &count) == rocblas_status_success && count > 0) {
        sols.resize((size_t)count);
        if (list(sols.data(), &count) != rocblas_status_success) count = 0;
        sols.resize((size_t)std::max<rocblas_int>(count, 0));
    }
    sols.insert(sols.begin(), 0);  // rocBLAS's own pick competes too
    // Every candidate's product is checked against rocBLAS's own pick: a candidate counts only when its result
    // matches to 1e-4 of the product's largest entry (a guard against a kernel that skips work or writes
    // nothing; an earlier version ran candidates with the check-only flag and timed calls that never computed).
    auto view = [&]() {
        return torch::from_blob(C.data_ptr<float>(), {batch, n, m}, {batch > 1 ? sC : 0, ldc, 1}, C.options());
    };
    TORCH_CHECK(run(0) == rocblas_status_success, "gemm_f32: rocBLAS's own kernel failed");
    const torch::Tensor ref = view().clone();
    const float ref_max = ref.abs().max().item<float>();
    float first_wrong = 0.f;  // the first rejected candidate's error (the log line's diagnostic)
    auto matches = [&]() {
        const float err = (view() - ref).abs().max().item<float>();
        const bool ok = std::isfinite(err) && err <= 1e-4f * ref_max;
        if (!ok && first_wrong == 0.f) first_wrong = std::isfinite(err) ? err : INFINITY;
        return ok;
    };
    hipEvent_t e0, e1;
    TORCH_CHECK(hipEventCreate(&e0) == hipSuccess && hipEventCreate(&e1) == hipSuccess, "gemm_f32: hipEventCreate");
    auto time_of = [&](int32_t sol, int reps) -> double {
        if (run(sol) != rocblas_status_success) return -1.0;  // warm-up (and the validity check)
        (void)hipEventRecord(e0, stream);
        for (int r = 0; r < reps; r++) run(sol);
        (void)hipEventRecord(e1, stream);
        (void)hipEventSynchronize(e1);
        float ms = 0.f;
        (void)hipEventElapsedTime(&ms, e0, e1);
        return 1e3 * ms / reps;
    };
    TunedGemm best;
    best.solution = 0;
    best.us = 1e30;
    int wrong = 0;
    for (const rocblas_int sol : sols) {
        // a kernel that writes nothing fails (a finite poison, so the log can report by how much)
        if (sol != 0) view().fill_(3.0e38f);
        double us = time_of(sol, 1);
        if (us < 0) continue;
        if (sol != 0 && !matches()) {
            wrong++;
            continue;
        }
        if (us < 1.5 * best.us) us = std::min(us, time_of(sol, 3));  // a contender: a steadier measurement
        if (sol == 0) best.default_us = us;
        if (us < best.us) {
            best.us = us;
            best.solution = sol;
        }
        best.candidates++;
    }
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    TORCH_CHECK(best.candidates > 0, "gemm_f32: no rocBLAS solution ran for ", xkey);
    bool rejected;
    {
        std::lock_guard<std::mutex> lk(g_tune_mu);
        rejected = g_tuned.count(ckey) != 0;  // the class's kernel did not serve this exact shape
        g_tuned[rejected ? xkey : ckey] = best;
        g_verified.insert(xkey);
    }
    fprintf(stderr,
            "gs4d gemm_f32: tuned %s: solution %d at %.1f us (rocBLAS's own pick %.1f us; %d candidates, %d with a "
            "wrong product, first error %.3g of max %.3g)\n",
            (rejected ? xkey : ckey).c_str(), best.solution, best.us, best.default_us, best.candidates, wrong,
            (double)first_wrong, (double)ref_max);
    // the result of the chosen kernel (the timing runs wrote C too, but leave no doubt which one did last)
    if (best.solution == 0) return run_default();
    TORCH_CHECK(run(best.solution) == rocblas_status_success, "gemm_f32: tuned solution failed");
    return best.solution;
}

// out[i] = sum over s of parts[s][i], s in order (a split-K GEMM's partials)
torch::Tensor sum_slices(torch::Tensor parts) {
    TORCH_CHECK(parts.is_cuda() && parts.scalar_type() == torch::kFloat32 && parts.is_contiguous() && parts.dim() >= 2,
                "sum_slices: contiguous f32 (S, ...) device tensor");
    const c10::hip::HIPGuard guard(parts.device().index());
    auto out = torch::empty(parts.sizes().slice(1), parts.options());
    const int64_t n = out.numel();
    check(gs4d_sum_slices(parts.data_ptr<float>(), (int)parts.size(0), n, out.data_ptr<float>(), stream_of(parts)),
          "gs4d_sum_slices");
    return out;
}

PYBIND11_MODULE(_C, m) {
    m.def("hexplane_points", &hexplane_points);
    m.def("hexplane_points_backward", &hexplane_points_backward, py::arg("dpts"), py::arg("aabb"),
          py::arg("add") = py::none());
    m.def("feature_relu_forward", &feature_relu_forward, py::arg("x"), py::arg("w"), py::arg("b"),
          py::arg("with_hb") = false);
    m.def("heads_forward", &heads_forward);
    m.def("heads_block_forward", &heads_block_forward);
    m.def("heads_block_forward_bf16", &heads_block_forward_bf16, py::arg("h"), py::arg("w1"), py::arg("b1"),
          py::arg("w2"), py::arg("b2"), py::arg("hb") = py::none());
    m.def("mlp_dx_bf16", &mlp_dx_bf16);
    m.def("mlp_dw_bf16", &mlp_dw_bf16);
    m.def("rows_assemble", &rows_assemble);
    m.def("mlp_dx_f32", &mlp_dx_f32);
    m.def("mlp_dw_f32", &mlp_dw_f32);
    m.def("feature_relu_backward", &feature_relu_backward);
    m.def("heads_backward", &heads_backward);
    m.def("linear_dw", &linear_dw);
    m.def("gemm_f32", &gemm_f32);
    m.def("gemm_tuned", &gemm_tuned);
    m.def("sum_slices", &sum_slices);
    m.def("hexplane_reg_forward", &hexplane_reg_forward);
    m.def("hexplane_reg_backward", &hexplane_reg_backward);
    m.def("hexplane_reg_accumulate", &hexplane_reg_accumulate, py::arg("planes"), py::arg("grads"), py::arg("w_smooth"),
          py::arg("w_l1"), py::arg("dloss"), py::arg("with_value") = false, py::arg("base") = py::none());
    m.def("deform_tail_forward", &deform_tail_forward);
    m.def("deform_tail_backward", &deform_tail_backward);
    m.def("hexplane_forward", &hexplane_forward, py::arg("pts"), py::arg("planes"), py::arg("order") = py::none());
    m.def("hexplane_backward", &hexplane_backward, py::arg("pts"), py::arg("planes"), py::arg("packed"),
          py::arg("dfeat"), py::arg("order"), py::arg("deterministic") = true);
    m.def("l1_forward", &l1_forward);
    m.def("l1_backward", &l1_backward);
    m.def("l1_loss_grad", &l1_loss_grad);
    m.def("densify_stats", &densify_stats);
    m.def("adam_step", &adam_step);
    m.def("version", []() { return std::string(gs4d_version()); });
}
