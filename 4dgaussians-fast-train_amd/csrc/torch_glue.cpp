// torch_glue.cpp -- the `_C` extension module: PyTorch-ROCm tensors -> libgs4d C ABI.
//
// Mirrors the reference's torch glue rasterize_points.cu:27-219 and its pybind table ext.cpp:15-18:
// same function names, positional arguments, return tuples and error behaviour (RuntimeError for
// AT_ERROR / runtime_error paths).  Differences: launches go to the *current* HIP stream instead of
// the legacy default stream; inputs must live on the GPU (there is no CPU fallback in the product
// path -- CPU tensors raise); gradient outputs are allocated uninitialised because libgs4d writes
// every element.
#include <ATen/ATen.h>
#include <c10/hip/HIPStream.h>
#include <c10/hip/HIPGuard.h>
#include <torch/extension.h>

#include <functional>
#include <string>
#include <tuple>

#include "../../include/gs4d.h"

namespace {

struct Resizer {
    torch::Tensor *t;
};
// rasterize_points.cu:27-33 resizeFunctional as a C callback.  The buffers start empty and are sized once per
// call, so a fresh allocation stands in for resize_ (same result; resize_ took ~8 us of host time per buffer)
char *resize_cb(void *ctx, size_t n) {
    auto *r = static_cast<Resizer *>(ctx);
    if (r->t->numel() == 0)
        *r->t = torch::empty({(long long)n}, r->t->options());
    else
        r->t->resize_({(long long)n});
    return reinterpret_cast<char *>(r->t->data_ptr());
}

void check_status(int st, const char *what) {
    if (st != GS4D_OK) throw std::runtime_error(std::string(what) + ": " + gs4d_last_error());
}

// Empty tensor -> nullptr (the reference's convention, rasterize_points.cu:95-106).
// Non-empty tensors must be float32 on the current HIP device; returns a contiguous, 16-byte
// aligned tensor that the caller keeps alive for the duration of the call.
torch::Tensor prep(const torch::Tensor &t, const char *name, const torch::Device &dev) {
    if (t.numel() == 0) return t;
    if (!t.is_cuda()) throw std::runtime_error(std::string(name) + " must be a HIP (GPU) tensor; the MI355X rasterizer has no CPU path");
    if (t.device() != dev) throw std::runtime_error(std::string(name) + " is on a different device than means3D");
    if (t.scalar_type() != torch::kFloat32) throw std::runtime_error(std::string(name) + " must be float32");
    torch::Tensor c = t.contiguous();
    if ((reinterpret_cast<uintptr_t>(c.data_ptr()) & 15) != 0) c = c.clone();
    return c;
}
const float *fptr(const torch::Tensor &t) { return t.numel() ? t.data_ptr<float>() : nullptr; }

// The view matrix as the reference's callers pass it: world_view_transform is a transposed 4x4 view
// (strides (1, 4)); such a matrix is read in place by the kernels (view_transposed = 1) instead of
// being copied by .contiguous().  Anything else goes through prep().
torch::Tensor prep_view(const torch::Tensor &t, const torch::Device &dev, int &transposed) {
    transposed = 0;
    if (t.numel() == 16 && t.dim() >= 2 && t.size(-1) == 4 && t.size(-2) == 4 && t.stride(-1) == 4 &&
        t.stride(-2) == 1 && t.is_cuda() && t.device() == dev && t.scalar_type() == torch::kFloat32 &&
        (reinterpret_cast<uintptr_t>(t.data_ptr()) & 15) == 0) {
        transposed = 1;
        return t;
    }
    return prep(t, "viewmatrix", dev);
}

}  // namespace

// rasterize_points.cu:35-117
std::tuple<int, torch::Tensor, torch::Tensor, torch::Tensor, torch::Tensor, torch::Tensor, torch::Tensor>
RasterizeGaussians(const torch::Tensor &background, const torch::Tensor &means3D, const torch::Tensor &colors,
                   const torch::Tensor &opacity, const torch::Tensor &scales, const torch::Tensor &rotations,
                   const float scale_modifier, const torch::Tensor &cov3D_precomp, const torch::Tensor &viewmatrix,
                   const torch::Tensor &projmatrix, const float tan_fovx, const float tan_fovy, const int image_height,
                   const int image_width, const torch::Tensor &sh, const int degree, const torch::Tensor &campos,
                   const bool prefiltered, const bool debug) {
    if (means3D.ndimension() != 2 || means3D.size(1) != 3) {
        AT_ERROR("means3D must have dimensions (num_points, 3)");
    }
    if (!means3D.is_cuda()) throw std::runtime_error("means3D must be a HIP (GPU) tensor; the MI355X rasterizer has no CPU path");
    const auto dev = means3D.device();
    c10::hip::HIPGuard guard(dev.index());
    const int P = means3D.size(0);
    const int H = image_height;
    const int W = image_width;
    auto float_opts = means3D.options().dtype(torch::kFloat32);
    auto byte_opts = means3D.options().dtype(torch::kByte);

    torch::Tensor geomBuffer = torch::empty({0}, byte_opts);
    torch::Tensor binningBuffer = torch::empty({0}, byte_opts);
    torch::Tensor imgBuffer = torch::empty({0}, byte_opts);
    torch::Tensor radii = torch::empty({P}, means3D.options().dtype(torch::kInt32));
    if (P == 0) {
        // the reference returns zero images when there is nothing to draw (forward never runs)
        return std::make_tuple(0, torch::zeros({3, H, W}, float_opts), torch::zeros({1, H, W}, float_opts), radii,
                               geomBuffer, binningBuffer, imgBuffer);
    }
    torch::Tensor out_color = torch::empty({3, H, W}, float_opts);
    torch::Tensor out_depth = torch::empty({1, H, W}, float_opts);

    int M = 0;
    if (sh.size(0) != 0) M = sh.size(1);
    auto bg = prep(background, "bg", dev), m3 = prep(means3D, "means3D", dev), col = prep(colors, "colors_precomp", dev),
         op = prep(opacity, "opacities", dev), sc = prep(scales, "scales", dev), rot = prep(rotations, "rotations", dev),
         c3 = prep(cov3D_precomp, "cov3D_precomp", dev), pm = prep(projmatrix, "projmatrix", dev),
         shc = prep(sh, "sh", dev), cp = prep(campos, "campos", dev);
    int vt = 0;
    auto vm = prep_view(viewmatrix, dev, vt);

    Resizer rg{&geomBuffer}, rb{&binningBuffer}, ri{&imgBuffer};
    hipStream_t stream = c10::hip::getCurrentHIPStream(dev.index()).stream();
    int rendered = 0;
    int st = gs4d_forward_ex(resize_cb, &rg, resize_cb, &rb, resize_cb, &ri, P, degree, M, fptr(bg), W, H, fptr(m3),
                             fptr(shc), fptr(col), fptr(op), fptr(sc), scale_modifier, fptr(rot), fptr(c3), fptr(vm),
                             fptr(pm), fptr(cp), tan_fovx, tan_fovy, prefiltered ? 1 : 0, out_color.data_ptr<float>(),
                             out_depth.data_ptr<float>(), radii.data_ptr<int>(), debug ? 1 : 0, (void *)stream,
                             &rendered, vt);
    check_status(st, "rasterize_gaussians");
    return std::make_tuple(rendered, out_color, out_depth, radii, geomBuffer, binningBuffer, imgBuffer);
}

// rasterize_points.cu:119-198
std::tuple<torch::Tensor, torch::Tensor, torch::Tensor, torch::Tensor, torch::Tensor, torch::Tensor, torch::Tensor,
           torch::Tensor>
RasterizeGaussiansBackward(const torch::Tensor &background, const torch::Tensor &means3D, const torch::Tensor &radii,
                           const torch::Tensor &colors, const torch::Tensor &scales, const torch::Tensor &rotations,
                           const float scale_modifier, const torch::Tensor &cov3D_precomp,
                           const torch::Tensor &viewmatrix, const torch::Tensor &projmatrix, const float tan_fovx,
                           const float tan_fovy, const torch::Tensor &dL_dout_color, const torch::Tensor &sh,
                           const int degree, const torch::Tensor &campos, const torch::Tensor &geomBuffer, const int R,
                           const torch::Tensor &binningBuffer, const torch::Tensor &imageBuffer, const bool debug) {
    if (!means3D.is_cuda()) throw std::runtime_error("means3D must be a HIP (GPU) tensor; the MI355X rasterizer has no CPU path");
    const auto dev = means3D.device();
    c10::hip::HIPGuard guard(dev.index());
    const int P = means3D.size(0);
    const int H = dL_dout_color.size(1);
    const int W = dL_dout_color.size(2);
    int M = 0;
    if (sh.size(0) != 0) M = sh.size(1);
    auto opts = means3D.options().dtype(torch::kFloat32);
    torch::Tensor dL_dmeans3D = torch::empty({P, 3}, opts);
    torch::Tensor dL_dmeans2D = torch::empty({P, 3}, opts);
    torch::Tensor dL_dcolors = torch::empty({P, 3}, opts);
    torch::Tensor dL_dopacity = torch::empty({P, 1}, opts);
    torch::Tensor dL_dcov3D = torch::empty({P, 6}, opts);
    torch::Tensor dL_dsh = torch::empty({P, M, 3}, opts);
    torch::Tensor dL_dscales = torch::empty({P, 3}, opts);
    torch::Tensor dL_drotations = torch::empty({P, 4}, opts);
    if (P != 0) {
        auto bg = prep(background, "bg", dev), m3 = prep(means3D, "means3D", dev), col = prep(colors, "colors_precomp", dev),
             sc = prep(scales, "scales", dev), rot = prep(rotations, "rotations", dev),
             c3 = prep(cov3D_precomp, "cov3D_precomp", dev), pm = prep(projmatrix, "projmatrix", dev),
             dl = prep(dL_dout_color, "grad_out_color", dev), shc = prep(sh, "sh", dev),
             cp = prep(campos, "campos", dev);
        int vt = 0;
        auto vm = prep_view(viewmatrix, dev, vt);
        torch::Tensor rad = radii.contiguous();
        if (rad.numel() && (rad.scalar_type() != torch::kInt32 || !rad.is_cuda()))
            throw std::runtime_error("radii must be an int32 GPU tensor");
        torch::Tensor scratch = torch::empty({0}, means3D.options().dtype(torch::kByte));
        Resizer rs{&scratch};
        hipStream_t stream = c10::hip::getCurrentHIPStream(dev.index()).stream();
        int st = gs4d_backward_ex(
            P, degree, M, R, fptr(bg), W, H, fptr(m3), fptr(shc), fptr(col), fptr(sc), scale_modifier, fptr(rot),
            fptr(c3), fptr(vm), fptr(pm), fptr(cp), tan_fovx, tan_fovy, rad.numel() ? rad.data_ptr<int>() : nullptr,
            reinterpret_cast<char *>(geomBuffer.data_ptr()),
            binningBuffer.numel() ? reinterpret_cast<char *>(binningBuffer.data_ptr()) : nullptr,
            reinterpret_cast<char *>(imageBuffer.data_ptr()), fptr(dl), dL_dmeans2D.data_ptr<float>(), nullptr,
            dL_dopacity.data_ptr<float>(), dL_dcolors.data_ptr<float>(), dL_dmeans3D.data_ptr<float>(),
            dL_dcov3D.data_ptr<float>(), M ? dL_dsh.data_ptr<float>() : nullptr, dL_dscales.data_ptr<float>(),
            dL_drotations.data_ptr<float>(), resize_cb, &rs, debug ? 1 : 0, (void *)stream, vt);
        check_status(st, "rasterize_gaussians_backward");
    }
    return std::make_tuple(dL_dmeans2D, dL_dcolors, dL_dopacity, dL_dmeans3D, dL_dcov3D, dL_dsh, dL_dscales,
                           dL_drotations);
}

// rasterize_points.cu:200-219
torch::Tensor MarkVisible(torch::Tensor &means3D, torch::Tensor &viewmatrix, torch::Tensor &projmatrix) {
    const int P = means3D.size(0);
    torch::Tensor present = torch::full({P}, false, means3D.options().dtype(at::kBool));
    if (P != 0) {
        if (!means3D.is_cuda()) throw std::runtime_error("means3D must be a HIP (GPU) tensor; the MI355X rasterizer has no CPU path");
        const auto dev = means3D.device();
        c10::hip::HIPGuard guard(dev.index());
        auto m3 = prep(means3D, "means3D", dev), pm = prep(projmatrix, "projmatrix", dev);
        int vt = 0;
        auto vm = prep_view(viewmatrix, dev, vt);
        hipStream_t stream = c10::hip::getCurrentHIPStream(dev.index()).stream();
        int st = gs4d_mark_visible_ex(P, fptr(m3), fptr(vm), fptr(pm),
                                      reinterpret_cast<uint8_t *>(present.data_ptr<bool>()), (void *)stream, vt);
        check_status(st, "mark_visible");
    }
    return present;
}

static std::vector<std::tuple<std::string, float>> last_timings() {
    const char *names[64];
    float ms[64];
    int n = gs4d_last_timings(names, ms, 64);
    std::vector<std::tuple<std::string, float>> out;
    for (int i = 0; i < n && i < 64; i++) out.emplace_back(names[i], ms[i]);
    return out;
}

// ext.cpp:15-18 plus three introspection helpers used by bench.py
// parity-test diagnostic: (o G, log2 G) of (Gaussian, pixel) pairs by the blend kernels' arithmetic
std::tuple<torch::Tensor, torch::Tensor> DebugPairAlpha(const torch::Tensor &geomBuffer, int P, int W, int H,
                                                        const torch::Tensor &gid_, const torch::Tensor &px_,
                                                        const torch::Tensor &py_) {
    TORCH_CHECK(geomBuffer.is_cuda() && gid_.is_cuda(), "debug_pair_alpha: device tensors");
    const c10::hip::HIPGuard guard(geomBuffer.device().index());
    auto gid = gid_.to(torch::kInt32).contiguous(), px = px_.to(torch::kInt32).contiguous(),
         py = py_.to(torch::kInt32).contiguous();
    TORCH_CHECK(gid.numel() == px.numel() && gid.numel() == py.numel(), "debug_pair_alpha: pair arrays differ");
    TORCH_CHECK(gid.numel() == 0 || (gid.min().item<int>() >= 0 && gid.max().item<int>() < P &&
                                     px.min().item<int>() >= 0 && py.min().item<int>() >= 0),
                "debug_pair_alpha: pair out of range");
    auto og = torch::empty({gid.numel()}, geomBuffer.options().dtype(torch::kFloat32));
    auto pw = torch::empty_like(og);
    const int st = gs4d_debug_pair_alpha(P, W, H, (const char *)geomBuffer.data_ptr(), (int)gid.numel(),
                                         gid.data_ptr<int>(), px.data_ptr<int>(), py.data_ptr<int>(),
                                         og.data_ptr<float>(), pw.data_ptr<float>(),
                                         c10::hip::getCurrentHIPStream(geomBuffer.device().index()).stream());
    TORCH_CHECK(st == 0, "debug_pair_alpha: ", gs4d_last_error());
    return {og, pw};
}

PYBIND11_MODULE(_C, m) {
    m.def("rasterize_gaussians", &RasterizeGaussians);
    m.def("debug_pair_alpha", &DebugPairAlpha);
    m.def("rasterize_gaussians_backward", &RasterizeGaussiansBackward);
    m.def("mark_visible", &MarkVisible);
    m.def("set_profiling", [](int level) { gs4d_set_profiling(level); });
    m.def("last_timings", &last_timings);
    m.def("version", []() { return std::string(gs4d_version()); });
}
