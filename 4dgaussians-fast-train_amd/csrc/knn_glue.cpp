// knn_glue.cpp -- the `simple_knn._C` extension module: distCUDA2 over the libgs4d C ABI.
//
// Mirrors submodules/simple-knn/spatial.cu:15-25 and ext.cpp:15-16: distCUDA2(points (P,3) float32)
// returns a (P,) float32 tensor of mean squared 3-NN distances on the points' device.  Launches go to
// the current HIP stream; CPU tensors raise (there is no CPU path).
#include <ATen/ATen.h>
#include <c10/hip/HIPGuard.h>
#include <c10/hip/HIPStream.h>
#include <torch/extension.h>

#include <string>

#include "../../include/gs4d.h"

namespace {
struct Scratch {
    torch::Tensor t;
};
char *alloc_cb(void *ctx, size_t n) {
    auto *s = static_cast<Scratch *>(ctx);
    s->t.resize_({(long long)n});
    return reinterpret_cast<char *>(s->t.data_ptr());
}
}  // namespace

torch::Tensor distCUDA2(const torch::Tensor &points) {
    if (points.ndimension() != 2 || points.size(1) != 3) throw std::runtime_error("points must have dimensions (num_points, 3)");
    if (!points.is_cuda()) throw std::runtime_error("points must be a HIP (GPU) tensor; simple_knn has no CPU path");
    const int P = (int)points.size(0);
    c10::hip::HIPGuard guard(points.device().index());
    torch::Tensor pts = points.to(torch::kFloat32).contiguous();
    torch::Tensor means = torch::full({P}, 0.0, pts.options());  // spatial.cu:20-21
    if (P == 0) return means;
    Scratch scratch{torch::empty({0}, pts.options().dtype(torch::kUInt8))};
    hipStream_t stream = c10::hip::getCurrentHIPStream(points.device().index()).stream();
    int st = gs4d_knn_mean_dist(P, pts.data_ptr<float>(), means.data_ptr<float>(), alloc_cb, &scratch, (void *)stream);
    if (st != GS4D_OK) throw std::runtime_error(std::string("distCUDA2: ") + gs4d_last_error());
    return means;
}

PYBIND11_MODULE(_C, m) { m.def("distCUDA2", &distCUDA2); }
