// train_tail.hip -- the train step after the rasterizer: fused L1 loss, the
// densification statistics and a multi-tensor Adam.
//
// Reference: utils/loss_utils.py:20-21 (l1_loss) with the L1 gradient torch's autograd derives
// (sign(x - y) / N), train.py:346-349 + scene/gaussian_model.py:521-523 (densification statistics),
// and torch.optim.Adam as configured by scene/gaussian_model.py:184 (betas (0.9, 0.999), eps 1e-15,
// no weight decay, no amsgrad), in the element-wise form of torch's multi-tensor ("foreach") path.
//
// All three are HBM-bound streams; each is ONE pass over its data where torch runs several:
//   l1:     reads x, y once, writes a 1-byte sign per element and one partial sum per workgroup;
//           a second launch sums the partials in a fixed order (deterministic loss); the backward
//           expands sign * (dL/dloss / N) (1 byte in, 4 bytes out per element);
//   adam:   per element reads p, g, m, v and writes p, m, v (28 bytes) for EVERY parameter tensor of
//           the model in one launch (tensor descriptors passed by value, chunk -> tensor lookup);
//   stats:  per Gaussian reads the viewspace gradient, visibility and radius and updates the three
//           accumulators in place.
#include <math.h>

#include "../../include/gs4d_train.h"
#include "gs4d_internal.h"

namespace gs4d {

constexpr int kTailThreads = 256;
constexpr int kL1PerThread = 8;
constexpr int kL1Chunk = kTailThreads * kL1PerThread;

__global__ __launch_bounds__(kTailThreads) void l1_partial_kernel(int64_t n, const float *__restrict__ x,
                                                                  const float *__restrict__ y,
                                                                  int8_t *__restrict__ sign, double *__restrict__ part) {
    const int64_t base = (int64_t)blockIdx.x * kL1Chunk;
    float acc = 0.f;
#pragma unroll
    for (int k = 0; k < kL1PerThread; k++) {
        const int64_t i = base + (int64_t)k * kTailThreads + threadIdx.x;
        if (i < n) {
            const float d = x[i] - y[i];
            acc += fabsf(d);
            sign[i] = (int8_t)((d > 0.f) - (d < 0.f));  // torch.sign; |x| has subgradient 0 at 0
        }
    }
    double s = acc;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off);
    __shared__ double s_w[kTailThreads / 64];
    if ((threadIdx.x & 63) == 0) s_w[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        double t = 0.0;
#pragma unroll
        for (int w = 0; w < kTailThreads / 64; w++) t += s_w[w];
        part[blockIdx.x] = t;
    }
}

__global__ __launch_bounds__(kTailThreads) void l1_final_kernel(int nblk, int64_t n, const double *__restrict__ part,
                                                                float *__restrict__ loss) {
    double s = 0.0;
    for (int i = threadIdx.x; i < nblk; i += kTailThreads) s += part[i];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off);
    __shared__ double s_w[kTailThreads / 64];
    if ((threadIdx.x & 63) == 0) s_w[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        double t = 0.0;
#pragma unroll
        for (int w = 0; w < kTailThreads / 64; w++) t += s_w[w];
        *loss = (float)(t / (double)n);
    }
}

__global__ __launch_bounds__(kTailThreads) void l1_backward_kernel(int64_t n, const int8_t *__restrict__ sign,
                                                                   const float *__restrict__ dloss,
                                                                   float *__restrict__ grad) {
    const float scale = *dloss / (float)n;  // d mean / dx = sign / N, times the upstream gradient
    for (int64_t i = (int64_t)blockIdx.x * kTailThreads + threadIdx.x; i < n; i += (int64_t)gridDim.x * kTailThreads)
        grad[i] = (float)sign[i] * scale;
}

// ---- densification statistics ------------------------------------------------------------------
__global__ __launch_bounds__(kTailThreads) void densify_stats_kernel(int P, const float *__restrict__ vs_grad,
                                                                     const uint8_t *__restrict__ visible,
                                                                     const int *__restrict__ radii,
                                                                     float *__restrict__ grad_accum,
                                                                     float *__restrict__ denom,
                                                                     float *__restrict__ max_radii) {
    const int i = blockIdx.x * kTailThreads + threadIdx.x;
    if (i >= P || !visible[i]) return;
    if (radii) max_radii[i] = fmaxf(max_radii[i], (float)radii[i]);  // train.py:348
    const float gx = vs_grad[3 * (size_t)i], gy = vs_grad[3 * (size_t)i + 1];
    grad_accum[i] += sqrtf(gx * gx + gy * gy);  // gaussian_model.py:522 torch.norm(grad[:, :2])
    denom[i] += 1.f;                            // gaussian_model.py:523
}

// ---- multi-tensor Adam --------------------------------------------------------------------------
constexpr int kAdamChunk = 4096;  // elements per workgroup

__global__ __launch_bounds__(kTailThreads) void adam_kernel(gs4d_adam_batch batch) {
    // chunk -> tensor: the descriptors carry their first chunk index (few dozen tensors: linear scan)
    const int64_t c = blockIdx.x;
    int t = 0;
    while (t + 1 < batch.count && batch.t[t + 1].first_chunk <= c) t++;
    const gs4d_adam_tensor d = batch.t[t];
    const int64_t base = (c - d.first_chunk) * kAdamChunk;
    const float b1 = batch.beta1, omb1 = batch.one_minus_beta1, b2 = batch.beta2, omb2 = batch.one_minus_beta2;
    const float eps = batch.eps, step_size = d.neg_step_size, bc2 = d.bias_correction2_sqrt;
    (void)b1;
    for (int k = threadIdx.x; k < kAdamChunk; k += kTailThreads) {
        const int64_t i = base + k;
        if (i >= d.n) break;
        const float g = d.grad[i];
        float m = d.exp_avg[i], v = d.exp_avg_sq[i];
        // exp_avg.lerp_(grad, 1 - beta1): weight < 0.5 -> self + weight * (end - self)
        m = fmaf(omb1, g - m, m);
        // exp_avg_sq.mul_(beta2).addcmul_(grad, grad, value=1 - beta2)
        v = v * b2;
        v = fmaf(omb2, g * g, v);
        // denom = exp_avg_sq.sqrt() / bias_correction2_sqrt + eps; param.addcdiv_(exp_avg, denom, -step_size)
        const float den = sqrtf(v) / bc2 + eps;
        d.param[i] = fmaf(step_size, m / den, d.param[i]);
        d.exp_avg[i] = m;
        d.exp_avg_sq[i] = v;
    }
}

}  // namespace gs4d

using namespace gs4d;

extern "C" {

size_t gs4d_l1_scratch_bytes(int64_t n) { return 8 * (size_t)((n + kL1Chunk - 1) / kL1Chunk) + 256; }

int gs4d_l1_loss_forward(int64_t n, const float *x, const float *y, int8_t *sign, float *loss, void *scratch,
                         void *stream) {
    if (n < 0 || (n > 0 && (!x || !y || !sign || !scratch)) || !loss) return 1;
    hipStream_t s = (hipStream_t)stream;
    if (n == 0) return hipMemsetAsync(loss, 0, 4, s) == hipSuccess ? 0 : 3;
    const int nblk = (int)((n + kL1Chunk - 1) / kL1Chunk);
    double *part = (double *)align_up((size_t)scratch, 8);
    hipLaunchKernelGGL(l1_partial_kernel, dim3(nblk), dim3(kTailThreads), 0, s, n, x, y, sign, part);
    hipLaunchKernelGGL(l1_final_kernel, dim3(1), dim3(kTailThreads), 0, s, nblk, n, part, loss);
    return hipGetLastError() == hipSuccess ? 0 : 3;
}

int gs4d_l1_loss_backward(int64_t n, const int8_t *sign, const float *dloss, float *grad, void *stream) {
    if (n < 0 || (n > 0 && (!sign || !dloss || !grad))) return 1;
    if (n == 0) return 0;
    const int nblk = (int)std::min<int64_t>((n + kTailThreads - 1) / kTailThreads, 8192);
    hipLaunchKernelGGL(l1_backward_kernel, dim3(nblk), dim3(kTailThreads), 0, (hipStream_t)stream, n, sign, dloss, grad);
    return hipGetLastError() == hipSuccess ? 0 : 3;
}

int gs4d_densify_stats(int P, const float *viewspace_grad, const uint8_t *visible, const int *radii, float *grad_accum,
                       float *denom, float *max_radii, void *stream) {
    if (P < 0 || (P > 0 && (!viewspace_grad || !visible || !grad_accum || !denom || (radii && !max_radii)))) return 1;
    if (P == 0) return 0;
    hipLaunchKernelGGL(densify_stats_kernel, dim3((P + kTailThreads - 1) / kTailThreads), dim3(kTailThreads), 0,
                       (hipStream_t)stream, P, viewspace_grad, visible, radii, grad_accum, denom, max_radii);
    return hipGetLastError() == hipSuccess ? 0 : 3;
}

int64_t gs4d_adam_chunks(int64_t n) { return (n + kAdamChunk - 1) / kAdamChunk; }

int gs4d_adam_step(const gs4d_adam_batch *batch, void *stream) {
    if (!batch || batch->count < 0 || batch->count > GS4D_ADAM_MAX_TENSORS) return 1;
    int64_t chunks = 0;
    for (int i = 0; i < batch->count; i++) {
        if (batch->t[i].first_chunk != chunks || batch->t[i].n < 0) return 1;
        chunks += gs4d_adam_chunks(batch->t[i].n);
    }
    if (chunks == 0) return 0;
    hipLaunchKernelGGL(adam_kernel, dim3((unsigned)chunks), dim3(kTailThreads), 0, (hipStream_t)stream, *batch);
    return hipGetLastError() == hipSuccess ? 0 : 3;
}

}  // extern "C"
