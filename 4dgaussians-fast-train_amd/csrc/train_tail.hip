// train_tail.hip -- the train step after the rasterizer: fused L1 loss, the
// densification statistics, a multi-tensor Adam and the HexPlane regularisers.
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
//           accumulators in place;
//   reg:    the 12 planes' smoothness + L1 terms (scene/gaussian_model.py:538-577), which torch runs as
//           ~100 slice / sub / square / mean kernels forward and their slice-backward zero-fills
//           backward: one launch per direction over every plane (plus one fixed-order final sum).
#include <math.h>

#include <algorithm>
#include <type_traits>
#include <cstdlib>

#include "../../include/gs4d_train.h"
#include "gs4d_internal.h"

namespace gs4d {

constexpr int kTailThreads = 256;
constexpr int kL1PerThread = 8;
constexpr int kL1Chunk = kTailThreads * kL1PerThread;

// ---- last-workgroup totals ------------------------------------------------------------------------
// A sum over a grid's per-workgroup partials without a second launch.  Each workgroup publishes its partial
// in its slot (agent-scope relaxed atomic store: coherent across the XCDs' L2s) and draws a ticket; the
// workgroup that draws the last ticket reads every slot and sums them in a fixed order -- thread-strided, then
// the wave tree, then the waves in order: the order of the separate one-workgroup final kernels these replace,
// so totals are unchanged bit for bit -- then puts every slot and ticket back to 0 for the next call.
// Tickets in two levels: workgroup b draws from sub-counter b % kTicketFan (each on its own 128-byte line),
// the last drawer of a sub-counter from the top counter -- one counter drawn by ~2000 workgroups serialised
// its atomics (~10 ns each, ~20 us per launch here).  No fences: an acquire/release pair at agent scope
// writes back the whole L2 in every workgroup (buffer_wbl2; ~70 us per launch here).  Instead a slot holds
// bits + 1 (never 0 for a partial: a double whose bits are all ones is not produced), and the last workgroup
// waits on any slot still reading 0 (a store issued before its workgroup's ticket, not yet visible); the wait
// is bounded.  Scratch layout: the counters at the 8-aligned start (kTicketWords words), the slots after them;
// all zero on entry and again on return (the callers keep the scratch).
constexpr int kTicketFan = 16, kTicketLine = 32;  // sub-counters; u32 words per counter (128 bytes)
constexpr int kTicketWords = (kTicketFan + 1) * kTicketLine;
struct TicketScratch {
    uint32_t *ticket;  // [0] top, [(j + 1) * kTicketLine] sub-counter j
    double *part;
};
__host__ __device__ inline TicketScratch ticket_scratch(void *scratch) {
    uint32_t *t = (uint32_t *)(((size_t)scratch + 7) & ~(size_t)7);
    return {t, (double *)(t + kTicketWords)};
}

// Thread 0 holds `t`, this workgroup's partial.  Returns true in every thread of the last workgroup, with
// the total in *total (all threads); false elsewhere.
__device__ __forceinline__ bool publish_and_total(double t, TicketScratch ts, int nblk, double *total) {
    __shared__ uint32_t s_last;
    __shared__ double s_w[kTailThreads / 64];
    unsigned long long *slot = (unsigned long long *)ts.part;
    if (threadIdx.x == 0) {
        __hip_atomic_store(slot + blockIdx.x, (unsigned long long)__double_as_longlong(t) + 1ull, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
        const uint32_t j = blockIdx.x % kTicketFan, nj = ((uint32_t)nblk - j + kTicketFan - 1) / kTicketFan;
        uint32_t *sub = ts.ticket + (j + 1) * kTicketLine;
        bool last = false;
        if (__hip_atomic_fetch_add(sub, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == nj - 1u) {
            __hip_atomic_store(sub, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // every draw on it is done
            const uint32_t nsub = nblk < kTicketFan ? (uint32_t)nblk : (uint32_t)kTicketFan;
            last = __hip_atomic_fetch_add(ts.ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == nsub - 1u;
        }
        s_last = last;
    }
    __syncthreads();
    if (!s_last) return false;
    // the slots in rounds of kRound per thread, all loads of a round in flight at once (then the rare waits)
    constexpr int kRound = 8;
    double s = 0.0;
    bool lost = false;  // a slot still 0 after the bounded wait
    for (int i0 = 0; i0 < nblk; i0 += kRound * kTailThreads) {
        unsigned long long v[kRound];
#pragma unroll
        for (int k = 0; k < kRound; k++) {
            const int i = i0 + k * kTailThreads + (int)threadIdx.x;
            v[k] = i < nblk ? __hip_atomic_load(slot + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 1ull;  // 1: +0.0
        }
#pragma unroll
        for (int k = 0; k < kRound; k++) {
            const int i = i0 + k * kTailThreads + (int)threadIdx.x;
            for (uint32_t spins = 0; v[k] == 0ull && spins < (1u << 22); spins++)
                v[k] = __hip_atomic_load(slot + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            lost |= v[k] == 0ull;
            if (i < nblk) __hip_atomic_store(slot + i, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (i < nblk && v[k] != 0ull) s += __longlong_as_double((long long)(v[k] - 1ull));
        }
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off);
    if ((threadIdx.x & 63) == 0) s_w[threadIdx.x >> 6] = s;
    // A slot that never arrived (the wait gave up: never seen, but possible in principle) leaves its late store
    // behind in the kept scratch, which would corrupt a later call's total silently.  Instead the scratch is
    // poisoned (word 1 of the top counter's line, sticky): this total and every later one with this scratch
    // are NaN, until the caller zeroes the scratch again.
    const bool any_lost = __syncthreads_or(lost);
    if (any_lost && threadIdx.x == 0) __hip_atomic_store(ts.ticket + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const bool poisoned = any_lost || __hip_atomic_load(ts.ticket + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u;
    double sum = 0.0;
#pragma unroll
    for (int w = 0; w < kTailThreads / 64; w++) sum += s_w[w];
    *total = poisoned ? __builtin_nan("") : sum;
    if (threadIdx.x == 0) __hip_atomic_store(ts.ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return true;
}

__global__ __launch_bounds__(kTailThreads) void l1_partial_kernel(int64_t n, const float *__restrict__ x,
                                                                  const float *__restrict__ y,
                                                                  int8_t *__restrict__ sign, TicketScratch ts,
                                                                  float *__restrict__ loss) {
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
    double t = 0.0;
#pragma unroll
    for (int w = 0; w < kTailThreads / 64; w++) t += s_w[w];
    double total;
    if (publish_and_total(t, ts, (int)gridDim.x, &total) && threadIdx.x == 0) *loss = (float)(total / (double)n);
}

// The same pass over 16-byte words (n % 4 == 0, 16-byte aligned x / y and 4-byte aligned sign): each
// thread takes two float4 of x and y and stores two char4 of signs -- a quarter of the memory
// instructions of the scalar form, the same partial layout (kL1Chunk elements per workgroup).
// GRAD: the loss's gradient for the upstream gradient `scale` = dloss * (1 / n) is stored instead of the signs
// (gs4d_l1_loss_grad: value and gradient in one pass, where l1_backward would read the signs back)
template <bool GRAD>
__global__ __launch_bounds__(kTailThreads) void l1_partial_v4_kernel(int64_t n4, const float4 *__restrict__ x,
                                                                     const float4 *__restrict__ y,
                                                                     char4 *__restrict__ sign, TicketScratch ts,
                                                                     float *__restrict__ loss, float4 *__restrict__ grad,
                                                                     float scale) {
    const int64_t base = (int64_t)blockIdx.x * (kL1Chunk / 4);
    float acc = 0.f;
#pragma unroll
    for (int k = 0; k < kL1PerThread / 4; k++) {
        const int64_t i = base + (int64_t)k * kTailThreads + threadIdx.x;
        if (i < n4) {
            const float4 a = x[i], b = y[i];
            const float d0 = a.x - b.x, d1 = a.y - b.y, d2 = a.z - b.z, d3 = a.w - b.w;
            acc += fabsf(d0);
            acc += fabsf(d1);
            acc += fabsf(d2);
            acc += fabsf(d3);
            auto sg = [](float d) { return (signed char)((d > 0.f) - (d < 0.f)); };  // torch.sign
            const char4 c = make_char4(sg(d0), sg(d1), sg(d2), sg(d3));
            if (GRAD)  // as l1_backward_v4_kernel: sign * (dloss * (1 / n))
                grad[i] = make_float4((float)c.x * scale, (float)c.y * scale, (float)c.z * scale, (float)c.w * scale);
            else
                sign[i] = c;
        }
    }
    double s = acc;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off);
    __shared__ double s_w[kTailThreads / 64];
    if ((threadIdx.x & 63) == 0) s_w[threadIdx.x >> 6] = s;
    __syncthreads();
    double t = 0.0;
#pragma unroll
    for (int w = 0; w < kTailThreads / 64; w++) t += s_w[w];
    double total;
    if (publish_and_total(t, ts, (int)gridDim.x, &total) && threadIdx.x == 0) *loss = (float)(total / (double)(4 * n4));
}

__global__ __launch_bounds__(kTailThreads) void l1_backward_kernel(int64_t n, const int8_t *__restrict__ sign,
                                                                   const float *__restrict__ dloss,
                                                                   float *__restrict__ grad) {
    // d mean / dx = sign / N, times the upstream gradient, rounded as torch's MeanBackward does it
    // (grad / numel with a scalar divisor: grad * (1 / numel))
    const float scale = *dloss * (1.0f / (float)n);
    for (int64_t i = (int64_t)blockIdx.x * kTailThreads + threadIdx.x; i < n; i += (int64_t)gridDim.x * kTailThreads)
        grad[i] = (float)sign[i] * scale;
}

__global__ __launch_bounds__(kTailThreads) void l1_backward_v4_kernel(int64_t n4, const char4 *__restrict__ sign,
                                                                      const float *__restrict__ dloss,
                                                                      float4 *__restrict__ grad, int64_t n) {
    const float scale = *dloss * (1.0f / (float)n);  // as l1_backward_kernel
    for (int64_t i = (int64_t)blockIdx.x * kTailThreads + threadIdx.x; i < n4; i += (int64_t)gridDim.x * kTailThreads) {
        const char4 c = sign[i];
        grad[i] = make_float4((float)c.x * scale, (float)c.y * scale, (float)c.z * scale, (float)c.w * scale);
    }
}

// ---- densification statistics ------------------------------------------------------------------
__global__ __launch_bounds__(kTailThreads) void densify_stats_kernel(int P, const float *__restrict__ vs_grad,
                                                                     const uint8_t *__restrict__ visible,
                                                                     const int *__restrict__ radii,
                                                                     float *__restrict__ grad_accum,
                                                                     float *__restrict__ denom,
                                                                     float *__restrict__ max_radii) {
    const int i = blockIdx.x * kTailThreads + threadIdx.x;
    if (i >= P) return;
    // without a visibility mask the filter is train.py's own definition of it, radii > 0 (:229-232; for a batch,
    // max over views of radii > 0 is any over views of visibility)
    if (visible ? !visible[i] : !(radii[i] > 0)) return;
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
    // one element: exactly the scalar sequence below, whichever width the loop loads at
    auto upd = [&](float g, float &p, float &m, float &v) {
        // exp_avg.lerp_(grad, 1 - beta1): weight < 0.5 -> self + weight * (end - self)
        m = fmaf(omb1, g - m, m);
        // exp_avg_sq.mul_(beta2).addcmul_(grad, grad, value=1 - beta2)
        v = v * b2;
        v = fmaf(omb2, g * g, v);
        // denom = exp_avg_sq.sqrt() / bias_correction2_sqrt + eps; param.addcdiv_(exp_avg, denom, -step_size)
        const float den = sqrtf(v) / bc2 + eps;
        p = fmaf(step_size, m / den, p);
    };
    const bool vec = (((uintptr_t)d.param | (uintptr_t)d.grad | (uintptr_t)d.exp_avg | (uintptr_t)d.exp_avg_sq) & 15) == 0;
    if (vec) {
        // 16-byte loads and stores (the chunk base is a multiple of 4); the tensor's last n % 4 elements by the
        // chunk that holds them
        const int64_t n4 = d.n >> 2;
        for (int k = threadIdx.x; k < kAdamChunk / 4; k += kTailThreads) {
            const int64_t i4 = (base >> 2) + k;
            if (i4 >= n4) break;
            const float4 g = reinterpret_cast<const float4 *>(d.grad)[i4];
            float4 p = reinterpret_cast<float4 *>(d.param)[i4];
            float4 m = reinterpret_cast<float4 *>(d.exp_avg)[i4];
            float4 v = reinterpret_cast<float4 *>(d.exp_avg_sq)[i4];
            upd(g.x, p.x, m.x, v.x);
            upd(g.y, p.y, m.y, v.y);
            upd(g.z, p.z, m.z, v.z);
            upd(g.w, p.w, m.w, v.w);
            reinterpret_cast<float4 *>(d.param)[i4] = p;
            reinterpret_cast<float4 *>(d.exp_avg)[i4] = m;
            reinterpret_cast<float4 *>(d.exp_avg_sq)[i4] = v;
        }
        const int64_t i = 4 * n4 + threadIdx.x;
        if (i < d.n && i >= base && i < base + kAdamChunk) {
            float p = d.param[i], m = d.exp_avg[i], v = d.exp_avg_sq[i];
            upd(d.grad[i], p, m, v);
            d.param[i] = p;
            d.exp_avg[i] = m;
            d.exp_avg_sq[i] = v;
        }
        return;
    }
    for (int k = threadIdx.x; k < kAdamChunk; k += kTailThreads) {
        const int64_t i = base + k;
        if (i >= d.n) break;
        float p = d.param[i], m = d.exp_avg[i], v = d.exp_avg_sq[i];
        upd(d.grad[i], p, m, v);
        d.param[i] = p;
        d.exp_avg[i] = m;
        d.exp_avg_sq[i] = v;
    }
}


// ---- deformation tail + activations (scene/deformation.py:140-146, gaussian_renderer/__init__.py:97-99)
// Blocks [0, nb_g) take one Gaussian per thread (means, scales, rotation, opacity); blocks [nb_g, ..)
// take the 3K SH values of the Gaussians as one flat, coalesced range.
__global__ __launch_bounds__(kTailThreads) void deform_tail_fwd_kernel(
    int P, int K, int nb_g, const float *__restrict__ xyz, const float *__restrict__ s, const float *__restrict__ r,
    const float *__restrict__ o, const float *__restrict__ f_dc, const float *__restrict__ f_rest,
    const float *__restrict__ dx, const float *__restrict__ ds, const float *__restrict__ dr,
    const float *__restrict__ d_o, const float *__restrict__ dshs, float *__restrict__ means,
    float *__restrict__ scales, float *__restrict__ rot, float *__restrict__ opac, float *__restrict__ shs, int v4) {
    if ((int)blockIdx.x < nb_g) {
        const int i = blockIdx.x * kTailThreads + threadIdx.x;
        if (i >= P) return;
#pragma unroll
        for (int c = 0; c < 3; c++) {
            const size_t k = 3 * (size_t)i + c;
            means[k] = dx ? xyz[k] + dx[k] : xyz[k];
            scales[k] = expf(ds ? s[k] + ds[k] : s[k]);
        }
        float q[4];
#pragma unroll
        for (int c = 0; c < 4; c++) {
            const size_t k = 4 * (size_t)i + c;
            q[c] = dr ? r[k] + dr[k] : r[k];
        }
        // F.normalize: x / max(||x||_2, eps)
        const float nrm = fmaxf(sqrtf(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]), 1e-12f);
#pragma unroll
        for (int c = 0; c < 4; c++) rot[4 * (size_t)i + c] = q[c] / nrm;
        const float x = d_o ? o[i] + d_o[i] : o[i];
        opac[i] = 1.f / (1.f + expf(-x));
        return;
    }
    const int64_t n = (int64_t)P * 3 * K;
    if (v4) {
        // four consecutive values per thread (3K % 4 == 0: they share a Gaussian), dshs / shs as 16-byte accesses
        const int64_t e0 = 4 * ((int64_t)(blockIdx.x - nb_g) * kTailThreads + threadIdx.x);
        if (e0 >= n) return;
        const int64_t g = (int64_t)((uint32_t)e0 / (uint32_t)(3 * K)), k0 = e0 - g * 3 * K;
        const float4 d = dshs ? reinterpret_cast<const float4 *>(dshs)[e0 / 4] : make_float4(0.f, 0.f, 0.f, 0.f);
        float b[4];
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int64_t k = k0 + j;
            b[j] = k < 3 ? f_dc[3 * g + k] : f_rest[g * 3 * (K - 1) + (k - 3)];
        }
        reinterpret_cast<float4 *>(shs)[e0 / 4] =
            dshs ? make_float4(b[0] + d.x, b[1] + d.y, b[2] + d.z, b[3] + d.w) : make_float4(b[0], b[1], b[2], b[3]);
        return;
    }
    const int64_t e = (int64_t)(blockIdx.x - nb_g) * kTailThreads + threadIdx.x;
    if (e >= n) return;
    // 32-bit quotient (a 64-bit division is a long software sequence): e < P * 3K < 2^32 by the host check
    const int64_t g = (int64_t)((uint32_t)e / (uint32_t)(3 * K)), k = e - g * 3 * K;
    const float base = k < 3 ? f_dc[3 * g + k] : f_rest[g * 3 * (K - 1) + (k - 3)];
    shs[e] = dshs ? base + dshs[e] : base;
}

__global__ __launch_bounds__(kTailThreads) void deform_tail_bwd_kernel(
    int P, int K, int nb_g, const float *__restrict__ scales, const float *__restrict__ r,
    const float *__restrict__ dr, const float *__restrict__ opac, const float *__restrict__ g_means,
    const float *__restrict__ g_scales, const float *__restrict__ g_rot, const float *__restrict__ g_opac,
    const float *__restrict__ g_shs, float *__restrict__ d_xyz, float *__restrict__ d_s, float *__restrict__ d_r,
    float *__restrict__ d_o, float *__restrict__ d_fdc, float *__restrict__ d_frest, float *__restrict__ g_dx,
    float *__restrict__ g_ds, float *__restrict__ g_dr, float *__restrict__ g_do, int v4) {
    if ((int)blockIdx.x < nb_g) {
        const int i = blockIdx.x * kTailThreads + threadIdx.x;
        if (i >= P) return;
#pragma unroll
        for (int c = 0; c < 3; c++) {
            const size_t k = 3 * (size_t)i + c;
            const float gm = g_means ? g_means[k] : 0.f;
            const float gs = g_scales ? g_scales[k] * scales[k] : 0.f;  // d exp(x) = exp(x) dx
            d_xyz[k] = gm;
            d_s[k] = gs;
            if (g_dx) g_dx[k] = gm;
            if (g_ds) g_ds[k] = gs;
        }
        float q[4], g[4];
#pragma unroll
        for (int c = 0; c < 4; c++) {
            const size_t k = 4 * (size_t)i + c;
            q[c] = dr ? r[k] + dr[k] : r[k];
            g[c] = g_rot ? g_rot[k] : 0.f;
        }
        // autograd of x / clamp_min(||x||, eps): g / n - x (x . g) / n^3 (the second term only when ||x|| > eps)
        const float n0 = sqrtf(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
        const float nrm = fmaxf(n0, 1e-12f);
        const float xg = q[0] * g[0] + q[1] * g[1] + q[2] * g[2] + q[3] * g[3];
        const float gn = n0 > 1e-12f ? -xg / (nrm * nrm) : 0.f;
#pragma unroll
        for (int c = 0; c < 4; c++) {
            const float v = g[c] / nrm + gn * (q[c] / n0);
            d_r[4 * (size_t)i + c] = v;
            if (g_dr) g_dr[4 * (size_t)i + c] = v;
        }
        const float y = opac[i];
        const float go = g_opac ? (g_opac[i] * (1.f - y)) * y : 0.f;  // sigmoid backward, torch's order
        d_o[i] = go;
        if (g_do) g_do[i] = go;
        return;
    }
    const int64_t n = (int64_t)P * 3 * K;
    if (v4) {  // as in deform_tail_fwd_kernel: g_shs as 16-byte loads
        const int64_t e0 = 4 * ((int64_t)(blockIdx.x - nb_g) * kTailThreads + threadIdx.x);
        if (e0 >= n) return;
        const int64_t gi = (int64_t)((uint32_t)e0 / (uint32_t)(3 * K)), k0 = e0 - gi * 3 * K;
        const float4 v4v = g_shs ? reinterpret_cast<const float4 *>(g_shs)[e0 / 4] : make_float4(0.f, 0.f, 0.f, 0.f);
        const float v[4] = {v4v.x, v4v.y, v4v.z, v4v.w};
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int64_t k = k0 + j;
            if (k < 3) d_fdc[3 * gi + k] = v[j];
            else d_frest[gi * 3 * (K - 1) + (k - 3)] = v[j];
        }
        return;
    }
    const int64_t e = (int64_t)(blockIdx.x - nb_g) * kTailThreads + threadIdx.x;
    if (e >= n) return;
    const int64_t gi = (int64_t)((uint32_t)e / (uint32_t)(3 * K)), k = e - gi * 3 * K;  // e < 2^32: host check
    const float v = g_shs ? g_shs[e] : 0.f;
    if (k < 3) d_fdc[3 * gi + k] = v;
    else d_frest[gi * 3 * (K - 1) + (k - 3)] = v;
}

// ---- HexPlane regularisers ------------------------------------------------------------------------
constexpr int kRegPerThread = 8;
constexpr int kRegBlock = kTailThreads * kRegPerThread;  // plane elements per workgroup

__device__ __forceinline__ int reg_plane_of(const gs4d_reg_batch &b, int64_t blk) {
    int t = 0;
    while (t + 1 < b.count && b.p[t + 1].first_block <= blk) t++;
    return t;
}

// second difference along H at row y (0 <= y <= H-3), in the reference's operation order
// (regulation.py:25-26): first[j] = t[j+1] - t[j], second[y] = first[y+1] - first[y]
__device__ __forceinline__ float second_diff(const float *__restrict__ col, int y, int W) {
    const float t0 = col[(size_t)y * W], t1 = col[(size_t)(y + 1) * W], t2 = col[(size_t)(y + 2) * W];
    return (t2 - t1) - (t1 - t0);
}

__global__ __launch_bounds__(kTailThreads) void reg_forward_kernel(gs4d_reg_batch b, TicketScratch ts, float *__restrict__ loss) {
    const int64_t blk = blockIdx.x;
    const gs4d_reg_plane d = b.p[reg_plane_of(b, blk)];
    const int64_t n = (int64_t)d.C * d.H * d.W, hw = (int64_t)d.H * d.W;
    const double cs = (double)d.w_smooth / ((double)d.C * (d.H - 2) * d.W), cl = (double)d.w_l1 / (double)n;
    double acc = 0.0;
    // rows y .. y + 2 of every element first (indices clamped into the plane: all loads in flight at once, none
    // behind the loop's exit), then the terms in element order
    float r[kRegPerThread][3];
    const int64_t i0 = (blk - d.first_block) * kRegBlock + threadIdx.x;
#pragma unroll
    for (int k = 0; k < kRegPerThread; k++) {
        const int64_t i = std::min<int64_t>(i0 + (int64_t)k * kTailThreads, n - 1);
        const int y = (int)(((uint32_t)i % (uint32_t)hw) / (uint32_t)d.W);  // 32-bit: a plane < 2^31 elements
        const float *col = d.data + (i - (int64_t)y * d.W);
#pragma unroll
        for (int q = 0; q < 3; q++) r[k][q] = col[(size_t)std::min(y + q, d.H - 1) * d.W];
    }
#pragma unroll
    for (int k = 0; k < kRegPerThread; k++) {
        const int64_t i = i0 + (int64_t)k * kTailThreads;
        if (i >= n) break;
        const float t = r[k][0];
        const int y = (int)(((uint32_t)i % (uint32_t)hw) / (uint32_t)d.W);
        if (y <= d.H - 3) {
            const float s2 = (r[k][2] - r[k][1]) - (r[k][1] - r[k][0]);  // second_diff at row y
            acc += cs * (double)(s2 * s2);
        }
        acc += cl * (double)fabsf(1.f - t);
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off);
    __shared__ double s_w[kTailThreads / 64];
    if ((threadIdx.x & 63) == 0) s_w[threadIdx.x >> 6] = acc;
    __syncthreads();
    double total;
    if (publish_and_total(s_w[0] + s_w[1] + s_w[2] + s_w[3], ts, (int)gridDim.x, &total) && threadIdx.x == 0)
        *loss = (float)total;
}

// d/dt of the batch loss, as autograd derives it from the reference's graph: mean -> g / N, square
// -> 2 s g, second[y] = first[y+1] - first[y] -> dfirst[j] = ds[j-1] - ds[j], first[j] = t[j+1] - t[j]
// -> dt[y] = dfirst[y-1] - dfirst[y] (out-of-range terms are 0); abs(1 - t) -> -sign(1 - t) g / N.
// loss (nullable): also the value, its per-workgroup partials exactly as reg_forward_kernel forms them (same
// workgroups, same per-thread order and terms: its second difference at row y is the ds[2] term below) and
// totalled by the last workgroup -- the value and the gradient from one read of the planes.  base (nullable):
// *loss = *base + value instead, the fp32 add of a loss term the value joins.
__global__ __launch_bounds__(kTailThreads) void reg_backward_kernel(gs4d_reg_batch b, const float *__restrict__ dloss,
                                                                    TicketScratch ts, float *__restrict__ loss,
                                                                    const float *__restrict__ base) {
    const bool part = loss != nullptr;
    const int64_t blk = blockIdx.x;
    const gs4d_reg_plane d = b.p[reg_plane_of(b, blk)];
    const int64_t n = (int64_t)d.C * d.H * d.W, hw = (int64_t)d.H * d.W;
    const float g = *dloss;
    const float gs = (g * d.w_smooth) / (float)((int64_t)d.C * (d.H - 2) * d.W);
    const float gl = (g * d.w_l1) / (float)n;
    const double cs = (double)d.w_smooth / ((double)d.C * (d.H - 2) * d.W), cl = (double)d.w_l1 / (double)n;
    double acc = 0.0;
    // rows y - 2 .. y + 2 of every element (and its gradient, when accumulating) first, indices clamped into the
    // plane: all loads in flight at once, none behind the loop's exit; out-of-range rows only feed masked terms
    float r[kRegPerThread][5], gv[kRegPerThread];
    const int64_t i0 = (blk - d.first_block) * kRegBlock + threadIdx.x;
#pragma unroll
    for (int k = 0; k < kRegPerThread; k++) {
        const int64_t i = std::min<int64_t>(i0 + (int64_t)k * kTailThreads, n - 1);
        const int y = (int)(((uint32_t)i % (uint32_t)hw) / (uint32_t)d.W);  // 32-bit: a plane < 2^31 elements
        const float *col = d.data + (i - (int64_t)y * d.W);
#pragma unroll
        for (int q = 0; q < 5; q++) r[k][q] = col[(size_t)std::min(std::max(y - 2 + q, 0), d.H - 1) * d.W];
        gv[k] = b.accumulate ? d.grad[i] : 0.f;
    }
#pragma unroll
    for (int k = 0; k < kRegPerThread; k++) {
        const int64_t i = i0 + (int64_t)k * kTailThreads;
        if (i >= n) break;
        const int y = (int)(((uint32_t)i % (uint32_t)hw) / (uint32_t)d.W);
        float ds[3], s2y = 0.f;  // ds[y-2], ds[y-1], ds[y]; s2y: the second difference at row y itself
#pragma unroll
        for (int q = 0; q < 3; q++) {
            const int yy = y - 2 + q;
            const bool in = yy >= 0 && yy <= d.H - 3;
            const float s2 = in ? (r[k][q + 2] - r[k][q + 1]) - (r[k][q + 1] - r[k][q]) : 0.f;  // second_diff at yy
            ds[q] = in ? 2.f * s2 * gs : 0.f;
            if (q == 2) s2y = s2;
        }
        const float df_prev = (y >= 1) ? ds[0] - ds[1] : 0.f;      // dfirst[y-1] = ds[y-2] - ds[y-1]
        const float df_cur = (y <= d.H - 2) ? ds[1] - ds[2] : 0.f;  // dfirst[y] = ds[y-1] - ds[y]
        const float t = r[k][2];
        const float one_m = 1.f - t;
        const float sg = (float)((one_m > 0.f) - (one_m < 0.f));
        const float v = (df_prev - df_cur) + (-sg) * gl;
        d.grad[i] = b.accumulate ? gv[k] + v : v;
        if (part) {  // reg_forward_kernel's terms, in its order
            if (y <= d.H - 3) acc += cs * (double)(s2y * s2y);
            acc += cl * (double)fabsf(1.f - t);
        }
    }
    if (part) {
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off);
        __shared__ double s_w[kTailThreads / 64];
        if ((threadIdx.x & 63) == 0) s_w[threadIdx.x >> 6] = acc;
        __syncthreads();
        double total;
        if (publish_and_total(s_w[0] + s_w[1] + s_w[2] + s_w[3], ts, (int)gridDim.x, &total) && threadIdx.x == 0)
            *loss = base ? *base + (float)total : (float)total;
    }
}

// ---- tall-skinny weight gradients -----------------------------------------------------------------
// dW = dy^T x and db = column sums of dy for Linear layers' backward, reduced over P ~ 1e5 rows with
// n <= 64 outputs and W in {64, 128, 256} inputs -- the deformation heads' second layers, which the
// GEMM library tiles only by their small output (~55 us per call whatever n, split-K included).  Up to
// kDwMaxProblems such products (same P and W) go in one launch, blockIdx.y picking the problem.  A
// workgroup takes a contiguous block of rows; inside it G = 512 / W thread groups take interleaved
// runs of kDwUnroll rows; a thread owns column c and accumulates all n outputs: x[p, c] is one
// coalesced vector load per row, the dy row is wave-uniform (scalar loads, the FMA's SGPR operand).
// db: lane l of each group's first wave adds dy[p, l].  Groups combine through LDS in group order and
// the per-workgroup partials are summed in a fixed order by a second launch: deterministic.
constexpr int kDwMaxProblems = 8;
constexpr int kDwThreads = 512;
constexpr int kDwMaxNW = 64 * 128;  // n * W bound (LDS combine buffer)

struct DwProblem {
    const float *dy;
    const float *x;
    float *dw;
    float *db;
    int n, ld_dy, ld_x, pad;
    int64_t part_off;  // floats into the partials buffer
};
struct DwBatch {
    DwProblem q[kDwMaxProblems];
};

template <int N, bool EXACT, int kDwUnroll>
__device__ __forceinline__ void dw_block(const DwProblem &q, int P, int W, int rows_per_wg, float *__restrict__ part,
                                         float *s_red, float *s_bs) {
    const int tid = threadIdx.x;
    const int G = kDwThreads / W;
    const int g = __builtin_amdgcn_readfirstlane(tid / W);  // W is a multiple of 64: wave-uniform
    const int c = tid - g * W;
    const bool lead = __builtin_amdgcn_readfirstlane(c) == 0;  // the group's first wave
    const int n = EXACT ? N : q.n;
    const float *__restrict__ dy = q.dy;
    const float *__restrict__ x = q.x;
    const int64_t p0 = (int64_t)blockIdx.x * rows_per_wg, p1 = min((int64_t)P, p0 + rows_per_wg);
    float acc[N];
#pragma unroll
    for (int j = 0; j < N; j++) acc[j] = 0.f;
    float bs = 0.f;
    for (int64_t p = p0 + (int64_t)g * kDwUnroll; p < p1; p += (int64_t)G * kDwUnroll) {
        float xv[kDwUnroll];
#pragma unroll
        for (int u = 0; u < kDwUnroll; u++) xv[u] = p + u < p1 ? x[(p + u) * q.ld_x + c] : 0.f;
#pragma unroll
        for (int u = 0; u < kDwUnroll; u++) {
            if (p + u < p1) {
                const float *d = dy + (p + u) * q.ld_dy;
#pragma unroll
                for (int j = 0; j < N; j++)
                    if (EXACT || j < n) acc[j] = fmaf(d[j], xv[u], acc[j]);
                if (lead && c < n) bs += d[c];
            }
        }
    }
    for (int h = 0; h < G; h++) {
        if (g == h) {
#pragma unroll
            for (int j = 0; j < N; j++)
                if (EXACT || j < n) s_red[j * W + c] = (h == 0 ? 0.f : s_red[j * W + c]) + acc[j];
            if (lead && c < n) s_bs[c] = (h == 0 ? 0.f : s_bs[c]) + bs;
        }
        __syncthreads();
    }
    float *out = part + q.part_off + (int64_t)blockIdx.x * n * (W + 1);
    for (int e = tid; e < n * (W + 1); e += kDwThreads) {
        const int r = e / (W + 1), cc = e - r * (W + 1);
        out[e] = cc < W ? s_red[r * W + cc] : s_bs[r];
    }
}

// FAMILY 0: n <= 8 (16 rows in flight per thread); FAMILY 1: n = 48 or n <= 16 (4 rows)
template <int FAMILY>
__global__ __launch_bounds__(kDwThreads) void linear_dw_kernel(DwBatch b, int P, int W, int rows_per_wg,
                                                                float *__restrict__ part) {
    __shared__ float s_red[kDwMaxNW];
    __shared__ float s_bs[64];
    const DwProblem &q = b.q[blockIdx.y];
    if constexpr (FAMILY == 0) {
        switch (q.n) {
        case 1: dw_block<1, true, 16>(q, P, W, rows_per_wg, part, s_red, s_bs); break;
        case 2: dw_block<2, true, 16>(q, P, W, rows_per_wg, part, s_red, s_bs); break;
        case 3: dw_block<3, true, 16>(q, P, W, rows_per_wg, part, s_red, s_bs); break;
        case 4: dw_block<4, true, 16>(q, P, W, rows_per_wg, part, s_red, s_bs); break;
        default: dw_block<8, false, 8>(q, P, W, rows_per_wg, part, s_red, s_bs);
        }
    } else {
        if (q.n == 48) dw_block<48, true, 4>(q, P, W, rows_per_wg, part, s_red, s_bs);
        else if (q.n <= 8) dw_block<8, false, 8>(q, P, W, rows_per_wg, part, s_red, s_bs);
        else dw_block<16, false, 4>(q, P, W, rows_per_wg, part, s_red, s_bs);
    }
}

// sum of the per-workgroup partials: 32 outputs (r, c | bias) of problem blockIdx.y per workgroup,
// 8 interleaved eighths of the workgroups combined in a fixed order
__global__ __launch_bounds__(256) void linear_dw_reduce_kernel(DwBatch b, int W, int nwg, const float *__restrict__ part) {
    __shared__ float s_sum[8][32];
    const DwProblem &q = b.q[blockIdx.y];
    const int per = q.n * (W + 1);
    if ((int)blockIdx.x * 32 >= per) return;  // uniform over the workgroup
    const int o = threadIdx.x & 31, k = threadIdx.x >> 5;
    const int i = blockIdx.x * 32 + o;
    const float *src = part + q.part_off;
    float v0 = 0.f, v1 = 0.f, v2 = 0.f, v3 = 0.f;  // four independent chains: loads in flight
    if (i < per) {
        int w = k;
        for (; w + 24 < nwg; w += 32) {
            v0 += src[(size_t)w * per + i];
            v1 += src[(size_t)(w + 8) * per + i];
            v2 += src[(size_t)(w + 16) * per + i];
            v3 += src[(size_t)(w + 24) * per + i];
        }
        for (; w < nwg; w += 8) v0 += src[(size_t)w * per + i];
    }
    s_sum[k][o] = (v0 + v1) + (v2 + v3);
    __syncthreads();
    if (k == 0 && i < per) {
        float t = 0.f;
#pragma unroll
        for (int e = 0; e < 8; e++) t += s_sum[e][o];
        const int r = i / (W + 1), cc = i - r * (W + 1);
        if (cc < W) q.dw[(size_t)r * W + cc] = t;
        else if (q.db) q.db[r] = t;
    }
}

// ---- the deformation heads' second layers, backward, in one pass over the first layers' output ------
// For k heads (scene/deformation.py:73-78: ReLU -> Linear(W, W) -> ReLU -> Linear(W, n_i)) evaluated as
// one block (gs4d_train/deformation.py _DeformHeads): a = relu(h W1^T + b1) is (P, kW), head i's output
// is a[:, iW:(i+1)W] W2_i^T + b2_i.  Given the output gradients g_i (P, n_i) this forms, reading `a` once:
//   da[:, iW + c] = (a > 0) * sum_r g_i[:, r] W2_i[r, c]   (mm + threshold_backward in autograd)
//   db1 = column sums of da,  dW2_i = g_i^T a_i,  db2_i = column sums of g_i.
// A workgroup takes a block of rows; thread c owns column c of a (kW <= 768 threads, head = c / W is
// wave-uniform): its W2_i column and dW2_i accumulators stay in registers, the g_i row is wave-uniform
// (scalar loads).  Per-workgroup partials are summed in a fixed order by a second launch.
constexpr int kHbMaxHeads = 8;
typedef float f4v __attribute__((ext_vector_type(4)));  // an MFMA 16x16 accumulator (4 per lane)
// One launch serves the heads [h0, h0 + hk) (columns h0 W .. (h0 + hk) W of a): the narrow heads and
// the 48-wide one go in separate launches, each with its own row blocking, so no workgroup waits on a
// few compute-heavy waves.
struct HbArgs {
    int P, W, k, rows_per_wg, h0, hk;
    int n[kHbMaxHeads];
    const float *w2[kHbMaxHeads];
    int poff[kHbMaxHeads + 1];  // local head i's partials: n_{h0+i} (W + 1) floats from poff[i]; poff[0] = hk W
};

// One wave's columns of head h.  The head's output-gradient rows for U rows at a time are one or a few
// coalesced vector loads (the U x n block is contiguous in g); each value reaches the FMAs as an SGPR
// through v_readlane.  The next block's loads are issued before the current block is used.  db2: the
// lead wave adds the blocks elementwise (flattened index i holds output i mod n) and folds them at the
// end in a fixed order.
// TA: the element type of a and da -- float, or __bf16 on the bf16 path (hyper.mlp_dtype = "bf16"), where
// the products still run in f32 on the bf16 values and da is rounded once when stored.
template <int N, bool EXACT, int U, class TA>
__device__ __forceinline__ void heads_bwd_cols(const HbArgs &A, int h, const TA *__restrict__ a,
                                               TA *__restrict__ da, const float *__restrict__ g,
                                               float *__restrict__ part, float *s_fold) {
    constexpr int KG = (U * N + 63) / 64;
    static_assert(EXACT || KG == 1, "runtime widths keep the block in one register");
    const int W = A.W, ld = A.k * W, hl = h - A.h0;
    const int col = A.h0 * W + threadIdx.x, c = (int)threadIdx.x - hl * W;
    const int lane = threadIdx.x & 63;
    const bool lead = c < 64;  // the head's first wave: db2 partials
    const int n = EXACT ? N : A.n[h];
    const float *__restrict__ w2 = A.w2[h];
    float w[N], acc[N];
#pragma unroll
    for (int r = 0; r < N; r++) {
        w[r] = (EXACT || r < n) ? w2[r * W + c] : 0.f;
        acc[r] = 0.f;
    }
    float gacc[KG];
#pragma unroll
    for (int k = 0; k < KG; k++) gacc[k] = 0.f;
    float csum = 0.f;
    const int64_t p0 = (int64_t)blockIdx.x * A.rows_per_wg, p1 = min((int64_t)A.P, p0 + A.rows_per_wg);
    const int64_t gend = p1 * n;
    // xn holds the raw elements: a bf16 value widened right after its (conditional) load would make the
    // compiler wait for that load inside the branch
    TA xn[U];
    float gn[KG];
    auto fetch = [&](int64_t p) {
#pragma unroll
        for (int u = 0; u < U; u++) xn[u] = p + u < p1 ? a[(p + u) * ld + col] : (TA)0.f;
#pragma unroll
        for (int k = 0; k < KG; k++) {
            const int64_t i = p * n + lane + 64 * k;
            gn[k] = (lane + 64 * k < U * n && i < gend) ? g[i] : 0.f;  // this block's U x n values only
        }
    };
    if (p0 < p1) fetch(p0);
    for (int64_t p = p0; p < p1; p += U) {
        float x[U], gv[KG];
#pragma unroll
        for (int u = 0; u < U; u++) x[u] = (float)xn[u];
#pragma unroll
        for (int k = 0; k < KG; k++) gv[k] = gn[k], gacc[k] += gn[k];
        if (p + U < p1) fetch(p + U);
#pragma unroll
        for (int u = 0; u < U; u++) {
            if (p + u < p1) {
                float sdot = 0.f;
#pragma unroll
                for (int r = 0; r < N; r++)
                    if (EXACT || r < n) {
                        const int idx = EXACT ? u * N + r : u * n + r;
                        const float dv = __builtin_bit_cast(
                            float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, gv[EXACT ? idx / 64 : 0]),
                                                             EXACT ? idx % 64 : idx));
                        sdot = fmaf(dv, w[r], sdot);
                        acc[r] = fmaf(dv, x[u], acc[r]);
                    }
                const float gvv = x[u] > 0.f ? sdot : 0.f;
                da[(p + u) * ld + col] = (TA)gvv;
                csum += gvv;
            }
        }
    }
    float *pw = part + (size_t)blockIdx.x * A.poff[A.hk];
    pw[threadIdx.x] = csum;
    float *ph = pw + A.poff[hl];
#pragma unroll
    for (int r = 0; r < N; r++)
        if (EXACT || r < n) ph[r * (W + 1) + c] = acc[r];
    if (lead) {
        // fold the flattened block sums: output r = sum over flattened indices i with i mod n == r
        float *f = s_fold + (threadIdx.x >> 6) * 64 * KG;
#pragma unroll
        for (int k = 0; k < KG; k++) f[lane + 64 * k] = gacc[k];
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        if (lane < n) {
            float t = 0.f;
            for (int i = lane; i < 64 * KG; i += n) t += f[i];
            ph[lane * (W + 1) + W] = t;
        }
    }
}

template <class TA>
__global__ __launch_bounds__(768) void heads_bwd_kernel(HbArgs A, const TA *__restrict__ a, TA *__restrict__ da,
                                                         const float *__restrict__ g0, const float *__restrict__ g1,
                                                         const float *__restrict__ g2, const float *__restrict__ g3,
                                                         const float *__restrict__ g4, const float *__restrict__ g5,
                                                         const float *__restrict__ g6, const float *__restrict__ g7,
                                                         float *__restrict__ part) {
    __shared__ float s_fold[16 * 64];  // per wave: the lead waves' flattened db2 block sums
    const int h = A.h0 + __builtin_amdgcn_readfirstlane((int)threadIdx.x / A.W);
    const float *__restrict__ g = h == 0 ? g0 : h == 1 ? g1 : h == 2 ? g2 : h == 3 ? g3 : h == 4 ? g4 : h == 5 ? g5
                                : h == 6 ? g6 : g7;
    switch (A.n[h]) {
    case 1: heads_bwd_cols<1, true, 8, TA>(A, h, a, da, g, part, s_fold); break;
    case 2: heads_bwd_cols<2, true, 8, TA>(A, h, a, da, g, part, s_fold); break;
    case 3: heads_bwd_cols<3, true, 8, TA>(A, h, a, da, g, part, s_fold); break;
    case 4: heads_bwd_cols<4, true, 8, TA>(A, h, a, da, g, part, s_fold); break;
    default:
        if (A.n[h] <= 8) heads_bwd_cols<8, false, 8, TA>(A, h, a, da, g, part, s_fold);
        else heads_bwd_cols<16, false, 4, TA>(A, h, a, da, g, part, s_fold);
    }
}

// The bf16 form with two columns per thread (W a multiple of 128: a head is whole waves of W / 2 threads):
// a and da move as bf16 pairs (4-byte loads and stores, half the memory instructions of one column per
// thread), the products and sums as in heads_bwd_cols, column by column.
typedef __attribute__((ext_vector_type(2))) __bf16 bf2v;
template <int N, bool EXACT, int U>
__device__ __forceinline__ void heads_bwd_cols2(const HbArgs &A, int h, const __bf16 *__restrict__ a,
                                                __bf16 *__restrict__ da, const float *__restrict__ g,
                                                float *__restrict__ part, float *s_fold) {
    constexpr int KG = (U * N + 63) / 64;
    static_assert(EXACT || KG == 1, "runtime widths keep the block in one register");
    const int W = A.W, ld = A.k * W, hl = h - A.h0;
    const int c = 2 * ((int)threadIdx.x - hl * (W / 2));  // this thread's first column in the head
    const int col = (A.h0 + hl) * W + c;
    const int lane = threadIdx.x & 63;
    const bool lead = c < 128;  // the head's first wave: db2 partials
    const int n = EXACT ? N : A.n[h];
    const float *__restrict__ w2 = A.w2[h];
    float w0[N], w1[N], acc0[N], acc1[N];
#pragma unroll
    for (int r = 0; r < N; r++) {
        const float2 wv = (EXACT || r < n) ? *reinterpret_cast<const float2 *>(w2 + r * W + c) : make_float2(0.f, 0.f);
        w0[r] = wv.x, w1[r] = wv.y;
        acc0[r] = acc1[r] = 0.f;
    }
    float gacc[KG];
#pragma unroll
    for (int k = 0; k < KG; k++) gacc[k] = 0.f;
    float csum0 = 0.f, csum1 = 0.f;
    const int64_t p0 = (int64_t)blockIdx.x * A.rows_per_wg, p1 = min((int64_t)A.P, p0 + A.rows_per_wg);
    const int64_t gend = p1 * n;
    bf2v xn[U];  // raw pairs until use (see heads_bwd_cols)
    float gn[KG];
    auto fetch = [&](int64_t p) {
#pragma unroll
        for (int u = 0; u < U; u++)
            xn[u] = p + u < p1 ? *reinterpret_cast<const bf2v *>(a + (p + u) * ld + col) : bf2v{(__bf16)0.f, (__bf16)0.f};
#pragma unroll
        for (int k = 0; k < KG; k++) {
            const int64_t i = p * n + lane + 64 * k;
            gn[k] = (lane + 64 * k < U * n && i < gend) ? g[i] : 0.f;
        }
    };
    if (p0 < p1) fetch(p0);
    for (int64_t p = p0; p < p1; p += U) {
        float x0[U], x1[U], gv[KG];
#pragma unroll
        for (int u = 0; u < U; u++) x0[u] = (float)xn[u][0], x1[u] = (float)xn[u][1];
#pragma unroll
        for (int k = 0; k < KG; k++) gv[k] = gn[k], gacc[k] += gn[k];
        if (p + U < p1) fetch(p + U);
#pragma unroll
        for (int u = 0; u < U; u++) {
            if (p + u < p1) {
                float sd0 = 0.f, sd1 = 0.f;
#pragma unroll
                for (int r = 0; r < N; r++)
                    if (EXACT || r < n) {
                        const int idx = EXACT ? u * N + r : u * n + r;
                        const float dv = __builtin_bit_cast(
                            float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, gv[EXACT ? idx / 64 : 0]),
                                                             EXACT ? idx % 64 : idx));
                        sd0 = fmaf(dv, w0[r], sd0);
                        sd1 = fmaf(dv, w1[r], sd1);
                        acc0[r] = fmaf(dv, x0[u], acc0[r]);
                        acc1[r] = fmaf(dv, x1[u], acc1[r]);
                    }
                const float g0 = x0[u] > 0.f ? sd0 : 0.f, g1 = x1[u] > 0.f ? sd1 : 0.f;
                *reinterpret_cast<bf2v *>(da + (p + u) * ld + col) = bf2v{(__bf16)g0, (__bf16)g1};
                csum0 += g0;
                csum1 += g1;
            }
        }
    }
    float *pw = part + (size_t)blockIdx.x * A.poff[A.hk];
    pw[hl * W + c] = csum0;
    pw[hl * W + c + 1] = csum1;
    float *ph = pw + A.poff[hl];
#pragma unroll
    for (int r = 0; r < N; r++)
        if (EXACT || r < n) ph[r * (W + 1) + c] = acc0[r], ph[r * (W + 1) + c + 1] = acc1[r];
    if (lead) {
        float *f = s_fold + (threadIdx.x >> 6) * 64 * KG;
#pragma unroll
        for (int k = 0; k < KG; k++) f[lane + 64 * k] = gacc[k];
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        if (lane < n) {
            float t = 0.f;
            for (int i = lane; i < 64 * KG; i += n) t += f[i];
            ph[lane * (W + 1) + W] = t;
        }
    }
}

__global__ __launch_bounds__(512) void heads_bwd2_kernel(HbArgs A, const __bf16 *__restrict__ a, __bf16 *__restrict__ da,
                                                        const float *__restrict__ g0, const float *__restrict__ g1,
                                                        const float *__restrict__ g2, const float *__restrict__ g3,
                                                        const float *__restrict__ g4, const float *__restrict__ g5,
                                                        const float *__restrict__ g6, const float *__restrict__ g7,
                                                        float *__restrict__ part) {
    __shared__ float s_fold[8 * 64];
    const int h = A.h0 + __builtin_amdgcn_readfirstlane((int)threadIdx.x / (A.W / 2));
    const float *__restrict__ g = h == 0 ? g0 : h == 1 ? g1 : h == 2 ? g2 : h == 3 ? g3 : h == 4 ? g4 : h == 5 ? g5
                                : h == 6 ? g6 : g7;
    switch (A.n[h]) {
    case 1: heads_bwd_cols2<1, true, 8>(A, h, a, da, g, part, s_fold); break;
    case 2: heads_bwd_cols2<2, true, 8>(A, h, a, da, g, part, s_fold); break;
    case 3: heads_bwd_cols2<3, true, 8>(A, h, a, da, g, part, s_fold); break;
    case 4: heads_bwd_cols2<4, true, 8>(A, h, a, da, g, part, s_fold); break;
    default:
        if (A.n[h] <= 8) heads_bwd_cols2<8, false, 8>(A, h, a, da, g, part, s_fold);
        else heads_bwd_cols2<16, false, 4>(A, h, a, da, g, part, s_fold);
    }
}

// The wide head (n = 48: the SH-coefficient deformation): the same products, VALU-bound rather than
// streaming (96 FMAs per row and column).  Thread c owns column c of the head (W threads); the head's
// output-gradient rows are staged in LDS in tiles of kWideTile rows (one coalesced load of a contiguous
// block of g) and read back as broadcasts, four values per ds_read_b128; the dot product (da) and the
// weight-gradient update (dW2) each take output pairs per v_pk_fma_f32.
constexpr int kWideTile = 8;
typedef float hf2 __attribute__((ext_vector_type(2)));

constexpr int kWideGroups = 2;  // row groups per workgroup: 2 x W threads (3 workgroups per CU at 152 VGPRs)

template <int N>
__global__ __launch_bounds__(512) void heads_bwd_wide_kernel(HbArgs A, const float *__restrict__ a,
                                                              float *__restrict__ da, const float *__restrict__ g,
                                                              float *__restrict__ part) {
    static_assert(N % 4 == 0, "rows of g read as float4");
    __shared__ float4 s_g[kWideGroups][kWideTile * N / 4];
    __shared__ float s_red[N * 128 + 2 * 128];  // row-group combine (W <= 128)
    const int W = A.W, ld = A.k * W, h = A.h0;
    const int rg = __builtin_amdgcn_readfirstlane((int)threadIdx.x / W);  // row group (wave-uniform)
    const int c = (int)threadIdx.x - rg * W, col = h * W + c;
    const float *__restrict__ w2 = A.w2[h];
    hf2 w[N / 2], acc[N / 2];
#pragma unroll
    for (int r = 0; r < N / 2; r++) {
        w[r] = hf2{w2[(2 * r) * W + c], w2[(2 * r + 1) * W + c]};
        acc[r] = hf2{0.f, 0.f};
    }
    float csum = 0.f, bsum = 0.f;
    const int64_t p0 = (int64_t)blockIdx.x * A.rows_per_wg, p1 = min((int64_t)A.P, p0 + A.rows_per_wg);
    // row group rg takes the tiles rg, rg + G, ... of the block; the next tile's x values and g block are
    // in registers while this one computes
    constexpr int kG4 = kWideTile * N / 4;  // float4 of g per tile
    constexpr int kGPer = (kG4 + 63) / 64;  // per thread, for W >= 64 threads
    const int64_t step = (int64_t)kWideGroups * kWideTile;
    float xn[kWideTile];
    float4 gn[kGPer];
    auto fetch = [&](int64_t t0) {
        const int nr = t0 < p1 ? (int)min((int64_t)kWideTile, p1 - t0) : 0;
#pragma unroll
        for (int u = 0; u < kWideTile; u++) xn[u] = u < nr ? a[(t0 + u) * ld + col] : 0.f;
        const float4 *src = reinterpret_cast<const float4 *>(g + t0 * N);
#pragma unroll
        for (int k = 0; k < kGPer; k++) {
            const int e = c + W * k;
            gn[k] = e < nr * N / 4 ? src[e] : make_float4(0.f, 0.f, 0.f, 0.f);
        }
    };
    fetch(p0 + rg * kWideTile);
    for (int64_t base = p0; base < p1; base += step) {  // uniform trip count over the workgroup
        const int64_t t0 = base + rg * kWideTile;
        const int nr = t0 < p1 ? (int)min((int64_t)kWideTile, p1 - t0) : 0;
        float x[kWideTile];
#pragma unroll
        for (int u = 0; u < kWideTile; u++) x[u] = xn[u];
        __syncthreads();  // the previous tile's LDS reads are done
#pragma unroll
        for (int k = 0; k < kGPer; k++) {
            const int e = c + W * k;
            if (e < kG4) s_g[rg][e] = gn[k];
        }
        __syncthreads();
        if (t0 + step < p1) fetch(t0 + step);
        const float4 *sg = s_g[rg];
        if (c < N)
            for (int u = 0; u < nr; u++) bsum += reinterpret_cast<const float *>(sg)[u * N + c];
        for (int u = 0; u < nr; u++) {
            hf2 sd0 = hf2{0.f, 0.f}, sd1 = hf2{0.f, 0.f};
            const hf2 xx = hf2{x[u], x[u]};
#pragma unroll
            for (int q = 0; q < N / 4; q++) {
                const float4 gv = sg[u * (N / 4) + q];
                const hf2 ga = hf2{gv.x, gv.y}, gb = hf2{gv.z, gv.w};
                sd0 = __builtin_elementwise_fma(ga, w[2 * q], sd0);
                sd1 = __builtin_elementwise_fma(gb, w[2 * q + 1], sd1);
                acc[2 * q] = __builtin_elementwise_fma(ga, xx, acc[2 * q]);
                acc[2 * q + 1] = __builtin_elementwise_fma(gb, xx, acc[2 * q + 1]);
            }
            const float gvv = x[u] > 0.f ? (sd0.x + sd0.y) + (sd1.x + sd1.y) : 0.f;
            da[(t0 + u) * ld + col] = gvv;
            csum += gvv;
        }
    }
    // combine the row groups in group order (deterministic) into group 0's registers
    for (int sgp = 1; sgp < kWideGroups; sgp++) {
        __syncthreads();
        if (rg == sgp) {
#pragma unroll
            for (int r = 0; r < N / 2; r++) {
                s_red[(2 * r) * 128 + c] = acc[r].x;
                s_red[(2 * r + 1) * 128 + c] = acc[r].y;
            }
            s_red[N * 128 + c] = csum;
            s_red[N * 128 + 128 + c] = bsum;
        }
        __syncthreads();
        if (rg == 0) {
#pragma unroll
            for (int r = 0; r < N / 2; r++) {
                acc[r].x += s_red[(2 * r) * 128 + c];
                acc[r].y += s_red[(2 * r + 1) * 128 + c];
            }
            csum += s_red[N * 128 + c];
            bsum += s_red[N * 128 + 128 + c];
        }
    }
    if (rg != 0) return;
    float *pw = part + (size_t)blockIdx.x * A.poff[1];
    pw[c] = csum;
    float *ph = pw + A.poff[0];
#pragma unroll
    for (int r = 0; r < N / 2; r++) {
        ph[(2 * r) * (W + 1) + c] = acc[r].x;
        ph[(2 * r + 1) * (W + 1) + c] = acc[r].y;
    }
    if (c < N) ph[c * (W + 1) + W] = bsum;
}

// The wide head on the f32 MFMA (v_mfma_f32_16x16x4_f32), for W in {64, 128} and N a multiple of 16:
// a wave takes 16-row blocks and forms
//   da (16 x W) = (a > 0) * (g (16 x N) W2 (N x W)):  lane group q = l >> 4 reads columns 4q..4q+3 of its
//       g row l & 15 per 16-column K chunk as one float4 (k index of step s = column 4q + s); W2^T in LDS
//       (row stride N + 4) is the B operand;
//   dW2 (N x W) += g^T a:  K = the 16 rows, lane group q takes rows 4q..4q+3 (k index of step s = row
//       4q + s), so the a values it needs are exactly the ones the da mask reads at the C positions
//       (rows 4q + j, columns 16t + c): loaded once, used twice;
//   db1 (column sums of da) and db2 (column sums of g) on the way.
// The waves' partials are added in wave order in LDS, the workgroups' by heads_bwd_reduce_kernel (the
// same partial layout as heads_bwd_wide_kernel).
template <int W, int N, class TA>
__global__ __launch_bounds__(256) void heads_bwd_wide_mfma_kernel(HbArgs A, const TA *__restrict__ a,
                                                                   TA *__restrict__ da,
                                                                   const float *__restrict__ g,
                                                                   float *__restrict__ part) {
    // each wave takes half of the head's W columns (CT tiles of 16) of a row block: waves 2i and 2i + 1
    // share block i's rows; only the first half accumulates db2 (g's column sums)
    constexpr int CT = W / 32, MT = N / 16, NKC = N / 16, WS = N + 4, NWV = 4;
    constexpr int PER = W + N * (W + 1);  // partial: db1 (W) then for each output r: dW2[r][0..W), db2[r]
    __shared__ float s_w2t[W * WS];
    __shared__ float s_red[PER];
    const int ld = A.k * W, h = A.h0;
    const float *__restrict__ w2 = A.w2[h];
    for (int e = threadIdx.x; e < N * W; e += 256) {  // W2 (N x W) -> W2^T rows
        const int r = e / W, col = e % W;
        s_w2t[col * WS + r] = w2[e];
    }
    __syncthreads();
    const int lane = threadIdx.x & 63, wv = (int)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6), q = lane >> 4, c = lane & 15;
    const int half = wv & 1, cb = half * (W / 2);  // this wave's first column
    f4v accw[MT][CT];
#pragma unroll
    for (int m = 0; m < MT; m++)
#pragma unroll
        for (int t = 0; t < CT; t++) accw[m][t] = f4v{0.f, 0.f, 0.f, 0.f};
    float csum[CT], bsum[MT];
#pragma unroll
    for (int t = 0; t < CT; t++) csum[t] = 0.f;
#pragma unroll
    for (int m = 0; m < MT; m++) bsum[m] = 0.f;
    const int P = A.P, nblk = (P + 15) / 16;
    const TA *acol = a + h * W + cb;
    TA *dacol = da + h * W + cb;
    // a block's loads: g rows as the da A operand, g at (row 4q + s, output 16m + c) as the dW2 A operand,
    // a at the C positions (row 4q + j, column 16t + c); issued one block ahead of their use
    float4 gA[NKC];
    float gT[MT][4];
    TA av[CT][4];  // raw elements, widened when the block comes up (see heads_bwd_cols)
    // rows past P (and the prefetch past the last block) read row P - 1: the loads are unconditional, so
    // the compiler's waits count exactly the loads issued after a block's (a branch around them made it wait
    // for every load in flight, the next block's prefetch included); such rows are masked when the block
    // comes up
    auto load_block = [&](int blk) {
        const int r0 = blk * 16, rg = min(r0 + c, P - 1);
#pragma unroll
        for (int kc = 0; kc < NKC; kc++) gA[kc] = *reinterpret_cast<const float4 *>(g + (size_t)rg * N + 16 * kc + 4 * q);
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int r = min(r0 + 4 * q + j, P - 1);
#pragma unroll
            for (int m = 0; m < MT; m++) gT[m][j] = g[(size_t)r * N + 16 * m + c];
#pragma unroll
            for (int t = 0; t < CT; t++) av[t][j] = acol[(size_t)r * ld + 16 * t + c];
        }
    };
    const int stride = gridDim.x * (NWV / 2);
    int blk = blockIdx.x * (NWV / 2) + (wv >> 1);
    load_block(blk);
    for (; blk < nblk; blk += stride) {
        const int r0 = blk * 16;
        float4 gAc[NKC];
        float gTc[MT][4], avc[CT][4];
#pragma unroll
        for (int kc = 0; kc < NKC; kc++) gAc[kc] = gA[kc];  // rows past P: da rows neither stored nor summed
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const bool ok = r0 + 4 * q + j < P;
#pragma unroll
            for (int m = 0; m < MT; m++) gTc[m][j] = ok ? gT[m][j] : 0.f;
#pragma unroll
            for (int t = 0; t < CT; t++) avc[t][j] = ok ? (float)av[t][j] : 0.f;
        }
        load_block(blk + stride);
        // da
#pragma unroll
        for (int t = 0; t < CT; t++) {
            f4v acc = f4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int kc = 0; kc < NKC; kc++) {
                const float4 bv = *reinterpret_cast<const float4 *>(s_w2t + (cb + 16 * t + c) * WS + 16 * kc + 4 * q);
                acc = __builtin_amdgcn_mfma_f32_16x16x4f32(gAc[kc].x, bv.x, acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_16x16x4f32(gAc[kc].y, bv.y, acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_16x16x4f32(gAc[kc].z, bv.z, acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_16x16x4f32(gAc[kc].w, bv.w, acc, 0, 0, 0);
            }
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const int r = r0 + 4 * q + j;
                const float v = avc[t][j] > 0.f ? acc[j] : 0.f;
                if (r < P) dacol[(size_t)r * ld + 16 * t + c] = (TA)v;
                csum[t] += v;
            }
        }
        // dW2 += g^T a, db2
#pragma unroll
        for (int m = 0; m < MT; m++) {
#pragma unroll
            for (int j = 0; j < 4; j++) bsum[m] += gTc[m][j];
#pragma unroll
            for (int t = 0; t < CT; t++)
#pragma unroll
                for (int j = 0; j < 4; j++)
                    accw[m][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(gTc[m][j], avc[t][j], accw[m][t], 0, 0, 0);
        }
    }
    // wave partials -> LDS: the two halves' column ranges are disjoint; waves of the same half are
    // added in wave order (accw C layout: row = output 16m + 4q + j, column cb + 16t + c); db1 / db2: the
    // 4 lane groups (q) of a column added in q order; db2 from the first half only
    for (int qw = 0; qw < NWV; qw++) {
        __syncthreads();
        if (wv == qw) {
            const bool first = qw < 2;  // the first wave of this half
#pragma unroll
            for (int m = 0; m < MT; m++)
#pragma unroll
                for (int t = 0; t < CT; t++)
#pragma unroll
                    for (int j = 0; j < 4; j++) {
                        float &d = s_red[W + (16 * m + 4 * q + j) * (W + 1) + cb + 16 * t + c];
                        d = first ? accw[m][t][j] : d + accw[m][t][j];
                    }
            for (int qq = 0; qq < 4; qq++) {
                if (q == qq) {
#pragma unroll
                    for (int t = 0; t < CT; t++) {
                        float &d = s_red[cb + 16 * t + c];
                        d = (first && qq == 0) ? csum[t] : d + csum[t];
                    }
                    if (half == 0) {
#pragma unroll
                        for (int m = 0; m < MT; m++) {
                            float &d = s_red[W + (16 * m + c) * (W + 1) + W];
                            d = (first && qq == 0) ? bsum[m] : d + bsum[m];
                        }
                    }
                }
                __builtin_amdgcn_s_waitcnt(0xc07f);
                __builtin_amdgcn_wave_barrier();
            }
        }
    }
    __syncthreads();
    float *pw = part + (size_t)blockIdx.x * PER;
    for (int i = threadIdx.x; i < PER; i += 256) pw[i] = s_red[i];
}

// the partials summed over the workgroups (32 record entries per workgroup, 8 eighths in a fixed
// order) and routed to db1 / dW2_i / db2_i
struct HbOut {
    float *db1;
    float *dw2[kHbMaxHeads];
    float *db2[kHbMaxHeads];
};
// 16 outputs per workgroup (16 interleaved sixteenths of the workgroups each, combined in a fixed order): the
// ~2k outputs of a launch then fill ~120 CUs instead of ~60
constexpr int kHbRedOut = 16, kHbRedSlices = 256 / kHbRedOut;
// One launch reduces the partials of up to kHbRedGroups launch groups (the narrow heads' and the wide head's):
// group g owns workgroups [blk0[g], blk0[g + 1]).
constexpr int kHbRedGroups = 2;
struct HbRed {
    HbArgs A[kHbRedGroups];
    const float *part[kHbRedGroups];
    int nwg[kHbRedGroups];
    int blk0[kHbRedGroups + 1];
    int count;
};
__global__ __launch_bounds__(256) void heads_bwd_reduce_kernel(HbRed R, HbOut O) {
    __shared__ float s_sum[kHbRedSlices][kHbRedOut];
    int gi = 0;
    while (gi + 1 < R.count && (int)blockIdx.x >= R.blk0[gi + 1]) gi++;
    const HbArgs &A = R.A[gi];
    const float *__restrict__ part = R.part[gi];
    const int nwg = R.nwg[gi];
    const int per = A.poff[A.hk];
    const int o = threadIdx.x % kHbRedOut, q = threadIdx.x / kHbRedOut;
    const int i = ((int)blockIdx.x - R.blk0[gi]) * kHbRedOut + o;
    float v0 = 0.f, v1 = 0.f, v2 = 0.f, v3 = 0.f;
    if (i < per) {
        int w = q;
        constexpr int K = kHbRedSlices;
        for (; w + 7 * K < nwg; w += 8 * K) {  // eight loads in flight per thread (the kernel is latency-bound)
            float x[8];
#pragma unroll
            for (int u = 0; u < 8; u++) x[u] = part[(size_t)(w + u * K) * per + i];
            v0 += x[0]; v1 += x[1]; v2 += x[2]; v3 += x[3];
            v0 += x[4]; v1 += x[5]; v2 += x[6]; v3 += x[7];
        }
        for (; w + 3 * K < nwg; w += 4 * K) {
            v0 += part[(size_t)w * per + i];
            v1 += part[(size_t)(w + K) * per + i];
            v2 += part[(size_t)(w + 2 * K) * per + i];
            v3 += part[(size_t)(w + 3 * K) * per + i];
        }
        for (; w < nwg; w += K) v0 += part[(size_t)w * per + i];
    }
    s_sum[q][o] = (v0 + v1) + (v2 + v3);
    __syncthreads();
    if (q == 0 && i < per) {
        float t = 0.f;
#pragma unroll
        for (int e = 0; e < kHbRedSlices; e++) t += s_sum[e][o];
        if (i < A.poff[0]) {
            O.db1[A.h0 * A.W + i] = t;
        } else {
            int hl = 0;
            while (hl + 1 < A.hk && i >= A.poff[hl + 1]) hl++;
            const int e = i - A.poff[hl], r = e / (A.W + 1), c = e - r * (A.W + 1);
            if (c < A.W) O.dw2[A.h0 + hl][r * A.W + c] = t;
            else O.db2[A.h0 + hl][r] = t;
        }
    }
}

static int dw_rows_per_wg(int P, int nmax) {
    // enough workgroups to cover the chip, few enough that the partials stay small next to x
    (void)P;
    return nmax <= 8 ? 256 : 1024;
}


// ---- the deformation field's first layer, backward (scene/deformation.py:51-55 with defor_depth <= 1:
// hidden = feature_out(x) = x W^T + b; every head starts with ReLU, so the heads read h = relu(hidden)).
// Given g = dL/dh, ONE pass over the rows forms dz = g * (h > 0) and both GEMMs on the f32 MFMA
// (v_mfma_f32_16x16x4_f32: exact f32, a k-ordered fma chain):
//   dx = dz W   (rows x Fin)   and   dW += dz^T x,  db += column sums of dz  (per-wave partials).
// A wave takes 16-row blocks: g and h rows are read coalesced (lanes along the outputs), dz is staged
// in an LDS tile, W lives in LDS.  At the end the
// workgroup's waves add their dW / db partials in wave order and a second launch sums the workgroups'
// partials in workgroup order (deterministic).
constexpr int kFbThreads = 256, kFbRows = 16;

template <int FIN, int FOUT>
__global__ __launch_bounds__(kFbThreads) void feature_bwd_kernel(int P, const float *__restrict__ g,
                                                                 const float *__restrict__ h,
                                                                 const float *__restrict__ x,
                                                                 const float *__restrict__ w, float *__restrict__ dx,
                                                                 float *__restrict__ part) {
    constexpr int NB = FIN / 16, MB = FOUT / 16, NW = kFbThreads / 64;
    // tile row stride = 17 (mod 64) words: the 16-row column reads of dx and the 4-row x 16-column reads
    // of dW both spread over the LDS banks
    constexpr int TS = FOUT + 17;
    constexpr int PER = FOUT * FIN + FOUT;  // one partial: dW (row-major) then db
    __shared__ float s_w[FOUT * FIN + FOUT];
    __shared__ float s_t[NW][kFbRows * TS];
    const int lane = threadIdx.x & 63, wv = (int)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    for (int i = threadIdx.x; i < FOUT * FIN / 4; i += kFbThreads)
        reinterpret_cast<float4 *>(s_w)[i] = reinterpret_cast<const float4 *>(w)[i];
    __syncthreads();
    float *t = s_t[wv];
    f4v accw[MB][NB];
#pragma unroll
    for (int m = 0; m < MB; m++)
#pragma unroll
        for (int n = 0; n < NB; n++) accw[m][n] = f4v{0.f, 0.f, 0.f, 0.f};
    float db0 = 0.f, db1 = 0.f;                  // this lane's output pair (o, o + 1)
    const int o = (2 * lane) % FOUT, rofs = (2 * lane) / FOUT;
    constexpr int RPI = 128 / FOUT;              // rows per coalesced load instruction
    const int nblk = (P + kFbRows - 1) / kFbRows;
    // block loads (g, h rows: lanes along the outputs; x rows as the B operand of dW:
    // B[k = row 4s + (l >> 4)][n = 16 nb + (l & 15)]), issued one block ahead of their use
    constexpr int NIT = kFbRows / RPI;
    float2 gv[NIT], hv[NIT];
    float xb[4][NB];
    // rows past P (and the prefetch past the last block) read row P - 1, masked when the block comes up:
    // unconditional loads let the compiler's waits count exactly the loads issued after a block's (with a
    // branch around them it waited for every load in flight, the next block's prefetch included)
    auto load_block = [&](int blk) {
        const int r0 = blk * kFbRows;
#pragma unroll
        for (int it = 0; it < NIT; it++) {
            const int r = min(r0 + it * RPI + rofs, P - 1);
            gv[it] = *reinterpret_cast<const float2 *>(g + (size_t)r * FOUT + o);
            hv[it] = *reinterpret_cast<const float2 *>(h + (size_t)r * FOUT + o);
        }
#pragma unroll
        for (int st = 0; st < 4; st++) {
            const int r = min(r0 + 4 * st + (lane >> 4), P - 1);
#pragma unroll
            for (int n = 0; n < NB; n++) xb[st][n] = x[(size_t)r * FIN + 16 * n + (lane & 15)];
        }
    };
    const int stride = gridDim.x * NW;
    int blk = blockIdx.x * NW + wv;
    load_block(blk);
    for (; blk < nblk; blk += stride) {
        const int r0 = blk * kFbRows;
        // dz = g * (h > 0) into the tile, column sums into db
#pragma unroll
        for (int it = 0; it < NIT; it++) {
            const int row = it * RPI + rofs;
            const bool ok = r0 + row < P;
            const float d0 = ok && hv[it].x > 0.f ? gv[it].x : 0.f, d1 = ok && hv[it].y > 0.f ? gv[it].y : 0.f;
            db0 += d0;
            db1 += d1;
            t[row * TS + o] = d0;
            t[row * TS + o + 1] = d1;
        }
        float xc[4][NB];
#pragma unroll
        for (int st = 0; st < 4; st++) {
            const bool ok = r0 + 4 * st + (lane >> 4) < P;
#pragma unroll
            for (int n = 0; n < NB; n++) xc[st][n] = ok ? xb[st][n] : 0.f;
        }
        load_block(blk + stride);  // the next block's loads fly while this one runs on the MFMA
        __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the tile is written (LDS is in order per wave)
        __builtin_amdgcn_wave_barrier();
        // dx = dz W: A[row l & 15][k = o 4s + (l >> 4)], B[k = o][n = 16 nb + (l & 15)]
        f4v accx[NB];
#pragma unroll
        for (int n = 0; n < NB; n++) accx[n] = f4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll 8
        for (int st = 0; st < FOUT / 4; st++) {
            const int ok = 4 * st + (lane >> 4);
            const float av = t[(lane & 15) * TS + ok];
#pragma unroll
            for (int n = 0; n < NB; n++)
                accx[n] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, s_w[ok * FIN + 16 * n + (lane & 15)], accx[n], 0, 0, 0);
        }
        // C[row (l >> 4) * 4 + i][col 16 nb + (l & 15)]
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const int r = r0 + (lane >> 4) * 4 + i;
            if (r < P) {
#pragma unroll
                for (int n = 0; n < NB; n++) dx[(size_t)r * FIN + 16 * n + (lane & 15)] = accx[n][i];
            }
        }
        // dW += dz^T x: A[m = o 16 mb + (l & 15)][k = row 4s + (l >> 4)], B = xb
#pragma unroll
        for (int st = 0; st < 4; st++) {
#pragma unroll
            for (int m = 0; m < MB; m++) {
                const float av = t[(4 * st + (lane >> 4)) * TS + 16 * m + (lane & 15)];
#pragma unroll
                for (int n = 0; n < NB; n++)
                    accw[m][n] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, xc[st][n], accw[m][n], 0, 0, 0);
            }
        }
        __builtin_amdgcn_wave_barrier();  // the tile's reads are done before the next block overwrites it
    }
    // the waves' partials added in wave order in LDS (W is no longer needed there)
    for (int q = 0; q < NW; q++) {
        __syncthreads();
        if (wv == q) {
#pragma unroll
            for (int m = 0; m < MB; m++)
#pragma unroll
                for (int n = 0; n < NB; n++)
#pragma unroll
                    for (int i = 0; i < 4; i++) {
                        float &dst = s_w[(16 * m + (lane >> 4) * 4 + i) * FIN + 16 * n + (lane & 15)];
                        dst = q == 0 ? accw[m][n][i] : dst + accw[m][n][i];
                    }
            // db: lanes with the same outputs (RPI > 1) add in lane order
#pragma unroll
            for (int rr = 0; rr < RPI; rr++) {
                if (rofs == rr) {
                    float &d0 = s_w[FOUT * FIN + o], &d1 = s_w[FOUT * FIN + o + 1];
                    d0 = (q == 0 && rr == 0) ? db0 : d0 + db0;
                    d1 = (q == 0 && rr == 0) ? db1 : d1 + db1;
                }
                __builtin_amdgcn_s_waitcnt(0xc07f);
                __builtin_amdgcn_wave_barrier();
            }
        }
    }
    __syncthreads();
    float *dst = part + (size_t)blockIdx.x * PER;
    for (int i = threadIdx.x; i < PER; i += kFbThreads) dst[i] = s_w[i];
}

// dW / db = the workgroups' partials summed in workgroup order: 16 outputs per workgroup, 16 threads per
// output each summing a strided slice of the partials (all loads independent), then the 16 slices
// added in slice order
__global__ __launch_bounds__(256) void feature_bwd_reduce_kernel(int nwg, int per, int nwb, const float *__restrict__ part,
                                                                 float *__restrict__ dw, float *__restrict__ db) {
    __shared__ float s_sum[16][17];
    const int oi = threadIdx.x & 15, sl = threadIdx.x >> 4;
    const int i = blockIdx.x * 16 + oi;
    float acc = 0.f;
    if (i < per) {
        int k = sl;
        for (; k + 112 < nwg; k += 128) {  // eight loads in flight per thread (the kernel is latency-bound)
            float x[8];
#pragma unroll
            for (int u = 0; u < 8; u++) x[u] = part[(size_t)(k + 16 * u) * per + i];
#pragma unroll
            for (int u = 0; u < 8; u++) acc += x[u];
        }
        for (; k + 48 < nwg; k += 64) {
            const float a0 = part[(size_t)k * per + i], a1 = part[(size_t)(k + 16) * per + i];
            const float a2 = part[(size_t)(k + 32) * per + i], a3 = part[(size_t)(k + 48) * per + i];
            acc += a0;
            acc += a1;
            acc += a2;
            acc += a3;
        }
        for (; k < nwg; k += 16) acc += part[(size_t)k * per + i];
    }
    s_sum[sl][oi] = acc;
    __syncthreads();
    if (sl == 0 && i < per) {
        float t = 0.f;
        for (int q = 0; q < 16; q++) t += s_sum[q][oi];
        if (i < nwb) dw[i] = t;
        else db[i - nwb] = t;
    }
}
// ---- the deformation heads' second layers, forward (scene/deformation.py:73-78 as one block: head i =
// a[:, iW:(i+1)W] W2_i^T + b2_i on a = relu(h W1^T + b1), (P, kW)) in ONE pass over a on the f32 MFMA
// (v_mfma_f32_16x16x4_f32), where torch runs k small GEMMs on column slices.  A wave takes 16-row
// blocks; for each head and 16-column K chunk the wave reads a as float4 straight from HBM (lane group
// q = l >> 4 holds columns 4q..4q+3 of its row l & 15: the MFMA's k index in step s is column 4q + s,
// so each lane's 4 steps come from one 16-byte load), the matching W2 rows (staged in LDS, row stride
// W + 4: conflict-free 16-byte reads) are the B operand, one accumulator per 16 outputs of the head.
struct HfArgs {
    int P, W, k, kW;  // kW: the row stride of a (floats)
    int n[kHbMaxHeads];
    int roff[kHbMaxHeads];  // head i's first row in the LDS copy of the W2s
    const float *w2[kHbMaxHeads];
    const float *b2[kHbMaxHeads];
    float *out[kHbMaxHeads];
};
constexpr int kHfThreads = 256, kHfMaxTiles = 4;  // up to 64 outputs per head

// NT...: tiles of 16 outputs per head, compile-time, so that every head's accumulators are registers
// and ALL heads advance together through each 16-column K chunk (sum NT independent MFMA chains; the
// next chunk's loads are issued before this chunk's MFMAs).
template <int W, int... NT>
__global__ __launch_bounds__(kHfThreads) void heads_fwd_kernel(HfArgs A, const float *__restrict__ a) {
    constexpr int K = sizeof...(NT);
    constexpr int nt[K] = {NT...};
    extern __shared__ float4 s_w2v[];
    float *s_w2 = reinterpret_cast<float *>(s_w2v);
    constexpr int WS = W + 4;
    for (int i = 0; i < K; i++)
        for (int e = threadIdx.x; e < A.n[i] * (W / 4); e += kHfThreads) {
            const int row = e / (W / 4), c4 = e % (W / 4);
            reinterpret_cast<float4 *>(s_w2 + (size_t)(A.roff[i] + row) * WS)[c4] =
                reinterpret_cast<const float4 *>(A.w2[i] + (size_t)row * W)[c4];
        }
    __syncthreads();
    const int lane = threadIdx.x & 63, wv = (int)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6), q = lane >> 4, c = lane & 15;
    const int nblk = (A.P + 15) / 16;
    for (int blk = blockIdx.x * (kHfThreads / 64) + wv; blk < nblk; blk += gridDim.x * (kHfThreads / 64)) {
        const int r0 = blk * 16, ra = r0 + c;
        const bool live = ra < A.P;
        const float *arow = a + (size_t)min(ra, A.P - 1) * A.kW + 4 * q;
        f4v acc[K][4];
#pragma unroll
        for (int i = 0; i < K; i++)
#pragma unroll
            for (int t = 0; t < 4; t++) acc[i][t] = f4v{0.f, 0.f, 0.f, 0.f};
        float4 av[K], an[K];
#pragma unroll
        for (int i = 0; i < K; i++) an[i] = *reinterpret_cast<const float4 *>(arow + i * W);
#pragma unroll 2
        for (int kc = 0; kc < W / 16; kc++) {
#pragma unroll
            for (int i = 0; i < K; i++) av[i] = live ? an[i] : make_float4(0.f, 0.f, 0.f, 0.f);
            if (kc + 1 < W / 16) {
#pragma unroll
                for (int i = 0; i < K; i++) an[i] = *reinterpret_cast<const float4 *>(arow + i * W + 16 * (kc + 1));
            }
#pragma unroll
            for (int i = 0; i < K; i++) {
#pragma unroll
                for (int t = 0; t < nt[i]; t++) {
                    const int nn = 16 * t + c;
                    const float4 bv = nn < A.n[i] ? *reinterpret_cast<const float4 *>(
                                                        s_w2 + (size_t)(A.roff[i] + nn) * WS + 16 * kc + 4 * q)
                                                  : make_float4(0.f, 0.f, 0.f, 0.f);
                    acc[i][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[i].x, bv.x, acc[i][t], 0, 0, 0);
                    acc[i][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[i].y, bv.y, acc[i][t], 0, 0, 0);
                    acc[i][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[i].z, bv.z, acc[i][t], 0, 0, 0);
                    acc[i][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[i].w, bv.w, acc[i][t], 0, 0, 0);
                }
            }
        }
        // C[row 4q + j][col 16 t + c]
#pragma unroll
        for (int i = 0; i < K; i++) {
#pragma unroll
            for (int t = 0; t < nt[i]; t++) {
                const int col = 16 * t + c, n = A.n[i];
                if (col < n) {
                    const float bias = A.b2[i][col];
#pragma unroll
                    for (int j = 0; j < 4; j++) {
                        const int r = r0 + 4 * q + j;
                        if (r < A.P) A.out[i][(size_t)r * n + col] = acc[i][t][j] + bias;
                    }
                }
            }
        }
    }
}
// ---- the whole heads block, forward (scene/deformation.py:73-78: head i = relu(h W1_i^T + b1_i) W2_i^T + b2_i
// on the shared h = relu(hidden)), first AND second layers in one pass on the f32 MFMA
// (v_mfma_f32_16x16x4_f32), where torch runs one (P x W) @ (W x kW) GEMM for the first layers and this
// library's heads_fwd pass read its (P, kW) result back.  Workgroup (x, head i): w1_i (W x W) and w2_i
// (n_i x W) staged in LDS, its waves each taking 16-point blocks.  Both layers are computed TRANSPOSED
// (features along the MFMA rows, the 16 points along its columns), so the first layer's accumulators are
// already the second layer's B operand: in k-step (t, v) lane l supplies feature 16 t + 4 (l >> 4) + v of
// point l & 15 -- the v-th register of its t-th accumulator (D[4 (l >> 4) + v][l & 15]) -- and the A operand
// (w1 / w2 rows from LDS, one 16-byte read per 4 MFMAs; row stride W + 8 floats, conflict-free for ds_read_b128's
// four 16-lane groups -- round 5's W + 4 put two lanes of a group on one bank slot: 9.4M conflict cycles per
// launch) uses the same feature order; 16 waves per workgroup, one workgroup per CU.  h is read as that
// B operand directly (one float4 per lane per 16 features); a = relu(z + b1) is written once, for the
// backward, and never read back.
constexpr int kHbfThreads = 512;
template <int W>
__global__ __launch_bounds__(kHbfThreads) void heads_block_fwd_kernel(HfArgs A, const float *__restrict__ h,
                                                                      const float *__restrict__ w1,
                                                                      const float *__restrict__ b1,
                                                                      float *__restrict__ a,
                                                                      float *__restrict__ w1t) {
    constexpr int NT = W / 16, WS = W + 8, NW = kHbfThreads / 64;
    extern __shared__ float4 s_v[];
    float *s_w1 = reinterpret_cast<float *>(s_v);  // W rows x WS
    float *s_b1 = s_w1 + W * WS;                   // W
    float *s_w2 = s_b1 + W;                        // n_pad rows x WS (rows >= n zero)
    const int head = blockIdx.y;
    const int n = A.n[head], npad = (n + 15) & ~15;
    float *s_b2 = s_w2 + npad * WS;  // n_pad (in LDS: a global load in the store loop would wait for every
                                     // load and store in flight, the next block's h prefetch included)
    const float *w1i = w1 + (size_t)head * W * W;
    for (int e = threadIdx.x; e < W * W / 4; e += kHbfThreads) {
        const int row = e / (W / 4), c4 = e % (W / 4);
        reinterpret_cast<float4 *>(s_w1 + row * WS)[c4] = reinterpret_cast<const float4 *>(w1i + (size_t)row * W)[c4];
    }
    for (int e = threadIdx.x; e < W; e += kHbfThreads) s_b1[e] = b1[head * W + e];
    for (int e = threadIdx.x; e < npad * (W / 4); e += kHbfThreads) {
        const int row = e / (W / 4), c4 = e % (W / 4);
        reinterpret_cast<float4 *>(s_w2 + row * WS)[c4] =
            row < n ? reinterpret_cast<const float4 *>(A.w2[head] + (size_t)row * W)[c4] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    for (int e = threadIdx.x; e < npad; e += kHbfThreads) s_b2[e] = e < n ? A.b2[head][e] : 0.f;
    __syncthreads();
    if (w1t && blockIdx.x == 0) {
        // workgroup 0 of each head also writes W1_i^T for the backward's input gradient (gs4d_mlp_dx_f32): 4 rows
        // of one column of the LDS image per 16-byte store
        for (int e = threadIdx.x; e < W * W / 4; e += kHbfThreads) {
            const int col = e / (W / 4), r4 = e % (W / 4);
            *reinterpret_cast<float4 *>(w1t + (size_t)col * A.kW + head * W + 4 * r4) =
                make_float4(s_w1[(4 * r4) * WS + col], s_w1[(4 * r4 + 1) * WS + col], s_w1[(4 * r4 + 2) * WS + col],
                            s_w1[(4 * r4 + 3) * WS + col]);
        }
    }
    const int lane = threadIdx.x & 63, wv = (int)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6), q = lane >> 4, c = lane & 15;
    const int nblk = (A.P + 15) / 16;
    const int stride = gridDim.x * NW;
    float *out = A.out[head];
    const bool v4out = (n & 3) == 0 && ((size_t)out & 15) == 0;
    float4 hn[NT];
    // rows past P (the last block's, and the prefetch past the last block) read row P - 1: every load is
    // unconditional, so the compiler's wait before a block's MFMAs counts exactly the loads issued after its
    // h (a branch around them made it wait for ALL loads, the next block's prefetch included); those rows'
    // results go to a's padding rows or are not stored
    auto load_h = [&](int blk) {
        const int pt = min(blk * 16 + c, A.P - 1);
#pragma unroll
        for (int t = 0; t < NT; t++) hn[t] = *reinterpret_cast<const float4 *>(h + (size_t)pt * W + 16 * t + 4 * q);
    };
    int blk = blockIdx.x * NW + wv;
    load_h(blk);
    for (; blk < nblk; blk += stride) {
        float4 hv[NT];
#pragma unroll
        for (int t = 0; t < NT; t++) hv[t] = hn[t];
        load_h(blk + stride);  // the next block's h loads fly while this one runs on the MFMA
        // z^T (W x 16) = W1_i h^T (a compiler barrier per 16-feature chunk keeps the LDS reads of one chunk,
        // 8 float4, in registers at a time)
        f4v acc[NT];
#pragma unroll
        for (int m = 0; m < NT; m++) acc[m] = f4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int t = 0; t < NT; t++) {
            asm volatile("" ::: "memory");
#pragma unroll
            for (int m = 0; m < NT; m++) {
                const float4 av = *reinterpret_cast<const float4 *>(s_w1 + (16 * m + c) * WS + 16 * t + 4 * q);
                acc[m] = __builtin_amdgcn_mfma_f32_16x16x4f32(av.x, hv[t].x, acc[m], 0, 0, 0);
                acc[m] = __builtin_amdgcn_mfma_f32_16x16x4f32(av.y, hv[t].y, acc[m], 0, 0, 0);
                acc[m] = __builtin_amdgcn_mfma_f32_16x16x4f32(av.z, hv[t].z, acc[m], 0, 0, 0);
                acc[m] = __builtin_amdgcn_mfma_f32_16x16x4f32(av.w, hv[t].w, acc[m], 0, 0, 0);
            }
        }
        // a = relu(z + b1): lane holds features 16 m + 4 q + j of point c; written as float4 per m
        const int pt = blk * 16 + c;
#pragma unroll
        for (int m = 0; m < NT; m++) {
            const float4 bb = *reinterpret_cast<const float4 *>(s_b1 + 16 * m + 4 * q);
            acc[m][0] = fmaxf(acc[m][0] + bb.x, 0.f);
            acc[m][1] = fmaxf(acc[m][1] + bb.y, 0.f);
            acc[m][2] = fmaxf(acc[m][2] + bb.z, 0.f);
            acc[m][3] = fmaxf(acc[m][3] + bb.w, 0.f);
            // a has ceil(P / 16) * 16 rows (gs4d_heads_block_forward): no condition on the store
            *reinterpret_cast<float4 *>(a + (size_t)pt * A.kW + head * W + 16 * m + 4 * q) =
                make_float4(acc[m][0], acc[m][1], acc[m][2], acc[m][3]);
        }
        // out^T (n_pad x 16) = W2_i a^T, B operand = the accumulators above
        for (int j = 0; j < npad; j += 16) {
            f4v o = f4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int m = 0; m < NT; m++) {
                const float4 wv4 = *reinterpret_cast<const float4 *>(s_w2 + (j + c) * WS + 16 * m + 4 * q);
                o = __builtin_amdgcn_mfma_f32_16x16x4f32(wv4.x, acc[m][0], o, 0, 0, 0);
                o = __builtin_amdgcn_mfma_f32_16x16x4f32(wv4.y, acc[m][1], o, 0, 0, 0);
                o = __builtin_amdgcn_mfma_f32_16x16x4f32(wv4.z, acc[m][2], o, 0, 0, 0);
                o = __builtin_amdgcn_mfma_f32_16x16x4f32(wv4.w, acc[m][3], o, 0, 0, 0);
            }
            // D[output j + 4 q + r][point c]: one float4 per lane when the rows are 16-byte aligned
            if (pt < A.P) {
                const int o0 = j + 4 * q;
                if (v4out && o0 + 3 < n) {
                    const float4 bb = *reinterpret_cast<const float4 *>(s_b2 + o0);
                    *reinterpret_cast<float4 *>(out + (size_t)pt * n + o0) =
                        make_float4(o[0] + bb.x, o[1] + bb.y, o[2] + bb.z, o[3] + bb.w);
                } else {
#pragma unroll
                    for (int r = 0; r < 4; r++)
                        if (o0 + r < n) out[(size_t)pt * n + o0 + r] = o[r] + s_b2[o0 + r];
                }
            }
        }
    }
}

// ---- the heads block forward on bf16 operands (hyper.mlp_dtype = "bf16", BASELINE C3's bf16 leg): the
// structure of heads_block_fwd_kernel on v_mfma_f32_16x16x32_bf16 (16x the f32 MFMA's rate), fp32
// accumulation, fp32 outputs.  Workgroup (x, head i): W1_i and W2_i converted to bf16 into LDS (row stride
// W + 8 elements); per 16-point block the first layer z^T (W x 16) = W1_i h^T is TRANSPOSED as in the f32
// kernel: in k-step t lane (q = l >> 4, c = l & 15) supplies h[point c][32 t + 8 q .. + 7] (converted to bf16
// on load) and W1_i[16 m + c][32 t + 8 q .. + 7] (one 16-byte LDS read); accumulator m then holds
// z[16 m + 4 q + v][point c], v = 0..3.  a = relu(z + b1) is rounded to bf16 once: stored (8 bytes per tile,
// for the backward) and used as the second layer's B operand straight from the registers -- k-step s of
// out^T = W2_i a^T takes the lane's values of accumulators 2s and 2s + 1, i.e. MFMA k index 8 q + j <->
// feature 16 (2 s + (j >> 2)) + 4 q + (j & 3), and the A operand (W2_i rows, two 8-byte LDS reads) uses
// that same feature order.
typedef __attribute__((ext_vector_type(8))) __bf16 bf8v;
typedef __attribute__((ext_vector_type(4))) __bf16 bf4v;
// HBIN: h arrives already rounded to bf16 in hb ((ceil(P / 16) * 16, W), gs4d_feature_relu_forward_hb), read as
// 16-byte loads (half the fp32 bytes per head) and not written
template <int W, bool HBIN>
__global__ __launch_bounds__(kHbfThreads) void heads_block_fwd_bf16_kernel(HfArgs A, const float *__restrict__ h,
                                                                           const float *__restrict__ w1,
                                                                           const float *__restrict__ b1,
                                                                           __bf16 *__restrict__ a,
                                                                           __bf16 *__restrict__ hb,
                                                                           __bf16 *__restrict__ w1t) {
    constexpr int NT = W / 16, NK = W / 32, WS = W + 8, NW = kHbfThreads / 64;
    extern __shared__ float4 s_v[];
    __bf16 *s_w1 = reinterpret_cast<__bf16 *>(s_v);       // W rows x WS
    const int head = blockIdx.y;
    const int n = A.n[head], npad = (n + 15) & ~15;
    __bf16 *s_w2 = s_w1 + W * WS;                            // npad rows x WS (rows >= n zero)
    float *s_b1 = reinterpret_cast<float *>(s_w2 + npad * WS);  // W
    float *s_b2 = s_b1 + W;                                  // npad
    const float *w1i = w1 + (size_t)head * W * W;
    for (int e = threadIdx.x; e < W * W / 4; e += kHbfThreads) {
        const int row = e / (W / 4), c4 = e % (W / 4);
        const float4 v = reinterpret_cast<const float4 *>(w1i + (size_t)row * W)[c4];
        const bf4v vb = bf4v{(__bf16)v.x, (__bf16)v.y, (__bf16)v.z, (__bf16)v.w};
        *reinterpret_cast<bf4v *>(s_w1 + row * WS + 4 * c4) = vb;
    }
    for (int e = threadIdx.x; e < npad * (W / 4); e += kHbfThreads) {
        const int row = e / (W / 4), c4 = e % (W / 4);
        const float4 v = row < n ? reinterpret_cast<const float4 *>(A.w2[head] + (size_t)row * W)[c4]
                                 : make_float4(0.f, 0.f, 0.f, 0.f);
        *reinterpret_cast<bf4v *>(s_w2 + row * WS + 4 * c4) = bf4v{(__bf16)v.x, (__bf16)v.y, (__bf16)v.z, (__bf16)v.w};
    }
    for (int e = threadIdx.x; e < W; e += kHbfThreads) s_b1[e] = b1[head * W + e];
    for (int e = threadIdx.x; e < npad; e += kHbfThreads) s_b2[e] = e < n ? A.b2[head][e] : 0.f;
    __syncthreads();
    if (w1t && blockIdx.x == 0) {
        // workgroup 0 of each head also writes W1_i^T in bf16 for the backward's input gradient
        // (gs4d_mlp_dx_bf16): 8 rows of one column of the LDS image per 16-byte store
        for (int e = threadIdx.x; e < W * W / 8; e += kHbfThreads) {
            const int col = e / (W / 8), r8 = e % (W / 8);
            bf8v v;
#pragma unroll
            for (int j = 0; j < 8; j++) v[j] = s_w1[(8 * r8 + j) * WS + col];
            *reinterpret_cast<bf8v *>(w1t + (size_t)col * A.kW + head * W + 8 * r8) = v;
        }
    }
    const int lane = threadIdx.x & 63, wv = (int)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6), q = lane >> 4, c = lane & 15;
    const int nblk = (A.P + 15) / 16;
    const int stride = gridDim.x * NW;
    float *out = A.out[head];
    const bool v4out = (n & 3) == 0 && ((size_t)out & 15) == 0;
    float4 hn[2 * NK];
    bf8v hbn[NK];
    // unconditional loads (rows past P read row P - 1), as in heads_block_fwd_kernel
    auto load_h = [&](int blk) {
        const int pt = min(blk * 16 + c, A.P - 1);
        if (HBIN) {
            const bf8v *src = reinterpret_cast<const bf8v *>(hb + (size_t)pt * W + 8 * q);
#pragma unroll
            for (int t = 0; t < NK; t++) hbn[t] = src[4 * t];
        } else {
            const float4 *src = reinterpret_cast<const float4 *>(h + (size_t)pt * W + 8 * q);
#pragma unroll
            for (int t = 0; t < NK; t++) {
                hn[2 * t] = src[8 * t];
                hn[2 * t + 1] = src[8 * t + 1];
            }
        }
    };
    int blk = blockIdx.x * NW + wv;
    load_h(blk);
    for (; blk < nblk; blk += stride) {
        bf8v hv[NK];
#pragma unroll
        for (int t = 0; t < NK; t++) {
            if (HBIN) {
                hv[t] = hbn[t];
            } else {
                const float4 x = hn[2 * t], y = hn[2 * t + 1];
                hv[t] = bf8v{(__bf16)x.x, (__bf16)x.y, (__bf16)x.z, (__bf16)x.w, (__bf16)y.x, (__bf16)y.y,
                             (__bf16)y.z, (__bf16)y.w};
            }
        }
        load_h(blk + stride);  // the next block's h loads fly while this one runs on the MFMA
        if (!HBIN && hb && head == 0) {  // bf16 h for the backward's weight-gradient GEMM (ceil(P / 16) * 16 rows)
            __bf16 *dst = hb + (size_t)(blk * 16 + c) * W + 8 * q;
#pragma unroll
            for (int t = 0; t < NK; t++) *reinterpret_cast<bf8v *>(dst + 32 * t) = hv[t];
        }
        f4v acc[NT];
#pragma unroll
        for (int m = 0; m < NT; m++) acc[m] = f4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int t = 0; t < NK; t++) {
            asm volatile("" ::: "memory");
#pragma unroll
            for (int m = 0; m < NT; m++) {
                const bf8v av = *reinterpret_cast<const bf8v *>(s_w1 + (16 * m + c) * WS + 32 * t + 8 * q);
                acc[m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, hv[t], acc[m], 0, 0, 0);
            }
        }
        // a = relu(z + b1) in bf16: lane holds features 16 m + 4 q + v of point c
        const int pt = blk * 16 + c;
        bf4v ab[NT];
#pragma unroll
        for (int m = 0; m < NT; m++) {
            const float4 bb = *reinterpret_cast<const float4 *>(s_b1 + 16 * m + 4 * q);
            ab[m] = bf4v{(__bf16)fmaxf(acc[m][0] + bb.x, 0.f), (__bf16)fmaxf(acc[m][1] + bb.y, 0.f),
                         (__bf16)fmaxf(acc[m][2] + bb.z, 0.f), (__bf16)fmaxf(acc[m][3] + bb.w, 0.f)};
            // a has ceil(P / 16) * 16 rows: no condition on the store
            *reinterpret_cast<bf4v *>(a + (size_t)pt * A.kW + head * W + 16 * m + 4 * q) = ab[m];
        }
        // out^T (n_pad x 16) = W2_i a^T, B operand = the lane's bf16 a values (k-step s: tiles 2s, 2s + 1)
        for (int j = 0; j < npad; j += 16) {
            f4v o = f4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int s2 = 0; s2 < NT / 2; s2++) {
                const __bf16 *wr = s_w2 + (j + c) * WS + 32 * s2 + 4 * q;
                const bf4v lo = *reinterpret_cast<const bf4v *>(wr), hi = *reinterpret_cast<const bf4v *>(wr + 16);
                const bf8v wa = bf8v{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
                const bf4v x0 = ab[2 * s2], x1 = ab[2 * s2 + 1];
                const bf8v xb = bf8v{x0[0], x0[1], x0[2], x0[3], x1[0], x1[1], x1[2], x1[3]};
                o = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa, xb, o, 0, 0, 0);
            }
            // D[output j + 4 q + r][point c]: one float4 per lane when the rows are 16-byte aligned
            if (pt < A.P) {
                const int o0 = j + 4 * q;
                if (v4out && o0 + 3 < n) {
                    const float4 bb = *reinterpret_cast<const float4 *>(s_b2 + o0);
                    *reinterpret_cast<float4 *>(out + (size_t)pt * n + o0) =
                        make_float4(o[0] + bb.x, o[1] + bb.y, o[2] + bb.z, o[3] + bb.w);
                } else {
#pragma unroll
                    for (int r = 0; r < 4; r++)
                        if (o0 + r < n) out[(size_t)pt * n + o0 + r] = o[r] + s_b2[o0 + r];
                }
            }
        }
    }
}

// ---- the bf16 heads block's input gradient: dh (P x W, fp32) = da (P x KW, bf16) W1 (KW x W, bf16), computed
// as dh^T = W1^T da^T on v_mfma_f32_16x16x32_bf16: the A operand is W1^T (W x KW, written by the block forward),
// the B operand da's rows as they lie in memory (lane (q, c): row c of a 16-row block, k = 32 s + 8 q .. + 7:
// one 16-byte load), and D[n = 16 m + 4 q + r][row c] leaves as one float4 per lane and tile.  A 512-thread
// workgroup takes 256 rows (32 per wave); W1^T is staged per 64-wide k chunk in LDS (16 KiB, double-buffered,
// row stride 144 B so the 16 rows of a fragment read fall on distinct banks) and shared by the 8 waves, so it
// is read from L2 once per workgroup instead of once per wave; da is prefetched one chunk ahead.  fp32
// accumulation over KW.
constexpr int kDxThreads = 512, kDxRowsPerWave = 32, kDxChunk = 64, kDxLdsStride = kDxChunk + 8;  // bf16 units
template <int W>
__global__ __launch_bounds__(kDxThreads) void mlp_dx_bf16_kernel(int P, int KW, const __bf16 *__restrict__ da,
                                                                 const __bf16 *__restrict__ w1t,
                                                                 float *__restrict__ dh) {
    constexpr int NT = W / 16, RB = kDxRowsPerWave / 16;
    constexpr int kPieces = W * kDxChunk / 8 / kDxThreads;  // 16-byte pieces of a chunk per thread (W = 128: 2)
    __shared__ __attribute__((aligned(16))) __bf16 s_a[2][W * kDxLdsStride];
    const int lane = threadIdx.x & 63, wv = (int)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6), q = lane >> 4, c = lane & 15;
    const int64_t row0 = (int64_t)blockIdx.x * (kDxThreads / 64) * kDxRowsPerWave + (int64_t)wv * kDxRowsPerWave;
    const __bf16 *brow[RB];
#pragma unroll
    for (int rb = 0; rb < RB; rb++)  // rows past P read row P - 1 (unconditional loads; not stored)
        brow[rb] = da + (size_t)min(row0 + 16 * rb + c, (int64_t)P - 1) * KW + 8 * q;
    f4v acc[NT][RB];
#pragma unroll
    for (int m = 0; m < NT; m++)
#pragma unroll
        for (int rb = 0; rb < RB; rb++) acc[m][rb] = f4v{0.f, 0.f, 0.f, 0.f};
    const int nch = KW / kDxChunk;
    bf8v ga[kPieces];
    auto load_a = [&](int ch) {  // piece e: W1^T row e / 8, 16-byte column piece e % 8 of the chunk
#pragma unroll
        for (int i = 0; i < kPieces; i++) {
            const int e = threadIdx.x + i * kDxThreads;
            ga[i] = *reinterpret_cast<const bf8v *>(w1t + (size_t)(e >> 3) * KW + ch * kDxChunk + 8 * (e & 7));
        }
    };
    auto store_a = [&](int buf) {
#pragma unroll
        for (int i = 0; i < kPieces; i++) {
            const int e = threadIdx.x + i * kDxThreads;
            *reinterpret_cast<bf8v *>(&s_a[buf][(e >> 3) * kDxLdsStride + 8 * (e & 7)]) = ga[i];
        }
    };
    bf8v bn[2][RB];
    auto load_b = [&](int ch) {
#pragma unroll
        for (int st = 0; st < 2; st++)
#pragma unroll
            for (int rb = 0; rb < RB; rb++)
                bn[st][rb] = *reinterpret_cast<const bf8v *>(brow[rb] + ch * kDxChunk + 32 * st);
    };
    load_a(0);
    load_b(0);
    store_a(0);
    __syncthreads();
    for (int ch = 0; ch < nch; ch++) {
        bf8v b[2][RB];
#pragma unroll
        for (int st = 0; st < 2; st++)
#pragma unroll
            for (int rb = 0; rb < RB; rb++) b[st][rb] = bn[st][rb];
        const int nx = min(ch + 1, nch - 1);  // the last chunk re-loads itself: loads stay unconditional
        load_a(nx);
        load_b(nx);
        const __bf16 *sa = s_a[ch & 1];
#pragma unroll
        for (int st = 0; st < 2; st++)
#pragma unroll
            for (int m = 0; m < NT; m++) {
                const bf8v a = *reinterpret_cast<const bf8v *>(sa + (16 * m + c) * kDxLdsStride + 32 * st + 8 * q);
#pragma unroll
                for (int rb = 0; rb < RB; rb++)
                    acc[m][rb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b[st][rb], acc[m][rb], 0, 0, 0);
            }
        if (ch + 1 < nch) store_a((ch + 1) & 1);  // the other buffer: read by nobody since the last barrier
        __syncthreads();
    }
#pragma unroll
    for (int rb = 0; rb < RB; rb++) {
        const int64_t row = row0 + 16 * rb + c;
        if (row < P)
#pragma unroll
            for (int m = 0; m < NT; m++)
                *reinterpret_cast<float4 *>(dh + (size_t)row * W + 16 * m + 4 * q) =
                    make_float4(acc[m][rb][0], acc[m][rb][1], acc[m][rb][2], acc[m][rb][3]);
    }
}

// ---- the bf16 heads block's first-layer weight gradient: dW1 (KW x W, fp32) = da^T hb, reduced over the P rows.
// Workgroup (row chunk s of 1024 rows, head i) forms the 128 x 128 block of head i's rows of dW1 over its chunk
// into parts[s] (summed over the chunks in order by gs4d_sum_slices): D[da feature 16 m + 4 q + r][hb feature
// 16 n + c] on v_mfma_f32_16x16x32_bf16 with K = rows.  Both operands need 8 consecutive ROWS of one column, so
// each 64-row step stages the da and hb tiles (64 x 128 bf16 each, row-major as loaded) in LDS and reads them
// back with ds_read_b64_tr_b16 (a 16-lane group reads a 4 x 16 block and receives it column-major): two
// transposed reads give an operand's 8 rows.  The tiles use the XOR-swizzled 256-byte rows of the guide's
// dual-use image (conflict-free transposed reads); rows past P are staged as zeros.  Double-buffered: the
// next step's tiles are loaded while this step's MFMAs run.
constexpr int kDwbThreads = 256, kDwbChunkRows = 1024, kDwbStepRows = 64;  // two MFMA k-steps per staged tile
typedef short s4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ int dwb_off(int row, int ch) {  // byte offset of 16-byte chunk ch of tile row `row`
    return 256 * row + 16 * (ch ^ (((row & 3) << 2) | ((row >> 2) & 3)));
}
__device__ __forceinline__ bf8v dwb_tr_frag(const unsigned char *tile, int rb, int g, int li, int c0) {
    // rows rb + 8 g .. + 7 of the 16 columns starting at chunk c0, as an MFMA operand fragment (lane li gets
    // column li): lane 4 q + p of the group addresses row (base + q), columns 4 p .. 4 p + 3
    const int q = li >> 2, p = li & 3;
    const unsigned char *a0 = tile + dwb_off(rb + 8 * g + q, c0 + (p >> 1)) + 8 * (p & 1);
    const unsigned char *a1 = tile + dwb_off(rb + 8 * g + 4 + q, c0 + (p >> 1)) + 8 * (p & 1);
    typedef __attribute__((address_space(3))) s4v lds_s4v;
    const s4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4v *)a0);
    const s4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4v *)a1);
    const s4v v[2] = {lo, hi};
    return __builtin_bit_cast(bf8v, v);
}
__global__ __launch_bounds__(kDwbThreads) void mlp_dw_bf16_kernel(int P, int KW, const __bf16 *__restrict__ da,
                                                                  const __bf16 *__restrict__ hb,
                                                                  float *__restrict__ parts) {
    constexpr int W = 128, NT = W / 16, MW = NT / (kDwbThreads / 64);  // m tiles per wave: 2
    constexpr int kPer = kDwbStepRows * 16 / kDwbThreads;  // 16-byte chunks per thread and tile
    __shared__ __attribute__((aligned(16))) unsigned char s_t[2][2][kDwbStepRows * 256];  // [buffer][da, hb][tile]
    const int head = blockIdx.y;
    const int64_t r0 = (int64_t)blockIdx.x * kDwbChunkRows;
    const int nst = (int)((min((int64_t)P, r0 + kDwbChunkRows) - r0 + kDwbStepRows - 1) / kDwbStepRows);
    const int lane = threadIdx.x & 63, wv = (int)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6), g = lane >> 4, li = lane & 15;
    f4v acc[MW][NT];
#pragma unroll
    for (int m = 0; m < MW; m++)
#pragma unroll
        for (int n = 0; n < NT; n++) acc[m][n] = f4v{0.f, 0.f, 0.f, 0.f};
    // staging: thread t moves chunks t, t + 256, ... of each tile: row e / 16, chunk e % 16
    bf8v ld[2][kPer];
    auto load = [&](int st) {
#pragma unroll
        for (int i = 0; i < kPer; i++) {
            const int e = threadIdx.x + i * kDwbThreads, row = e >> 4, ch = e & 15;
            const int64_t pr = r0 + kDwbStepRows * st + row;
            const bool ok = pr < P;
            const int64_t prc = ok ? pr : 0;
            const bf8v z = bf8v{};
            const bf8v va = *reinterpret_cast<const bf8v *>(da + (size_t)prc * KW + head * W + 8 * ch);
            const bf8v vh = *reinterpret_cast<const bf8v *>(hb + (size_t)prc * W + 8 * ch);
            ld[0][i] = ok ? va : z;
            ld[1][i] = ok ? vh : z;
        }
    };
    auto store = [&](int buf) {
#pragma unroll
        for (int i = 0; i < kPer; i++) {
            const int e = threadIdx.x + i * kDwbThreads, row = e >> 4, ch = e & 15;
            *reinterpret_cast<bf8v *>(&s_t[buf][0][dwb_off(row, ch)]) = ld[0][i];
            *reinterpret_cast<bf8v *>(&s_t[buf][1][dwb_off(row, ch)]) = ld[1][i];
        }
    };
    if (nst > 0) {
        load(0);
        store(0);
    }
    __syncthreads();
    for (int st = 0; st < nst; st++) {
        if (st + 1 < nst) load(st + 1);
        const unsigned char *ta = s_t[st & 1][0], *th = s_t[st & 1][1];
#pragma unroll
        for (int kk = 0; kk < kDwbStepRows / 32; kk++) {
            bf8v a[MW];
#pragma unroll
            for (int m = 0; m < MW; m++) a[m] = dwb_tr_frag(ta, 32 * kk, g, li, 2 * (wv * MW + m));
#pragma unroll
            for (int n = 0; n < NT; n++) {
                const bf8v b = dwb_tr_frag(th, 32 * kk, g, li, 2 * n);
#pragma unroll
                for (int m = 0; m < MW; m++)
                    acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[m], b, acc[m][n], 0, 0, 0);
            }
        }
        if (st + 1 < nst) store((st + 1) & 1);  // the other buffer: nobody reads it since the last barrier
        __syncthreads();
    }
    // D[da feature 16 m + 4 g + r][hb feature 16 n + li] of head `head` -> parts[s]
    float *o = parts + (size_t)blockIdx.x * KW * W + (size_t)head * W * W;
#pragma unroll
    for (int m = 0; m < MW; m++)
#pragma unroll
        for (int n = 0; n < NT; n++)
#pragma unroll
            for (int r = 0; r < 4; r++)
                o[(size_t)(16 * (wv * MW + m) + 4 * g + r) * W + 16 * n + li] = acc[m][n][r];
}

// ---- the fp32 heads block's input gradient: dh (P x W) = da (P x KW) W1 (KW x W) on v_mfma_f32_16x16x4_f32
// (f32 products and sums in one fixed order per element: the same bits in every process, where the library
// GEMM this replaces was picked per process by timing).  Computed transposed as mlp_dx_bf16_kernel does:
// dh^T = W1^T da^T.  In the 16-wide k slice kk, lane (q = l >> 4, c = l & 15) supplies k = 16 kk + 4 q + s in
// MFMA step s, so one float4 load of da row c gives the lane's 4 steps of the B operand, and the A operand
// W1^T[16 m + c][16 kk + 4 q .. + 3] is one 16-byte LDS read.  The operand is W1^T (W x KW, written by the heads
// block forward): its k-runs are staged with coalesced 16-byte loads and 16-byte LDS stores, row stride KC + 8
// floats, which is conflict-free for both (ds_read_b128's four 16-lane groups; 8-lane store groups).  (Round 6
// first staged W1 itself, transposing with scalar stores at stride KC + 4: 2-way conflicts on every read, 38M
// conflict cycles per launch, 63 % MFMA busy.)
// A workgroup is 4 waves on ONE 64-feature group of dh (4 m tiles) and 64 rows (16 per wave): small units of
// work (3136 workgroups at P = 100k, W = 128) keep the per-CU share even.  The group's 64 x KC block of W1^T is
// staged per k chunk, double-buffered; da is prefetched a chunk ahead.  Workgroups b and b + 8 (same XCD) take the
// two feature groups of the same rows, so the second read of those da rows is an L2 hit.
// KC: the k chunk, 64, or 32 when KW / 64 is odd (the loop runs chunks in pairs: an even count keeps both halves
// unconditional, so the compiler cannot sink the second half's loads into a branch).
constexpr int kDxfThreads = 256;
// RB: 16-row blocks per wave (2: each W1^T LDS read feeds twice the MFMAs)
template <int W, int KC, int RB>
__global__ __launch_bounds__(kDxfThreads) void mlp_dx_f32_kernel(int P, int KW, int nrg, const float *__restrict__ da,
                                                                 const float *__restrict__ w1t, float *__restrict__ dh) {
    constexpr int NG = W / 64;  // feature groups
    constexpr int S = KC + 8, KK = KC / 16, NP = KC / 16, Q = KC / 4;  // NP: staging float4 per thread; Q per row
    __shared__ __attribute__((aligned(16))) float s_a[2][64 * S];
    int rg = blockIdx.x, fg = 0;
    if (NG == 2) {
        const int i = blockIdx.x & 15;
        fg = i >> 3;
        rg = (int)(blockIdx.x >> 4) * 8 + (i & 7);
    }
    if (rg >= nrg) return;  // the grid is padded to whole groups of 8 row groups (uniform over the workgroup)
    const int lane = threadIdx.x & 63, wv = (int)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6), q = lane >> 4,
              c = lane & 15;
    int64_t row[RB];
    const float *brow[RB];
#pragma unroll
    for (int rb = 0; rb < RB; rb++) {
        row[rb] = (int64_t)rg * 64 * RB + wv * 16 * RB + 16 * rb + c;
        // rows past P read row P - 1 (unconditional loads; not stored)
        brow[rb] = da + (size_t)min(row[rb], (int64_t)P - 1) * KW + 4 * q;
    }
    f4v acc[4][RB];
#pragma unroll
    for (int m = 0; m < 4; m++)
#pragma unroll
        for (int rb = 0; rb < RB; rb++) acc[m][rb] = f4v{0.f, 0.f, 0.f, 0.f};
    const int nch = KW / KC;
    // staging: piece e = t + 256 i is W1^T row 64 fg + e / Q (a feature), k 4 (e % Q) .. + 3 of the chunk.
    // Chunks run in pairs, the pair's two halves unrolled with compile-time buffer and register-set indices (no
    // lambdas: captured register arrays were left in scratch memory), each half issuing the next chunk's loads
    // ahead of its own MFMAs.  nch is even (KC), so both halves are straight-line code.
    float4 bb[2][RB][KK];
    {
        float4 ga[NP];
#pragma unroll
        for (int i = 0; i < NP; i++) {
            const int e = (int)threadIdx.x + kDxfThreads * i;
            ga[i] = *reinterpret_cast<const float4 *>(w1t + (size_t)(64 * fg + e / Q) * KW + 4 * (e % Q));
        }
#pragma unroll
        for (int rb = 0; rb < RB; rb++)
#pragma unroll
            for (int kk = 0; kk < KK; kk++) bb[0][rb][kk] = *reinterpret_cast<const float4 *>(brow[rb] + 16 * kk);
#pragma unroll
        for (int i = 0; i < NP; i++) {
            const int e = (int)threadIdx.x + kDxfThreads * i;
            *reinterpret_cast<float4 *>(&s_a[0][(e / Q) * S + 4 * (e % Q)]) = ga[i];
        }
    }
    __syncthreads();
    for (int ch = 0; ch < nch; ch += 2) {
#pragma unroll
        for (int hf = 0; hf < 2; hf++) {
            const int nx = min(ch + hf + 1, nch - 1);  // the last chunk re-loads itself: loads stay unconditional
            float4 ga[NP];
#pragma unroll
            for (int i = 0; i < NP; i++) {
                const int e = (int)threadIdx.x + kDxfThreads * i;
                ga[i] = *reinterpret_cast<const float4 *>(w1t + (size_t)(64 * fg + e / Q) * KW + nx * KC + 4 * (e % Q));
            }
#pragma unroll
            for (int rb = 0; rb < RB; rb++)
#pragma unroll
                for (int kk = 0; kk < KK; kk++)
                    bb[hf ^ 1][rb][kk] = *reinterpret_cast<const float4 *>(brow[rb] + nx * KC + 16 * kk);
            __builtin_amdgcn_sched_barrier(0);  // left to itself the scheduler sank the loads below the MFMAs
            const float *sa = s_a[hf];
#pragma unroll
            for (int kk = 0; kk < KK; kk++)
#pragma unroll
                for (int m = 0; m < 4; m++) {
                    const float4 av = *reinterpret_cast<const float4 *>(sa + (16 * m + c) * S + 16 * kk + 4 * q);
#pragma unroll
                    for (int rb = 0; rb < RB; rb++) {
                        const float4 bv = bb[hf][rb][kk];
                        acc[m][rb] = __builtin_amdgcn_mfma_f32_16x16x4f32(av.x, bv.x, acc[m][rb], 0, 0, 0);
                        acc[m][rb] = __builtin_amdgcn_mfma_f32_16x16x4f32(av.y, bv.y, acc[m][rb], 0, 0, 0);
                        acc[m][rb] = __builtin_amdgcn_mfma_f32_16x16x4f32(av.z, bv.z, acc[m][rb], 0, 0, 0);
                        acc[m][rb] = __builtin_amdgcn_mfma_f32_16x16x4f32(av.w, bv.w, acc[m][rb], 0, 0, 0);
                    }
                }
            // the other buffer: read by nobody since the last barrier (after the last chunk, by nobody at all)
#pragma unroll
            for (int i = 0; i < NP; i++) {
                const int e = (int)threadIdx.x + kDxfThreads * i;
                *reinterpret_cast<float4 *>(&s_a[hf ^ 1][(e / Q) * S + 4 * (e % Q)]) = ga[i];
            }
            __syncthreads();
        }
    }
    // D[feature 16 m + 4 q + r][row c]
#pragma unroll
    for (int rb = 0; rb < RB; rb++)
        if (row[rb] < P)
#pragma unroll
            for (int m = 0; m < 4; m++)
                *reinterpret_cast<float4 *>(dh + (size_t)row[rb] * W + 64 * fg + 16 * m + 4 * q) =
                    make_float4(acc[m][rb][0], acc[m][rb][1], acc[m][rb][2], acc[m][rb][3]);
}

// ---- the fp32 heads block's first-layer weight gradient: dW1 (KW x W) = da^T h reduced over the P rows, on
// v_mfma_f32_16x16x4_f32 with K = rows.  Workgroup (row chunk s, 64-row block mb of dW1): 4 waves, wave w owning
// the 64 x (W / 4) block of columns w W/4 ..; the chunk's rows pass through LDS in 16-row stages (da's 64 columns
// and h's W columns of each row, coalesced 16-byte loads and stores, double-buffered, the next stage's loads
// issued ahead of this stage's MFMAs).  In the MFMA k-step over stage rows r .. r + 3, lane (q, c) reads
// A[feature c][row q] = da[r + q][64 mb + 16 mt + c] and B[row q][feature c] = h[r + q][16 nt + c] as single
// dwords (row strides of 80 and W + 16 floats: the two rows a 32-lane half reads fall on opposite bank halves,
// conflict-free).  Rows past P are staged as zeros.  Each wave writes its block of parts[s]; gs4d_sum_slices adds
// the chunks in order.  Deterministic by construction.  The m blocks of one chunk sit on one XCD (they share its
// h rows).  (Round 6 first read both operands straight from HBM as dwords at 2 waves/SIMD: 50 % MFMA busy.)
constexpr int kDwfThreads = 256, kDwfStage = 16;
// v, or zeros: component selects (a select between two float4 values became a select of scratch addresses)
__device__ __forceinline__ float4 keep4(bool ok, float4 v) {
    return make_float4(ok ? v.x : 0.f, ok ? v.y : 0.f, ok ? v.z : 0.f, ok ? v.w : 0.f);
}
// MB: dW1 rows per workgroup, 64 (waves side by side over the W columns) or 128 (waves 2 x 2, each a 64 x W/2
// block: twice the MFMAs per stage and per LDS read)
template <int W, int MB>
__global__ __launch_bounds__(kDwfThreads) void mlp_dw_f32_kernel(int P, int KW, int S, int chunk_rows,
                                                                 const float *__restrict__ da,
                                                                 const float *__restrict__ h,
                                                                 float *__restrict__ parts) {
    constexpr int MT = 4, NTW = MB == 64 ? W / 64 : W / 32;  // m tiles and n tiles per wave
    constexpr int SD = MB + 16, SH = W + 16, QD = MB / 4;    // QD: float4 per staged da row
    constexpr int PD = kDwfStage * QD / kDwfThreads, PH = kDwfStage * (W / 4) / kDwfThreads;  // float4 per thread
    __shared__ __attribute__((aligned(16))) float s_d[2][kDwfStage * SD];
    __shared__ __attribute__((aligned(16))) float s_h[2][kDwfStage * SH];
    const int nmb = KW / MB;
    // b = 8 (nmb j + mb) + x: chunk s = 8 j + x, so the nmb blocks of a chunk share b % 8 (the XCD)
    const int b = blockIdx.x, x = b & 7, jm = b >> 3, mb = jm % nmb, s = 8 * (jm / nmb) + x;
    if (s >= S) return;  // padding of the grid to whole groups of 8 chunks (uniform over the workgroup)
    const int lane = threadIdx.x & 63, wv = (int)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6), q = lane >> 4,
              c = lane & 15;
    const int wm = MB == 64 ? 0 : wv >> 1, wn = MB == 64 ? wv : wv & 1;  // the wave's m and n block
    const int64_t r0 = (int64_t)s * chunk_rows, r1 = min((int64_t)P, r0 + chunk_rows);
    f4v acc[MT][NTW];
#pragma unroll
    for (int mt = 0; mt < MT; mt++)
#pragma unroll
        for (int nt = 0; nt < NTW; nt++) acc[mt][nt] = f4v{0.f, 0.f, 0.f, 0.f};
    // staging: da piece e: stage row e / QD, float4 e % QD; h piece e: stage row e / (W / 4), float4 e % (W / 4).
    // Stages run in pairs, each half unrolled with compile-time buffer indices (see mlp_dx_f32_kernel): the next
    // stage's loads, this stage's MFMAs from LDS, then the next stage into the other buffer (rows past r1 read row
    // r1 - 1 and are stored as zeros; past the last stage a padding stage, zeros, read by nobody).
    const int nst = (int)((r1 - r0 + 2 * kDwfStage - 1) / (2 * kDwfStage)) * 2;
#pragma unroll
    for (int pre = 0; pre < 1; pre++) {  // stage 0 into buffer 0
        float4 gd[PD], gh[PH];
#pragma unroll
        for (int i = 0; i < PD; i++) {
            const int e = (int)threadIdx.x + kDwfThreads * i;
            const int64_t r = r0 + e / QD;
            gd[i] = *reinterpret_cast<const float4 *>(da + (size_t)min(r, r1 - 1) * KW + MB * mb + 4 * (e % QD));
            *reinterpret_cast<float4 *>(&s_d[0][(e / QD) * SD + 4 * (e % QD)]) = keep4(r < r1, gd[i]);
        }
#pragma unroll
        for (int i = 0; i < PH; i++) {
            const int e = (int)threadIdx.x + kDwfThreads * i;
            const int64_t r = r0 + e / (W / 4);
            gh[i] = *reinterpret_cast<const float4 *>(h + (size_t)min(r, r1 - 1) * W + 4 * (e % (W / 4)));
            *reinterpret_cast<float4 *>(&s_h[0][(e / (W / 4)) * SH + 4 * (e % (W / 4))]) = keep4(r < r1, gh[i]);
        }
    }
    __syncthreads();
    for (int st = 0; st < nst; st += 2) {
#pragma unroll
        for (int hf = 0; hf < 2; hf++) {
            const int64_t rn = r0 + (int64_t)kDwfStage * (st + hf + 1);  // the next stage's first row
            float4 gd[PD], gh[PH];
#pragma unroll
            for (int i = 0; i < PD; i++) {
                const int e = (int)threadIdx.x + kDwfThreads * i;
                gd[i] = *reinterpret_cast<const float4 *>(da + (size_t)min(rn + e / QD, r1 - 1) * KW + MB * mb +
                                                          4 * (e % QD));
            }
#pragma unroll
            for (int i = 0; i < PH; i++) {
                const int e = (int)threadIdx.x + kDwfThreads * i;
                gh[i] = *reinterpret_cast<const float4 *>(h + (size_t)min(rn + e / (W / 4), r1 - 1) * W +
                                                          4 * (e % (W / 4)));
            }
            __builtin_amdgcn_sched_barrier(0);
            const float *sd = s_d[hf], *sh = s_h[hf];
#pragma unroll
            for (int u = 0; u < kDwfStage / 4; u++) {
                float av[MT], hv[NTW];
#pragma unroll
                for (int mt = 0; mt < MT; mt++) av[mt] = sd[(4 * u + q) * SD + 64 * wm + 16 * mt + c];
#pragma unroll
                for (int nt = 0; nt < NTW; nt++) hv[nt] = sh[(4 * u + q) * SH + 16 * (NTW * wn + nt) + c];
#pragma unroll
                for (int mt = 0; mt < MT; mt++)
#pragma unroll
                    for (int nt = 0; nt < NTW; nt++)
                        acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[mt], hv[nt], acc[mt][nt], 0, 0, 0);
            }
#pragma unroll
            for (int i = 0; i < PD; i++) {
                const int e = (int)threadIdx.x + kDwfThreads * i;
                *reinterpret_cast<float4 *>(&s_d[hf ^ 1][(e / QD) * SD + 4 * (e % QD)]) = keep4(rn + e / QD < r1, gd[i]);
            }
#pragma unroll
            for (int i = 0; i < PH; i++) {
                const int e = (int)threadIdx.x + kDwfThreads * i;
                *reinterpret_cast<float4 *>(&s_h[hf ^ 1][(e / (W / 4)) * SH + 4 * (e % (W / 4))]) =
                    keep4(rn + e / (W / 4) < r1, gh[i]);
            }
            __syncthreads();
        }
    }
    // D[feature 64 wm + 16 mt + 4 q + r][column 16 (NTW wn + nt) + c] of rows MB mb .. of dW1
    float *o = parts + (size_t)s * KW * W + (size_t)(MB * mb + 64 * wm) * W;
#pragma unroll
    for (int mt = 0; mt < MT; mt++)
#pragma unroll
        for (int nt = 0; nt < NTW; nt++)
#pragma unroll
            for (int r = 0; r < 4; r++)
                o[(size_t)(16 * mt + 4 * q + r) * W + 16 * (NTW * wn + nt) + c] = acc[mt][nt][r];
}

// ---- the wide head's second-layer backward on the bf16 path (n = 48, W = 128): heads_bwd_wide_mfma_kernel's
// products on v_mfma_f32_16x16x32_bf16 with g rounded to bf16 (the bf16 leg's operands), sums in fp32.  A
// workgroup takes 32-row steps (grid-stride): the a tile (32 x 128 bf16) and the g tile (32 x 48 -> bf16,
// columns 48..63 zero) are staged in LDS (the swizzled 256-byte rows of mlp_dw_bf16_kernel), W2^T (128 x 64
// bf16, zero-padded k) once per workgroup.
//   da^T = W2^T g^T: A = W2^T rows (LDS row reads), B = g rows (LDS row reads), D = 4 consecutive columns of one
//        row per lane: masked by a > 0 and stored as 8 bytes; db1 summed from the fp32 results;
//   dW2 += g^T a: both operands by ds_read_b64_tr_b16 (K = the 32 rows);
//   db2: the fp32 g values summed as staged.
// Partials in heads_bwd_reduce_kernel's layout (fixed-order sums: deterministic).
__global__ __launch_bounds__(256) void heads_bwd_wide_bf16_kernel(HbArgs A, const __bf16 *__restrict__ a,
                                                                  __bf16 *__restrict__ da, const float *__restrict__ g,
                                                                  float *__restrict__ part) {
    constexpr int W = 128, N = 48, KS = 72;  // W2^T row stride (bf16): 64 + 8 (144 B)
    __shared__ __attribute__((aligned(16))) __bf16 s_w2t[W * KS];
    __shared__ __attribute__((aligned(16))) unsigned char s_ta[32 * 256], s_tg[32 * 256];
    __shared__ float4 s_red[192];
    const int ld = A.k * W, h = A.h0;
    const float *__restrict__ w2 = A.w2[h];
    const int lane = threadIdx.x & 63, wv = (int)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6), q = lane >> 4, c = lane & 15;
    for (int e = threadIdx.x; e < W * 64; e += 256) {
        const int n = e / 64, k = e % 64;
        s_w2t[n * KS + k] = (__bf16)(k < N ? w2[k * W + n] : 0.f);
    }
    for (int e = threadIdx.x; e < 32 * 10; e += 256) {  // g tile chunks 6..15 stay zero
        const int row = e / 10, ch = 6 + e % 10;
        *reinterpret_cast<bf8v *>(&s_tg[dwb_off(row, ch)]) = bf8v{};
    }
    f4v accw[3][2];
#pragma unroll
    for (int m = 0; m < 3; m++) accw[m][0] = accw[m][1] = f4v{0.f, 0.f, 0.f, 0.f};
    float4 dsum[2][2];  // [n local][row block]: this lane's da column sums (4 columns)
#pragma unroll
    for (int i = 0; i < 2; i++) dsum[i][0] = dsum[i][1] = make_float4(0.f, 0.f, 0.f, 0.f);
    float4 gsum = make_float4(0.f, 0.f, 0.f, 0.f);  // threads < 192: fp32 column sums of g, columns 4 (t % 12) ..
    const int P = A.P, nb32 = (P + 31) / 32;
    for (int blk = blockIdx.x; blk < nb32; blk += gridDim.x) {
        const int64_t r0 = (int64_t)blk * 32;
        // stage the a tile (512 16-byte chunks, two per thread) and the g tile (384 float4, two per thread < 192)
#pragma unroll
        for (int i = 0; i < 2; i++) {
            const int e = threadIdx.x + 256 * i, row = e >> 4, ch = e & 15;
            const int64_t pr = r0 + row;
            bf8v v = bf8v{};
            if (pr < P) v = *reinterpret_cast<const bf8v *>(a + (size_t)pr * ld + h * W + 8 * ch);
            *reinterpret_cast<bf8v *>(&s_ta[dwb_off(row, ch)]) = v;
        }
        if (threadIdx.x < 192) {
            const int c4 = threadIdx.x % 12;
#pragma unroll
            for (int i = 0; i < 2; i++) {
                const int row = threadIdx.x / 12 + 16 * i;
                const int64_t pr = r0 + row;
                float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
                if (pr < P) v = *reinterpret_cast<const float4 *>(g + (size_t)pr * N + 4 * c4);
                gsum.x += v.x; gsum.y += v.y; gsum.z += v.z; gsum.w += v.w;
                *reinterpret_cast<bf4v *>(&s_tg[dwb_off(row, c4 >> 1) + 8 * (c4 & 1)]) =
                    bf4v{(__bf16)v.x, (__bf16)v.y, (__bf16)v.z, (__bf16)v.w};
            }
        }
        __syncthreads();
        // da^T: wave wv takes columns tiles n = 2 wv, 2 wv + 1 for both 16-row blocks
#pragma unroll
        for (int nl = 0; nl < 2; nl++) {
            const int n = 2 * wv + nl;
#pragma unroll
            for (int rb = 0; rb < 2; rb++) {
                f4v d = f4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int st = 0; st < 2; st++) {
                    const bf8v wa = *reinterpret_cast<const bf8v *>(&s_w2t[(16 * n + c) * KS + 32 * st + 8 * q]);
                    const bf8v gb = *reinterpret_cast<const bf8v *>(&s_tg[dwb_off(16 * rb + c, 4 * st + q)]);
                    d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa, gb, d, 0, 0, 0);
                }
                // D[column 16 n + 4 q + r][row 16 rb + c]
                const int row = 16 * rb + c;
                const bf4v av = *reinterpret_cast<const bf4v *>(&s_ta[dwb_off(row, 2 * n + (q >> 1)) + 8 * (q & 1)]);
                const float v0 = (float)av[0] > 0.f ? d[0] : 0.f, v1 = (float)av[1] > 0.f ? d[1] : 0.f;
                const float v2 = (float)av[2] > 0.f ? d[2] : 0.f, v3 = (float)av[3] > 0.f ? d[3] : 0.f;
                if (r0 + row < P) {
                    *reinterpret_cast<bf4v *>(da + (size_t)(r0 + row) * ld + h * W + 16 * n + 4 * q) =
                        bf4v{(__bf16)v0, (__bf16)v1, (__bf16)v2, (__bf16)v3};
                    dsum[nl][rb].x += v0; dsum[nl][rb].y += v1; dsum[nl][rb].z += v2; dsum[nl][rb].w += v3;
                }
            }
        }
        // dW2 += g^T a: tiles (m = 0..2, n = 2 wv, 2 wv + 1), K = the 32 rows
#pragma unroll
        for (int m = 0; m < 3; m++) {
            const bf8v ga = dwb_tr_frag(s_tg, 0, q, c, 2 * m);
#pragma unroll
            for (int nl = 0; nl < 2; nl++) {
                const bf8v ab = dwb_tr_frag(s_ta, 0, q, c, 2 * (2 * wv + nl));
                accw[m][nl] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ga, ab, accw[m][nl], 0, 0, 0);
            }
        }
        __syncthreads();  // the tiles are restaged by the next step
    }
    float *pw = part + (size_t)blockIdx.x * (W + N * (W + 1));
    // db1: the 16 lanes of a lane group (rows) summed by a fixed butterfly, both row blocks in order
#pragma unroll
    for (int nl = 0; nl < 2; nl++) {
        float4 t = make_float4(dsum[nl][0].x + dsum[nl][1].x, dsum[nl][0].y + dsum[nl][1].y,
                               dsum[nl][0].z + dsum[nl][1].z, dsum[nl][0].w + dsum[nl][1].w);
#pragma unroll
        for (int off = 1; off < 16; off <<= 1) {
            t.x += __shfl_xor(t.x, off, 16); t.y += __shfl_xor(t.y, off, 16);
            t.z += __shfl_xor(t.z, off, 16); t.w += __shfl_xor(t.w, off, 16);
        }
        if (c == 0) {
            const int col = 16 * (2 * wv + nl) + 4 * q;
            pw[col] = t.x, pw[col + 1] = t.y, pw[col + 2] = t.z, pw[col + 3] = t.w;
        }
    }
    // dW2: D[output 16 m + 4 q + r][column 16 n + c]
#pragma unroll
    for (int m = 0; m < 3; m++)
#pragma unroll
        for (int nl = 0; nl < 2; nl++)
#pragma unroll
            for (int r = 0; r < 4; r++)
                pw[W + (16 * m + 4 * q + r) * (W + 1) + 16 * (2 * wv + nl) + c] = accw[m][nl][r];
    // db2: the 16 threads of each column group summed in thread order
    if (threadIdx.x < 192) s_red[threadIdx.x] = gsum;
    __syncthreads();
    if (threadIdx.x < 12) {
        float4 t = s_red[threadIdx.x];
        for (int j = 1; j < 16; j++) {
            const float4 v = s_red[threadIdx.x + 12 * j];
            t.x += v.x; t.y += v.y; t.z += v.z; t.w += v.w;
        }
        const int o = 4 * threadIdx.x;
        pw[W + (o + 0) * (W + 1) + W] = t.x;
        pw[W + (o + 1) * (W + 1) + W] = t.y;
        pw[W + (o + 2) * (W + 1) + W] = t.z;
        pw[W + (o + 3) * (W + 1) + W] = t.w;
    }
}

// ---- the deformation field's first layer, forward: h = relu(x W^T + b) (P, FOUT) from x (P, FIN) on the
// f32 MFMA.  Per 16-row block: lane group q = l >> 4 reads columns 4q..4q+3 of its row l & 15 of a 16-column
// K chunk as one float4 (the MFMA's k index in step s is column 4q + s), the matching W rows (LDS, row stride
// FIN + 4) are the B operand, FOUT / 16 accumulators; bias and ReLU on the way out.
// hb (nullable): h rounded to bf16 as well, (ceil(P / 16) * 16, FOUT): the bf16 heads block reads it instead of
// converting h once per head; its padding rows hold row P - 1's values (every x load reads row min(r, P - 1)).
template <int FIN, int FOUT>
__global__ __launch_bounds__(kFbThreads) void feature_fwd_kernel(int P, const float *__restrict__ x,
                                                                 const float *__restrict__ w,
                                                                 const float *__restrict__ b, float *__restrict__ h,
                                                                 __bf16 *__restrict__ hb) {
    constexpr int WS = FIN + 4, NT = FOUT / 16, NW = kFbThreads / 64;
    __shared__ float s_w[FOUT * WS];
    for (int e = threadIdx.x; e < FOUT * FIN / 4; e += kFbThreads) {
        const int row = e / (FIN / 4), c4 = e % (FIN / 4);
        reinterpret_cast<float4 *>(s_w + row * WS)[c4] = reinterpret_cast<const float4 *>(w + (size_t)row * FIN)[c4];
    }
    __syncthreads();
    const int lane = threadIdx.x & 63, wv = (int)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6), q = lane >> 4, c = lane & 15;
    float bias[NT];
#pragma unroll
    for (int t = 0; t < NT; t++) bias[t] = b[16 * t + c];
    const int nblk = (P + 15) / 16;
    for (int blk = blockIdx.x * NW + wv; blk < nblk; blk += gridDim.x * NW) {
        const int r0 = blk * 16, ra = r0 + c;
        float4 xv[FIN / 16];
#pragma unroll
        for (int kc = 0; kc < FIN / 16; kc++)
            xv[kc] = *reinterpret_cast<const float4 *>(x + (size_t)min(ra, P - 1) * FIN + 16 * kc + 4 * q);
        f4v acc[NT];
#pragma unroll
        for (int t = 0; t < NT; t++) acc[t] = f4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kc = 0; kc < FIN / 16; kc++) {
#pragma unroll
            for (int t = 0; t < NT; t++) {
                const float4 bv = *reinterpret_cast<const float4 *>(s_w + (16 * t + c) * WS + 16 * kc + 4 * q);
                acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(xv[kc].x, bv.x, acc[t], 0, 0, 0);
                acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(xv[kc].y, bv.y, acc[t], 0, 0, 0);
                acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(xv[kc].z, bv.z, acc[t], 0, 0, 0);
                acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(xv[kc].w, bv.w, acc[t], 0, 0, 0);
            }
        }
        // C[row 4q + j][col 16 t + c]
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int r = r0 + 4 * q + j;
            if (r < P) {
#pragma unroll
                for (int t = 0; t < NT; t++) h[(size_t)r * FOUT + 16 * t + c] = fmaxf(acc[t][j] + bias[t], 0.f);
            }
            if (hb) {
#pragma unroll
                for (int t = 0; t < NT; t++) hb[(size_t)r * FOUT + 16 * t + c] = (__bf16)fmaxf(acc[t][j] + bias[t], 0.f);
            }
        }
    }
}

// ---- the HexPlane field's input points: scene/hexplane.py:20-21 normalize_aabb + :166 torch.cat((pts, t)) in
// one pass, pts4[n] = ((xyz[n] - aabb[0]) * s - 1, t[n]) with s = (1 / (aabb[1] - aabb[0])) * 2 (torch's
// 2.0 / tensor is reciprocal-then-multiply), the same float operations as the reference's graph; backward:
// dxyz = dpts[:, 0:3] * s (the mul's gradient; the time column takes none).
__device__ __forceinline__ float3 hex_scale(const float *aabb) {
    return make_float3((1.0f / (aabb[3] - aabb[0])) * 2.0f, (1.0f / (aabb[4] - aabb[1])) * 2.0f,
                       (1.0f / (aabb[5] - aabb[2])) * 2.0f);
}
__global__ __launch_bounds__(256) void hex_points_kernel(int N, const float *__restrict__ xyz, int64_t ld_xyz,
                                                         const float *__restrict__ t, int64_t ld_t,
                                                         const float *__restrict__ aabb, float4 *__restrict__ pts) {
    const int n = blockIdx.x * 256 + threadIdx.x;
    if (n >= N) return;
    const float3 sc = hex_scale(aabb);
    const float *x = xyz + (size_t)n * ld_xyz;
    pts[n] = make_float4((x[0] - aabb[0]) * sc.x - 1.0f, (x[1] - aabb[1]) * sc.y - 1.0f, (x[2] - aabb[2]) * sc.z - 1.0f,
                         t[(size_t)n * ld_t]);
}
// add (nullable): another gradient of xyz, summed in (the add autograd would launch for xyz's two uses)
__global__ __launch_bounds__(256) void hex_points_bwd_kernel(int N, const float4 *__restrict__ dpts,
                                                             const float *__restrict__ aabb,
                                                             const float *__restrict__ add, float *__restrict__ dxyz) {
    const int n = blockIdx.x * 256 + threadIdx.x;
    if (n >= N) return;
    const float3 sc = hex_scale(aabb);
    const float4 d = dpts[n];
    float g0 = d.x * sc.x, g1 = d.y * sc.y, g2 = d.z * sc.z;
    if (add) {
        g0 = add[3 * (size_t)n] + g0;
        g1 = add[3 * (size_t)n + 1] + g1;
        g2 = add[3 * (size_t)n + 2] + g2;
    }
    dxyz[3 * (size_t)n] = g0;
    dxyz[3 * (size_t)n + 1] = g1;
    dxyz[3 * (size_t)n + 2] = g2;
}

}  // namespace gs4d

using namespace gs4d;

// sum of S slices of n floats in slice order (gs4d_sum_slices): four slices in flight per thread, float4
// columns when n and the pointers allow
// 64-thread workgroups: a column per thread, so the (P / 1024)-slice sums of the MLP's 128 x 640 weight
// gradient (20480 float4 columns) spread over 320 workgroups, every CU, where 256-thread ones filled 80 CUs
constexpr int kSumThreads = 64;
// ---- row surgery of densification / pruning (gs4d_rows_assemble, scene/gaussian_model.py:316-506): tensor
// blockIdx.y, its output elements grid-strided over blockIdx.x.  Element c of output row r: r < K takes old
// row keep[r]; r = K + j takes, by the tensor's mode, old row append[j] or (the last given_rows) given rows,
// or zero.  Pure copies
// (4-byte words or bytes): bitwise the reference's cat / boolean-index results.  The batch is passed by value.
constexpr int64_t kRowsPerBlock = (int64_t)kTailThreads * 8;
template <class T>
__device__ __forceinline__ void rows_copy(const gs4d_rows_batch &b, const gs4d_rows_tensor &t) {
    const int64_t w = t.width, n = (b.K + b.A) * w;
    const T *__restrict__ src = (const T *)t.src;
    const T *__restrict__ given = (const T *)t.given;
    T *__restrict__ dst = (T *)t.dst;
    for (int64_t e = (int64_t)blockIdx.x * kTailThreads + threadIdx.x; e < n; e += (int64_t)gridDim.x * kTailThreads) {
        const int64_t r = e / w, c = e - r * w;
        T v = T(0);
        if (t.mode != GS4D_ROWS_ZERO) {
            if (r < b.K) {
                v = src[(int64_t)b.keep[r] * w + c];
            } else if (t.mode == GS4D_ROWS_GATHER) {
                const int64_t j = r - b.K, jg = j - (b.A - t.given_rows);
                v = jg < 0 ? src[(int64_t)b.append[j] * w + c] : given[jg * w + c];
            }
        }
        dst[e] = v;
    }
}
__global__ __launch_bounds__(kTailThreads) void rows_assemble_kernel(gs4d_rows_batch b) {
    const gs4d_rows_tensor &t = b.t[blockIdx.y];
    if (t.esize == 4) rows_copy<uint32_t>(b, t);
    else rows_copy<uint8_t>(b, t);
}

template <bool V4>
__global__ __launch_bounds__(kSumThreads) void sum_slices_kernel(const float *__restrict__ parts, int S, int64_t n,
                                                                 float *__restrict__ out) {
    const int64_t m = V4 ? n / 4 : n;
    for (int64_t i = (int64_t)blockIdx.x * kSumThreads + threadIdx.x; i < m; i += (int64_t)gridDim.x * kSumThreads) {
        if (V4) {
            const float4 *p = reinterpret_cast<const float4 *>(parts) + i;
            float4 acc = p[0];
            int s = 1;
            for (; s + 7 < S; s += 8) {  // the loads of eight slices issued together, added in order
                float4 v[8];
#pragma unroll
                for (int k = 0; k < 8; k++) v[k] = p[(size_t)(s + k) * m];
#pragma unroll
                for (int k = 0; k < 8; k++) {
                    acc.x += v[k].x; acc.y += v[k].y; acc.z += v[k].z; acc.w += v[k].w;
                }
            }
            for (; s < S; s++) {
                const float4 a = p[(size_t)s * m];
                acc.x += a.x; acc.y += a.y; acc.z += a.z; acc.w += a.w;
            }
            reinterpret_cast<float4 *>(out)[i] = acc;
        } else {
            float acc = parts[i];
            for (int s = 1; s < S; s++) acc += parts[(size_t)s * n + i];
            out[i] = acc;
        }
    }
}

// Many slices (S >= 16) over few outputs (the split-K weight gradients: 200 slices of 82k floats): a wave per
// 16 float4 outputs, its four 16-lane groups summing a quarter of the slices each in slice order, then the
// quarters as (q0 + q1) + (q2 + q3) through two lane swaps -- a fixed tree, so every run gives the same bits, and
// four times the loads in flight of one thread per output (which left most CUs idle: 80 workgroups).
__global__ __launch_bounds__(kSumThreads) void sum_slices_quarters_kernel(const float *__restrict__ parts, int S,
                                                                          int64_t m, float4 *__restrict__ out) {
    const int lane = threadIdx.x & 63, g = lane >> 4;
    const int64_t i = (((int64_t)blockIdx.x * kSumThreads + threadIdx.x) >> 6) * 16 + (lane & 15);
    const int s0 = g * S / 4, s1 = (g + 1) * S / 4;
    const float4 *p = reinterpret_cast<const float4 *>(parts) + (i < m ? i : 0);
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    int s = s0;
    for (; s + 7 < s1; s += 8) {  // eight slices' loads issued together, added in order
        float4 v[8];
#pragma unroll
        for (int k = 0; k < 8; k++) v[k] = p[(size_t)(s + k) * m];
#pragma unroll
        for (int k = 0; k < 8; k++) {
            acc.x += v[k].x; acc.y += v[k].y; acc.z += v[k].z; acc.w += v[k].w;
        }
    }
    for (; s < s1; s++) {
        const float4 a = p[(size_t)s * m];
        acc.x += a.x; acc.y += a.y; acc.z += a.z; acc.w += a.w;
    }
    // (q0 + q1) + (q2 + q3): float addition commutes exactly, so both lanes of a swap hold the same bits
#pragma unroll
    for (int off = 16; off <= 32; off <<= 1) {
        acc.x += __shfl_xor(acc.x, off);
        acc.y += __shfl_xor(acc.y, off);
        acc.z += __shfl_xor(acc.z, off);
        acc.w += __shfl_xor(acc.w, off);
    }
    if (g == 0 && i < m) out[i] = acc;
}

extern "C" {

// the launches: maximal runs of heads of one class (narrow: n <= 16; wide: n = 48)
static bool hb_wide(int n) { return n > 16; }  // n = 48 (validated), one head per launch
static bool hb_mfma(int W, int n) { return (W == 64 || W == 128) && n == 48; }  // heads_bwd_wide_mfma_kernel
#ifndef HB_WIDE_BF16
#define HB_WIDE_BF16 1
#endif
static const bool hb_wide_bf16 = HB_WIDE_BF16 != 0;  // the bf16 path's wide head on heads_bwd_wide_bf16_kernel
static int hb_rows_per_wg(int P, bool wide, bool bf) {
    // narrow heads stream a: about two (fp32) or four (bf16: half the bytes per row) workgroups per CU; the wide
    // head's waves are compute-heavy and its per-workgroup partials large (9 KB per block of rows): 512-row
    // blocks on the fp32 MFMA kernel, 256 on the bf16 one (tools/ab_heads.sh at P = 100k: the fp32 heads
    // backward 160 -> 148 us, the bf16 one 106 -> 97 us against 128-row blocks and P / 512 narrow rows)
    if (wide) return bf ? 256 : 512;
    return bf ? std::max(64, (P + 1023) / 1024) : std::max(64, (P + 511) / 512);
}
extern "C++" {
template <class Fn>
static void hb_groups(int k, const int *n, Fn fn) {  // fn(h0, hk)
    for (int h0 = 0; h0 < k;) {
        int h1 = h0 + 1;
        while (h1 < k && !hb_wide(n[h0]) && !hb_wide(n[h1])) h1++;
        fn(h0, h1 - h0);
        h0 = h1;
    }
}
}

size_t gs4d_heads_backward_scratch_bytes(int P, int W, int k, const int *n) {
    if (P < 0 || W < 1 || k < 1 || k > kHbMaxHeads || !n) return 0;
    size_t total = 256;
    hb_groups(k, n, [&](int h0, int hk) {
        size_t per = (size_t)hk * W;
        for (int i = h0; i < h0 + hk; i++) per += (size_t)std::max(n[i], 0) * (W + 1);
        // one size for both element types: the smaller row block (more workgroups, more partials)
        const int rows = std::min(hb_rows_per_wg(P, hb_wide(n[h0]), false), hb_rows_per_wg(P, hb_wide(n[h0]), true));
        const size_t nwg = std::max<size_t>(1, ((size_t)P + rows - 1) / rows);
        total += align_up(4 * nwg * per, 256);
    });
    return total;
}

extern "C++" {
template <class TA, class Args>
static int heads_backward_t(const Args *args, void *scratch, void *stream) {
    if (!args || !scratch) return 1;
    const Args &b = *args;
    const TA *ba = reinterpret_cast<const TA *>(b.a);
    TA *bda = reinterpret_cast<TA *>(b.da);
    if (b.P < 0 || (b.W != 64 && b.W != 128 && b.W != 256) || b.k < 1 || b.k > kHbMaxHeads || b.k * b.W > 768 ||
        !b.db1)
        return 1;
    if (b.P > 0 && (!b.a || !b.da)) return 1;
    HbArgs A{};
    HbOut O{};
    A.P = b.P, A.W = b.W, A.k = b.k;
    const float *g[kHbMaxHeads] = {};
    for (int i = 0; i < b.k; i++) {
        if (b.n[i] < 1 || (b.n[i] > 16 && b.n[i] != 48) || !b.w2[i] || !b.dw2[i] || !b.db2[i] || (b.P > 0 && !b.g[i]))
            return 1;
        if (b.n[i] == 48 && (((size_t)b.g[i] & 15) || b.W > 128)) return 1;  // rows read as float4; LDS combine
        A.n[i] = b.n[i], A.w2[i] = b.w2[i], g[i] = b.g[i];
        O.dw2[i] = b.dw2[i], O.db2[i] = b.db2[i];
    }
    O.db1 = b.db1;
    hipStream_t s = (hipStream_t)stream;
    char *q = (char *)align_up((size_t)scratch, 256);
    int err = 0;
    HbRed R{};
    auto flush = [&]() {  // the pending groups' reduction, one launch
        if (!R.count) return;
        hipLaunchKernelGGL(heads_bwd_reduce_kernel, dim3(R.blk0[R.count]), dim3(256), 0, s, R, O);
        R = HbRed{};
    };
    hb_groups(b.k, b.n, [&](int h0, int hk) {
        A.h0 = h0, A.hk = hk;
        A.rows_per_wg = hb_rows_per_wg(b.P, hb_wide(b.n[h0]), std::is_same<TA, __bf16>::value);
        A.poff[0] = hk * b.W;
        for (int i = 0; i < hk; i++) A.poff[i + 1] = A.poff[i] + b.n[h0 + i] * (b.W + 1);
        const int nwg = std::max(1, (int)(((int64_t)b.P + A.rows_per_wg - 1) / A.rows_per_wg));
        float *part = (float *)q;
        q += align_up(4 * (size_t)nwg * A.poff[hk], 256);
        if (b.P == 0) {  // empty sums: the partials of one empty workgroup
            if (hipMemsetAsync(part, 0, 4 * (size_t)A.poff[hk], s) != hipSuccess) err = 3;
        } else {
            if (hb_wide(b.n[h0]) && hb_mfma(b.W, b.n[h0]) && std::is_same<TA, __bf16>::value && b.W == 128 &&
                hb_wide_bf16) {
                hipLaunchKernelGGL(heads_bwd_wide_bf16_kernel, dim3(nwg), dim3(256), 0, s, A, (const __bf16 *)ba,
                                   (__bf16 *)bda, g[h0], part);
            } else if (hb_wide(b.n[h0]) && hb_mfma(b.W, b.n[h0])) {
                if (b.W == 128)
                    hipLaunchKernelGGL((heads_bwd_wide_mfma_kernel<128, 48, TA>), dim3(nwg), dim3(256), 0, s, A, ba,
                                       bda, g[h0], part);
                else
                    hipLaunchKernelGGL((heads_bwd_wide_mfma_kernel<64, 48, TA>), dim3(nwg), dim3(256), 0, s, A, ba, bda,
                                       g[h0], part);
            } else if (hb_wide(b.n[h0])) {
                if constexpr (std::is_same<TA, float>::value)
                    hipLaunchKernelGGL(heads_bwd_wide_kernel<48>, dim3(nwg), dim3(kWideGroups * b.W), 0, s, A, ba, bda,
                                       g[h0], part);
                else
                    err = 1;  // the bf16 path serves the wide head on the MFMA kernel only (W in {64, 128})
            } else if (std::is_same<TA, __bf16>::value && b.W % 128 == 0 && hk * b.W <= 1024)
                hipLaunchKernelGGL(heads_bwd2_kernel, dim3(nwg), dim3(hk * b.W / 2), 0, s, A, (const __bf16 *)ba,
                                   (__bf16 *)bda, g[0], g[1], g[2], g[3], g[4], g[5], g[6], g[7], part);
            else
                hipLaunchKernelGGL(heads_bwd_kernel<TA>, dim3(nwg), dim3(hk * b.W), 0, s, A, ba, bda, g[0], g[1], g[2],
                                   g[3], g[4], g[5], g[6], g[7], part);
        }
        if (R.count == kHbRedGroups) flush();
        R.A[R.count] = A, R.part[R.count] = part, R.nwg[R.count] = nwg;
        R.blk0[R.count + 1] = R.blk0[R.count] + (A.poff[hk] + kHbRedOut - 1) / kHbRedOut;
        R.count++;
    });
    flush();
    if (err) return err;
    return hipGetLastError() == hipSuccess ? 0 : 3;
}
}

int gs4d_heads_backward(const gs4d_heads_bwd *args, void *scratch, void *stream) {
    return heads_backward_t<float>(args, scratch, stream);
}

int gs4d_heads_backward_bf16(const gs4d_heads_bwd_bf16 *args, void *scratch, void *stream) {
    if (args)
        for (int i = 0; i < args->k && i < kHbMaxHeads; i++)
            if (hb_wide(args->n[i]) && !hb_mfma(args->W, args->n[i])) return 1;
    return heads_backward_t<__bf16>(args, scratch, stream);
}

size_t gs4d_linear_dw_scratch_bytes(int P, int W, int count, const int *n) {
    if (P < 0 || W < 1 || count < 1 || count > kDwMaxProblems || !n) return 0;
    int nmax = 0, nsum = 0;
    for (int i = 0; i < count; i++) nmax = std::max(nmax, n[i]), nsum += std::max(n[i], 0);
    const size_t nwg = std::max<size_t>(1, ((size_t)P + dw_rows_per_wg(P, nmax) - 1) / dw_rows_per_wg(P, nmax));
    return 4 * nwg * (size_t)nsum * (W + 1) + 256;
}

int gs4d_linear_dw(int P, int W, int count, const gs4d_dw_problem *problems, void *scratch, void *stream) {
    if (P < 0 || (W != 64 && W != 128 && W != 256) || count < 1 || count > kDwMaxProblems || !problems || !scratch)
        return 1;
    DwBatch b{};
    int nmax = 0, nsum = 0;
    for (int i = 0; i < count; i++) {
        const gs4d_dw_problem &p = problems[i];
        if (p.n < 1 || (p.n > 16 && p.n != 48) || p.n * W > kDwMaxNW || (P > 0 && (!p.dy || !p.x)) || !p.dw || p.ld_dy < p.n || p.ld_x < W)
            return 1;
        nmax = std::max(nmax, p.n);
        b.q[i] = DwProblem{p.dy, p.x, p.dw, p.db, p.n, p.ld_dy, p.ld_x, 0, 0};
    }
    hipStream_t s = (hipStream_t)stream;
    if (P == 0) {
        for (int i = 0; i < count; i++) {
            if (hipMemsetAsync(b.q[i].dw, 0, 4 * (size_t)b.q[i].n * W, s) != hipSuccess) return 3;
            if (b.q[i].db && hipMemsetAsync(b.q[i].db, 0, 4 * (size_t)b.q[i].n, s) != hipSuccess) return 3;
        }
        return 0;
    }
    const int rows = dw_rows_per_wg(P, nmax);
    const int nwg = (int)(((int64_t)P + rows - 1) / rows);
    for (int i = 0; i < count; i++) b.q[i].part_off = (int64_t)nwg * nsum * (W + 1), nsum += b.q[i].n;
    float *part = (float *)align_up((size_t)scratch, 256);
    if (nmax <= 8) hipLaunchKernelGGL(linear_dw_kernel<0>, dim3(nwg, count), dim3(kDwThreads), 0, s, b, P, W, rows, part);
    else hipLaunchKernelGGL(linear_dw_kernel<1>, dim3(nwg, count), dim3(kDwThreads), 0, s, b, P, W, rows, part);
    hipLaunchKernelGGL(linear_dw_reduce_kernel, dim3((nmax * (W + 1) + 31) / 32, count), dim3(256), 0, s, b, W, nwg,
                       (const float *)part);
    return hipGetLastError() == hipSuccess ? 0 : 3;
}

int64_t gs4d_reg_blocks(int C, int H, int W) { return ((int64_t)C * H * W + kRegBlock - 1) / kRegBlock; }

static int reg_check(const gs4d_reg_batch *b, int64_t *nblk) {
    if (!b || b->count < 1 || b->count > GS4D_REG_MAX_PLANES) return 1;
    int64_t blocks = 0;
    for (int i = 0; i < b->count; i++) {
        const gs4d_reg_plane &p = b->p[i];
        if (!p.data || p.C < 1 || p.H < 3 || p.W < 1 || p.first_block != blocks) return 1;
        if ((int64_t)p.C * p.H * p.W > INT32_MAX) return 1;  // the kernels index a plane in 32 bits
        blocks += gs4d_reg_blocks(p.C, p.H, p.W);
    }
    *nblk = blocks;
    return 0;
}

size_t gs4d_reg_scratch_bytes(const gs4d_reg_batch *batch) {
    int64_t nblk = 0;
    if (reg_check(batch, &nblk)) return 0;
    return 8 * (size_t)nblk + 4 * kTicketWords + 256;
}

int gs4d_hexplane_reg_forward(const gs4d_reg_batch *batch, float *loss, void *scratch, void *stream) {
    int64_t nblk = 0;
    if (reg_check(batch, &nblk) || !loss || !scratch) return 1;
    hipLaunchKernelGGL(reg_forward_kernel, dim3((unsigned)nblk), dim3(kTailThreads), 0, (hipStream_t)stream, *batch,
                       ticket_scratch(scratch), loss);
    return hipGetLastError() == hipSuccess ? 0 : 3;
}

int gs4d_hexplane_reg_backward(const gs4d_reg_batch *batch, const float *dloss, void *stream) {
    int64_t nblk = 0;
    if (reg_check(batch, &nblk) || !dloss) return 1;
    for (int i = 0; i < batch->count; i++)
        if (!batch->p[i].grad) return 1;
    hipLaunchKernelGGL(reg_backward_kernel, dim3((unsigned)nblk), dim3(kTailThreads), 0, (hipStream_t)stream, *batch,
                       dloss, TicketScratch{nullptr, nullptr}, (float *)nullptr, (const float *)nullptr);
    return hipGetLastError() == hipSuccess ? 0 : 3;
}

int gs4d_hexplane_reg_backward_value(const gs4d_reg_batch *batch, const float *dloss, float *loss, const float *base,
                                     void *scratch, void *stream) {
    int64_t nblk = 0;
    if (reg_check(batch, &nblk) || !dloss || !loss || !scratch) return 1;
    for (int i = 0; i < batch->count; i++)
        if (!batch->p[i].grad) return 1;
    hipLaunchKernelGGL(reg_backward_kernel, dim3((unsigned)nblk), dim3(kTailThreads), 0, (hipStream_t)stream, *batch,
                       dloss, ticket_scratch(scratch), loss, base);
    return hipGetLastError() == hipSuccess ? 0 : 3;
}


size_t gs4d_l1_scratch_bytes(int64_t n) { return 8 * (size_t)((n + kL1Chunk - 1) / kL1Chunk) + 4 * kTicketWords + 256; }

int gs4d_l1_loss_forward(int64_t n, const float *x, const float *y, int8_t *sign, float *loss, void *scratch,
                         void *stream) {
    if (n < 0 || (n > 0 && (!x || !y || !sign || !scratch)) || !loss) return 1;
    hipStream_t s = (hipStream_t)stream;
    if (n == 0) return hipMemsetAsync(loss, 0, 4, s) == hipSuccess ? 0 : 3;
    const int64_t nblk = (n + kL1Chunk - 1) / kL1Chunk;
    if (nblk > INT32_MAX) return 1;
    if (n % 4 == 0 && (((size_t)x | (size_t)y) & 15) == 0 && ((size_t)sign & 3) == 0)
        hipLaunchKernelGGL(l1_partial_v4_kernel<false>, dim3((unsigned)nblk), dim3(kTailThreads), 0, s, n / 4,
                           (const float4 *)x, (const float4 *)y, (char4 *)sign, ticket_scratch(scratch), loss,
                           (float4 *)nullptr, 0.f);
    else
        hipLaunchKernelGGL(l1_partial_kernel, dim3((unsigned)nblk), dim3(kTailThreads), 0, s, n, x, y, sign,
                           ticket_scratch(scratch), loss);
    return hipGetLastError() == hipSuccess ? 0 : 3;
}

int gs4d_l1_loss_grad(int64_t n, const float *x, const float *y, float dloss, float *loss, float *grad, void *scratch,
                      void *stream) {
    if (n < 0 || (n > 0 && (!x || !y || !grad || !scratch)) || !loss) return 1;
    hipStream_t s = (hipStream_t)stream;
    if (n == 0) return hipMemsetAsync(loss, 0, 4, s) == hipSuccess ? 0 : 3;
    if (n % 4 != 0 || (((size_t)x | (size_t)y | (size_t)grad) & 15) != 0) return 1;  // the float4 form only
    const int64_t nblk = (n + kL1Chunk - 1) / kL1Chunk;
    if (nblk > INT32_MAX) return 1;
    const float scale = dloss * (1.0f / (float)n);  // torch's MeanBackward rounding, as l1_backward
    hipLaunchKernelGGL(l1_partial_v4_kernel<true>, dim3((unsigned)nblk), dim3(kTailThreads), 0, s, n / 4,
                       (const float4 *)x, (const float4 *)y, (char4 *)nullptr, ticket_scratch(scratch), loss,
                       (float4 *)grad, scale);
    return hipGetLastError() == hipSuccess ? 0 : 3;
}

int gs4d_l1_loss_backward(int64_t n, const int8_t *sign, const float *dloss, float *grad, void *stream) {
    if (n < 0 || (n > 0 && (!sign || !dloss || !grad))) return 1;
    if (n == 0) return 0;
    if (n % 4 == 0 && ((size_t)sign & 3) == 0 && ((size_t)grad & 15) == 0) {
        const int nblk = (int)std::min<int64_t>((n / 4 + kTailThreads - 1) / kTailThreads, 8192);
        hipLaunchKernelGGL(l1_backward_v4_kernel, dim3(nblk), dim3(kTailThreads), 0, (hipStream_t)stream, n / 4,
                           (const char4 *)sign, dloss, (float4 *)grad, n);
        return hipGetLastError() == hipSuccess ? 0 : 3;
    }
    const int nblk = (int)std::min<int64_t>((n + kTailThreads - 1) / kTailThreads, 8192);
    hipLaunchKernelGGL(l1_backward_kernel, dim3(nblk), dim3(kTailThreads), 0, (hipStream_t)stream, n, sign, dloss, grad);
    return hipGetLastError() == hipSuccess ? 0 : 3;
}

int gs4d_deform_tail_forward(int P, int K, const float *xyz, const float *s, const float *r, const float *o,
                             const float *f_dc, const float *f_rest, const float *dx, const float *ds, const float *dr,
                             const float *d_o, const float *dshs, float *means, float *scales, float *rot,
                             float *opac, float *shs, void *stream) {
    if (P < 0 || K < 1 || (P > 0 && (!xyz || !s || !r || !o || !f_dc || (K > 1 && !f_rest) || !means || !scales ||
                                     !rot || !opac || !shs)))
        return 1;
    if (P == 0) return 0;
    if ((int64_t)P * 3 * K > UINT32_MAX) return 1;  // the SH range is indexed in 32 bits
    const int nb_g = (P + kTailThreads - 1) / kTailThreads;
    const int v4 = (3 * K) % 4 == 0 && (((size_t)dshs | (size_t)shs) & 15) == 0;
    const int64_t nb_s = ((int64_t)P * 3 * K / (v4 ? 4 : 1) + kTailThreads - 1) / kTailThreads;
    hipLaunchKernelGGL(deform_tail_fwd_kernel, dim3((unsigned)(nb_g + nb_s)), dim3(kTailThreads), 0, (hipStream_t)stream,
                       P, K, nb_g, xyz, s, r, o, f_dc, f_rest, dx, ds, dr, d_o, dshs, means, scales, rot, opac, shs, v4);
    return hipGetLastError() == hipSuccess ? 0 : 3;
}

int gs4d_deform_tail_backward(int P, int K, const float *scales, const float *r, const float *dr, const float *opac,
                              const float *g_means, const float *g_scales, const float *g_rot, const float *g_opac,
                              const float *g_shs, float *d_xyz, float *d_s, float *d_r, float *d_o, float *d_fdc,
                              float *d_frest, float *g_dx, float *g_ds, float *g_dr, float *g_do, void *stream) {
    if (P < 0 || K < 1 || (P > 0 && (!scales || !r || !opac || !d_xyz || !d_s || !d_r || !d_o || !d_fdc ||
                                     (K > 1 && !d_frest))))
        return 1;
    if (P == 0) return 0;
    if ((int64_t)P * 3 * K > UINT32_MAX) return 1;  // the SH range is indexed in 32 bits
    const int nb_g = (P + kTailThreads - 1) / kTailThreads;
    const int v4 = (3 * K) % 4 == 0 && ((size_t)g_shs & 15) == 0;
    const int64_t nb_s = ((int64_t)P * 3 * K / (v4 ? 4 : 1) + kTailThreads - 1) / kTailThreads;
    hipLaunchKernelGGL(deform_tail_bwd_kernel, dim3((unsigned)(nb_g + nb_s)), dim3(kTailThreads), 0, (hipStream_t)stream,
                       P, K, nb_g, scales, r, dr, opac, g_means, g_scales, g_rot, g_opac, g_shs, d_xyz, d_s, d_r, d_o,
                       d_fdc, d_frest, g_dx, g_ds, g_dr, g_do, v4);
    return hipGetLastError() == hipSuccess ? 0 : 3;
}

int gs4d_rows_assemble(const gs4d_rows_batch *batch, void *stream) {
    if (!batch || batch->count < 0 || batch->count > GS4D_ROWS_MAX_TENSORS || batch->K < 0 || batch->A < 0) return 1;
    const gs4d_rows_batch &b = *batch;
    const int64_t rows = b.K + b.A;
    if (rows > INT32_MAX || (b.K > 0 && !b.keep)) return 1;
    int64_t most = 0;
    for (int i = 0; i < b.count; i++) {
        const gs4d_rows_tensor &t = b.t[i];
        if (t.width < 1 || (t.esize != 1 && t.esize != 4) || t.mode < GS4D_ROWS_GATHER || t.mode > GS4D_ROWS_ZERO) return 1;
        if (rows > 0 && !t.dst) return 1;
        if (t.mode != GS4D_ROWS_ZERO && b.K > 0 && !t.src) return 1;
        if (t.mode == GS4D_ROWS_GATHER) {
            if (t.given_rows < 0 || t.given_rows > b.A || (t.given_rows > 0 && !t.given)) return 1;
            if (t.given_rows < b.A && (!b.append || !t.src)) return 1;
        }
        most = std::max(most, rows * t.width);
    }
    if (b.count == 0 || most == 0) return 0;
    const unsigned gx = (unsigned)std::min<int64_t>((most + kRowsPerBlock - 1) / kRowsPerBlock, 4096);
    hipLaunchKernelGGL(rows_assemble_kernel, dim3(gx, b.count), dim3(kTailThreads), 0, (hipStream_t)stream, b);
    return hipGetLastError() == hipSuccess ? 0 : 3;
}

int gs4d_sum_slices(const float *parts, int S, int64_t n, float *out, void *stream) {
    if (S < 1 || n < 0 || (n > 0 && (!parts || !out))) return 1;
    if (n == 0) return 0;
    const bool v4 = n % 4 == 0 && ((uintptr_t)parts % 16) == 0 && ((uintptr_t)out % 16) == 0;
    const int64_t m = v4 ? n / 4 : n;
    if (v4 && S >= 16 && m <= ((int64_t)1 << 24)) {
        const unsigned g4 = (unsigned)((m + 15) / 16 * 64 + kSumThreads - 1) / kSumThreads;
        hipLaunchKernelGGL(sum_slices_quarters_kernel, dim3(g4), dim3(kSumThreads), 0, (hipStream_t)stream, parts, S,
                           m, reinterpret_cast<float4 *>(out));
        return hipGetLastError() == hipSuccess ? 0 : 3;
    }
    const unsigned grid = (unsigned)std::min<int64_t>((m + kSumThreads - 1) / kSumThreads, 16384);
    if (v4)
        hipLaunchKernelGGL(sum_slices_kernel<true>, dim3(grid), dim3(kSumThreads), 0, (hipStream_t)stream, parts, S, n, out);
    else
        hipLaunchKernelGGL(sum_slices_kernel<false>, dim3(grid), dim3(kSumThreads), 0, (hipStream_t)stream, parts, S, n,
                           out);
    return hipGetLastError() == hipSuccess ? 0 : 3;
}

int gs4d_densify_stats(int P, const float *viewspace_grad, const uint8_t *visible, const int *radii, float *grad_accum,
                       float *denom, float *max_radii, void *stream) {
    if (P < 0 || (P > 0 && (!viewspace_grad || (!visible && !radii) || !grad_accum || !denom || (radii && !max_radii))))
        return 1;
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

static int fb_grid(int P) {
    const int nblk = (P + kFbRows - 1) / kFbRows;
    return std::max(1, std::min(512, (nblk + 3) / 4));
}
size_t gs4d_feature_relu_backward_scratch_bytes(int P, int Fin, int Fout) {
    return 4 * (size_t)fb_grid(std::max(P, 0)) * ((size_t)Fout * Fin + Fout) + 256;
}

int gs4d_feature_relu_backward(int P, int Fin, int Fout, const float *g, const float *h, const float *x,
                               const float *w, float *dx, float *dw, float *db, void *scratch, void *stream) {
    if (P < 0 || !w || !dw || !db || !scratch) return 1;
    if (!((Fin == 32 && Fout == 128) || (Fin == 64 && Fout == 64) || (Fin == 32 && Fout == 64))) return 1;
    if (P > 0 && (!g || !h || !x || !dx)) return 1;
    if ((((size_t)g | (size_t)h | (size_t)w) & 15) != 0) return 1;
    hipStream_t s = (hipStream_t)stream;
    const int nwg = fb_grid(P), per = Fout * Fin + Fout;
    float *part = (float *)align_up((size_t)scratch, 256);
    if (P == 0) {
        if (hipMemsetAsync(part, 0, 4 * (size_t)per, s) != hipSuccess) return 3;
    } else if (Fin == 32 && Fout == 128) {
        hipLaunchKernelGGL((feature_bwd_kernel<32, 128>), dim3(nwg), dim3(kFbThreads), 0, s, P, g, h, x, w, dx, part);
    } else if (Fin == 64) {
        hipLaunchKernelGGL((feature_bwd_kernel<64, 64>), dim3(nwg), dim3(kFbThreads), 0, s, P, g, h, x, w, dx, part);
    } else {
        hipLaunchKernelGGL((feature_bwd_kernel<32, 64>), dim3(nwg), dim3(kFbThreads), 0, s, P, g, h, x, w, dx, part);
    }
    hipLaunchKernelGGL(feature_bwd_reduce_kernel, dim3((per + 15) / 16), dim3(256), 0, s, P == 0 ? 1 : nwg, per,
                       Fout * Fin, (const float *)part, dw, db);
    return hipGetLastError() == hipSuccess ? 0 : 3;
}

int gs4d_heads_forward(const gs4d_heads_fwd *args, void *stream) {
    if (!args) return 1;
    const gs4d_heads_fwd &b = *args;
    if (b.P < 0 || (b.W != 64 && b.W != 128 && b.W != 256) || b.k < 1 || b.k > kHbMaxHeads) return 1;
    HfArgs A{};
    A.P = b.P, A.W = b.W, A.k = b.k, A.kW = b.k * b.W;
    int rows = 0;
    for (int i = 0; i < b.k; i++) {
        if (b.n[i] < 1 || b.n[i] > 16 * kHfMaxTiles || !b.w2[i] || !b.b2[i] || (b.P > 0 && !b.out[i])) return 1;
        if (((size_t)b.w2[i] & 15) != 0) return 1;
        A.n[i] = b.n[i], A.w2[i] = b.w2[i], A.b2[i] = b.b2[i], A.out[i] = b.out[i], A.roff[i] = rows;
        rows += b.n[i];
    }
    const size_t lds = 4 * (size_t)rows * (b.W + 4);
    if (lds > 64 * 1024) return 1;
    if (b.P == 0) return 0;
    if (!b.a || ((size_t)b.a & 15) != 0) return 1;
    const int nblk = (b.P + 15) / 16;
    const int nwg = std::max(1, std::min(1024, (nblk + 3) / 4));
    hipStream_t s = (hipStream_t)stream;
    int tiles[kHbMaxHeads];
    for (int i = 0; i < b.k; i++) tiles[i] = (b.n[i] + 15) / 16;
    auto is = [&](std::initializer_list<int> cfg) {
        if ((int)cfg.size() != b.k) return false;
        int i = 0;
        for (int t : cfg) if (tiles[i++] != t) return false;
        return true;
    };
    auto launch = [&](auto kernel, const HfArgs &args, const float *ap) {
        hipLaunchKernelGGL(kernel, dim3(nwg), dim3(kHfThreads), lds, s, args, ap);
    };
    // the reference's head sets: arguments/dynerf (pos, scales, rotations, opacity, shs: 3,3,4,1,48 outputs)
    // and the defaults (pos, scales, rotations); any other set runs head by head
    if (b.W == 128 && is({1, 1, 1, 1, 3})) launch(heads_fwd_kernel<128, 1, 1, 1, 1, 3>, A, b.a);
    else if (b.W == 64 && is({1, 1, 1, 1, 3})) launch(heads_fwd_kernel<64, 1, 1, 1, 1, 3>, A, b.a);
    else if (b.W == 64 && is({1, 1, 1})) launch(heads_fwd_kernel<64, 1, 1, 1>, A, b.a);
    else if (b.W == 128 && is({1, 1, 1})) launch(heads_fwd_kernel<128, 1, 1, 1>, A, b.a);
    else {
        for (int i = 0; i < b.k; i++) {  // one head per launch: a's row stride stays k W
            HfArgs H{};
            H.P = b.P, H.W = b.W, H.k = 1, H.n[0] = b.n[i], H.roff[0] = 0, H.w2[0] = b.w2[i], H.b2[0] = b.b2[i];
            H.out[0] = b.out[i];
            const float *ap = b.a + (size_t)i * b.W;
            const int t = tiles[i];
            H.kW = b.k * b.W;
            auto one = [&](auto k64, auto k128, auto k256) {
                if (b.W == 64) launch(k64, H, ap);
                else if (b.W == 128) launch(k128, H, ap);
                else launch(k256, H, ap);
            };
            if (t == 1) one(heads_fwd_kernel<64, 1>, heads_fwd_kernel<128, 1>, heads_fwd_kernel<256, 1>);
            else if (t == 2) one(heads_fwd_kernel<64, 2>, heads_fwd_kernel<128, 2>, heads_fwd_kernel<256, 2>);
            else if (t == 3) one(heads_fwd_kernel<64, 3>, heads_fwd_kernel<128, 3>, heads_fwd_kernel<256, 3>);
            else one(heads_fwd_kernel<64, 4>, heads_fwd_kernel<128, 4>, heads_fwd_kernel<256, 4>);
        }
    }
    return hipGetLastError() == hipSuccess ? 0 : 3;
}

static int cu_count() {  // compute units of the current device (cached per device)
    static int cus[64] = {};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
    if (cus[dev] == 0) {
        int n = 0;
        if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
        cus[dev] = n;
    }
    return cus[dev];
}

// hipFuncSetAttribute(MaxDynamicSharedMemorySize) is per device: done once per (device, kernel set), and
// false when the device's per-workgroup LDS cannot hold `need` bytes
constexpr int kErrLds = 4;
static bool raise_lds_limit(const void *k0, const void *k1, int set, size_t need) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return false;
    static int state[3][64] = {};  // [set][device]: 0 unknown, 1 raised, 2 unavailable
    int &st = state[set][dev];
    if (st == 0) {
        int maxlds = 0;
        (void)hipDeviceGetAttribute(&maxlds, hipDeviceAttributeMaxSharedMemoryPerBlock, dev);
        const bool ok = hipFuncSetAttribute(k0, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) == hipSuccess &&
                        hipFuncSetAttribute(k1, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) == hipSuccess;
        (void)hipGetLastError();
        st = ok ? 1 : 2;
        if (ok && maxlds > 0 && (size_t)maxlds < 96 * 1024) st = 2;  // not a gfx950-class LDS
    }
    return st == 1 && need <= 160 * 1024;
}

int gs4d_heads_block_forward(const gs4d_heads_block_fwd *args, void *stream) {
    if (!args) return 1;
    const gs4d_heads_block_fwd &b = *args;
    if (b.P < 0 || (b.W != 64 && b.W != 128) || b.k < 1 || b.k > kHbMaxHeads || !b.w1 || !b.b1) return 1;
    HfArgs A{};
    A.P = b.P, A.W = b.W, A.k = b.k, A.kW = b.k * b.W;
    int npad_max = 0;
    for (int i = 0; i < b.k; i++) {
        if (b.n[i] < 1 || b.n[i] > 64 || !b.w2[i] || !b.b2[i] || (b.P > 0 && !b.out[i])) return 1;
        if (((size_t)b.w2[i] & 15) != 0) return 1;
        A.n[i] = b.n[i], A.w2[i] = b.w2[i], A.b2[i] = b.b2[i], A.out[i] = b.out[i];
        npad_max = std::max(npad_max, (b.n[i] + 15) & ~15);
    }
    if (((size_t)b.w1 & 15) != 0 || ((size_t)b.b1 & 15) != 0) return 1;
    if (b.P == 0) return 0;
    if (!b.h || !b.a || (((size_t)b.h | (size_t)b.a | (size_t)b.w1t) & 15) != 0) return 1;
    const size_t lds = 4 * ((size_t)(b.W + npad_max) * (b.W + 8) + b.W + npad_max);
    const int nblk = (b.P + 15) / 16;
    // ~1024 workgroups over the heads, one resident per CU (LDS): each stages its head's weights once and
    // takes a few blocks per wave (measured at P = 100k, k = 5: 237 / 218 / 207 us for 256 / 512 / 1024)
    // (16-wave workgroups measured no faster: 185-196 us for 256-1024 of them)
    const int per_head = std::max(1, std::min((nblk + 7) / 8, std::max(1, 1024 / b.k)));
    hipStream_t s = (hipStream_t)stream;
    // dynamic LDS above 64 KiB (gfx950: 160 KiB per CU), set once per device; a device that cannot give it
    // returns GS4D_TRAIN_ERR_LDS (the caller falls back to the GEMM formulation)
    if (!raise_lds_limit((const void *)heads_block_fwd_kernel<128>, (const void *)heads_block_fwd_kernel<64>, 0, lds))
        return kErrLds;
    if (b.W == 128)
        hipLaunchKernelGGL(heads_block_fwd_kernel<128>, dim3(per_head, b.k), dim3(kHbfThreads), lds, s, A, b.h, b.w1,
                           b.b1, b.a, b.w1t);
    else
        hipLaunchKernelGGL(heads_block_fwd_kernel<64>, dim3(per_head, b.k), dim3(kHbfThreads), lds, s, A, b.h, b.w1,
                           b.b1, b.a, b.w1t);
    return hipGetLastError() == hipSuccess ? 0 : 3;
}

int gs4d_heads_block_forward_bf16(const gs4d_heads_block_fwd_bf16 *args, void *stream) {
    if (!args) return 1;
    const gs4d_heads_block_fwd_bf16 &b = *args;
    if (b.P < 0 || (b.W != 64 && b.W != 128) || b.k < 1 || b.k > kHbMaxHeads || !b.w1 || !b.b1) return 1;
    HfArgs A{};
    A.P = b.P, A.W = b.W, A.k = b.k, A.kW = b.k * b.W;
    int npad_max = 0;
    for (int i = 0; i < b.k; i++) {
        if (b.n[i] < 1 || b.n[i] > 64 || !b.w2[i] || !b.b2[i] || (b.P > 0 && !b.out[i])) return 1;
        if (((size_t)b.w2[i] & 15) != 0) return 1;
        A.n[i] = b.n[i], A.w2[i] = b.w2[i], A.b2[i] = b.b2[i], A.out[i] = b.out[i];
        npad_max = std::max(npad_max, (b.n[i] + 15) & ~15);
    }
    if (((size_t)b.w1 & 15) != 0 || ((size_t)b.b1 & 15) != 0) return 1;
    if (b.P == 0) return 0;
    // h NULL: hb is the input (h already rounded to bf16, gs4d_feature_relu_forward_hb)
    const bool hbin = !b.h;
    if ((hbin && !b.hb) || !b.a || (((size_t)b.h | (size_t)b.a | (size_t)b.hb | (size_t)b.w1t) & 15) != 0) return 1;
    const size_t lds = 2 * (size_t)(b.W + npad_max) * (b.W + 8) + 4 * (size_t)(b.W + npad_max);
    const int nblk = (b.P + 15) / 16;
    // two workgroups per CU (the bf16 kernel's VGPRs allow two 512-thread workgroups): one round of
    // workgroups, each loading and converting its head's weights once (measured 85 -> 80 us at P = 100k, five
    // heads, against the fp32 kernel's 1024 / k)
    const int per_head = std::max(1, std::min((nblk + 7) / 8, std::max(1, 2 * cu_count() / b.k)));
    hipStream_t s = (hipStream_t)stream;
    if (!raise_lds_limit((const void *)heads_block_fwd_bf16_kernel<128, false>,
                         (const void *)heads_block_fwd_bf16_kernel<64, false>, 1, lds) ||
        !raise_lds_limit((const void *)heads_block_fwd_bf16_kernel<128, true>,
                         (const void *)heads_block_fwd_bf16_kernel<64, true>, 2, lds))
        return kErrLds;
    auto go = [&](auto kern) {
        hipLaunchKernelGGL(kern, dim3(per_head, b.k), dim3(kHbfThreads), lds, s, A, b.h, b.w1, b.b1, (__bf16 *)b.a,
                           (__bf16 *)b.hb, (__bf16 *)b.w1t);
    };
    if (b.W == 128) hbin ? go(heads_block_fwd_bf16_kernel<128, true>) : go(heads_block_fwd_bf16_kernel<128, false>);
    else hbin ? go(heads_block_fwd_bf16_kernel<64, true>) : go(heads_block_fwd_bf16_kernel<64, false>);
    return hipGetLastError() == hipSuccess ? 0 : 3;
}

int gs4d_mlp_dx_bf16(int P, int KW, int W, const uint16_t *da, const uint16_t *w1t, float *dh, void *stream) {
    if (P < 0 || KW < kDxChunk || KW % kDxChunk != 0 || (W != 64 && W != 128)) return 1;
    if (P == 0) return 0;
    if (!da || !w1t || !dh || (((size_t)da | (size_t)w1t | (size_t)dh) & 15) != 0) return 1;
    const int64_t rows_per_wg = (kDxThreads / 64) * kDxRowsPerWave;
    const dim3 grid((unsigned)(((int64_t)P + rows_per_wg - 1) / rows_per_wg));
    if (W == 128)
        hipLaunchKernelGGL(mlp_dx_bf16_kernel<128>, grid, dim3(kDxThreads), 0, (hipStream_t)stream, P, KW,
                           (const __bf16 *)da, (const __bf16 *)w1t, dh);
    else
        hipLaunchKernelGGL(mlp_dx_bf16_kernel<64>, grid, dim3(kDxThreads), 0, (hipStream_t)stream, P, KW,
                           (const __bf16 *)da, (const __bf16 *)w1t, dh);
    return hipGetLastError() == hipSuccess ? 0 : 3;
}

size_t gs4d_mlp_dw_bf16_scratch_bytes(int P, int KW, int W) {
    if (P <= 0 || KW <= 0 || W <= 0) return 256;
    const size_t S = ((size_t)P + kDwbChunkRows - 1) / kDwbChunkRows;
    return 4 * S * (size_t)KW * W + 256;
}

int gs4d_mlp_dw_bf16(int P, int KW, int W, const uint16_t *da, const uint16_t *hb, float *dw, void *scratch,
                     void *stream) {
    if (P < 0 || W != 128 || KW < W || KW % W != 0 || !dw) return 1;
    hipStream_t s = (hipStream_t)stream;
    if (P == 0) return hipMemsetAsync(dw, 0, 4 * (size_t)KW * W, s) == hipSuccess ? 0 : 3;
    if (!da || !hb || !scratch || (((size_t)da | (size_t)hb) & 15) != 0) return 1;
    const int S = (int)(((int64_t)P + kDwbChunkRows - 1) / kDwbChunkRows);
    float *parts = (float *)align_up((size_t)scratch, 256);
    hipLaunchKernelGGL(mlp_dw_bf16_kernel, dim3(S, KW / W), dim3(kDwbThreads), 0, s, P, KW, (const __bf16 *)da,
                       (const __bf16 *)hb, parts);
    if (hipGetLastError() != hipSuccess) return 3;
    return gs4d_sum_slices(parts, S, (int64_t)KW * W, dw, stream);
}

// A/B switch of the kernels' shapes (development only; 0 = the kept shapes): GS4D_MLP_SHAPE bit 0 = one 16-row
// block per wave in gs4d_mlp_dx_f32, bit 1 = 64-row m blocks in gs4d_mlp_dw_f32
static int mlp_shape() {
    static const int v = [] {
        const char *e = getenv("GS4D_MLP_SHAPE");
        return e ? atoi(e) : 0;
    }();
    return v;
}

int gs4d_mlp_dx_f32(int P, int KW, int W, const float *da, const float *w1t, float *dh, void *stream) {
    if (P < 0 || KW < 64 || KW % 64 != 0 || (W != 64 && W != 128)) return 1;
    if (P == 0) return 0;
    if (!da || !w1t || !dh || (((size_t)da | (size_t)w1t | (size_t)dh) & 15) != 0) return 1;
    hipStream_t s = (hipStream_t)stream;
    const bool k64 = KW % 128 == 0;  // an even number of 64-wide chunks, else 32-wide ones
    const int RB = (mlp_shape() & 1) ? 1 : 2;
    const int nrg = (int)(((int64_t)P + 64 * RB - 1) / (64 * RB));
    // W = 128: two feature groups per row group, the grid padded to whole groups of 8 row groups
    const dim3 grid((unsigned)(W == 128 ? (nrg + 7) / 8 * 16 : nrg));
    auto go = [&](auto kern) { hipLaunchKernelGGL(kern, grid, dim3(kDxfThreads), 0, s, P, KW, nrg, da, w1t, dh); };
    if (RB == 2) {  // 32-wide k chunks: two register sets of B for two row blocks fit 4 waves/SIMD
        if (W == 128) go(mlp_dx_f32_kernel<128, 32, 2>);
        else go(mlp_dx_f32_kernel<64, 32, 2>);
    } else {
        if (W == 128) k64 ? go(mlp_dx_f32_kernel<128, 64, 1>) : go(mlp_dx_f32_kernel<128, 32, 1>);
        else k64 ? go(mlp_dx_f32_kernel<64, 64, 1>) : go(mlp_dx_f32_kernel<64, 32, 1>);
    }
    return hipGetLastError() == hipSuccess ? 0 : 3;
}

// the m-block rows of gs4d_mlp_dw_f32's workgroups
static int dwf_mb(int KW, int W) { return (KW % 128 == 0 && W == 128 && !(mlp_shape() & 2)) ? 128 : 64; }
// the row chunks of gs4d_mlp_dw_f32: one resident round of workgroups over (chunk, m block) -- four per CU (a
// wave per SIMD each, <= 128 registers) -- so that every workgroup runs once and all finish together; chunks a
// multiple of 32 rows, at least 256
static void dwf_chunks(int P, int KW, int W, int *S, int *rows) {
    const int nmb = std::max(1, KW / dwf_mb(KW, W));
    const int64_t target = std::max<int64_t>(1, (4 * (int64_t)cu_count()) / nmb);
    int64_t c = ((int64_t)P + target - 1) / target;
    c = std::max<int64_t>(256, (c + 31) / 32 * 32);
    *rows = (int)c;
    *S = (int)std::max<int64_t>(1, ((int64_t)P + c - 1) / c);
}

size_t gs4d_mlp_dw_f32_scratch_bytes(int P, int KW, int W) {
    if (P <= 0 || KW <= 0 || W <= 0) return 256;
    int S = 1, rows = 0;
    dwf_chunks(P, KW, W, &S, &rows);
    return 4 * (size_t)S * KW * W + 256;
}

int gs4d_mlp_dw_f32(int P, int KW, int W, const float *da, const float *h, float *dw, void *scratch, void *stream) {
    if (P < 0 || (W != 64 && W != 128) || KW < 64 || KW % 64 != 0 || !dw) return 1;
    hipStream_t s = (hipStream_t)stream;
    if (P == 0) return hipMemsetAsync(dw, 0, 4 * (size_t)KW * W, s) == hipSuccess ? 0 : 3;
    if (!da || !h || !scratch) return 1;
    int S = 1, rows = 0;
    dwf_chunks(P, KW, W, &S, &rows);
    float *parts = (float *)align_up((size_t)scratch, 256);
    const int MB = dwf_mb(KW, W);
    const unsigned grid = (unsigned)(8 * (KW / MB) * ((S + 7) / 8));
    auto go = [&](auto kern) {
        hipLaunchKernelGGL(kern, dim3(grid), dim3(kDwfThreads), 0, s, P, KW, S, rows, da, h, parts);
    };
    if (W == 128) MB == 128 ? go(mlp_dw_f32_kernel<128, 128>) : go(mlp_dw_f32_kernel<128, 64>);
    else go(mlp_dw_f32_kernel<64, 64>);
    if (hipGetLastError() != hipSuccess) return 3;
    return gs4d_sum_slices(parts, S, (int64_t)KW * W, dw, stream);
}

int gs4d_feature_relu_forward_hb(int P, int Fin, int Fout, const float *x, const float *w, const float *b, float *h,
                                 uint16_t *hb, void *stream) {
    if (P < 0 || !w || !b) return 1;
    if (!((Fin == 32 && Fout == 128) || (Fin == 64 && Fout == 64) || (Fin == 32 && Fout == 64))) return 1;
    if (P == 0) return 0;
    if (!x || !h || (((size_t)x | (size_t)w) & 15) != 0) return 1;
    hipStream_t s = (hipStream_t)stream;
    const int nwg = std::max(1, std::min(1024, ((P + 15) / 16 + 3) / 4));
    __bf16 *hbb = reinterpret_cast<__bf16 *>(hb);
    if (Fin == 32 && Fout == 128)
        hipLaunchKernelGGL((feature_fwd_kernel<32, 128>), dim3(nwg), dim3(kFbThreads), 0, s, P, x, w, b, h, hbb);
    else if (Fin == 64)
        hipLaunchKernelGGL((feature_fwd_kernel<64, 64>), dim3(nwg), dim3(kFbThreads), 0, s, P, x, w, b, h, hbb);
    else
        hipLaunchKernelGGL((feature_fwd_kernel<32, 64>), dim3(nwg), dim3(kFbThreads), 0, s, P, x, w, b, h, hbb);
    return hipGetLastError() == hipSuccess ? 0 : 3;
}
int gs4d_feature_relu_forward(int P, int Fin, int Fout, const float *x, const float *w, const float *b, float *h,
                              void *stream) {
    return gs4d_feature_relu_forward_hb(P, Fin, Fout, x, w, b, h, nullptr, stream);
}

int gs4d_hexplane_points(int N, const float *xyz, int64_t ld_xyz, const float *t, int64_t ld_t, const float *aabb,
                         float *pts, void *stream) {
    if (N < 0 || !aabb) return 1;
    if (N == 0) return 0;
    if (!xyz || !t || !pts || ((size_t)pts & 15) != 0 || ld_xyz < 3 || ld_t < 0) return 1;
    hipLaunchKernelGGL(hex_points_kernel, dim3((N + 255) / 256), dim3(256), 0, (hipStream_t)stream, N, xyz, ld_xyz, t,
                       ld_t, aabb, (float4 *)pts);
    return hipGetLastError() == hipSuccess ? 0 : 3;
}

int gs4d_hexplane_points_backward_add(int N, const float *dpts, const float *aabb, const float *add, float *dxyz,
                                      void *stream) {
    if (N < 0 || !aabb) return 1;
    if (N == 0) return 0;
    if (!dpts || !dxyz || ((size_t)dpts & 15) != 0) return 1;
    hipLaunchKernelGGL(hex_points_bwd_kernel, dim3((N + 255) / 256), dim3(256), 0, (hipStream_t)stream, N,
                       (const float4 *)dpts, aabb, add, dxyz);
    return hipGetLastError() == hipSuccess ? 0 : 3;
}

int gs4d_hexplane_points_backward(int N, const float *dpts, const float *aabb, float *dxyz, void *stream) {
    return gs4d_hexplane_points_backward_add(N, dpts, aabb, nullptr, dxyz, stream);
}

}  // extern "C"
