// Micro-benchmark of the radix-sort pass (binning.hip) in isolation: per-pass time for the depth sort
// (100k keys) and the tile sort (940k keys) shapes.  Build: hipcc -O3 --offload-arch=gfx950 -I include
// tools/bench/sortbench.hip -o /tmp/sortbench
#include "../../4dgaussians-fast-train_amd/csrc/binning.hip"

#include <stdio.h>
#include <stdlib.h>

#include <vector>

using namespace gs4d;

#define CK(x)                                                                         \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                  \
        }                                                                             \
    } while (0)

template <int THREADS, int ITEMS, int MODE = 0>
static void run(const char *name, int n, int bits, bool sorted_hi) {
    std::vector<uint32_t> h(n), hist(kHistWords, 0);
    uint32_t seed = 1234567;
    for (int i = 0; i < n; i++) {
        seed = seed * 1664525u + 1013904223u;
        h[i] = sorted_hi ? (seed >> 8) & ((1u << bits) - 1) : seed & (bits == 32 ? 0xFFFFFFFFu : ((1u << bits) - 1));
        for (int p = 0; p < (bits + 7) / 8; p++) hist[(i % 8) * kMaxPasses * 256 + p * 256 + ((h[i] >> (8 * p)) & 255)]++;
    }
    uint32_t *k0, *k1, *v0, *v1, *zero;
    const int nblk = sort_nblk(n, THREADS * ITEMS);
    const size_t zw = kZeroHist + kHistWords + 64 + (size_t)kMaxPasses * 256 * nblk + 64;
    CK(hipMalloc(&k0, 4 * n)); CK(hipMalloc(&k1, 4 * n)); CK(hipMalloc(&v0, 4 * n)); CK(hipMalloc(&v1, 4 * n));
    CK(hipMalloc(&zero, 4 * zw));
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    const int npass = (bits + 7) / 8;
    float best = 1e9;
    for (int it = 0; it < 20; it++) {
        CK(hipMemcpy(k0, h.data(), 4 * n, hipMemcpyHostToDevice));
        CK(hipMemset(zero, 0, 4 * zw));
        CK(hipMemcpy(zero + kZeroHist, hist.data(), 4 * kHistWords, hipMemcpyHostToDevice));
        CK(hipDeviceSynchronize());
        uint32_t *keys[2] = {k0, k1}, *vals[2] = {v0, v1};
        CK(hipEventRecord(a, 0));
        onesweep_sort<THREADS, ITEMS, MODE>(keys, vals, n, nullptr, bits, zero + kZeroHist,
                                                     zero + kZeroHist + kHistWords + 64, zero + kZeroHist + kHistWords,
                                                     0);
        CK(hipEventRecord(b, 0));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        if (it > 2 && ms < best) best = ms;
    }
    // check sortedness
    std::vector<uint32_t> out(n);
    CK(hipMemcpy(out.data(), (npass & 1) ? k1 : k0, 4 * n, hipMemcpyDeviceToHost));
    bool ok = true;
    for (int i = 1; i < n; i++) ok &= out[i - 1] <= out[i];
    uint32_t err;
    CK(hipMemcpy(&err, zero + kZeroHist + kHistWords + 1, 4, hipMemcpyDeviceToHost));
    printf("mode=%d %-22s n=%7d bits=%2d threads=%4d items=%2d nblk=%4d  %7.1f us total  %6.1f us/pass  sorted=%d err=%u\n",
           MODE, name, n, bits, THREADS, ITEMS, nblk, best * 1e3, best * 1e3 / npass, ok, err);
    hipFree(k0); hipFree(k1); hipFree(v0); hipFree(v1); hipFree(zero);
}

__global__ void copy_kernel(const uint32_t *__restrict__ a, const uint32_t *__restrict__ b, uint32_t *__restrict__ c,
                            uint32_t *__restrict__ d, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
        c[i] = a[i];
        d[i] = b[i];
    }
}
static void run_copy(int n) {
    uint32_t *k0, *k1, *v0, *v1;
    CK(hipMalloc(&k0, 4 * n)); CK(hipMalloc(&k1, 4 * n)); CK(hipMalloc(&v0, 4 * n)); CK(hipMalloc(&v1, 4 * n));
    CK(hipMemset(k0, 0, 4 * n)); CK(hipMemset(v0, 0, 4 * n));
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    float best = 1e9;
    for (int it = 0; it < 20; it++) {
        CK(hipEventRecord(a, 0));
        hipLaunchKernelGGL(copy_kernel, dim3((n + 255) / 256), dim3(256), 0, 0, k0, v0, k1, v1, n);
        CK(hipEventRecord(b, 0));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        if (it > 2 && ms < best) best = ms;
    }
    // 10 back-to-back launches
    CK(hipEventRecord(a, 0));
    for (int it = 0; it < 10; it++)
        hipLaunchKernelGGL(copy_kernel, dim3((n + 255) / 256), dim3(256), 0, 0, k0, v0, k1, v1, n);
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms10;
    CK(hipEventElapsedTime(&ms10, a, b));
    printf("copy n=%d: single %.1f us, back-to-back %.1f us/launch\n", n, best * 1e3, ms10 * 1e2);
    hipFree(k0); hipFree(k1); hipFree(v0); hipFree(v1);
}

int main() {
    run_copy(100000);
    run_copy(940000);
    run<256, 4>("depth 256x4", 100000, 32, false);
    run<1024, 4>("depth 1024x4", 100000, 32, false);
    run<1024, 4, 1>("depth 1024x4", 100000, 32, false);
    run<1024, 2>("depth 1024x2", 100000, 32, false);
    run<256, 8>("tile 256x8", 940000, 13, false);
    run<1024, 8>("tile 1024x8", 940000, 13, false);
    run<1024, 8, 1>("tile 1024x8", 940000, 13, false);
    run<1024, 4>("tile 1024x4", 940000, 13, false);
    run<1024, 16>("tile 1024x16", 940000, 13, false);
    return 0;
}
