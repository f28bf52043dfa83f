// Microbenchmark: global no-return atomic add throughput on gfx950, f32 (-munsafe-fp-atomics: the hardware
// float add) against u64 (the fixed-point sums of a deterministic reduction), over a region of R words (the
// contention of the HexPlane backward's plane gradients: a few 10^5 addresses, each hit by several workgroups).
// hipcc --offload-arch=gfx950 -O3 -munsafe-fp-atomics tools/bench/global_atomics.hip -o /tmp/ga && /tmp/ga
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr int kIters = 16;

template <int MODE>  // 0 f32, 1 u64, 2 u32
__global__ __launch_bounds__(256) void k(void *buf, int R, int salt) {
    uint32_t a = (blockIdx.x * 256 + threadIdx.x) * 2654435761u + salt;
    for (int i = 0; i < kIters; i++) {
        const uint32_t idx = (a >> 7) % R;
        if (MODE == 0) unsafeAtomicAdd((float *)buf + idx, 1.5f);
        if (MODE == 1) atomicAdd((unsigned long long *)buf + idx, 3ull);
        if (MODE == 2) atomicAdd((uint32_t *)buf + idx, 3u);
        a = a * 1664525u + 1013904223u;
    }
}

template <int MODE>
static float run(void *buf, int R) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    hipLaunchKernelGGL(k<MODE>, dim3(4096), dim3(256), 0, 0, buf, R, 1);
    (void)hipEventRecord(e0, 0);
    for (int r = 0; r < 5; r++) hipLaunchKernelGGL(k<MODE>, dim3(4096), dim3(256), 0, 0, buf, R, r);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms; (void)hipEventElapsedTime(&ms, e0, e1);
    return ms / 5;
}

int main() {
    void *buf;
    (void)hipMalloc(&buf, (size_t)8 << 22);
    (void)hipMemset(buf, 0, (size_t)8 << 22);
    const double ops = 4096.0 * 256 * kIters;
    for (int R : {4096, 65536, 1 << 20}) {
        float t0 = run<0>(buf, R), t1 = run<1>(buf, R), t2 = run<2>(buf, R);
        printf("R=%8d  f32 %7.3f ms (%6.1f G atomics/s)  u64 %7.3f ms (%6.1f)  u32 %7.3f ms (%6.1f)\n", R, t0,
               ops / t0 * 1e-6, t1, ops / t1 * 1e-6, t2, ops / t2 * 1e-6);
    }
    return 0;
}
