// Microbenchmark: LDS atomic add throughput on gfx950 by type (u32, u64, f32) against plain LDS
// read-modify-write, for the HexPlane backward's accumulation design.  hipcc --offload-arch=gfx950 -O3
// tools/bench/lds_atomics.hip -o /tmp/lds_atomics && /tmp/lds_atomics
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr int kWin = 4096, kIters = 256;

template <int MODE>  // 0 u32 atomic, 1 u64 atomic, 2 f32 atomic, 3 plain f32 rmw (racy, timing only), 4 u64 with 4-way conflicts
__global__ __launch_bounds__(256) void k(uint64_t *out, int salt) {
    __shared__ uint64_t win[kWin];
    for (int i = threadIdx.x; i < kWin; i += 256) win[i] = 0;
    __syncthreads();
    uint32_t *w32 = reinterpret_cast<uint32_t *>(win);
    float *wf = reinterpret_cast<float *>(win);
    uint32_t a = threadIdx.x * 17u + blockIdx.x + salt;
    for (int i = 0; i < kIters; i++) {
        const uint32_t idx = (MODE == 4 ? (a >> 2) : a) & (kWin - 1);
        if (MODE == 0) atomicAdd(&w32[idx], 3u);
        if (MODE == 1 || MODE == 4) atomicAdd((unsigned long long *)&win[idx], 3ull);
        if (MODE == 2) atomicAdd(&wf[idx], 1.5f);
        if (MODE == 3) wf[idx] += 1.5f;
        a += 97u;
    }
    __syncthreads();
    uint64_t s = 0;
    for (int i = threadIdx.x; i < kWin; i += 256) s += win[i];
    if (s == 12345) out[blockIdx.x] = s;
}

template <int MODE>
static float run(uint64_t *out) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    hipLaunchKernelGGL(k<MODE>, dim3(2048), dim3(256), 0, 0, out, 1);
    (void)hipEventRecord(e0, 0);
    for (int r = 0; r < 5; r++) hipLaunchKernelGGL(k<MODE>, dim3(2048), dim3(256), 0, 0, out, r);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms; (void)hipEventElapsedTime(&ms, e0, e1);
    return ms / 5;
}

int main() {
    uint64_t *out;
    (void)hipMalloc(&out, 2048 * 8);
    const double ops = 2048.0 * 256 * kIters;
    const char *names[] = {"ds_add_u32", "ds_add_u64", "ds_add_f32", "plain f32 rmw", "ds_add_u64 4-way conflict"};
    float t[5] = {run<0>(out), run<1>(out), run<2>(out), run<3>(out), run<4>(out)};
    for (int m = 0; m < 5; m++)
        printf("%-28s %8.3f ms  %6.2f lane-ops per clock per CU (2.4 GHz, 256 CUs)\n", names[m], t[m],
               ops / (t[m] * 1e-3) / 2.4e9 / 256);
    return 0;
}
