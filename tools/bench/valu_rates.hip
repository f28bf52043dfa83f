// valu_rates.hip -- issue throughput of the instructions the blend kernels are made of (diagnostic).
//
// Each kernel runs a loop of 8 independent chains of ONE instruction kind (inline asm, so the compiler
// keeps exactly that instruction), on every SIMD of the chip at a chosen number of waves per SIMD.
// Prints ns per wave-instruction per SIMD and cycles at the measured in-kernel clock (s_memtime ticks
// / s_memrealtime 100 MHz ticks).  Answers: is v_pk_fma_f32 worth two v_fma_f32, what do v_exp_f32,
// v_rcp_f32, v_cndmask, v_cmp, v_permlane*_swap and DPP adds cost relative to them.
//
//   hipcc -O3 --offload-arch=gfx950 tools/bench/valu_rates.hip -o tools/bench/valu_rates && ./tools/bench/valu_rates
#include <hip/hip_runtime.h>
#include <stdio.h>

#define ITERS 4096
#define CHECK(x)                                                                  \
    do {                                                                          \
        hipError_t e_ = (x);                                                      \
        if (e_ != hipSuccess) {                                                   \
            printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__);      \
            return 1;                                                             \
        }                                                                         \
    } while (0)

typedef float f2 __attribute__((ext_vector_type(2)));

template <int KIND>
__global__ __launch_bounds__(256) void rate_kernel(float *out, unsigned long long *clk, float seed) {
    float a[8];
    f2 p[8];
#pragma unroll
    for (int i = 0; i < 8; i++) {
        a[i] = seed + threadIdx.x * 1e-3f + i;
        p[i] = f2{a[i], a[i] + 0.5f};
    }
    const float m = 0.999f, c = 1e-3f;
    const f2 m2 = f2{m, m}, c2 = f2{c, c};
    unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < ITERS; it++) {
#pragma unroll
        for (int i = 0; i < 8; i++) {
            if constexpr (KIND == 0) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(m), "v"(c));
            if constexpr (KIND == 1) asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(p[i]) : "v"(m2), "v"(c2));
            if constexpr (KIND == 2) asm volatile("v_exp_f32 %0, %0" : "+v"(a[i]));
            if constexpr (KIND == 3) asm volatile("v_rcp_f32 %0, %0" : "+v"(a[i]));
            if constexpr (KIND == 4) asm volatile("v_add_f32 %0, %0, %1" : "+v"(a[i]) : "v"(c));
            if constexpr (KIND == 5) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(p[i]) : "v"(c2));
            if constexpr (KIND == 6) asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(p[i]) : "v"(m2));
            if constexpr (KIND == 7)
                asm volatile("v_cmp_le_f32 vcc, %1, %0\n\tv_cndmask_b32 %0, 0, %0, vcc" : "+v"(a[i]) : "v"(c) : "vcc");
            if constexpr (KIND == 8) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a[i]) : "v"(c) : "vcc");
            if constexpr (KIND == 9) {
                float b = a[(i + 1) & 7];
                asm volatile("v_permlane32_swap_b32 %0, %1" : "+v"(a[i]), "+v"(b));
                a[(i + 1) & 7] = b;
            }
            if constexpr (KIND == 10)
                asm volatile("v_add_f32_dpp %0, %0, %0 row_ror:8 row_mask:0xf bank_mask:0xf" : "+v"(a[i]));
            if constexpr (KIND == 11) asm volatile("v_mul_f32 %0, %0, %1" : "+v"(a[i]) : "v"(m));
            if constexpr (KIND == 12) {  // mixed: 2 fma + 1 exp (the blend's ratio)
                asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(m), "v"(c));
            }
        }
        if constexpr (KIND == 12) {
            asm volatile("v_exp_f32 %0, %0" : "+v"(a[0]));
            asm volatile("v_exp_f32 %0, %0" : "+v"(a[4]));
        }
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 8; i++) s += a[i] + p[i].x + p[i].y;
    if (s == 12345.f) out[threadIdx.x] = s;
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        clk[0] = t1 - t0;
        clk[1] = r1 - r0;
    }
}

template <int KIND>
int run(const char *name, int waves_per_simd, float *out, unsigned long long *clk, int cus, double per_iter) {
    // 256-thread workgroups = 4 waves, one per SIMD; blocks = CUs * waves_per_simd
    const int blocks = cus * waves_per_simd;
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    hipLaunchKernelGGL(rate_kernel<KIND>, dim3(blocks), dim3(256), 0, 0, out, clk, 1.0f);
    CHECK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int r = 0; r < 5; r++) {
        CHECK(hipEventRecord(e0));
        hipLaunchKernelGGL(rate_kernel<KIND>, dim3(blocks), dim3(256), 0, 0, out, clk, 1.0f);
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        float ms;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        best = ms < best ? ms : best;
    }
    unsigned long long h[2];
    CHECK(hipMemcpy(h, clk, 16, hipMemcpyDeviceToHost));
    const double ghz = (double)h[0] / ((double)h[1] * 10.0);  // memrealtime is 100 MHz
    // wave-instructions issued per SIMD: waves_per_simd * ITERS * per_iter
    const double inst = (double)waves_per_simd * ITERS * per_iter;
    const double ns = best * 1e6 / inst;
    printf("%-28s waves/SIMD %2d  %.3f ns/inst/SIMD  %.2f cyc @ %.2f GHz (in-kernel clock)\n", name, waves_per_simd,
           ns, ns * ghz, ghz);
    return 0;
}

int main() {
    hipDeviceProp_t prop;
    CHECK(hipGetDeviceProperties(&prop, 0));
    const int cus = prop.multiProcessorCount;
    printf("device %s, %d CUs\n", prop.gcnArchName, cus);
    float *out;
    unsigned long long *clk;
    CHECK(hipMalloc(&out, 4096));
    CHECK(hipMalloc(&clk, 16));
    for (int w : {1, 4, 8}) {
        run<0>("v_fma_f32", w, out, clk, cus, 8);
        run<11>("v_mul_f32", w, out, clk, cus, 8);
        run<4>("v_add_f32", w, out, clk, cus, 8);
        run<1>("v_pk_fma_f32", w, out, clk, cus, 8);
        run<5>("v_pk_add_f32", w, out, clk, cus, 8);
        run<6>("v_pk_mul_f32", w, out, clk, cus, 8);
        run<2>("v_exp_f32", w, out, clk, cus, 8);
        run<3>("v_rcp_f32", w, out, clk, cus, 8);
        run<7>("v_cmp+v_cndmask (pair)", w, out, clk, cus, 8);
        run<8>("v_cndmask_b32", w, out, clk, cus, 8);
        run<9>("v_permlane32_swap", w, out, clk, cus, 8);
        run<10>("v_add_f32_dpp row_ror", w, out, clk, cus, 8);
        run<12>("8 fma + 2 exp (per 10)", w, out, clk, cus, 10);
    }
    return 0;
}
