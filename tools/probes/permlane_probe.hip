// Probe: semantics of v_permlane32_swap / v_permlane16_swap and DPP row ops on gfx950.
#include <hip/hip_runtime.h>
#include <stdio.h>
__global__ void k(int *out) {
    int l = threadIdx.x;
    int a = 1000 + l, b = 2000 + l;
    auto r32 = __builtin_amdgcn_permlane32_swap(a, b, false, false);
    auto r16 = __builtin_amdgcn_permlane16_swap(a, b, false, false);
    out[l] = r32[0]; out[64 + l] = r32[1]; out[128 + l] = r16[0]; out[192 + l] = r16[1];
}
int main() {
    int *d; hipMalloc(&d, 256 * 4);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
    int h[256]; hipMemcpy(h, d, 1024, hipMemcpyDeviceToHost);
    const char *nm[4] = {"p32 vdst", "p32 src ", "p16 vdst", "p16 src "};
    for (int q = 0; q < 4; q++) { printf("%s:", nm[q]); for (int l = 0; l < 64; l += 8) printf(" [%d]=%d", l, h[q * 64 + l]); printf("\n"); }
    return 0;
}
