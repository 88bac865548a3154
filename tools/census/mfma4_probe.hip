// Dev tool: lane layout and issue rate of v_mfma_f32_4x4x1_16b_f32 on gfx950.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f4 __attribute__((ext_vector_type(4)));
__global__ void k(float *out, int mode) {
    const int l = threadIdx.x;
    float a = mode == 0 ? (float)(l + 1) : 1.f;
    float b = mode == 1 ? (float)(l + 1) : 1.f;
    f4 c = {0, 0, 0, 0};
    c = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c, 0, 0, 0);
    for (int r = 0; r < 4; ++r) out[l * 4 + r] = c[r];
}
// N back-to-back MFMAs on NACC independent accumulators; cycles per MFMA (s_memtime)
template <int NACC>
__global__ void rate(float *out, long long *cyc, int n) {
    const int l = threadIdx.x;
    float a = 1.f + l * 1e-3f, b = 1.f - l * 1e-3f;
    f4 c[NACC];
    for (int q = 0; q < NACC; ++q) c[q] = f4{0, 0, 0, 0};
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < n; ++i)
#pragma unroll
        for (int q = 0; q < NACC; ++q) c[q] = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c[q], 0, 0, 0);
    long long t1 = __builtin_amdgcn_s_memtime();
    float s = 0;
    for (int q = 0; q < NACC; ++q) s += c[q][0] + c[q][1] + c[q][2] + c[q][3];
    out[blockIdx.x * 64 + l] = s;
    if (l == 0) cyc[blockIdx.x] = t1 - t0;
}
int main() {
    float *d, h[256];
    hipMalloc(&d, 1 << 20);
    long long *cy, hc[1024];
    hipMalloc(&cy, 1024 * 8);
    for (int mode = 0; mode < 2; ++mode) {
        hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, mode);
        hipMemcpy(h, d, 256 * 4, hipMemcpyDeviceToHost);
        printf("mode %d (%s = value-1 = source lane):\n", mode, mode == 0 ? "A" : "B");
        for (int l = 0; l < 64; ++l) {
            printf("l%2d:", l);
            for (int r = 0; r < 4; ++r) printf(" %3d", (int)h[l * 4 + r] - 1);
            printf(l % 4 == 3 ? "\n" : " |");
        }
    }
    const int n = 4096;
    hipLaunchKernelGGL(rate<1>, dim3(1), dim3(64), 0, 0, d, cy, n);
    hipMemcpy(hc, cy, 8, hipMemcpyDeviceToHost);
    printf("1 acc, 1 wave: %.2f cycles per MFMA\n", (double)hc[0] / n);
    hipLaunchKernelGGL(rate<4>, dim3(1), dim3(64), 0, 0, d, cy, n);
    hipMemcpy(hc, cy, 8, hipMemcpyDeviceToHost);
    printf("4 acc, 1 wave: %.2f cycles per MFMA\n", (double)hc[0] / (4.0 * n));
    hipLaunchKernelGGL(rate<8>, dim3(1), dim3(64), 0, 0, d, cy, n);
    hipMemcpy(hc, cy, 8, hipMemcpyDeviceToHost);
    printf("8 acc, 1 wave: %.2f cycles per MFMA\n", (double)hc[0] / (8.0 * n));
    return 0;
}
