// Dev tool: print the operand/result lane layout of v_mfma_f32_4x4x1_16b_f32.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f4 __attribute__((ext_vector_type(4)));
__global__ void k(float *out, int mode) {
    const int l = threadIdx.x;
    // mode 0: A = lane id + 1, B = 1 -> D[i][j] = A of (block, i)
    // mode 1: A = 1, B = lane id + 1 -> D[i][j] = B of (block, j)
    float a = mode == 0 ? (float)(l + 1) : 1.f;
    float b = mode == 1 ? (float)(l + 1) : 1.f;
    f4 c = {0, 0, 0, 0};
    c = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c, 0, 0, 0);
    for (int r = 0; r < 4; ++r) out[l * 4 + r] = c[r];
}
int main() {
    float *d, h[256];
    hipMalloc(&d, 256 * 4);
    for (int mode = 0; mode < 2; ++mode) {
        hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, mode);
        hipMemcpy(h, d, 256 * 4, hipMemcpyDeviceToHost);
        printf("mode %d (value-1 = source lane):\n", mode);
        for (int l = 0; l < 64; ++l) {
            printf("l%2d:", l);
            for (int r = 0; r < 4; ++r) printf(" %3d", (int)h[l * 4 + r] - 1);
            printf(l % 4 == 3 ? "\n" : " |");
        }
    }
    return 0;
}
