// Dev tool: issue rate of the f32 MFMAs the head projection can use, one wave per
// SIMD, cycles per MFMA by s_memtime: v_mfma_f32_4x4x1_16b_f32 and
// v_mfma_f32_16x16x4_f32 on 8 independent accumulators, bare and with the dW kernel's
// two VALU per MFMA (v_bfe_i32 + v_and on the A value).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f4 __attribute__((ext_vector_type(4)));
template <int KIND, int VALU>
__global__ void rate(float *out, long long *cyc, int n, unsigned mword) {
    const int l = threadIdx.x;
    float a = 1.f + l * 1e-3f, b = 1.f - l * 1e-3f;
    f4 c[8];
    for (int q = 0; q < 8; ++q) c[q] = f4{0, 0, 0, 0};
    unsigned w = mword ^ l;
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < n; ++i) {
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            float aa = a;
            if (VALU) {
                const int keep = __builtin_amdgcn_sbfe((int)w, q * 3 + (i & 3), 1);
                aa = __uint_as_float(__float_as_uint(a + q) & (unsigned)keep);
            }
            if (KIND == 0) c[q] = __builtin_amdgcn_mfma_f32_4x4x1f32(aa, b, c[q], 0, 0, 0);
            else c[q] = __builtin_amdgcn_mfma_f32_16x16x4f32(aa, b, c[q], 0, 0, 0);
        }
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    float s = 0;
    for (int q = 0; q < 8; ++q) s += c[q][0] + c[q][1] + c[q][2] + c[q][3];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}
template <int KIND, int VALU>
void run(const char *name, float *d, long long *cy, int waves) {
    const int n = 2048;
    long long hc[1024];
    // one block per CU (many CUs), `waves` waves per block = waves per SIMD / 4 ... use
    // 4 * waves threads-of-64 so each SIMD holds `waves` waves
    hipLaunchKernelGGL((rate<KIND, VALU>), dim3(256), dim3(64 * 4 * waves), 0, 0, d, cy, n, 0x5a5a5a5au);
    hipDeviceSynchronize();
    hipMemcpy(hc, cy, 8 * 256, hipMemcpyDeviceToHost);
    double m = 0;
    for (int i = 0; i < 256; ++i) m += hc[i];
    m /= 256;
    printf("%-34s %d wave(s)/SIMD: %.2f cycles per MFMA per wave\n", name, waves, m / (8.0 * n));
}
int main() {
    float *d;
    long long *cy;
    hipMalloc(&d, 1 << 24);
    hipMalloc(&cy, 8 * 1024);
    for (int w = 1; w <= 4; w *= 2) {
        run<0, 0>("4x4x1_16b bare", d, cy, w);
        run<0, 1>("4x4x1_16b + bfe/and", d, cy, w);
        run<1, 0>("16x16x4 bare", d, cy, w);
        run<1, 1>("16x16x4 + bfe/and", d, cy, w);
    }
    return 0;
}
