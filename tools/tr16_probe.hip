// Dev probe: what ds_read_b64_tr_b16 (through the clang builtin) returns per lane
// for an LDS image whose element (r, c) holds r * 100 + c, with lane 4q + p of each
// 16-lane group addressing row q (+ 4 for the upper 32 lanes), columns 4p..4p+3
// (+ 16 for lane groups 1 and 3).  Build: hipcc --offload-arch=gfx950 -O2 -o
// tools/tr16_probe tools/tr16_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>

typedef short v4s16 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4s16 lds_v4s16;

__global__ void k(short *out) {
    __shared__ __attribute__((aligned(16))) short img[8 * 40];
    for (int i = threadIdx.x; i < 8 * 40; i += 64) img[i] = (short)((i / 40) * 100 + i % 40);
    __syncthreads();
    const int lane = threadIdx.x, i = lane & 15, q = i >> 2, p = i & 3;
    const int row = q + 4 * (lane >> 5), col = 16 * ((lane >> 4) & 1) + 4 * p;
    v4s16 r = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s16 *)&img[row * 40 + col]);
    for (int e = 0; e < 4; ++e) out[lane * 4 + e] = r[e];
}

int main() {
    short *d, h[256];
    hipMalloc(&d, 512);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
    hipMemcpy(h, d, 512, hipMemcpyDeviceToHost);
    for (int l = 0; l < 64; ++l) {
        printf("lane %2d:", l);
        for (int e = 0; e < 4; ++e) printf(" %4d", h[l * 4 + e]);
        printf("%s", (l % 4 == 3) ? "\n" : "   ");
    }
    hipFree(d);
    return 0;
}
