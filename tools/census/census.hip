// Dev tool: how many 256-thread workgroups are co-resident per CU for a given static
// LDS footprint.  Each block records (CU id, start, end) with s_memtime; the host
// prints the max overlap per CU.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>

template <int LDSF>
__global__ __launch_bounds__(256) void k_census(unsigned long long *rec, int spin) {
    __shared__ float buf[LDSF];
    unsigned long long t0 = __builtin_readcyclecounter();
    buf[threadIdx.x % LDSF] = (float)threadIdx.x;
    __syncthreads();
    float acc = buf[(threadIdx.x * 7) % LDSF];
    for (int i = 0; i < spin; ++i) { __builtin_amdgcn_s_sleep(10); acc += 1.f; }
    buf[(threadIdx.x * 3) % LDSF] = acc;
    __syncthreads();
    unsigned long long t1 = __builtin_readcyclecounter();
    if (threadIdx.x == 0) {
        unsigned hw;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
        unsigned xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        rec[blockIdx.x * 4 + 0] = hw;
        rec[blockIdx.x * 4 + 1] = xcc;
        rec[blockIdx.x * 4 + 2] = t0;
        rec[blockIdx.x * 4 + 3] = t1 + (unsigned long long)(buf[0] * 0);
    }
}

template <int LDSF>
void run(int nb, int spin) {
    unsigned long long *d;
    hipMalloc(&d, nb * 4 * 8);
    hipLaunchKernelGGL(k_census<LDSF>, dim3(nb), dim3(256), 0, 0, d, spin);
    hipDeviceSynchronize();
    std::vector<unsigned long long> h(nb * 4);
    hipMemcpy(h.data(), d, nb * 32, hipMemcpyDeviceToHost);
    // CU key: xcc, se_id, cu_id from HW_ID (gfx9: cu_id bits 8-11, sh_id 12, se_id 13-15)
    struct E { unsigned long long key, t; int d; };
    std::vector<E> ev;
    for (int b = 0; b < nb; ++b) {
        unsigned hw = (unsigned)h[b * 4], xcc = (unsigned)h[b * 4 + 1];
        unsigned long long key = ((unsigned long long)xcc << 32) | (hw & 0xFF00u) | ((hw >> 13) & 7u) << 16 | ((hw >> 12) & 1u) << 20;
        ev.push_back({key, h[b * 4 + 2], +1});
        ev.push_back({key, h[b * 4 + 3], -1});
    }
    std::sort(ev.begin(), ev.end(), [](const E &a, const E &b) { return a.key != b.key ? a.key < b.key : (a.t != b.t ? a.t < b.t : a.d < b.d); });
    int maxc = 0, cus = 0; unsigned long long cur = ~0ull; int c = 0; long sum = 0;
    for (auto &e : ev) {
        if (e.key != cur) { if (cur != ~0ull) sum += maxc; cur = e.key; c = 0; cus++; maxc = 0; }
        c += e.d; maxc = std::max(maxc, c);
    }
    sum += maxc;
    printf("LDS %6d B  blocks %d  distinct CUs %d  mean max-resident/CU %.2f\n", LDSF * 4, nb, cus, (double)sum / cus);
    hipFree(d);
}

int main() {
    run<1024>(4096, 2000);
    run<4608>(4096, 2000);
    run<6912>(4096, 2000);
    run<9216>(4096, 2000);
    run<12288>(4096, 2000);
    return 0;
}
