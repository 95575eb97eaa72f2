// census.hip -- how many one-wave workgroups (and multi-wave ones) a CU holds at once.
// Every wave spins ~T us on s_memrealtime (100 MHz) and records the XCC/CU it ran on and
// its start/end; the kernel time for N waves gives the resident waves per CU.
// usage: ./census [threads_per_wg] [lds_bytes_per_wg] [spin_us] [workgroups (launch-rate mode)]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>

__global__ void k_spin(uint64_t ticks, uint32_t *out, int lds_bytes) {
    extern __shared__ uint32_t dyn[];
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(2);
    if (lds_bytes) dyn[threadIdx.x % (lds_bytes / 4)] = (uint32_t)t0;
    if ((threadIdx.x & 63) == 0) {
        uint32_t hw;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
        uint32_t xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        const uint32_t w = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
        out[2 * w] = hw;
        out[2 * w + 1] = xcc;
    }
}

int main(int argc, char **argv) {
    const int tpb = argc > 1 ? atoi(argv[1]) : 64;
    const int lds = argc > 2 ? atoi(argv[2]) : 0;
    const int spin_us = argc > 3 ? atoi(argv[3]) : 200;
    const uint64_t ticks = 100ull * spin_us;  // s_memrealtime runs at 100 MHz
    const int fixed_wgs = argc > 4 ? atoi(argv[4]) : 0;  // launch-rate mode: this many workgroups
    for (int waves_per_cu : {8, 16, 24, 32, 40, 48, 64}) {
        if (fixed_wgs && waves_per_cu != 8) break;
        const int nblk = fixed_wgs ? fixed_wgs : 256 * waves_per_cu / (tpb / 64), nw = nblk * (tpb / 64);
        uint32_t *d;
        hipMalloc(&d, nw * 8);
        hipEvent_t a, b;
        hipEventCreate(&a);
        hipEventCreate(&b);
        hipLaunchKernelGGL(k_spin, dim3(nblk), dim3(tpb), lds, 0, ticks, d, lds);  // warm
        hipEventRecord(a);
        hipLaunchKernelGGL(k_spin, dim3(nblk), dim3(tpb), lds, 0, ticks, d, lds);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms = 0;
        hipEventElapsedTime(&ms, a, b);
        printf("tpb %4d lds %6d spin %4d us: %7d workgroups -> %.3f ms (%.2f spin rounds, %.1f ns per workgroup)\n",
               tpb, lds, spin_us, nblk, ms, ms * 1000.0 / spin_us, ms * 1e6 / nblk);
        hipFree(d);
    }
    return 0;
}
