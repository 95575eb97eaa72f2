// Microbenchmark: LDS-DMA (global_load_lds) completion latency seen by
// "s_waitcnt vmcnt(N)" with two iterations of slack, under VALU-only or
// LDS-heavy work between issue and wait.  Mirrors the K2 prefetch pattern.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>

__device__ __forceinline__ void dma4(const void *g, uint32_t lds_base) {
    uint32_t tmp;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\tglobal_load_lds_dword %2, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(tmp) : "s"(__builtin_amdgcn_readfirstlane(lds_base)), "v"(g) : "memory");
}
__device__ __forceinline__ void dma16(const void *g, uint32_t lds_base) {
    uint32_t tmp;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\tglobal_load_lds_dwordx4 %2, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(tmp) : "s"(__builtin_amdgcn_readfirstlane(lds_base)), "v"(g) : "memory");
}

template <int MODE>
__global__ void __launch_bounds__(64) k(const uint8_t *buf, size_t bufsize, const uint8_t *rec, unsigned long long *out,
                                        int work, int iters, int stride_mode) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[4500];
    const uint32_t lane = threadIdx.x, blk = blockIdx.x;
    unsigned long long wait = 0;
    uint32_t acc = lane;
    for (int i = 0; i < 4500; i += 64) if (i + lane < 4500) lds[i + lane] = 0;
    __syncthreads();
    for (int it = 0; it < iters; it++) {
        size_t a;
        if (stride_mode == 0) a = ((size_t)blk * 8192 + (size_t)it * 260 + lane * 4) % (bufsize - 16);
        else a = ((size_t)(blk % 16384) * 8192 + (size_t)it * 260 + lane * 4 + (lane * 7) % 4) % (bufsize - 16);
        dma4(buf + a, (uint32_t)(uintptr_t)&lds[(it & 3) * 64]);
        if (lane < 4) dma16(rec + (size_t)blk * 8704 + (size_t)it * 32 + lane * 16, (uint32_t)(uintptr_t)&lds[256 + (it % 7) * 16]);
        if (MODE == 0) {
            for (int w = 0; w < work; w++) acc = acc * 1664525u + 1013904223u;
        } else if (MODE == 2) {  // K2-like sub-rounds: 6 reads + 5 mskor, one wait each
            for (int w = 0; w < work / 8; w++) {
                const uint32_t base = 512 + ((acc >> 5) + lane * 61) % 3800;
                const uint32_t x0 = lds[base], x1 = lds[base + 1], x2 = lds[base + 2], x3 = lds[base + 3],
                               x4 = lds[base + 4], x5 = lds[base + 5];
                const uint32_t db = 512 + ((acc >> 7) + lane * 37) % 3800;
                asm volatile("ds_mskor_b32 %0, %1, %2" ::"v"((uint32_t)(uintptr_t)&lds[db]), "v"(0xffu), "v"(x0 ^ x1) : "memory");
                asm volatile("ds_mskor_b32 %0, %1, %2" ::"v"((uint32_t)(uintptr_t)&lds[db + 1]), "v"(0xffu), "v"(x1 ^ x2) : "memory");
                asm volatile("ds_mskor_b32 %0, %1, %2" ::"v"((uint32_t)(uintptr_t)&lds[db + 2]), "v"(0xffu), "v"(x2 ^ x3) : "memory");
                asm volatile("ds_mskor_b32 %0, %1, %2" ::"v"((uint32_t)(uintptr_t)&lds[db + 3]), "v"(0xffu), "v"(x3 ^ x4) : "memory");
                asm volatile("ds_mskor_b32 %0, %1, %2" ::"v"((uint32_t)(uintptr_t)&lds[db + 4]), "v"(0xffu), "v"(x4 ^ x5) : "memory");
                acc = acc * 1664525u + x0 + 1013904223u;
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            }
        } else {
            for (int w = 0; w < work / 8; w++) {
                const uint32_t idx = 512 + ((acc >> 3) + lane * 61) % 3900;
                const uint32_t v = lds[idx];
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                asm volatile("ds_mskor_b32 %0, %1, %2" ::"v"((uint32_t)(uintptr_t)&lds[idx ^ 1]), "v"(0xffu), "v"(v) : "memory");
                acc = acc * 1664525u + v + 1013904223u;
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            }
        }
        const unsigned long long t0 = __builtin_amdgcn_s_memtime();
        asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        const unsigned long long t1 = __builtin_amdgcn_s_memtime();
        wait += t1 - t0;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (lane == 0) { atomicAdd(&out[0], wait); if (acc == 12345) out[1] = acc; }
}

int main(int argc, char **argv) {
    const int nblk = argc > 1 ? atoi(argv[1]) : 131072;
    const int iters = 60;
    size_t bufsize = (size_t)16384 * 8192 + 4096;
    uint8_t *buf, *rec;
    unsigned long long *out;
    hipMalloc(&buf, bufsize);
    hipMalloc(&rec, (size_t)nblk * 8704 + 4096);
    hipMalloc(&out, 16);
    hipMemset(buf, 1, bufsize);
    hipMemset(rec, 2, (size_t)nblk * 8704 + 4096);
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    for (int mode = 0; mode < 3; mode++)
        for (int work : {0, 100, 400, 1600})
            for (int sm = 0; sm < 2; sm++) {
                hipMemset(out, 0, 16);
                auto kern = mode == 2 ? k<2> : mode ? k<1> : k<0>;
                hipLaunchKernelGGL(kern, dim3(nblk), dim3(64), 0, 0, buf, bufsize, rec, out, work, iters, sm);
                hipMemset(out, 0, 16);
                hipEventRecord(e0);
                hipLaunchKernelGGL(kern, dim3(nblk), dim3(64), 0, 0, buf, bufsize, rec, out, work, iters, sm);
                hipEventRecord(e1);
                hipEventSynchronize(e1);
                float ms; hipEventElapsedTime(&ms, e0, e1);
                unsigned long long w; hipMemcpy(&w, out, 8, hipMemcpyDeviceToHost);
                printf("mode %s work %5d src %s: kernel %.3f ms, wait/iter %.0f cycles, kernel cycles/iter/wave %.0f\n",
                       mode == 2 ? "lds2" : mode ? "lds " : "valu", work, sm ? "16k-unal" : "linear  ", ms, (double)w / nblk / iters,
                       ms * 1e-3 * 2.4e9 / ((double)nblk / (256.0 * 9)) / iters);
            }
    return 0;
}
