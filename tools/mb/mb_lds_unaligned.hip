// Microbenchmark: ds_read_b32 at byte-unaligned LDS addresses vs two aligned reads + v_alignbyte.
// Checks the values and times both forms (s_memtime cycles per wave-instruction).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

// throughput form: 8 independent reads per iteration, 16 waves per workgroup
__global__ void kt(uint32_t *out, unsigned long long *cyc, int mode, int iters) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[8192];
    for (int i = threadIdx.x; i < 8192; i += blockDim.x) lds[i] = (uint8_t)(i * 131 + 7);
    __syncthreads();
    uint32_t acc = 0;
    uint32_t a = threadIdx.x * 61 + 1;
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int u = 0; u < 8; u++) {
            const uint32_t ad = (a + u * 517) & 4095;
            uint32_t v;
            if (mode == 0) v = *(const uint32_t *)(lds + ad);
            else {
                const uint32_t *w = (const uint32_t *)(lds + (ad & ~3u));
                v = __builtin_amdgcn_alignbyte(w[1], w[0], ad & 3u);
            }
            acc += v;
        }
        a += 77;
    }
    __syncthreads();
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

__global__ void k(uint32_t *out, unsigned long long *cyc, int mode, int iters) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[8192];
    for (int i = threadIdx.x; i < 8192; i++) lds[i] = (uint8_t)(i * 131 + 7);
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63;
    uint32_t acc = 0, bad = 0;
    uint32_t a = lane * 61 + 1;
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; it++) {
        const uint32_t ad = a & 4095;
        uint32_t v;
        if (mode == 0) {
            v = *(const uint32_t *)(lds + ad);  // unaligned ds_read_b32
        } else {
            const uint32_t *w = (const uint32_t *)(lds + (ad & ~3u));
            v = __builtin_amdgcn_alignbyte(w[1], w[0], ad & 3u);
        }
        const uint32_t e = (uint32_t)(uint8_t)(ad * 131 + 7) | ((uint32_t)(uint8_t)((ad + 1) * 131 + 7) << 8) |
                           ((uint32_t)(uint8_t)((ad + 2) * 131 + 7) << 16) | ((uint32_t)(uint8_t)((ad + 3) * 131 + 7) << 24);
        bad += v != e;
        acc += v;
        a = a * 1103515245u + (v & 7u) + 12345u;  // dependent chain through the value
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
    out[blockIdx.x * blockDim.x + threadIdx.x] = bad * 1000000u + (acc & 0xff);
}

int main() {
    uint32_t *out;
    unsigned long long *cyc;
    hipMalloc(&out, 1024 * 1024 * 4);
    hipMalloc(&cyc, 1024 * 8);
    for (int mode = 0; mode < 2; mode++) {
        hipLaunchKernelGGL(k, dim3(256), dim3(64), 0, 0, out, cyc, mode, 4096);
        hipDeviceSynchronize();
        uint32_t h[64 * 256];
        unsigned long long c[256];
        hipMemcpy(h, out, sizeof(h), hipMemcpyDeviceToHost);
        hipMemcpy(c, cyc, sizeof(c), hipMemcpyDeviceToHost);
        unsigned bad = 0;
        for (int i = 0; i < 64 * 256; i++) bad += h[i] / 1000000u;
        printf("mode %d (%s): bad %u, cycles/iter %.1f\n", mode, mode == 0 ? "unaligned ds_read_b32" : "2 reads + alignbyte",
               bad, (double)c[0] / 4096);
    }
    for (int mode = 0; mode < 2; mode++) {
        hipLaunchKernelGGL(kt, dim3(256), dim3(1024), 0, 0, out, cyc, mode, 2048);
        hipDeviceSynchronize();
        unsigned long long c[256];
        hipMemcpy(c, cyc, sizeof(c), hipMemcpyDeviceToHost);
        printf("throughput mode %d (%s): cycles per 16-wave x 8 reads iteration %.1f -> %.2f cycles per wave-read\n", mode,
               mode == 0 ? "unaligned ds_read_b32" : "2 reads + alignbyte", (double)c[0] / 2048, (double)c[0] / 2048 / 128);
    }
    return 0;
}
