// Microbenchmark (tools only): calibrates the PMC FETCH_SIZE counter on gfx950 for the access
// patterns the decode kernels use, against a known byte count.  Each kernel reads every byte of
// a 512 MiB buffer exactly once from HBM (far larger than L2 and MALL), so the true fetch is
// 512 MiB per kernel; FETCH_SIZE (KiB per dispatch, rocprofv3 --pmc FETCH_SIZE) divided by it
// is the factor to correct a measured FETCH_SIZE with.
//   x4        16 B per lane, 1 KiB contiguous per wave instruction (the guide's streaming case)
//   dword     4 B per lane, contiguous
//   dword_u   4 B per lane, contiguous but 1 byte off dword alignment (K2's far/literal loads)
//   dma4      global_load_lds_dword, 4 B per lane, contiguous (K2's record DMA)
//   dma4_tok  global_load_lds_dword at K2-token-like positions: lane l of a wave reads 4 B at
//             byte 3l/2 of a 96-B stretch (overlapping, unaligned), stretches back to back
//   dma16     global_load_lds_dwordx4, 16 B per lane (K1's ring DMA)
// usage: rocprofv3 --pmc FETCH_SIZE -- ./mb_fetch
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#include "../../gobeansdb_amd/csrc/qlzx_device.h"

constexpr size_t kBytes = 512ull << 20;

__global__ void k_x4(const uint8_t *p, uint32_t *out) {
    const size_t g = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t s = 0;
    for (size_t o = g * 16; o < kBytes; o += (size_t)gridDim.x * blockDim.x * 16) {
        const uint4 v = *(const uint4 *)(p + o);
        s += v.x ^ v.y ^ v.z ^ v.w;
    }
    if (s == 0x12345678u) out[0] = s;
}
__global__ void k_dword(const uint8_t *p, uint32_t *out, uint32_t mis) {
    const size_t g = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t s = 0;
    for (size_t o = g * 4; o + 4 + mis <= kBytes; o += (size_t)gridDim.x * blockDim.x * 4)
        s += *(const uint32_t *)(p + o + mis);
    if (s == 0x12345678u) out[0] = s;
}
__global__ void __launch_bounds__(64) k_dma4(const uint8_t *p, uint32_t *out) {
    __shared__ uint32_t lds[4][64];
    const size_t g = (size_t)blockIdx.x * 64 + threadIdx.x;
    uint32_t s = 0, k = 0;
    for (size_t o = g * 4; o < kBytes; o += (size_t)gridDim.x * 64 * 4, k++) {
        qlzx::dma4(p + o, qlzx::lds_addr(lds[k & 3]));
        if ((k & 3) == 3) {
            qlzx::vm_sync();
            s += lds[0][threadIdx.x] ^ lds[3][threadIdx.x];
        }
    }
    qlzx::vm_sync();
    if (s == 0x12345678u) out[0] = s;
}
__global__ void __launch_bounds__(64) k_dma4_tok(const uint8_t *p, uint32_t *out) {
    __shared__ uint32_t lds[4][64];
    uint32_t s = 0, k = 0;
    const size_t nstretch = kBytes / 96;
    for (size_t st = blockIdx.x; st < nstretch; st += gridDim.x, k++) {
        const size_t o = st * 96 + (threadIdx.x * 3) / 2;
        qlzx::dma4(p + (o + 4 <= kBytes ? o : kBytes - 4), qlzx::lds_addr(lds[k & 3]));
        if ((k & 3) == 3) {
            qlzx::vm_sync();
            s += lds[1][threadIdx.x] ^ lds[2][threadIdx.x];
        }
    }
    qlzx::vm_sync();
    if (s == 0x12345678u) out[0] = s;
}
__global__ void __launch_bounds__(64) k_dma16(const uint8_t *p, uint32_t *out) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[4][256];
    const size_t g = (size_t)blockIdx.x * 64 + threadIdx.x;
    uint32_t s = 0, k = 0;
    for (size_t o = g * 16; o < kBytes; o += (size_t)gridDim.x * 64 * 16, k++) {
        qlzx::dma16(p + o, qlzx::lds_addr(lds[k & 3]));
        if ((k & 3) == 3) {
            qlzx::vm_sync();
            s += lds[0][threadIdx.x] ^ lds[3][threadIdx.x];
        }
    }
    qlzx::vm_sync();
    if (s == 0x12345678u) out[0] = s;
}

int main() {
    uint8_t *p;
    uint32_t *out;
    if (hipMalloc(&p, kBytes + 64) != hipSuccess || hipMalloc(&out, 64) != hipSuccess) return 1;
    (void)hipMemset(p, 1, kBytes + 64);
    (void)hipDeviceSynchronize();
    const int grid = 256 * 32;
    hipLaunchKernelGGL(k_x4, dim3(grid), dim3(256), 0, 0, p, out);
    hipLaunchKernelGGL(k_dword, dim3(grid), dim3(256), 0, 0, p, out, 0u);
    hipLaunchKernelGGL(k_dword, dim3(grid), dim3(256), 0, 0, p, out, 1u);
    hipLaunchKernelGGL(k_dma4, dim3(grid), dim3(64), 0, 0, p, out);
    hipLaunchKernelGGL(k_dma4_tok, dim3(grid), dim3(64), 0, 0, p, out);
    hipLaunchKernelGGL(k_dma16, dim3(grid), dim3(64), 0, 0, p, out);
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    printf("true bytes per kernel: %zu (%.1f KiB)\n", kBytes, kBytes / 1024.0);
    return 0;
}
