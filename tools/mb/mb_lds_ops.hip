// Microbenchmark: LDS throughput per wave-instruction for the DS forms a decoder copy can use.
// 16 waves per CU (1024-thread workgroups, one per CU), each issuing a stream of independent
// DS instructions at scattered dword-aligned addresses (a match copy's pattern), 8 per
// lgkmcnt(0) drain.  Prints CU cycles per wave-instruction (s_memtime / (16 waves x count)).
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

typedef uint32_t v4u __attribute__((ext_vector_type(4)));

template <int MODE>
__global__ void __launch_bounds__(1024) k(uint32_t *out, unsigned long long *cyc, int iters, int active, int pat) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[16384];  // 64 KiB
    for (int i = threadIdx.x; i < 16384; i += blockDim.x) lds[i] = i * 2654435761u;
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t wbase = wave * 4096;  // 4 KiB per wave
    uint32_t h = lane * 0x9E3779B9u + wave * 77u;
    uint32_t acc = 0;
    const bool on = (int)lane < active;
    __syncthreads();
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    if (on) {
        for (int it = 0; it < iters; it++) {
            h = h * 1664525u + 1013904223u;
            // pat 0: random dword addresses; pat 1: consecutive ~5.3-B items (a match batch's dests)
            const uint32_t a4 = wbase + (pat ? (((uint32_t)it * 344u + lane * 21u / 4u) & 2044u) : ((h >> 8) & 2044u));
            const uint32_t a8 = a4 & ~7u;
#define U(o) OP(o)
#pragma unroll
            for (int u = 0; u < 1; u++) {
                uint32_t v0;
                uint64_t r;
                v4u qv;
                if (MODE == 0) {
#define OP(o) asm volatile("ds_read_b32 %0, %1 offset:" #o : "=v"(v0) : "v"(a4)); acc += v0;
                    U(0) U(136) U(272) U(408) U(544) U(680) U(816) U(952)
#undef OP
                } else if (MODE == 1) {
#define OP(o) asm volatile("ds_read2_b32 %0, %1 offset0:" #o "/4 offset1:" #o "/4+1" : "=v"(r) : "v"(a4)); acc += (uint32_t)r;
                    U(0) U(136) U(272) U(408) U(544) U(680) U(816) U(952)
#undef OP
                } else if (MODE == 2) {
#define OP(o) asm volatile("ds_read_b64 %0, %1 offset:" #o : "=v"(r) : "v"(a4)); acc += (uint32_t)r;
                    U(0) U(136) U(272) U(408) U(544) U(680) U(816) U(952)
#undef OP
                } else if (MODE == 3) {
#define OP(o) asm volatile("ds_read_b64 %0, %1 offset:" #o : "=v"(r) : "v"(a8)); acc += (uint32_t)r;
                    U(0) U(136) U(272) U(408) U(544) U(680) U(816) U(952)
#undef OP
                } else if (MODE == 4) {
#define OP(o) asm volatile("ds_write_b32 %0, %1 offset:" #o ::"v"(a4), "v"(h) : "memory");
                    U(0) U(136) U(272) U(408) U(544) U(680) U(816) U(952)
#undef OP
                } else if (MODE == 5) {
#define OP(o) asm volatile("ds_mskor_b32 %0, %1, %2 offset:" #o ::"v"(a4), "v"(h & 0xff00u), "v"(h & 0x0100u) : "memory");
                    U(0) U(136) U(272) U(408) U(544) U(680) U(816) U(952)
#undef OP
                } else if (MODE == 6) {
#define OP(o) asm volatile("ds_or_b32 %0, %1 offset:" #o ::"v"(a4), "v"(h) : "memory");
                    U(0) U(136) U(272) U(408) U(544) U(680) U(816) U(952)
#undef OP
                } else if (MODE == 7) {
#define OP(o) asm volatile("ds_write_b8 %0, %1 offset:" #o ::"v"(a4), "v"(h) : "memory");
                    U(1) U(138) U(275) U(408) U(545) U(682) U(819) U(952)
#undef OP
                } else if (MODE == 8) {
#define OP(o) asm volatile("ds_read2_b64 %0, %1 offset0:" #o "/8 offset1:" #o "/8+1" : "=v"(qv) : "v"(a8)); acc += qv.x;
                    U(0) U(136) U(272) U(408) U(544) U(680) U(816) U(952)
#undef OP
                } else if (MODE == 9) {
#define OP(o) asm volatile("ds_write_b64 %0, %1 offset:" #o ::"v"(a8), "v"(((uint64_t)h << 32) | h) : "memory");
                    U(0) U(136) U(272) U(408) U(544) U(680) U(816) U(952)
#undef OP
                } else if (MODE == 10) {
#define OP(o) asm volatile("ds_read_b128 %0, %1 offset:" #o : "=v"(qv) : "v"(a4 & ~15u)); acc += qv.x;
                    U(0) U(144) U(288) U(432) U(576) U(720) U(864) U(1008)
#undef OP
                } else if (MODE == 11) {
#define OP(o) asm volatile("ds_read_u8 %0, %1 offset:" #o : "=v"(v0) : "v"(a4)); acc += v0;
                    U(1) U(138) U(275) U(408) U(545) U(682) U(819) U(952)
#undef OP
                } else if (MODE == 12) {
                    v4u hv; hv.x = h; hv.y = h ^ 1u; hv.z = h ^ 2u; hv.w = h ^ 3u;
#define OP(o) asm volatile("ds_write_b128 %0, %1 offset:" #o ::"v"(a4 & ~15u), "v"(hv) : "memory");
                    U(0) U(144) U(288) U(432) U(576) U(720) U(864) U(1008)
#undef OP
                }
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        }
    }
    __syncthreads();
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc + lds[threadIdx.x];
}

static const char *names[] = {"ds_read_b32",          "ds_read2_b32 (4-al)",  "ds_read_b64 (4-aligned)",
                              "ds_read_b64 (8-al)",   "ds_write_b32",         "ds_mskor_b32",
                              "ds_or_b32",            "ds_write_b8",          "ds_read2_b64 (8-al)",
                              "ds_write_b64 (8-al) ",  "ds_read_b128 (16-al)",  "ds_read_u8",
                              "ds_write_b128 (16-al)"};

template <int MODE>
void run(uint32_t *out, unsigned long long *cyc, int active, int pat) {
    const int iters = 2048;
    hipLaunchKernelGGL(k<MODE>, dim3(256), dim3(1024), 0, 0, out, cyc, iters, active, pat);
    hipDeviceSynchronize();
    unsigned long long c[256];
    hipMemcpy(c, cyc, sizeof(c), hipMemcpyDeviceToHost);
    double s = 0;
    for (int i = 0; i < 256; i++) s += c[i];
    s /= 256;
    printf("%-26s %s active %2d: %.2f CU cycles per wave-instruction\n", names[MODE], pat ? "consec" : "random", active, s / (16.0 * iters * 8));
}

int main() {
    uint32_t *out;
    unsigned long long *cyc;
    hipMalloc(&out, 256 * 1024 * 4);
    hipMalloc(&cyc, 256 * 8);
    for (int pat : {0, 1})
    for (int active : {64, 8}) {
        run<0>(out, cyc, active, pat);
        run<1>(out, cyc, active, pat);
        run<2>(out, cyc, active, pat);
        run<3>(out, cyc, active, pat);
        run<4>(out, cyc, active, pat);
        run<5>(out, cyc, active, pat);
        run<6>(out, cyc, active, pat);
        run<7>(out, cyc, active, pat);
        run<8>(out, cyc, active, pat);
        run<9>(out, cyc, active, pat);
        run<10>(out, cyc, active, pat);
        run<11>(out, cyc, active, pat);
        run<12>(out, cyc, active, pat);
    }
    return 0;
}
