// Microbenchmark: instruction issue rates per CU on gfx950 -- SALU vs VALU vs mixed, with
// W waves per CU (one workgroup of W*64 threads per CU).  Each wave runs 16 independent
// instructions per iteration (no dependencies between them, so issue, not latency, bounds).
// Prints CU cycles per wave-instruction.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

template <int MODE>
__global__ void k(uint32_t *out, unsigned long long *cyc, int iters) {
    uint32_t s0 = blockIdx.x, s1 = 1, s2 = 2, s3 = 3, s4 = 4, s5 = 5, s6 = 6, s7 = 7;
    uint32_t v0 = threadIdx.x, v1 = 1, v2 = 2, v3 = 3, v4 = 4, v5 = 5, v6 = 6, v7 = 7;
    __syncthreads();
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; it++) {
        if (MODE == 0) {  // 16 SALU
            asm volatile(
                "s_add_u32 %0, %0, 3\n s_add_u32 %1, %1, 5\n s_add_u32 %2, %2, 7\n s_add_u32 %3, %3, 9\n"
                "s_add_u32 %4, %4, 3\n s_add_u32 %5, %5, 5\n s_add_u32 %6, %6, 7\n s_add_u32 %7, %7, 9\n"
                "s_add_u32 %0, %0, 3\n s_add_u32 %1, %1, 5\n s_add_u32 %2, %2, 7\n s_add_u32 %3, %3, 9\n"
                "s_add_u32 %4, %4, 3\n s_add_u32 %5, %5, 5\n s_add_u32 %6, %6, 7\n s_add_u32 %7, %7, 9\n"
                : "+s"(s0), "+s"(s1), "+s"(s2), "+s"(s3), "+s"(s4), "+s"(s5), "+s"(s6), "+s"(s7)::"scc");
        } else if (MODE == 1) {  // 16 VALU
            asm volatile(
                "v_add_u32 %0, %0, 3\n v_add_u32 %1, %1, 5\n v_add_u32 %2, %2, 7\n v_add_u32 %3, %3, 9\n"
                "v_add_u32 %4, %4, 3\n v_add_u32 %5, %5, 5\n v_add_u32 %6, %6, 7\n v_add_u32 %7, %7, 9\n"
                "v_add_u32 %0, %0, 3\n v_add_u32 %1, %1, 5\n v_add_u32 %2, %2, 7\n v_add_u32 %3, %3, 9\n"
                "v_add_u32 %4, %4, 3\n v_add_u32 %5, %5, 5\n v_add_u32 %6, %6, 7\n v_add_u32 %7, %7, 9\n"
                : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7));
        } else if (MODE == 2) {  // 8 SALU + 8 VALU interleaved
            asm volatile(
                "s_add_u32 %0, %0, 3\n v_add_u32 %8, %8, 3\n s_add_u32 %1, %1, 5\n v_add_u32 %9, %9, 5\n"
                "s_add_u32 %2, %2, 7\n v_add_u32 %10, %10, 7\n s_add_u32 %3, %3, 9\n v_add_u32 %11, %11, 9\n"
                "s_add_u32 %4, %4, 3\n v_add_u32 %12, %12, 3\n s_add_u32 %5, %5, 5\n v_add_u32 %13, %13, 5\n"
                "s_add_u32 %6, %6, 7\n v_add_u32 %14, %14, 7\n s_add_u32 %7, %7, 9\n v_add_u32 %15, %15, 9\n"
                : "+s"(s0), "+s"(s1), "+s"(s2), "+s"(s3), "+s"(s4), "+s"(s5), "+s"(s6), "+s"(s7), "+v"(v0),
                  "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7)::"scc");
        } else if (MODE == 3) {  // 16 v_cmp writing SGPR pairs (ballot-like)
            uint64_t m0, m1, m2, m3;
            asm volatile(
                "v_cmp_lt_u32 %0, %4, %5\n v_cmp_lt_u32 %1, %5, %6\n v_cmp_lt_u32 %2, %6, %7\n v_cmp_lt_u32 %3, %7, %4\n"
                "v_cmp_lt_u32 %0, %4, %5\n v_cmp_lt_u32 %1, %5, %6\n v_cmp_lt_u32 %2, %6, %7\n v_cmp_lt_u32 %3, %7, %4\n"
                "v_cmp_lt_u32 %0, %4, %5\n v_cmp_lt_u32 %1, %5, %6\n v_cmp_lt_u32 %2, %6, %7\n v_cmp_lt_u32 %3, %7, %4\n"
                "v_cmp_lt_u32 %0, %4, %5\n v_cmp_lt_u32 %1, %5, %6\n v_cmp_lt_u32 %2, %6, %7\n v_cmp_lt_u32 %3, %7, %4\n"
                : "=s"(m0), "=s"(m1), "=s"(m2), "=s"(m3)
                : "v"(v0), "v"(v1), "v"(v2), "v"(v3));
            s0 += (uint32_t)(m0 ^ m1 ^ m2 ^ m3);
        } else if (MODE == 4) {  // 16 SALU 64-bit ops
            uint64_t a = s0, b = s1, c = s2, d = s3;
            asm volatile(
                "s_and_b64 %0, %0, %1\n s_or_b64 %1, %1, %2\n s_xor_b64 %2, %2, %3\n s_and_b64 %3, %3, %0\n"
                "s_and_b64 %0, %0, %1\n s_or_b64 %1, %1, %2\n s_xor_b64 %2, %2, %3\n s_and_b64 %3, %3, %0\n"
                "s_and_b64 %0, %0, %1\n s_or_b64 %1, %1, %2\n s_xor_b64 %2, %2, %3\n s_and_b64 %3, %3, %0\n"
                "s_and_b64 %0, %0, %1\n s_or_b64 %1, %1, %2\n s_xor_b64 %2, %2, %3\n s_and_b64 %3, %3, %0\n"
                : "+s"(a), "+s"(b), "+s"(c), "+s"(d)::"scc");
            s0 = (uint32_t)(a ^ b ^ c ^ d);
        }
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    __syncthreads();
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
    out[blockIdx.x * blockDim.x + threadIdx.x] = s0 + s1 + s2 + s3 + s4 + s5 + s6 + s7 + v0 + v1 + v2 + v3 + v4 + v5 + v6 + v7;
}

static const char *names[] = {"16 s_add_u32", "16 v_add_u32", "8 s_add + 8 v_add", "16 v_cmp -> sgpr",
                              "16 s_*_b64"};

template <int MODE>
void run(uint32_t *out, unsigned long long *cyc, int waves) {
    const int iters = 4096;
    hipLaunchKernelGGL(k<MODE>, dim3(256), dim3(64 * waves), 0, 0, out, cyc, iters);
    hipDeviceSynchronize();
    unsigned long long c[256];
    hipMemcpy(c, cyc, sizeof(c), hipMemcpyDeviceToHost);
    double s = 0;
    for (int i = 0; i < 256; i++) s += c[i];
    s /= 256;
    printf("%-20s waves/CU %2d: %.3f CU cycles per wave-instruction (%.2f per SIMD)\n", names[MODE], waves,
           s / (waves * 16.0 * iters), s / (waves * 16.0 * iters) * 4);
}

int main() {
    uint32_t *out;
    unsigned long long *cyc;
    hipMalloc(&out, 256 * 1024 * 4);
    hipMalloc(&cyc, 256 * 8);
    for (int w : {1, 4, 8, 16}) {
        run<0>(out, cyc, w);
        run<1>(out, cyc, w);
        run<2>(out, cyc, w);
        run<3>(out, cyc, w);
        run<4>(out, cyc, w);
    }
    return 0;
}
