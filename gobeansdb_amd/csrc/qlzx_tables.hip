// qlzx_tables.hip -- constant tables for the CRC32 kernels, built at compile time.
#include "qlzx_device.h"

namespace qlzx {

struct CrcTables {
    uint32_t table[256];
    uint32_t pow8[64];
};

__host__ __device__ constexpr uint32_t mulmod_c(uint32_t a, uint32_t b) {
    uint32_t p = 0;
    for (int i = 0; i < 32; i++) {
        if (a & 0x80000000u) p ^= b;
        a <<= 1;
        b = (b & 1u) ? (b >> 1) ^ CRC_POLY : (b >> 1);
    }
    return p;
}

__host__ __device__ constexpr CrcTables make_tables() {
    CrcTables t{};
    for (uint32_t i = 0; i < 256; i++) {
        uint32_t c = i;
        for (int k = 0; k < 8; k++) c = (c & 1u) ? (c >> 1) ^ CRC_POLY : (c >> 1);
        t.table[i] = c;
    }
    // x^1 in reflected form is bit 30; square 3 times -> x^8 (one byte of zeros)
    uint32_t x = 0x40000000u;
    for (int k = 0; k < 3; k++) x = mulmod_c(x, x);
    for (int k = 0; k < 64; k++) {
        t.pow8[k] = x;  // x^(8 * 2^k)
        x = mulmod_c(x, x);
    }
    return t;
}

constexpr CrcTables kTables = make_tables();
static_assert(kTables.table[1] == 0x77073096u, "crc table");    // store/crc32.go:7
static_assert(kTables.table[255] == 0x2d02ef8du, "crc table");  // store/crc32.go:58

__device__ uint32_t g_crc_table[256] = {
#define R(i) kTables.table[i]
#define R8(i) R(i), R(i + 1), R(i + 2), R(i + 3), R(i + 4), R(i + 5), R(i + 6), R(i + 7)
#define R64(i) R8(i), R8(i + 8), R8(i + 16), R8(i + 24), R8(i + 32), R8(i + 40), R8(i + 48), R8(i + 56)
    R64(0), R64(64), R64(128), R64(192)
#undef R64
#undef R8
#undef R
};

__device__ uint32_t g_crc_pow[64] = {
#define P(i) kTables.pow8[i]
#define P8(i) P(i), P(i + 1), P(i + 2), P(i + 3), P(i + 4), P(i + 5), P(i + 6), P(i + 7)
    P8(0), P8(8), P8(16), P8(24), P8(32), P8(40), P8(48), P8(56)
#undef P8
#undef P
};

}  // namespace qlzx

// Host copies (used by the single-call crc32_write path's self-check and tests).
extern "C" uint32_t qlzx_host_crc_table(int i) { return qlzx::kTables.table[i & 255]; }
