// qlzx_tables.hip -- constant tables for the CRC32 kernels, built at compile time.
#include "qlzx_device.h"

namespace qlzx {

struct CrcTables {
    uint32_t table[256];
    uint32_t pow8[64];
    uint32_t piece[64];  // piece[k] = x^(8 * 64 * k): shifts a 64-B piece's CRC over k later pieces
    uint32_t byte[64];   // byte[j] = x^(8 * j): with piece[], x^(8 n) for n < 4096 in one product
    uint32_t stripe[64]; // stripe[k] = x^(8 * 4096 * k): shifts a 4 KiB stripe's CRC over k stripes
    uint32_t slice[8][256];  // slice[k][b]: CRC of byte b followed by k zero bytes (slicing-by-8)
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
    for (uint32_t i = 0; i < 256; i++) t.slice[0][i] = t.table[i];
    for (int k = 1; k < 8; k++)
        for (uint32_t i = 0; i < 256; i++) {
            const uint32_t c = t.slice[k - 1][i];
            t.slice[k][i] = (c >> 8) ^ t.table[c & 0xffu];
        }
    // x^1 in reflected form is bit 30; square 3 times -> x^8 (one byte of zeros)
    uint32_t x = 0x40000000u;
    for (int k = 0; k < 3; k++) x = mulmod_c(x, x);
    for (int k = 0; k < 64; k++) {
        t.pow8[k] = x;  // x^(8 * 2^k)
        x = mulmod_c(x, x);
    }
    t.piece[0] = 0x80000000u;  // x^0
    for (int k = 1; k < 64; k++) t.piece[k] = mulmod_c(t.piece[k - 1], t.pow8[6]);  // * x^(8*64)
    t.byte[0] = 0x80000000u;
    for (int k = 1; k < 64; k++) t.byte[k] = mulmod_c(t.byte[k - 1], t.pow8[0]);     // * x^8
    t.stripe[0] = 0x80000000u;
    for (int k = 1; k < 64; k++) t.stripe[k] = mulmod_c(t.stripe[k - 1], t.pow8[12]);  // * x^(8*4096)
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

__device__ uint32_t g_crc_slice8[8 * 256] = {
#define S(k, i) kTables.slice[k][i]
#define S8(k, i) S(k, i), S(k, i + 1), S(k, i + 2), S(k, i + 3), S(k, i + 4), S(k, i + 5), S(k, i + 6), S(k, i + 7)
#define S64(k, i) S8(k, i), S8(k, i + 8), S8(k, i + 16), S8(k, i + 24), S8(k, i + 32), S8(k, i + 40), S8(k, i + 48), S8(k, i + 56)
#define S256(k) S64(k, 0), S64(k, 64), S64(k, 128), S64(k, 192)
    S256(0), S256(1), S256(2), S256(3), S256(4), S256(5), S256(6), S256(7)
#undef S256
#undef S64
#undef S8
#undef S
};

__device__ uint32_t g_crc_pow[64] = {
#define P(i) kTables.pow8[i]
#define P8(i) P(i), P(i + 1), P(i + 2), P(i + 3), P(i + 4), P(i + 5), P(i + 6), P(i + 7)
    P8(0), P8(8), P8(16), P8(24), P8(32), P8(40), P8(48), P8(56)
#undef P8
#undef P
};

__device__ uint32_t g_crc_piece[64] = {
#define Q(i) kTables.piece[i]
#define Q8(i) Q(i), Q(i + 1), Q(i + 2), Q(i + 3), Q(i + 4), Q(i + 5), Q(i + 6), Q(i + 7)
    Q8(0), Q8(8), Q8(16), Q8(24), Q8(32), Q8(40), Q8(48), Q8(56)
#undef Q8
#undef Q
};

#define T8(a, i) kTables.a[i], kTables.a[i + 1], kTables.a[i + 2], kTables.a[i + 3], kTables.a[i + 4], \
    kTables.a[i + 5], kTables.a[i + 6], kTables.a[i + 7]
#define T64(a) T8(a, 0), T8(a, 8), T8(a, 16), T8(a, 24), T8(a, 32), T8(a, 40), T8(a, 48), T8(a, 56)
__device__ uint32_t g_crc_byte[64] = {T64(byte)};
__device__ uint32_t g_crc_stripe[64] = {T64(stripe)};
#undef T64
#undef T8

// Multiply-by-constant tables for wave_crc: g_crc_mul[i * 1024 + j * 256 + b] = (b << 8 j) *
// x^(8 kMulBytes[i]) mod P, so a register c times that power is four lookups, one per byte.
// i = 0..5: 64 * 2^i bytes (the lane-combine tree), i = 6: 4032 bytes (the other 63 lanes'
// pieces of a 4 KiB stripe).
constexpr int kMulTabs = 7;
struct CrcMul {
    uint32_t t[kMulTabs * 1024];
};
__host__ __device__ constexpr CrcMul make_mul() {
    CrcMul m{};
    const uint32_t pieces[kMulTabs] = {1, 2, 4, 8, 16, 32, 63};
    for (int i = 0; i < kMulTabs; i++) {
        const uint32_t k = kTables.piece[pieces[i]];
        // b -> (b << 8 j) * k is linear in b: build from the 8 single-bit products
        for (int j = 0; j < 4; j++) {
            uint32_t bit[8] = {};
            for (int q = 0; q < 8; q++) bit[q] = mulmod_c(k, 1u << (8 * j + q));
            for (uint32_t b = 0; b < 256; b++) {
                uint32_t v = 0;
                for (int q = 0; q < 8; q++)
                    if (b & (1u << q)) v ^= bit[q];
                m.t[i * 1024 + j * 256 + b] = v;
            }
        }
    }
    return m;
}
constexpr CrcMul kMul = make_mul();
static_assert(kMul.t[0] == 0 && kMul.t[6 * 1024 + 256 + 1] == mulmod_c(kTables.piece[63], 1u << 8), "crc mul");

#define M8(i) kMul.t[i], kMul.t[i + 1], kMul.t[i + 2], kMul.t[i + 3], kMul.t[i + 4], kMul.t[i + 5], \
    kMul.t[i + 6], kMul.t[i + 7]
#define M64(i) M8(i), M8(i + 8), M8(i + 16), M8(i + 24), M8(i + 32), M8(i + 40), M8(i + 48), M8(i + 56)
#define M1K(i) M64(i), M64(i + 64), M64(i + 128), M64(i + 192), M64(i + 256), M64(i + 320), M64(i + 384), \
    M64(i + 448), M64(i + 512), M64(i + 576), M64(i + 640), M64(i + 704), M64(i + 768), M64(i + 832), \
    M64(i + 896), M64(i + 960)
__device__ uint32_t g_crc_mul[kMulTabs * 1024] = {M1K(0), M1K(1024), M1K(2048), M1K(3072), M1K(4096),
                                                  M1K(5120), M1K(6144)};

// The same for x^(8 * 32): wave_crc_rep's two half-piece chains meet through it.
__host__ __device__ constexpr CrcMul make_mul32() {
    CrcMul m{};
    const uint32_t k = kTables.byte[32];
    for (int j = 0; j < 4; j++) {
        uint32_t bit[8] = {};
        for (int q = 0; q < 8; q++) bit[q] = mulmod_c(k, 1u << (8 * j + q));
        for (uint32_t b = 0; b < 256; b++) {
            uint32_t v = 0;
            for (int q = 0; q < 8; q++)
                if (b & (1u << q)) v ^= bit[q];
            m.t[j * 256 + b] = v;
        }
    }
    return m;
}
constexpr CrcMul kMul32 = make_mul32();
#undef M8
#define M8(i) kMul32.t[i], kMul32.t[i + 1], kMul32.t[i + 2], kMul32.t[i + 3], kMul32.t[i + 4], kMul32.t[i + 5], \
    kMul32.t[i + 6], kMul32.t[i + 7]
__device__ uint32_t g_crc_mul32[1024] = {M1K(0)};
#undef M1K
#undef M64
#undef M8

}  // namespace qlzx

// Host copies (used by the single-call crc32_write path's self-check and tests).
extern "C" uint32_t qlzx_host_crc_table(int i) { return qlzx::kTables.table[i & 255]; }
