// qlzx_device.h -- device-side helpers shared by the gfx950 kernels.
//
// QuickLZ level-3 format facts used here (SURVEY.md §8 "Format facts"):
//   header byte 0 = 01SSLLHC (quicklz.c:771-772); 9-byte header if H
//   control word: 32-bit LE, LSB-first item bits, bit 31 sentinel (quicklz.c:203,221)
//   level-3 match tokens (quicklz.c:579-610)
//   last 10 output bytes are always literals (quicklz.c:204, 503)
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/qlzx.h"

#define QLZX_TAIL 10u         // UNCONDITIONAL_MATCHLEN + UNCOMPRESSED_END (quicklz.c:24-25)
#define QLZX_BUCKETS 4096u    // QLZ_HASH_VALUES (quicklz.h:62)
#define QLZX_SLOTS 16u        // QLZ_POINTERS    (quicklz.h:61)
#define QLZX_MAX_OFFSET 131071u
#define QLZX_STR_(x) #x
#define QLZX_STR(x) QLZX_STR_(x)

namespace qlzx {

// CRC-32/IEEE reflected table, poly 0xEDB88320 (store/crc32.go:5-59).
extern __device__ uint32_t g_crc_table[256];
// g_crc_x8n[k] = x^(8 * 2^k) mod P in reflected form, for CRC shift/combine.
extern __device__ uint32_t g_crc_pow[64];
// g_crc_slice8[k * 256 + b]: CRC of byte b followed by k zero bytes (slicing-by-8).
extern __device__ uint32_t g_crc_slice8[8 * 256];
// g_crc_piece[k] = x^(8 * 64 * k) mod P: shift of a 64-B piece's CRC over k later 64-B pieces.
extern __device__ uint32_t g_crc_piece[64];
// g_crc_byte[j] = x^(8 j); g_crc_stripe[k] = x^(8 * 4096 * k).
extern __device__ uint32_t g_crc_byte[64];
extern __device__ uint32_t g_crc_stripe[64];

constexpr uint32_t CRC_POLY = 0xEDB88320u;

// GF(2) product a*b mod P, reflected representation (bit 31 = x^0).
__device__ __forceinline__ uint32_t gf2_mulmod(uint32_t a, uint32_t b) {
    uint32_t p = 0;
#pragma unroll 8
    for (int i = 0; i < 32; i++) {
        p ^= (a & 0x80000000u) ? b : 0u;
        a <<= 1;
        b = (b & 1u) ? (b >> 1) ^ CRC_POLY : (b >> 1);
    }
    return p;
}

// Raw CRC state advanced over `nbytes` zero bytes: s * x^(8n) mod P.
__device__ __forceinline__ uint32_t crc_shift(uint32_t s, uint64_t nbytes) {
    uint32_t k = 0;
    while (nbytes) {
        if (nbytes & 1u) s = gf2_mulmod(g_crc_pow[k], s);
        nbytes >>= 1;
        k++;
    }
    return s;
}

// x^(8 n) for n <= 4096 in at most one product (tables above).
__device__ __forceinline__ uint32_t crc_xpow_bytes(uint32_t n) {
    return n == 4096 ? g_crc_pow[12] : gf2_mulmod(g_crc_piece[n >> 6], g_crc_byte[n & 63]);
}

__device__ __forceinline__ uint32_t crc_byte(const uint32_t *tab, uint32_t c, uint32_t b) {
    return tab[(c ^ b) & 0xffu] ^ (c >> 8);
}

__device__ __forceinline__ uint32_t crc_word(const uint32_t *tab, uint32_t c, uint32_t w) {
    c = crc_byte(tab, c, w & 0xff);
    c = crc_byte(tab, c, (w >> 8) & 0xff);
    c = crc_byte(tab, c, (w >> 16) & 0xff);
    return crc_byte(tab, c, w >> 24);
}

// Load the slicing-by-8 tables into LDS (call by the whole block, then __syncthreads()).
__device__ __forceinline__ void load_crc_slice8(uint32_t *lds_tab8) {
    for (uint32_t i = threadIdx.x; i < 8 * 256; i += blockDim.x) lds_tab8[i] = g_crc_slice8[i];
}

// Load the CRC table into LDS (call by the whole block, then __syncthreads()).
__device__ __forceinline__ void load_crc_table(uint32_t *lds_tab) {
    for (uint32_t i = threadIdx.x; i < 256; i += blockDim.x) lds_tab[i] = g_crc_table[i];
}

// Slicing-by-8 update over 8 bytes (lo = bytes 0..3, hi = bytes 4..7), tables in LDS.
__device__ __forceinline__ uint32_t crc_slice8(const uint32_t *t, uint32_t c, uint32_t lo, uint32_t hi) {
    const uint32_t x = lo ^ c;
    return t[7 * 256 + (x & 0xff)] ^ t[6 * 256 + ((x >> 8) & 0xff)] ^ t[5 * 256 + ((x >> 16) & 0xff)] ^
           t[4 * 256 + (x >> 24)] ^ t[3 * 256 + (hi & 0xff)] ^ t[2 * 256 + ((hi >> 8) & 0xff)] ^
           t[1 * 256 + ((hi >> 16) & 0xff)] ^ t[hi >> 24];
}

// LDS DMA (global -> LDS, no VGPR destination): each lane's bytes land at
// lds_base + 16*lane (dwordx4) or + 4*lane (dword); lds_base must be
// wave-uniform.  Issued as inline asm so the compiler's waitcnt pass does not
// serialise later LDS reads behind it; callers wait with vm_sync()/vmcnt(N).
// M0 is saved and restored around the DMA.
__device__ __forceinline__ void dma16(const void *g, uint32_t lds_base) {
    uint32_t tmp;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\tglobal_load_lds_dwordx4 %2, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(tmp)
                 : "s"(__builtin_amdgcn_readfirstlane(lds_base)), "v"(g)
                 : "memory");
}
__device__ __forceinline__ void dma4(const void *g, uint32_t lds_base) {
    uint32_t tmp;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\tglobal_load_lds_dword %2, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(tmp)
                 : "s"(__builtin_amdgcn_readfirstlane(lds_base)), "v"(g)
                 : "memory");
}
__device__ __forceinline__ uint32_t lds_addr(const void *p) { return (uint32_t)(uintptr_t)p; }

// ---- optional in-kernel phase timing (profiling build: -DQLZX_PROFILE) ----
// Stamps are s_memtime (shader clock) deltas summed per phase into a debug
// buffer; they never feed any output.  Release builds compile them away.
#ifdef QLZX_PROFILE
extern __device__ unsigned long long *g_prof;
#define PROF_DECL unsigned long long _pt = __builtin_amdgcn_s_memtime(), _pacc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#define PROF_MARK(ph)                                             \
    do {                                                          \
        const unsigned long long _n = __builtin_amdgcn_s_memtime(); \
        _pacc[ph] += _n - _pt;                                    \
        _pt = _n;                                                 \
    } while (0)
#define PROF_FLUSH(slot)                                                            \
    do {                                                                            \
        if (g_prof && (threadIdx.x & 63) == 0)                                      \
            for (int _j = 0; _j < 8; _j++) atomicAdd(&g_prof[(slot) * 8 + _j], _pacc[_j]); \
    } while (0)
#define PROF_COUNT(i, v) (_pacc[i] += (v))
#else
#define PROF_DECL
#define PROF_MARK(ph) \
    do {              \
    } while (0)
#define PROF_FLUSH(slot) \
    do {                 \
    } while (0)
#define PROF_COUNT(i, v) ((void)0)
#endif

// s_waitcnt on LDS only (no vmcnt), plus a compiler memory barrier.
__device__ __forceinline__ void lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
__device__ __forceinline__ void vm_sync() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

__device__ __forceinline__ uint32_t ld_u8(const uint8_t *p) { return *p; }
__device__ __forceinline__ uint32_t ld_u32_bytes(const uint8_t *p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

// Level-3 token decode (quicklz.c:579-610): returns token length in bytes.
__device__ __forceinline__ uint32_t decode_token(uint32_t t, uint32_t &off, uint32_t &len) {
    if ((t & 3u) == 0) { off = (t & 0xffu) >> 2; len = 3; return 1; }
    if ((t & 2u) == 0) { off = (t & 0xffffu) >> 2; len = 3; return 2; }
    if ((t & 1u) == 0) { off = (t & 0xffffu) >> 6; len = ((t >> 2) & 15u) + 3; return 2; }
    if ((t & 127u) != 3) { off = (t >> 7) & 0x1ffffu; len = ((t >> 2) & 0x1fu) + 2; return 3; }
    off = t >> 15; len = ((t >> 7) & 255u) + 3; return 4;
}

// Token length from its first byte alone.
__device__ __forceinline__ uint32_t token_bytes(uint32_t b0) {
    if ((b0 & 3u) == 0) return 1;
    if ((b0 & 3u) != 3) return 2;
    return ((b0 & 127u) != 3) ? 3 : 4;
}

struct Header {
    uint32_t hdr, csize, dsize;
    bool compressed;
    uint32_t level;
};

__device__ __forceinline__ Header parse_header(const uint8_t *s) {
    Header h;
    const uint32_t b0 = s[0];
    h.hdr = (b0 & 2u) ? 9u : 3u;
    h.compressed = (b0 & 1u) != 0;
    h.level = (b0 >> 2) & 3u;
    if (h.hdr == 9) {
        h.csize = ld_u32_bytes(s + 1);
        h.dsize = ld_u32_bytes(s + 5);
    } else {
        h.csize = s[1];
        h.dsize = s[2];
    }
    return h;
}

}  // namespace qlzx
