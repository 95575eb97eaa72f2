// qlzx_crc.hip -- batched CRC32 (store/crc32.go:61-68 semantics) and the
// synthetic workload generator.
//
// CRC layout: one wavefront per buffer.  The buffer is cut into 4 KiB stripes;
// lane l owns bytes [64 l, 64 l + 64) of a stripe (4 x 16-B loads), runs the
// byte table from a zero state, and the 64 partial CRCs are merged with
// GF(2) shifts: crc(A||B) = shift(crc(A), |B|) ^ crc(B) for the raw (linear)
// state.  The initial state is folded in at the end: raw(B, s) =
// raw(B, 0) ^ shift(s, |B|).
#include "qlzx_device.h"

namespace qlzx {

constexpr uint32_t kStripe = 4096;
constexpr uint32_t kPiece = 64;

// CRC of one lane's piece of n bytes (n <= 64) at q, from state 0.  q is 4-aligned: the piece
// arrives as 16 dwords (four 16-B loads, all issued before any is used; dwords past n are
// clamped to the piece's last dword so nothing past the buffer is read), then slicing-by-8
// over its whole 8-B words and the table-driven byte step for the rest.
__device__ __forceinline__ uint32_t piece_crc_a4(const uint32_t *t8, const uint8_t *q, uint32_t n) {
    uint32_t w[16];
    const uint32_t *qw = (const uint32_t *)q;
    if (n == kPiece) {
        const uint4 *q4 = (const uint4 *)q;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const uint4 v = q4[k];
            w[4 * k] = v.x, w[4 * k + 1] = v.y, w[4 * k + 2] = v.z, w[4 * k + 3] = v.w;
        }
    } else {
        const uint32_t lastw = (n + 3) / 4 - 1;  // last dword holding a byte of the piece
#pragma unroll
        for (uint32_t k = 0; k < 16; k++) w[k] = qw[k < lastw ? k : lastw];
    }
    uint32_t c = 0;
#pragma unroll
    for (uint32_t k = 0; k < 16; k += 2)
        if (4 * k + 8 <= n) c = crc_slice8(t8, c, w[k], w[k + 1]);
    // the < 8 trailing bytes of a partial piece
    for (uint32_t b = n & ~7u; b < n; b++) c = crc_byte(t8, c, (w[b >> 2] >> (8 * (b & 3))) & 0xffu);
    return c;
}

// Raw CRC from state 0 of `len` bytes at p, wave-cooperative; all lanes return the result.
// t8 = slicing-by-8 tables in LDS.  Each 4 KiB stripe: lane l takes bytes [64 l, 64 l + 64)
// (piece_crc_a4 when p is 4-aligned), then crc(stripe) = XOR_l piece_crc_l * x^(8 * bytes
// after the piece) (one or two GF(2) products per lane from the g_crc_piece / g_crc_byte
// tables) and run = run * x^(8 * |stripe|) ^ crc(stripe).
__device__ uint32_t wave_crc_raw(const uint32_t *t8, const uint8_t *p, uint64_t len, uint32_t lane) {
    uint32_t run = 0;
    const bool al4 = (((uintptr_t)p) & 3u) == 0;
    for (uint64_t base = 0; base < len; base += kStripe) {
        const uint32_t slen = (uint32_t)((len - base) < kStripe ? (len - base) : kStripe);
        const uint32_t lo = lane * kPiece;
        const uint32_t mine = lo < slen ? ((slen - lo) < kPiece ? (slen - lo) : kPiece) : 0u;
        uint32_t c = 0;
        if (mine) {
            const uint8_t *q = p + base + lo;
            if (al4) c = piece_crc_a4(t8, q, mine);
            else for (uint32_t k = 0; k < mine; k++) c = crc_byte(t8, c, q[k]);
            // shift past the rest of the stripe: whole pieces, then bytes
            const uint32_t after = slen - lo - mine;
            if (after & 63u) c = gf2_mulmod(g_crc_byte[after & 63u], c);
            if (after >> 6) c = gf2_mulmod(g_crc_piece[after >> 6], c);
        }
        for (int m = 32; m >= 1; m >>= 1) c ^= __shfl_xor(c, m, 64);
        run = (base ? gf2_mulmod(crc_xpow_bytes(slen), run) : 0u) ^ c;
    }
    return run;
}

// ---- wave_crc: one wave, any length, the initial state folded into the data ----
// The buffer M (len bytes) is viewed as nst = ceil(len / 4 KiB) stripes of a virtual stream
// pad zeros ‖ M (pad < 4096 leading zeros: a raw CRC from state 0 is unchanged by them).  Lane
// l owns piece l (64 B) of every stripe and keeps ONE register for all its pieces: between
// stripes it skips the other lanes' 4032 bytes (x^(8*4032), one table multiply) and then runs
// slicing-by-8 over its next piece from that state.  A 6-level tree (x^(8*64*2^k)) merges the
// 64 registers at the end.  The initial state is XORed into M's first dword (for a reflected
// CRC, crc(s, M) = crc(0, M ^ s in bytes 0..3)), so there is no per-buffer shift.  Pieces are
// read as dwords at 4-aligned addresses and realigned with v_alignbyte when pad % 4 != 0.
constexpr uint32_t kCrcLdsWords = 8 * 256 + kMulTabs * 1024;  // slice8 tables, then g_crc_mul

__device__ __forceinline__ void load_crc_lds(uint32_t *lds) {
    for (uint32_t i = threadIdx.x; i < 8 * 256; i += blockDim.x) lds[i] = g_crc_slice8[i];
    for (uint32_t i = threadIdx.x; i < kMulTabs * 1024; i += blockDim.x) lds[8 * 256 + i] = g_crc_mul[i];
}

__device__ __forceinline__ uint32_t crc_mul_tab(const uint32_t *m, uint32_t c) {
    return m[c & 0xffu] ^ m[256 + ((c >> 8) & 0xffu)] ^ m[512 + ((c >> 16) & 0xffu)] ^ m[768 + (c >> 24)];
}

// CRC register after the len bytes at p from state init (no final inversion); every lane
// returns it.  lds = load_crc_lds's tables.  p need not be aligned: the dword view starts at
// p rounded down, the m = p % 4 bytes before p are masked to zero.
__device__ uint32_t wave_crc(const uint32_t *lds, const uint8_t *p, uint64_t len, uint32_t init, uint32_t lane) {
    const uint32_t *t8 = lds, *mul = lds + 8 * 256;
    if (len < 4) {
        uint32_t c = init;
        for (uint32_t b = 0; b < len; b++) c = crc_byte(t8, c, p[b]);
        return c;
    }
    const uint32_t m = (uint32_t)((uintptr_t)p & 3u);
    const uint32_t *w32 = (const uint32_t *)(p - m);
    const uint64_t nst = (len + kStripe - 1) / kStripe;
    const uint32_t pad = (uint32_t)(nst * kStripe - len);
    const uint32_t sh = (m - pad) & 3u;  // every piece starts sh bytes past a dword boundary
    const int64_t lastdw = (int64_t)((len + m - 1) >> 2);
    const uint64_t ini = (uint64_t)init << (8 * m);  // init over M's bytes 0..3 in the dword view
    const uint32_t keep0 = 0xffffffffu << (8 * m);    // dword 0: the bytes that belong to M
    uint32_t c = 0;
    for (uint64_t t = 0; t < nst; t++) {
        const int64_t a = (int64_t)(t * kStripe + kPiece * lane) - (int64_t)pad + m;  // in the dword view
        c = crc_mul_tab(mul + 6 * 1024, c);
        if (a + (int64_t)kPiece <= (int64_t)m) continue;  // the piece is all leading zeros
        const int64_t d0 = (a - (int64_t)sh) >> 2;
        uint32_t w[17];
        if (d0 >= 2 && d0 + 16 <= lastdw) {
            const uint4 *q4 = (const uint4 *)(w32 + d0);
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const uint4 v = q4[k];
                w[4 * k] = v.x, w[4 * k + 1] = v.y, w[4 * k + 2] = v.z, w[4 * k + 3] = v.w;
            }
            w[16] = sh ? w32[d0 + 16] : 0u;
        } else {  // the first or the last pieces: dwords outside [0, lastdw] read as 0
#pragma unroll
            for (int k = 0; k < 17; k++) {
                const int64_t i = d0 + k;
                uint32_t v = (i >= 0 && i <= lastdw) ? w32[i] : 0u;
                if (i == 0) v = (v & keep0) ^ (uint32_t)ini;
                if (i == 1) v ^= (uint32_t)(ini >> 32);
                w[k] = v;
            }
        }
        if (sh) {
#pragma unroll
            for (int k = 0; k < 16; k++) w[k] = __builtin_amdgcn_alignbyte(w[k + 1], w[k], sh);
        }
#pragma unroll
        for (int k = 0; k < 16; k += 2) c = crc_slice8(t8, c, w[k], w[k + 1]);
    }
#pragma unroll
    for (int k = 0; k < 6; k++) c = crc_mul_tab(mul + k * 1024, c) ^ __shfl_xor(c, 1 << k, 64);
    return __shfl(c, 0, 64);
}

// ---- wave_crc_rep: wave_crc with the byte table replicated across LDS banks ----
// Same layout, initial-state fold and lane-combine tree as wave_crc, but each lane runs its 64-B
// piece through ONE byte table (c = T[(c ^ b) & 0xff] ^ c >> 8) held R times over, lane l reading
// copy l % R: entry e of copy q sits at dword R e + q.  R = 4 (inside K2, in its 4 KiB window):
// bank q + 4 (e & 7) of the 32 a half-wave uses, eight lanes per copy over eight banks (R = 16
// would leave only lanes l and l + 16 to collide but needs 16 KiB).  slice8's eight tables serve
// random indices at about four conflicts per half-wave: the lookups, not the data, bound it (one
// lookup per byte either way).  mul = the g_crc_mul tables (LDS or global).  The two 32-B halves
// of a piece run as two independent chains (the lookups are a dependent-latency chain), joined
// through g_crc_mul32 (global).
// S4: tab holds the slicing-by-4 tables instead (g_crc_slice8[0..1023], 4 KiB, no copies): four
// independent lookups per dword instead of a chain of four, one VALU less per byte, more conflicts.
template <uint32_t R, bool S4 = false>
__device__ __forceinline__ uint32_t wave_crc_rep(const uint32_t *tab, const uint32_t *mul, const uint8_t *p, uint64_t len,
                                 uint32_t init, uint32_t lane) {
    const uint32_t *tr = S4 ? tab : tab + (lane & (R - 1));
    if (len < 4) {
        uint32_t c = init;
        for (uint32_t b = 0; b < len; b++) c = tr[((c ^ p[b]) & 0xffu) * (S4 ? 1u : R)] ^ (c >> 8);
        return c;
    }
    const uint32_t m = (uint32_t)((uintptr_t)p & 3u);
    const uint32_t *w32 = (const uint32_t *)(p - m);
    const uint64_t nst = (len + kStripe - 1) / kStripe;
    const uint32_t pad = (uint32_t)(nst * kStripe - len);
    const uint32_t sh = (m - pad) & 3u;
    const int64_t lastdw = (int64_t)((len + m - 1) >> 2);
    const uint64_t ini = (uint64_t)init << (8 * m);
    const uint32_t keep0 = 0xffffffffu << (8 * m);
    uint32_t c = 0;
    for (uint64_t t = 0; t < nst; t++) {
        const int64_t a = (int64_t)(t * kStripe + kPiece * lane) - (int64_t)pad + m;
        c = crc_mul_tab(mul + 6 * 1024, c);
        if (a + (int64_t)kPiece <= (int64_t)m) continue;
        const int64_t d0 = (a - (int64_t)sh) >> 2;
        uint32_t w[17];
        if (d0 >= 2 && d0 + 16 <= lastdw) {
            const uint4 *q4 = (const uint4 *)(w32 + d0);
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const uint4 v = q4[k];
                w[4 * k] = v.x, w[4 * k + 1] = v.y, w[4 * k + 2] = v.z, w[4 * k + 3] = v.w;
            }
            w[16] = sh ? w32[d0 + 16] : 0u;
        } else {
#pragma unroll
            for (int k = 0; k < 17; k++) {
                const int64_t i = d0 + k;
                uint32_t v = (i >= 0 && i <= lastdw) ? w32[i] : 0u;
                if (i == 0) v = (v & keep0) ^ (uint32_t)ini;
                if (i == 1) v ^= (uint32_t)(ini >> 32);
                w[k] = v;
            }
        }
        if (sh) {
#pragma unroll
            for (int k = 0; k < 16; k++) w[k] = __builtin_amdgcn_alignbyte(w[k + 1], w[k], sh);
        }
        uint32_t d = 0;
#pragma unroll
        for (int k = 0; k < 8; k++) {
            c ^= w[k];
            d ^= w[k + 8];
            if constexpr (S4) {
                c = tr[768 + (c & 0xffu)] ^ tr[512 + ((c >> 8) & 0xffu)] ^ tr[256 + ((c >> 16) & 0xffu)] ^ tr[c >> 24];
                d = tr[768 + (d & 0xffu)] ^ tr[512 + ((d >> 8) & 0xffu)] ^ tr[256 + ((d >> 16) & 0xffu)] ^ tr[d >> 24];
            } else {
#pragma unroll
                for (int b = 0; b < 4; b++) {
                    c = tr[(c & 0xffu) * R] ^ (c >> 8);
                    d = tr[(d & 0xffu) * R] ^ (d >> 8);
                }
            }
        }
        c = crc_mul_tab(g_crc_mul32, c) ^ d;
    }
#pragma unroll
    for (int k = 0; k < 6; k++) c = crc_mul_tab(mul + k * 1024, c) ^ __shfl_xor(c, 1 << k, 64);
    return __shfl(c, 0, 64);
}

#ifndef QLZX_K2_ONLY
__global__ void __launch_bounds__(256) k_crc32(const uint8_t *src, const uint64_t *off,
                                               const uint32_t *len, uint32_t n,
                                               const uint32_t *init, uint32_t final_xor,
                                               uint32_t *out) {
    __shared__ uint32_t tab[kCrcLdsWords];
    load_crc_lds(tab);
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t i = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
    if (i >= n) return;
    const uint32_t reg = wave_crc(tab, src + off[i], len[i], init ? init[i] : 0xffffffffu, lane);
    if (lane == 0) out[i] = reg ^ final_xor;
}
#endif  // QLZX_K2_ONLY

// ---------------- synthetic workloads ----------------
__device__ __forceinline__ uint64_t sm64(uint64_t &s) {
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
__device__ __forceinline__ uint64_t block_seed(uint64_t seed, uint64_t id) {
    uint64_t s = seed ^ (id * 0xD1B54A32D192ED03ull);
    return sm64(s);
}
__device__ __forceinline__ uint32_t zipf_pick(const uint32_t *cdf, uint32_t nw, uint32_t u) {
    uint32_t lo = 0, hi = nw - 1;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (cdf[mid] > u) hi = mid; else lo = mid + 1;
    }
    return lo;
}
__device__ void gen_text(uint64_t s, const uint8_t *vocab, const uint32_t *voff, const uint32_t *cdf,
                         uint32_t nw, uint8_t *out, uint32_t n) {
    uint32_t p = 0;
    while (p < n) {
        const uint64_t r = sm64(s);
        const uint32_t w = zipf_pick(cdf, nw, (uint32_t)r);
        for (uint32_t i = voff[w]; i < voff[w + 1] && p < n; i++) out[p++] = vocab[i];
        if ((uint32_t)(r >> 32) % 100u < 8u && p < n) out[p++] = '.';
        if (p < n) out[p++] = ' ';
    }
}
__device__ void gen_image(uint64_t s, const uint8_t *vocab, const uint32_t *voff, const uint32_t *cdf,
                          uint32_t nw, uint8_t *out, uint32_t n) {
    const uint64_t kind = sm64(s);
    if ((kind & 3) != 0) {
        for (uint32_t p = 0; p < n; p += 8) {
            const uint64_t r = sm64(s);
            for (uint32_t b = 0; b < 8 && p + b < n; b++) out[p + b] = (uint8_t)(r >> (8 * b));
        }
        return;
    }
    gen_text(sm64(s), vocab, voff, cdf, nw, out, n);
    const uint32_t pct = 40u + (uint32_t)((kind >> 8) % 6u);
    for (uint32_t p = 0; p < n; p++) {
        const uint64_t r = sm64(s);
        if ((uint32_t)r % 100u < pct) out[p] = (uint8_t)(r >> 32);
    }
}

#ifndef QLZX_K2_ONLY
__global__ void __launch_bounds__(64) k_synth(int kind, uint64_t seed, uint64_t first, uint8_t *dst,
                                              const uint64_t *off, const uint32_t *len, uint32_t n,
                                              const uint8_t *vocab, const uint32_t *voff,
                                              const uint32_t *cdf, uint32_t nw) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t s = block_seed(seed, first + i);
    if (kind == 0) gen_text(s, vocab, voff, cdf, nw, dst + off[i], len[i]);
    else gen_image(s, vocab, voff, cdf, nw, dst + off[i], len[i]);
}
#endif  // QLZX_K2_ONLY

}  // namespace qlzx
