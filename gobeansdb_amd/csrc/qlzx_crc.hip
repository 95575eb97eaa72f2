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

// Raw CRC from state 0 of `len` bytes at p, wave-cooperative; all lanes return
// the result.  t8 = slicing-by-8 tables in LDS.  Full 4-KiB stripes: lane l
// runs slicing-by-8 over its 64-B piece (16-B loads when p is 4-aligned), then
// crc(stripe) = XOR_l piece_crc_l * x^(8*64*(63-l)) (one GF(2) product per
// lane, g_crc_piece) and run = run * x^(8*4096) ^ crc(stripe).  The last,
// partial stripe takes the byte path with a general shift.
__device__ uint32_t wave_crc_raw(const uint32_t *t8, const uint8_t *p, uint64_t len, uint32_t lane) {
    uint32_t run = 0;
    const bool al4 = (((uintptr_t)p) & 3u) == 0;
    const uint32_t kshift = g_crc_piece[63 - lane];
    const uint32_t kstripe = g_crc_pow[12];  // x^(8 * 4096)
    uint64_t base = 0;
    for (; base + kStripe <= len; base += kStripe) {
        const uint8_t *q = p + base + lane * kPiece;
        uint32_t c = 0;
        if (al4) {
            const uint32_t *w = (const uint32_t *)q;
#pragma unroll
            for (int k = 0; k < 16; k += 2) c = crc_slice8(t8, c, w[k], w[k + 1]);
        } else {
            for (uint32_t k = 0; k < kPiece; k++) c = crc_byte(t8, c, q[k]);
        }
        c = gf2_mulmod(kshift, c);
        for (int m = 32; m >= 1; m >>= 1) c ^= __shfl_xor(c, m, 64);
        run = gf2_mulmod(kstripe, run) ^ c;
    }
    if (base < len) {  // partial stripe
        const uint32_t slen = (uint32_t)(len - base);
        const uint32_t lo = lane * kPiece;
        uint32_t c = 0;
        if (lo < slen) {
            const uint32_t mine = (slen - lo) < kPiece ? (slen - lo) : kPiece;
            const uint8_t *q = p + base + lo;
            for (uint32_t k = 0; k < mine; k++) c = crc_byte(t8, c, q[k]);
            c = crc_shift(c, slen - lo - mine);
        }
        for (int m = 32; m >= 1; m >>= 1) c ^= __shfl_xor(c, m, 64);
        run = crc_shift(run, slen) ^ c;
    }
    return run;
}

__global__ void __launch_bounds__(256) k_crc32(const uint8_t *src, const uint64_t *off,
                                               const uint32_t *len, uint32_t n,
                                               const uint32_t *init, uint32_t final_xor,
                                               uint32_t *out) {
    __shared__ uint32_t tab[8 * 256];
    load_crc_slice8(tab);
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t i = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
    if (i >= n) return;
    const uint32_t l = len[i];
    const uint32_t raw = wave_crc_raw(tab, src + off[i], l, lane);
    const uint32_t s = init ? init[i] : 0xffffffffu;
    if (lane == 0) out[i] = (raw ^ crc_shift(s, l)) ^ final_xor;
}

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

}  // namespace qlzx
