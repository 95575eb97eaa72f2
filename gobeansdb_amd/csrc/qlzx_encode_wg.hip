// qlzx_encode_wg.hip -- position-parallel level-3 encoder, one workgroup per block.
//
// Bit-exact restatement of qlz_compress_core level 3 (quicklz.c:197-494) for
// blocks of up to QLZX_WG_MAX_LEN bytes, organised for CDNA4 instead of as the
// reference's serial loop.  The enabling fact: every position
// 0..size-11 is inserted into the hash table in position order, whether it is
// a literal, a match start or inside a match (quicklz.c:356-372).  So the
// candidate set at position p is a pure function of the input prefix: the d
// most recent earlier positions with the same 12-bit hash, d = min(c, 16) with
// c = (their count mod 256) (the u8 hash_counter and the c > k loop bound,
// quicklz.c:316-331).  The best match (longest, ties to the larger position,
// quicklz.c:344) can therefore be found for all positions at once; only the
// greedy parse that picks which positions emit items is sequential, and it is
// resolved by segment walkers with a fix-up pass.
//
// Per block (one workgroup, block + working set in LDS, input read once):
//   S. stored-block proof (incompressible input): a bound on the
//      bytes any parse could save, from a count of repeated 3-grams, shows the
//      bail-out test of quicklz.c:218 must fire -> emit the stored block.
//   0. input -> LDS.
//   1. stable partition of positions by bucket group (hash >> 4, 256 groups)
//      into a per-workgroup global scratch list (wave-ballot ranks).
//   2. each wave takes groups dynamically and walks the group's positions in
//      64-position batches with a 16-bucket x 16-slot ring (packed position +
//      upper 12 fetch bits, so the 3-byte compare needs no input read);
//      candidates from the same batch come from peer lanes (ballot match).
//      Result: best length per position in LDS, offset in global scratch.
//   3. greedy parse: one walker per 64-position segment, converged by
//      re-walking segments whose entry point changed (usually 1-2 rounds).
//   4. item sizes -> block scan -> bail-out test at control-word boundaries
//      (quicklz.c:216-219) -> emission of tokens, literals and control words.
//   5. fused CRC32 (store/crc32.go:61) of the emitted bytes, 4 KiB stripe per wave.
#include "qlzx_device.h"

#ifndef QLZX_WG_MAX_LEN
#define QLZX_WG_MAX_LEN 65536
#endif

namespace qlzx {

__device__ __forceinline__ uint32_t ld32u(const uint8_t *lds, uint32_t a) {
    const uint32_t *w = (const uint32_t *)(lds + (a & ~3u));
    return __builtin_amdgcn_alignbyte(w[1], w[0], a & 3u);
}
__device__ __forceinline__ uint32_t fetch24(const uint8_t *lds, uint32_t p) { return ld32u(lds, p) & 0xFFFFFFu; }
__device__ __forceinline__ uint32_t hash12(uint32_t f) { return ((f >> 12) ^ f) & (QLZX_BUCKETS - 1); }

// Lanes (within `act`) whose NB-bit key equals this lane's key.
template <int NB>
__device__ __forceinline__ uint64_t match_peers(uint32_t key, uint64_t act) {
    uint64_t m = act;
#pragma unroll
    for (int bi = 0; bi < NB; bi++) {
        const bool set = (key >> bi) & 1u;
        const uint64_t B = __ballot(set);
        m &= set ? B : ~B;
    }
    return m;
}

__device__ __forceinline__ uint64_t shfl_up64(uint64_t x, uint32_t d) {
    const uint32_t lo = __shfl_up((uint32_t)x, d, 64), hi = __shfl_up((uint32_t)(x >> 32), d, 64);
    return ((uint64_t)hi << 32) | lo;
}

// Exclusive block-wide scan of one u64 per thread (W waves); `total` = sum.
template <uint32_t W>
__device__ uint64_t block_scan_excl(uint64_t v, uint64_t *wsum, uint64_t &total) {
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint64_t x = v;
#pragma unroll
    for (uint32_t d = 1; d < 64; d <<= 1) {
        const uint64_t y = shfl_up64(x, d);
        if (lane >= d) x += y;
    }
    if (lane == 63) wsum[wave] = x;
    __syncthreads();
    uint64_t pre = 0, tot = 0;
#pragma unroll
    for (uint32_t w = 0; w < W; w++) {
        const uint64_t u = wsum[w];
        if (w < wave) pre += u;
        tot += u;
    }
    __syncthreads();
    total = tot;
    return pre + x - v;
}

// Level-3 match token (quicklz.c:377-406); returns its byte count.
__device__ __forceinline__ uint32_t token_of(uint32_t ml, uint32_t off, uint32_t &t) {
    if (ml == 3 && off <= 63) { t = off << 2; return 1; }
    if (ml == 3 && off <= 16383) { t = (off << 2) | 1u; return 2; }
    if (ml <= 18 && off <= 1023) { t = ((ml - 3) << 2) | (off << 6) | 2u; return 2; }
    if (ml <= 33) { t = ((ml - 2) << 2) | (off << 7) | 3u; return 3; }
    t = ((ml - 3) << 7) | (off << 15) | 3u;
    return 4;
}

// Stored-block proof ("incompressible blocks").  D = number of
// positions whose 3-gram hashes (h') to a value seen at another position: an
// upper bound on the positions whose 3-gram repeats an earlier one.  Any match
// of length L covers L-2 such positions, so every parse saves at most 2D bytes
// and spends at most 2D extra input bytes per control word; with T = 3(n>>2),
// the first control word past T then exists inside the main loop and fails
// the ratio test of quicklz.c:218 whenever both inequalities hold.
__host__ __device__ inline bool stored_proof(uint32_t n, uint32_t D) {
    const uint64_t T = 3ull * (n >> 2);
    return 2ull * D + 31 + T + 11 <= n && 70ull * D < 4ull * (T + 1) + 31ull * ((T + 1) >> 5);
}

constexpr uint32_t kEncGroups = 256;  // bucket groups (hash >> 4), 16 buckets each

template <uint32_t CAP>
struct WgCfg {
    static constexpr uint32_t T = CAP / 64;  // threads = walkers (one 64-position segment each)
    static constexpr uint32_t W = T / 64;    // waves
    static constexpr uint32_t IN_B = CAP + 64;
    static constexpr uint32_t L8_B = (CAP + 64) > 8192 ? CAP + 64 : 8192;  // reused for CRC tables
    static constexpr uint32_t U_B = IN_B + L8_B;                          // s_in | s_l8
    static constexpr uint32_t BM_LOG2 = CAP >= 65536 ? 20 : (CAP >= 16384 ? 18 : 16);  // proof bitmap bits
    static constexpr uint32_t NCW = (CAP + 30) / 31;
    static constexpr uint32_t SC1 = kEncGroups * W;  // phase 1 counters
    static constexpr uint32_t SC2 = W * (256 + 16);  // phase 2 rings + counters
    static constexpr uint32_t SC4 = 2 * NCW;         // phase 4 control words + positions
    static constexpr uint32_t SC12 = SC1 > SC2 ? SC1 : SC2;
    static constexpr uint32_t SCR = SC12 > SC4 ? SC12 : SC4;
    static constexpr size_t SLOT_BYTES = (size_t)CAP * 4;  // gpos u16[CAP] + goff u16[CAP]
    static_assert((1u << BM_LOG2) / 8 <= U_B, "proof bitmap overlays s_in|s_l8");
};

template <uint32_t CAP>
__global__ void __launch_bounds__(CAP / 64) k_encode_wg(qlzx_blocks b, uint32_t *csize_out, int32_t *status,
                                                         const uint32_t *crc_state, uint32_t *crc_out,
                                                         uint8_t *ws) {
    using C = WgCfg<CAP>;
    constexpr uint32_t T = C::T, W = C::W;
    __shared__ __attribute__((aligned(16))) uint8_t s_u[C::U_B];
    __shared__ __attribute__((aligned(16))) uint32_t s_scr[C::SCR];
    __shared__ uint32_t s_gstart[kEncGroups + 1];
    __shared__ uint64_t s_wsum[W];
    __shared__ uint32_t s_misc[24];  // [0] next group, [1] proof count, [4..] CRC stripes
    uint8_t *const s_in = s_u, *const s_l8 = s_u + C::IN_B;

    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint64_t ltm = (1ull << lane) - 1ull;
    uint16_t *gpos = (uint16_t *)(ws + (size_t)blockIdx.x * C::SLOT_BYTES);
    uint16_t *goff = gpos + CAP;

    for (uint32_t i = blockIdx.x; i < b.n; i += gridDim.x) {
        const uint32_t n = b.src_len[i];
        __syncthreads();        // LDS of the previous block is free
        if (n > CAP) continue;  // general (lane) path
        if (n == 0) {           // cquicklz.go:36 panics on &src[0]
            if (tid == 0) {
                csize_out[i] = 0;
                if (status) status[i] = QLZX_E_EMPTY;
                if (crc_state && crc_out) crc_out[i] = ~crc_state[i];
            }
            continue;
        }
        uint8_t *dst = b.dst + b.dst_off[i];
        const uint8_t *src = b.src + b.src_off[i];
        const uint32_t hdr = n < 216 ? 3u : 9u;  // quicklz.c:708-711
        if (tid == 0) {
            s_misc[0] = 0;
            s_misc[1] = 0;
        }
        bool stored = false;

        // ---- S. stored-block proof on incompressible input ----
        if (n >= 256 && (((uintptr_t)src) & 15u) == 0) {
            uint32_t *bm = (uint32_t *)s_u;
            constexpr uint32_t BMW = (1u << C::BM_LOG2) / 32;
            for (uint32_t k = tid * 4; k < BMW; k += T * 4) *(uint4 *)(bm + k) = make_uint4(0, 0, 0, 0);
            __syncthreads();
            uint32_t dup = 0;
            const uint32_t ny = n - 2;  // positions holding a whole 3-gram
            for (uint32_t y0 = tid * 16; y0 < ny; y0 += T * 16) {
                uint32_t w[5];
                if (y0 + 20 <= n) {
                    const uint4 v = *(const uint4 *)(src + y0);
                    w[0] = v.x, w[1] = v.y, w[2] = v.z, w[3] = v.w;
                    w[4] = *(const uint32_t *)(src + y0 + 16);
                } else {
#pragma unroll
                    for (int j = 0; j < 5; j++) {
                        uint32_t x = 0;
                        for (int k = 0; k < 4; k++) {
                            const uint32_t o = y0 + 4 * j + k;
                            x |= (o < n ? (uint32_t)src[o] : 0u) << (8 * k);
                        }
                        w[j] = x;
                    }
                }
#pragma unroll 4
                for (uint32_t j = 0; j < 16; j++) {
                    if (y0 + j < ny) {
                        const uint32_t f = __builtin_amdgcn_alignbyte(w[j / 4 + 1], w[j / 4], j & 3) & 0xFFFFFFu;
                        const uint32_t h = (f * 0x9E3779B1u) >> (32 - C::BM_LOG2);
                        const uint32_t bit = 1u << (h & 31u);
                        dup += (atomicOr(&bm[h >> 5], bit) & bit) ? 1u : 0u;
                    }
                }
            }
            for (int m = 32; m >= 1; m >>= 1) dup += __shfl_xor(dup, m, 64);
            if (lane == 0) atomicAdd(&s_misc[1], dup);
            __syncthreads();
            stored = stored_proof(n, s_misc[1]);
            if (stored) {  // quicklz.c:722-727 from the global copy of the input
                if ((((uintptr_t)dst) & 3u) == 0) {
                    const uint32_t tot = n + hdr, a0 = (hdr + 3u) & ~3u;
                    for (uint32_t o = a0 + tid * 4; o + 4 <= tot; o += T * 4)
                        *(uint32_t *)(dst + o) = *(const uint32_t *)(src + o - hdr);  // unaligned load
                    for (uint32_t o = hdr + tid; o < tot; o += T)
                        if (o < a0 || o >= (tot & ~3u)) dst[o] = src[o - hdr];
                } else {
                    for (uint32_t o = tid; o < n; o += T) dst[hdr + o] = src[o];
                }
                if (tid == 0) write_header(dst, hdr, false, n + hdr, n);
            }
            __syncthreads();  // the bitmap region becomes s_in / s_l8
        }

        uint32_t csz = n + hdr;
        if (!stored) {
            // ---- 0. input -> LDS (zero padded for word over-reads) ----
            if ((((uintptr_t)src) & 15u) == 0) {
                for (uint32_t o = tid * 16; o < n; o += T * 16) {
                    if (o + 16 <= n) *(uint4 *)(s_in + o) = *(const uint4 *)(src + o);
                    else for (uint32_t k = o; k < n; k++) s_in[k] = src[k];
                }
            } else {
                for (uint32_t o = tid; o < n; o += T) s_in[o] = src[o];
            }
            for (uint32_t o = n + tid; o < ((n + 15u) & ~15u) + 48u; o += T) s_in[o] = 0;
            const uint32_t P = n >= 11 ? n - 10 : 0;  // searched positions: 0 .. size-11 (quicklz.c:204)
            __syncthreads();

            if (P) {
                // ---- 1. stable partition of positions by bucket group ----
                uint32_t *cnt1 = s_scr;  // [group * W + wave]
                for (uint32_t k = tid; k < kEncGroups * W; k += T) cnt1[k] = 0;
                const uint32_t per = (P + 64 * W - 1) / (64 * W) * 64;
                const uint32_t r0 = min(P, wave * per), r1 = min(P, r0 + per);
                __syncthreads();
                for (uint32_t base = r0; base < r1; base += 64) {
                    const uint32_t p = base + lane;
                    if (p < r1) atomicAdd(&cnt1[(hash12(fetch24(s_in, p)) >> 4) * W + wave], 1u);
                }
                __syncthreads();
                {
                    uint32_t v[4];
                    uint32_t sum = 0;
#pragma unroll
                    for (int j = 0; j < 4; j++) {
                        v[j] = cnt1[4 * tid + j];
                        sum += v[j];
                    }
                    uint64_t tot;
                    uint32_t ex = (uint32_t)block_scan_excl<W>(sum, s_wsum, tot);
#pragma unroll
                    for (int j = 0; j < 4; j++) {
                        cnt1[4 * tid + j] = ex;
                        ex += v[j];
                    }
                }
                __syncthreads();
                for (uint32_t g = tid; g < kEncGroups; g += T) s_gstart[g] = cnt1[g * W];
                if (tid == 0) s_gstart[kEncGroups] = P;
                __syncthreads();
                for (uint32_t base = r0; base < r1; base += 64) {  // wave-uniform
                    const uint32_t p = base + lane;
                    const bool valid = p < r1;
                    const uint32_t g = valid ? hash12(fetch24(s_in, p)) >> 4 : 0u;
                    const uint64_t peers = match_peers<8>(g, __ballot(valid));
                    const uint32_t intra = __popcll(peers & ltm);
                    uint32_t cur = 0;
                    if (valid) cur = cnt1[g * W + wave];
                    // every lane's read is issued before the leader's write (in-order LDS per wave)
                    if (valid && intra == 0) cnt1[g * W + wave] = cur + (uint32_t)__popcll(peers);
                    if (valid) gpos[cur + intra] = (uint16_t)p;
                }
                __syncthreads();

                // ---- 2. best match per position, group by group ----
                uint32_t *ring = s_scr + wave * (256 + 16);  // [bucket(16)][slot(16)] = pos | fetch[23:12] << 16
                uint32_t *cntb = ring + 256;                  // hash_counter (mod 256) per bucket
                for (;;) {
                    uint32_t g = 0;
                    if (lane == 0) g = atomicAdd(&s_misc[0], 1u);
                    g = __shfl(g, 0, 64);
                    if (g >= kEncGroups) break;
                    const uint32_t gs = s_gstart[g], ge = s_gstart[g + 1];
                    if (gs == ge) continue;
                    if (lane < 16) cntb[lane] = 0;
                    for (uint32_t base = gs; base < ge; base += 64) {  // wave-uniform
                        const uint32_t j = base + lane;
                        const bool valid = j < ge;
                        const uint32_t p = valid ? (uint32_t)gpos[j] : 0u;
                        const uint32_t f = valid ? fetch24(s_in, p) : 0u;
                        const uint32_t bk = hash12(f) & 15u, fh = f >> 12;
                        const uint64_t peers = match_peers<4>(bk, __ballot(valid));
                        const uint64_t below = peers & ltm;
                        const uint32_t intra = __popcll(below);
                        const uint32_t above = (uint32_t)__popcll(peers & ~ltm) - (valid ? 1u : 0u);
                        const uint32_t c0 = valid ? cntb[bk] : 0u;
                        const uint32_t r = c0 + intra;  // this position's insertion index (mod 256)
                        const uint32_t rm = r & 255u;
                        const uint32_t d = valid ? (rm < 16u ? rm : 16u) : 0u;  // candidates (c > k bound)
                        const uint32_t dr = d > intra ? d - intra : 0u;        // of them in the ring
                        const uint32_t limit = valid ? min(255u, n - 4u - p) : 0u;  // quicklz.c:310
                        const uint32_t packed = p | (fh << 16);
                        uint32_t best = 0, bpos = 0;
                        // ring candidates: insertion ranks c0-dr .. c0-1 live in slots rank & 15
                        uint32_t fm = 0;
                        if (__ballot(dr != 0)) {
                            const uint4 *row = (const uint4 *)(ring + bk * 16);
#pragma unroll 1
                            for (uint32_t q4 = 0; q4 < 4; q4++) {
                                const uint4 v = row[q4];
                                const uint32_t e[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
                                for (uint32_t t = 0; t < 4; t++) {
                                    const uint32_t s = 4 * q4 + t;
                                    const bool ok = ((e[t] ^ (fh << 16)) < 0x10000u) && (((c0 - 1u - s) & 15u) < dr);
                                    fm |= ok ? (1u << s) : 0u;
                                }
                            }
                        }
                        // same-batch candidates (peer lanes, most recent first), then the ring
                        uint64_t tmp = below;
                        uint32_t kk = 0;
                        for (;;) {
                            const bool use_intra = tmp != 0 && kk < d;
                            if (__ballot(use_intra || fm != 0) == 0) break;
                            uint32_t ei = 0;
                            if (__ballot(use_intra)) {
                                const int sl = use_intra ? 63 - __builtin_clzll(tmp) : (int)lane;
                                ei = __shfl(packed, sl, 64);
                                if (use_intra) tmp &= ~(1ull << sl);
                            }
                            uint32_t q = 0xFFFFFFFFu;
                            if (use_intra) {
                                kk++;
                                if ((ei >> 16) == fh) q = ei & 0xFFFFu;
                            } else if (fm) {
                                const uint32_t s = __builtin_ctz(fm);
                                fm &= fm - 1;
                                q = ring[bk * 16 + s] & 0xFFFFu;
                            }
                            // quicklz.c:318-354: longest match, ties to the larger position
                            // (candidates arrive in no particular order); o < src - MINOFFSET.
                            // A lower position than the best so far must be strictly longer.
                            if (q != 0xFFFFFFFFu && q + 3u <= p &&
                                (best == 0 || q > bpos || (best < limit && s_in[q + best] == s_in[p + best]))) {
                                uint32_t m = 3;
                                for (;;) {
                                    const uint32_t x = ld32u(s_in, q + m) ^ ld32u(s_in, p + m);
                                    if (x) {
                                        m += (uint32_t)__builtin_ctz(x) >> 3;
                                        break;
                                    }
                                    m += 4;
                                    if (m >= limit) break;
                                }
                                if (m > limit) m = limit;
                                if (m > best || (m == best && q > bpos)) {
                                    best = m;
                                    bpos = q;
                                }
                            }
                        }
                        if (valid) {
                            s_l8[p] = (uint8_t)best;  // 0 = literal, else 3..255
                            if (best) goff[p] = (uint16_t)(p - bpos);
                            if (above < 16u) ring[bk * 16 + (r & 15u)] = packed;  // quicklz.c:356-358
                            if (above == 0u) cntb[bk] = (r + 1u) & 255u;
                        }
                    }
                }
            }
            __syncthreads();

            // ---- 3. greedy parse (quicklz.c:361-372,449-485): segment walkers + fix-up ----
            const uint32_t nseg = (n + 63) / 64;
            const uint32_t s0 = tid * 64, e0 = min(n, s0 + 64);
            uint64_t bits = 0;
            uint32_t from = s0, xit = s0;
            uint32_t *ex = s_scr;
            auto walk = [&](uint32_t a) {
                uint64_t bb = 0;
                uint32_t p = a;
                while (p < e0) {  // 8 positions per LDS read; literal stretches skip ahead
                    const uint32_t pa = p & ~7u, sh = p - pa;
                    uint64_t w = *(const uint64_t *)(s_l8 + pa) >> (8 * sh);
                    const uint32_t span = min(8u - sh, e0 - p);
                    if (span < 8) w &= (1ull << (8 * span)) - 1ull;
                    if (p + span > P) {  // positions >= P are never searched (tail literals)
                        const uint32_t keep = P > p ? P - p : 0u;
                        w = keep ? (w & ((1ull << (8 * keep)) - 1ull)) : 0ull;
                    }
                    if (w == 0) {
                        bb |= ((1ull << span) - 1ull) << (p - s0);
                        p += span;
                    } else {
                        const uint32_t z = (uint32_t)__builtin_ctzll(w) >> 3;
                        bb |= ((1ull << (z + 1)) - 1ull) << (p - s0);
                        p += z + (uint32_t)((w >> (8 * z)) & 0xFFu);
                    }
                }
                bits = bb;
                return p;
            };
            // round 0 walks every segment from its own start; later rounds re-walk (or trim)
            // the segments whose entry, the exit of the segment before, changed
            for (uint32_t round = 0;; round++) {
                uint32_t entry = s0;
                if (round) {
                    __syncthreads();
                    entry = (tid == 0 || tid >= nseg) ? from : ex[tid - 1];
                    __syncthreads();
                }
                int changed = 0;
                if (tid < nseg && (round == 0 || entry != from)) {
                    uint32_t nx;
                    if (entry >= e0) {  // a match covers the whole segment
                        bits = 0;
                        nx = entry;
                    } else if (round && entry > from && ((bits >> (entry - s0)) & 1ull)) {  // paths merge
                        bits &= ~((1ull << (entry - s0)) - 1ull);
                        nx = xit;
                    } else {
                        nx = walk(entry);
                    }
                    from = entry;
                    if (round == 0 || nx != xit) {
                        xit = nx;
                        ex[tid] = nx;
                        changed = 1;
                    }
                }
                if (!__syncthreads_or(changed)) break;
            }

            // ---- 4. sizes, bail-out test, emission ----
            uint32_t items = 0, bytes = 0;
            if (tid < nseg) {
                items = __popcll(bits);
                for (uint64_t t = bits; t; t &= t - 1) {
                    const uint32_t p = s0 + (uint32_t)__builtin_ctzll(t);
                    const uint32_t L = p < P ? (uint32_t)s_l8[p] : 0u;
                    uint32_t tk;
                    bytes += L ? token_of(L, goff[p], tk) : 1u;
                }
            }
            uint64_t tot;
            const uint64_t exs = block_scan_excl<W>(((uint64_t)items << 32) | bytes, s_wsum, tot);
            const uint32_t I0 = (uint32_t)(exs >> 32), B0 = (uint32_t)exs;
            const uint32_t Itot = (uint32_t)(tot >> 32), Btot = (uint32_t)tot;
            int bail = 0;
            if (tid < nseg) {  // quicklz.c:216-219: at each new control word inside the main loop
                uint32_t idx = I0, bb = B0;
                for (uint64_t t = bits; t; t &= t - 1) {
                    const uint32_t p = s0 + (uint32_t)__builtin_ctzll(t);
                    const uint32_t L = p < P ? (uint32_t)s_l8[p] : 0u;
                    uint32_t tk;
                    const uint32_t sz = L ? token_of(L, goff[p], tk) : 1u;
                    if (idx && idx % 31u == 0 && p < P) {
                        const uint32_t op = 4u * (idx / 31u) + bb;
                        if (p > 3u * (n >> 2) && op > p - (p >> 5)) bail = 1;
                    }
                    idx++;
                    bb += sz;
                }
            }
            bail = __syncthreads_or(bail);
            if (bail) {  // stored block (quicklz.c:722-727)
                for (uint32_t o = tid; o < n; o += T) dst[hdr + o] = s_in[o];
                if (tid == 0) write_header(dst, hdr, false, n + hdr, n);
                csz = n + hdr;
            } else {
                const uint32_t ncw = (Itot + 30) / 31;
                uint32_t core = 4 * ncw + Btot;
                uint32_t *cw = s_scr, *cwpos = s_scr + C::NCW;
                for (uint32_t c = tid; c < ncw; c += T) cw[c] = 0;
                __syncthreads();
                if (tid < nseg) {
                    uint32_t idx = I0, bb = B0;
                    for (uint64_t t = bits; t; t &= t - 1) {
                        const uint32_t p = s0 + (uint32_t)__builtin_ctzll(t);
                        const uint32_t L = p < P ? (uint32_t)s_l8[p] : 0u;
                        const uint32_t c = idx / 31u, bit = idx % 31u;
                        const uint32_t op = hdr + 4u * (c + 1u) + bb;
                        if (bit == 0) cwpos[c] = op - 4u;
                        if (L) {
                            uint32_t tk;
                            const uint32_t sz = token_of(L, goff[p], tk);
                            atomicOr(&cw[c], 1u << bit);
                            for (uint32_t k = 0; k < sz; k++) dst[op + k] = (uint8_t)(tk >> (8 * k));
                            bb += sz;
                        } else {
                            dst[op] = s_in[p];
                            bb += 1;
                        }
                        idx++;
                    }
                }
                __syncthreads();
                for (uint32_t c = tid; c < ncw; c += T) st32(dst + cwpos[c], cw[c] | 0x80000000u);
                if (core < 9) {  // quicklz.c:493: 9-byte core minimum, zero filled
                    for (uint32_t o = core + tid; o < 9; o += T) dst[hdr + o] = 0;
                    core = 9;
                }
                if (tid == 0) write_header(dst, hdr, true, core + hdr, n);
                csz = core + hdr;
            }
        }

        // ---- 5. fused CRC of the emitted value (store/crc32.go:61-68) ----
        if (crc_state && crc_out) {
            __syncthreads();  // emitted bytes visible to the whole workgroup
            uint32_t *t8 = (uint32_t *)s_l8;
            load_crc_slice8(t8);
            __syncthreads();
            const uint32_t nst = (csz + 4095) / 4096;
            for (uint32_t st = wave; st < nst; st += W) {
                const uint32_t len = min(4096u, csz - st * 4096);
                const uint32_t raw = wave_crc_raw(t8, dst + (size_t)st * 4096, len, lane);
                if (lane == 0) s_misc[4 + st] = raw;
            }
            __syncthreads();
            if (tid == 0) {
                uint32_t run = crc_state[i];
                for (uint32_t st = 0; st < nst; st++) {
                    const uint32_t len = min(4096u, csz - st * 4096);
                    run = (len == 4096 ? gf2_mulmod(g_crc_pow[12], run) : crc_shift(run, len)) ^ s_misc[4 + st];
                }
                crc_out[i] = ~run;
            }
        }
        if (tid == 0) {
            csize_out[i] = csz;
            if (status) status[i] = QLZX_OK;
        }
    }
}

inline bool encode_wg_enabled() { return true; }

inline uint32_t encode_wg_cap(uint32_t max_len) {
    if (max_len > QLZX_WG_MAX_LEN) max_len = QLZX_WG_MAX_LEN;
    return max_len <= 4096 ? 4096u : (max_len <= 16384 ? 16384u : 65536u);
}
// Persistent workgroups per class: LDS-bound residency x 256 CUs.
inline uint32_t encode_wg_slots(uint32_t cap) { return cap == 65536 ? 256u : (cap == 16384 ? 1024u : 2560u); }

inline size_t encode_wg_ws_bytes(uint32_t n, uint32_t max_len) {
    const uint32_t cap = encode_wg_cap(max_len);
    const uint32_t slots = std::min<uint32_t>(std::max<uint32_t>(n, 1), encode_wg_slots(cap));
    return (size_t)slots * cap * 4;
}

inline int launch_encode_wg(const qlzx_blocks &b, uint32_t *csize, int32_t *status, const uint32_t *crc_state,
                            uint32_t *crc_out, uint32_t max_len, uint32_t flags, void *ws, hipStream_t s) {
    (void)flags;
    const uint32_t cap = encode_wg_cap(max_len);
    const uint32_t grid = std::min<uint32_t>(b.n, encode_wg_slots(cap));
    if (grid == 0) return 0;
    uint8_t *w = (uint8_t *)ws;
    if (cap == 4096)
        hipLaunchKernelGGL(k_encode_wg<4096>, dim3(grid), dim3(64), 0, s, b, csize, status, crc_state, crc_out, w);
    else if (cap == 16384)
        hipLaunchKernelGGL(k_encode_wg<16384>, dim3(grid), dim3(256), 0, s, b, csize, status, crc_state, crc_out, w);
    else
        hipLaunchKernelGGL(k_encode_wg<65536>, dim3(grid), dim3(1024), 0, s, b, csize, status, crc_state, crc_out, w);
    return (int)hipGetLastError();
}

}  // namespace qlzx
