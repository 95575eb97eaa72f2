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
// Per block (one workgroup, block + working set in LDS, input read once;
// blocks are handed to persistent workgroups by a global ticket counter):
//   S. stored-block proof (incompressible input): a bound on the
//      bytes any parse could save, from a count of repeated 3-gram hashes
//      (bitmap of no-return LDS ORs, then a popcount), shows the bail-out test
//      of quicklz.c:218 must fire -> emit the stored block.
//   0. input -> LDS.
//   1. the searched positions sorted by 12-bit bucket, stable in position
//      (two LSD radix passes: low 4 hash bits, then the bucket group), into a
//      per-workgroup global scratch list, plus each bucket's start in it.
//   2. every position in parallel: its candidates are the preceding <= 16
//      entries of its bucket in the sorted list; longest match wins, ties to
//      the larger position.  No per-bucket serial walk, so a block whose
//      positions all share one bucket (zeros, runs) spreads like any other.
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

// The thread index behind an opaque move.  Read afresh in every phase, so the compiler cannot hoist
// tid-derived addresses and lane masks out of the persistent block loop and keep them live (the
// 64 KiB kernel sits at the 128-VGPR cap of a 1024-thread workgroup: they were what it spilled).
__device__ __forceinline__ uint32_t tid_here() {
    uint32_t t;
    asm volatile("v_mov_b32 %0, %1" : "=v"(t) : "v"((uint32_t)threadIdx.x));
    return t;
}

// An opaque zero: a constant zero register pair or quad is otherwise hoisted out of the block
// loop and spilled rather than rematerialised.
__device__ __forceinline__ uint32_t zero_here() {
    uint32_t z;
    asm volatile("v_mov_b32 %0, 0" : "=v"(z));
    return z;
}

__device__ __forceinline__ uint32_t ld32u(const uint8_t *lds, uint32_t a) {
    const uint32_t *w = (const uint32_t *)(lds + (a & ~3u));
    return __builtin_amdgcn_alignbyte(w[1], w[0], a & 3u);
}
__device__ __forceinline__ uint32_t fetch24(const uint8_t *lds, uint32_t p) { return ld32u(lds, p) & 0xFFFFFFu; }
__device__ __forceinline__ uint32_t hash12(uint32_t f) { return ((f >> 12) ^ f) & (QLZX_BUCKETS - 1); }

// Lanes (within `act`) whose NB-bit key equals this lane's key.
// Per key bit: an all-ones / zero lane mask from one sign-extending bit extract, the ballot of
// it, and m &= ~(B ^ mask) on each 32-bit half (one three-input bit op each; the select form
// `set ? B : ~B` compiled to nine VALU ops per bit).
template <int NB>
__device__ __forceinline__ uint64_t match_peers(uint32_t key, uint64_t act) {
    uint32_t lo = (uint32_t)act, hi = (uint32_t)(act >> 32);
#pragma unroll
    for (int bi = 0; bi < NB; bi++) {
        const uint32_t sm = (uint32_t)((int32_t)(key << (31 - bi)) >> 31);  // all ones iff bit bi set
        const uint64_t B = __ballot(sm != 0u);
        lo &= ~((uint32_t)B ^ sm);
        hi &= ~((uint32_t)(B >> 32) ^ sm);
    }
    return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ uint64_t shfl_up64(uint64_t x, uint32_t d) {
    const uint32_t lo = __shfl_up((uint32_t)x, d, 64), hi = __shfl_up((uint32_t)(x >> 32), d, 64);
    return ((uint64_t)hi << 32) | lo;
}

// Exclusive block-wide scan of one u64 per thread (W waves); `total` = sum.
template <uint32_t W>
__device__ uint64_t block_scan_excl(uint64_t v, uint64_t *wsum, uint64_t &total) {
    const uint32_t tid0 = tid_here(), lane = tid0 & 63, wave = tid0 >> 6;
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

// Position (0..63) of the r-th set bit of x (r < popcount(x)), by halving.
__device__ __forceinline__ uint32_t select64(uint64_t x, uint32_t r) {
    uint32_t pos = 0;
#pragma unroll
    for (uint32_t w = 32; w >= 1; w >>= 1) {
        const uint32_t c = (uint32_t)__popcll(x & ((1ull << w) - 1ull));
        if (r >= c) {
            r -= c;
            x >>= w;
            pos += w;
        }
    }
    return pos;
}

// Sum of the first r 2-bit fields of the 64-item code array sc[4] (16 fields per word).
__device__ __forceinline__ uint32_t fields2_prefix(const uint32_t sc[4], uint32_t r) {
    uint32_t s = 0;
#pragma unroll
    for (uint32_t q = 0; q < 4; q++) {
        const uint32_t lim = r > 16 * q ? min(r - 16 * q, 16u) : 0u;  // fields of word q below r
        const uint32_t w = sc[q] & (lim >= 16 ? 0xFFFFFFFFu : ((1u << (2 * lim)) - 1u));
        s += (uint32_t)__popc(w & 0x55555555u) + 2u * (uint32_t)__popc(w & 0xAAAAAAAAu);
    }
    return s;
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
// Prefix-first pass (phase 4): blocks of >= kPrefixMinLen bytes whose 3-gram repeat count (the
// stored proof's D) is below kPrefixRepeatPct % of their positions parse only the positions below
// 3/4 of the input + kPrefixMargin first.  On the c3 noisy blocks (40-45 % random bytes) 256 of
// the 263 in 387 that end stored bail out at that first test, within 53 B of 3/4 of the input
// (instrumented oracle), and D < 28 % flags them with 3 false positives.
constexpr bool kSpecCopy = true;
constexpr bool kPrefixPass = true;
// Best match in poorly compressible blocks (3-gram repeats, the stored proof's D, below
// kCompactPct % of the positions; 0 = never): a wave whose lanes all have at most
// kMatchCompactMax candidates that can match (same 3 bytes, far enough back) visits only those,
// in a per-lane bit loop, instead of all 16.
constexpr uint32_t kCompactPct = 60;
constexpr uint32_t kMatchCompactN = 10;
constexpr uint32_t kMatchCompactMax = kMatchCompactN;
// Stored proof: 16-position steps per thread whose input loads are issued together.
constexpr uint32_t kProofSteps = 4;
// Bail-out after a parse: reuse the stored proof's speculative copy (only the edges written).
constexpr bool kBailSpec = true;
// Radix scatter: 64-element batches per iteration whose list loads are in flight together (the
// second pass; the first reads no list).
constexpr uint32_t kScatterU = 4;
// Best match: sorted entries staged in LDS for this many consecutive 64-entry steps of a wave per
// global-load wait (1 = one step per wait, the steps of a wave T entries apart).
constexpr uint32_t kMatchStage = 4;
// Bucket starts of the 64 KiB kernel in LDS (8 KiB) rather than in the workgroup's global slot.
constexpr bool kBstLds = true;
constexpr uint32_t kPrefixPct = 28;
constexpr uint32_t kPrefixMarginB = 1024;
constexpr uint32_t kPrefixMinLen = kPrefixPass ? 16384 : 0xFFFFFFFFu, kPrefixRepeatPct = kPrefixPct,
                   kPrefixMargin = kPrefixMarginB;
constexpr uint32_t kParseRounds = 4;  // segment-walker rounds before the serial item walk

// One pass of a stable LSD radix partition of the searched positions by
// NB_LOG2 bits of their hash (starting at bit `shift`): out[] lists the
// positions of in[] (or 0..P-1) grouped by key, each group in input order.
// Each wave owns a contiguous input range; counters are [key][wave] so the
// exclusive scan over them is stable.  cnt holds (1 << NB_LOG2) * W words.
//   hist      (nullable) u16-pair histogram of the full 12-bit hash, counted
//             in this pass's count loop (bucket starts, bucket_sort)
//   next_cnt  (nullable) [key'][wave'] counts of the NEXT pass (key' = hash >> 4,
//             wave' = the wave owning the output index), accumulated while
//             scattering so the next pass needs no count loop
//   counted   cnt already holds this pass's counts (from the previous scatter)
// Counter slot of logical counter L = key * W + wave: one padding word per key row, so the
// lanes of one wave (same wave, different keys) hit different LDS banks.  Without it a
// 16-wave workgroup's row stride of 16 words put all 64 lanes on 4 banks.
template <uint32_t W>
__device__ __forceinline__ uint32_t cslot(uint32_t L) {
    return L + L / W;
}
constexpr uint32_t cslots(uint32_t nkeys, uint32_t W) { return nkeys * (W + 1); }

template <uint32_t W, uint32_t NB_LOG2, typename OUT>
__device__ void stable_partition(const uint8_t *s_in, uint32_t P, const uint16_t *in, OUT *out, uint32_t shift,
                                 uint32_t *cnt, uint64_t *wsum, unsigned long long *sub, uint32_t *hist,
                                 uint32_t *next_cnt, bool counted) {
#ifdef QLZX_PROFILE
#define SUB_MARK(k)                                                         \
    do {                                                                    \
        if (sub) {                                                          \
            const unsigned long long _n = __builtin_amdgcn_s_memtime();     \
            sub[k] += _n - sub[7];                                          \
            sub[7] = _n;                                                    \
        }                                                                   \
    } while (0)
#else
#define SUB_MARK(k) do { } while (0)
#endif
    constexpr uint32_t T = 64 * W, NB = 1u << NB_LOG2, NC = NB * W;
    constexpr uint32_t CPT = NC >= T ? NC / T : 1;  // counters per scanning thread
    static_assert(NC % CPT == 0 && NC / CPT <= T, "counter layout");
    const uint32_t tid = tid_here(), lane = tid & 63, wave = tid >> 6;
    const uint64_t ltm = (1ull << lane) - 1ull;
    const uint32_t per = (P + 64 * W - 1) / (64 * W) * 64;
    const uint32_t r0 = min(P, wave * per), r1 = min(P, r0 + per);
    const uint32_t per_magic = 0xFFFFFFFFu / per + 1u;  // umulhi(x, per_magic) = x / per for x < 2^16
    constexpr uint32_t U = sizeof(OUT) == 4 ? kScatterU : 4;  // 64-element batches per iteration
    SUB_MARK(0);
    if (!counted) {
        for (uint32_t k = tid; k < cslots(NB, W); k += T) cnt[k] = 0;
        __syncthreads();
        for (uint32_t base = r0; base < r1; base += 64 * U) {
            uint32_t pv[U];
#pragma unroll
            for (uint32_t u = 0; u < U; u++) {
                const uint32_t j = base + 64 * u + lane;
                pv[u] = j < r1 ? (in ? (uint32_t)in[j] : j) : 0u;
            }
#pragma unroll
            for (uint32_t u = 0; u < U; u++) {
                if (base + 64 * u + lane < r1) {
                    const uint32_t h = hash12(fetch24(s_in, pv[u]));
                    atomicAdd(&cnt[cslot<W>(((h >> shift) & (NB - 1)) * W + wave)], 1u);
                    if (hist) atomicAdd(&hist[h >> 1], 1u << (16 * (h & 1u)));
                }
            }
        }
        __syncthreads();
    }
    SUB_MARK(1);  // count
    {
        const bool own = tid * CPT < NC;
        uint32_t v[CPT];
        uint32_t sum = 0;
#pragma unroll
        for (uint32_t j = 0; j < CPT; j++) {
            v[j] = own ? cnt[cslot<W>(CPT * tid + j)] : 0u;
            sum += v[j];
        }
        uint64_t tot;
        uint32_t ex = (uint32_t)block_scan_excl<W>(sum, wsum, tot);
        if (own) {
#pragma unroll
            for (uint32_t j = 0; j < CPT; j++) {
                cnt[cslot<W>(CPT * tid + j)] = ex;
                ex += v[j];
            }
        }
    }
    __syncthreads();
    SUB_MARK(2);  // scan
    for (uint32_t base0 = r0; base0 < r1; base0 += 64 * U) {  // wave-uniform
      uint32_t pv[U];
#pragma unroll
      for (uint32_t u = 0; u < U; u++) {
          const uint32_t j = base0 + 64 * u + lane;
          pv[u] = j < r1 ? (in ? (uint32_t)in[j] : j) : 0u;
      }
#pragma unroll
      for (uint32_t u = 0; u < U; u++) {
        const uint32_t j = base0 + 64 * u + lane;
        const bool valid = j < r1;
        const uint32_t p = pv[u];
        const uint32_t f = fetch24(s_in, p);
        const uint32_t h = hash12(f);
        const uint32_t key = valid ? (h >> shift) & (NB - 1) : 0u;
        const uint64_t peers = match_peers<NB_LOG2>(key, __ballot(valid));
        const uint32_t intra = __popcll(peers & ltm);
        uint32_t cur = 0;
        if (valid) cur = cnt[cslot<W>(key * W + wave)];
        // every lane's read is issued before the leader's write (in-order LDS per wave)
        if (valid && intra == 0) cnt[cslot<W>(key * W + wave)] = cur + (uint32_t)__popcll(peers);
        if (valid) {
            out[cur + intra] = (OUT)(sizeof(OUT) == 2 ? p : p | ((f >> 12) << 16));
            if (next_cnt) atomicAdd(&next_cnt[cslot<W>((h >> 4) * W + __umulhi(cur + intra, per_magic))], 1u);
        }
      }
    }
    __syncthreads();
    SUB_MARK(3);  // scatter
}

// Searched positions sorted by 12-bit bucket, stable in position (two LSD radix
// passes: low 4 hash bits, then the bucket group), as gl[t] = pos | fetch[23:12] << 16,
// plus bst[h] = the sorted index where bucket h starts (exclusive scan of the
// bucket histogram counted in the first pass).  tmp: u16[P] scratch; s_hist:
// 2048 words of LDS free during the sort; s_cnt: 272 * (W + 1) words.
template <uint32_t W, uint32_t L8_BYTES>
__device__ void bucket_sort(const uint8_t *s_in, uint32_t P, uint16_t *tmp, uint32_t *gl, uint16_t *bst,
                            uint32_t *s_cnt, uint32_t *s_hist, uint64_t *wsum, unsigned long long *subA,
                            unsigned long long *subB) {
    constexpr uint32_t T = 64 * W;
    const uint32_t tid = tid_here();
    uint32_t *cntB = s_cnt, *cntA = s_cnt + cslots(kEncGroups, W);
    // LDS peer slots after the histogram, where the workgroup's LDS has room for them
    for (uint32_t k = tid; k < QLZX_BUCKETS / 2; k += T) s_hist[k] = 0;
    for (uint32_t k = tid; k < cslots(kEncGroups, W); k += T) cntB[k] = 0;
    // (pass A zeroes its own counters and syncs before counting)
    stable_partition<W, 4>(s_in, P, nullptr, tmp, 0, cntA, wsum, subA, s_hist, cntB, false);
    // bucket starts: exclusive scan of the u16-pair histogram, bucket order = sorted order
    {
        constexpr uint32_t PT = QLZX_BUCKETS / 2 / T > 0 ? QLZX_BUCKETS / 2 / T : 1;  // words per thread
        const bool own = tid * PT < QLZX_BUCKETS / 2;
        uint32_t sum = 0;
        if (own)
            for (uint32_t j = 0; j < PT; j++) {
                const uint32_t w = s_hist[tid * PT + j];
                sum += (w & 0xFFFFu) + (w >> 16);
            }
        uint64_t tot;
        uint32_t ex = (uint32_t)block_scan_excl<W>(sum, wsum, tot);
        if (own)
            for (uint32_t j = 0; j < PT; j++) {
                const uint32_t w = s_hist[tid * PT + j], h0 = 2 * (tid * PT + j);
                bst[h0] = (uint16_t)ex;
                ex += w & 0xFFFFu;
                bst[h0 + 1] = (uint16_t)ex;
                ex += w >> 16;
            }
    }
#ifdef QLZX_PROFILE
    if (subB) subB[7] = __builtin_amdgcn_s_memtime();
#endif
    stable_partition<W, 8>(s_in, P, tmp, gl, 4, cntB, wsum, subB, nullptr, nullptr, true);
}

template <uint32_t CAP>
struct WgCfg {
    static constexpr uint32_t T = CAP / 64;  // threads = walkers (one 64-position segment each)
    static constexpr uint32_t W = T / 64;    // waves
    static constexpr uint32_t IN_B = CAP + 64;
    static constexpr uint32_t L8_B = (CAP + 64) > 8192 ? CAP + 64 : 8192;  // reused for CRC tables
    static constexpr uint32_t U_B = IN_B + L8_B;                          // s_in | s_l8
    static constexpr uint32_t BM_LOG2 = CAP >= 65536 ? 20 : (CAP >= 16384 ? 18 : 16);  // proof bitmap bits
    static constexpr uint32_t NCW = (CAP + 30) / 31;
    static constexpr uint32_t SC1 = cslots(kEncGroups + 16, W);  // phase 1 counters (both radix passes)
    static constexpr uint32_t SC4 = 2 * NCW;         // phase 4 control words + positions
    static constexpr uint32_t SC3 = (T + 2) + 2 * T;  // phase 3 exits + serial-walk segment bits
    static constexpr uint32_t SCR = SC1 > SC4 ? (SC1 > SC3 ? SC1 : SC3) : (SC4 > SC3 ? SC4 : SC3);
    // gl u32[CAP] (sorted positions | fetch[23:12] << 16) | goff u16[CAP] | bst u16[4096]
    static constexpr size_t SLOT_BYTES = (size_t)CAP * 6 + QLZX_BUCKETS * 2;
    static_assert((1u << BM_LOG2) / 8 <= U_B, "proof bitmap overlays s_in|s_l8");
};

// Next block for a persistent workgroup: one ticket per block from a global
// counter (blocks differ in cost by 100x: stored-proof vs full parse), so the
// expensive ones spread over the workgroups instead of a static stride.
__device__ __forceinline__ uint32_t next_block(uint32_t *ticket, uint32_t *s_slot) {
    __syncthreads();  // every thread has read the previous ticket
    if (tid_here() == 0) *s_slot = atomicAdd(ticket, 1u);
    __syncthreads();
    return __builtin_amdgcn_readfirstlane(*s_slot);  // uniform: the block's pointers and sizes in SGPRs
}

template <uint32_t CAP>
__global__ void __launch_bounds__(CAP / 64) k_encode_wg(qlzx_blocks b, uint32_t *csize_out, int32_t *status,
                                                         const uint32_t *crc_state, uint32_t *crc_out,
                                                         uint8_t *ws, uint32_t *ticket) {
    using C = WgCfg<CAP>;
    constexpr uint32_t T = C::T, W = C::W;
    __shared__ __attribute__((aligned(16))) uint8_t s_u[C::U_B];
    __shared__ __attribute__((aligned(16))) uint32_t s_scr[C::SCR];
    __shared__ uint64_t s_wsum[W];
    __shared__ uint32_t s_misc[24];  // [0] next group, [1] proof count, [4..] CRC stripes
    constexpr bool BL = kBstLds && CAP == 65536;  // (the smaller kernels' occupancy is LDS-bound)
    __shared__ uint16_t s_bst[BL ? QLZX_BUCKETS : 1];
    uint8_t *const s_in = s_u, *const s_l8 = s_u + C::IN_B;

    uint32_t *gl = (uint32_t *)(ws + (size_t)blockIdx.x * C::SLOT_BYTES);
    uint16_t *goff = (uint16_t *)(gl + CAP);
    uint16_t *bst = BL ? s_bst : goff + CAP;  // sorted-list start of each bucket

    PROF_DECL
#ifdef QLZX_PROFILE
    unsigned long long _pacc_sub[16] = {};
#endif
    for (uint32_t i = next_block(ticket, &s_misc[22]); i < b.n; i = next_block(ticket, &s_misc[22])) {
        uint32_t tid = tid_here(), lane = tid & 63, wave = tid >> 6;
#define QLZX_TID_REFRESH() (tid = tid_here(), lane = tid & 63, wave = tid >> 6)
        const uint32_t n = b.src_len[i];  // LDS of the previous block is free (next_block synced)
        if (n > CAP) continue;            // general (lane) path
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
            const uint32_t z = zero_here();
            s_misc[0] = z;
            s_misc[1] = z;
        }
        bool stored = false;
        bool prefix = false;  // try the prefix-only pass first (below, phase 4)
        bool cmode = false;   // compact best-match loop (phase 2)
        bool spec = false;    // the proof wrote the stored value's aligned 16-B chunks

        PROF_MARK(0);  // 0: ticket + setup
        QLZX_TID_REFRESH();
        // ---- S. stored-block proof on incompressible input ----
        if (n >= 256 && (((uintptr_t)src) & 15u) == 0) {
            uint32_t *bm = (uint32_t *)s_u;
            constexpr uint32_t BMW = (1u << C::BM_LOG2) / 32;
            const uint32_t z0 = zero_here();
            for (uint32_t k = tid * 4; k < BMW; k += T * 4) *(uint4 *)(bm + k) = make_uint4(z0, z0, z0, z0);
            __syncthreads();
            const uint32_t ny = n - 2;  // positions holding a whole 3-gram
            auto load20 = [&](uint32_t y0, uint32_t w[6]) {  // w[5] only with kSpecCopy
                if (y0 + 24 <= n) {
                    const uint4 v = *(const uint4 *)(src + y0);
                    w[0] = v.x, w[1] = v.y, w[2] = v.z, w[3] = v.w;
                    w[4] = *(const uint32_t *)(src + y0 + 16);
                    if (kSpecCopy) w[5] = *(const uint32_t *)(src + y0 + 20);
                } else {
#pragma unroll
                    for (int j = 0; j < (kSpecCopy ? 6 : 5); j++) {
                        uint32_t x = 0;
                        for (int k = 0; k < 4; k++) {
                            const uint32_t o = y0 + 4 * j + k;
                            x |= (o < n ? (uint32_t)src[o] : 0u) << (8 * k);
                        }
                        w[j] = x;
                    }
                }
            };
            auto mark16 = [&](uint32_t y0, const uint32_t w[6]) {
                // fully unrolled (w[] indices static: a partial unroll turned every w[j / 4] into a
                // select chain); the per-position range test only in the block's last piece
                if (y0 + 16 <= ny) {
#pragma unroll
                    for (uint32_t j = 0; j < 16; j++) {
                        const uint32_t f = __builtin_amdgcn_alignbyte(w[j / 4 + 1], w[j / 4], j & 3) & 0xFFFFFFu;
                        const uint32_t h = (f * 0x9E3779B1u) >> (32 - C::BM_LOG2);
                        atomicOr(&bm[h >> 5], 1u << (h & 31u));  // no return: D = ny - distinct hashes
                    }
                } else {
#pragma unroll
                    for (uint32_t j = 0; j < 16; j++) {
                        if (y0 + j < ny) {
                            const uint32_t f = __builtin_amdgcn_alignbyte(w[j / 4 + 1], w[j / 4], j & 3) & 0xFFFFFFu;
                            const uint32_t h = (f * 0x9E3779B1u) >> (32 - C::BM_LOG2);
                            atomicOr(&bm[h >> 5], 1u << (h & 31u));
                        }
                    }
                }
            };
            // Speculative stored copy: most blocks the proof sees end stored, and the proof already
            // has their bytes in registers, so the 16-B destination chunks [16, a1) of the stored
            // value (header + input: chunk o holds input bytes o - 9 ..) go out now, each from the
            // window of the step 16 bytes before it.  A block that is not stored overwrites them
            // (its output is shorter; dst capacity is >= n + 400).
            spec = kSpecCopy && hdr == 9 && (((uintptr_t)dst) & 15u) == 0;
            const uint32_t sa1 = (n + hdr) & ~15u;
            auto spec16 = [&](uint32_t y0, const uint32_t w[6]) {
                if (spec && y0 + 32 <= sa1)
                    *(uint4 *)(dst + y0 + 16) = make_uint4(
                        __builtin_amdgcn_alignbyte(w[2], w[1], 3), __builtin_amdgcn_alignbyte(w[3], w[2], 3),
                        __builtin_amdgcn_alignbyte(w[4], w[3], 3), __builtin_amdgcn_alignbyte(w[5], w[4], 3));
            };
            // kProofSteps 16-position steps per iteration (4: a whole block of any class
            // in one iteration), every load in flight before any step is hashed
            constexpr uint32_t PS = kProofSteps;
            for (uint32_t y0 = tid * 16; y0 < ny; y0 += PS * T * 16) {
                uint32_t w[PS][6];
#pragma unroll
                for (uint32_t j = 0; j < PS; j++) {
#pragma unroll
                    for (uint32_t k = 0; k < 6; k++) w[j][k] = 0;
                    if (y0 + j * T * 16 < ny) load20(y0 + j * T * 16, w[j]);
                }
#pragma unroll
                for (uint32_t j = 0; j < PS; j++) {
                    if (y0 + j * T * 16 < ny) {
                        mark16(y0 + j * T * 16, w[j]);
                        spec16(y0 + j * T * 16, w[j]);
                    }
                }
            }
            __syncthreads();
            uint32_t ones = 0;
            for (uint32_t k = tid * 4; k < BMW; k += T * 4) {
                const uint4 v = *(const uint4 *)(bm + k);
                ones += __popc(v.x) + __popc(v.y) + __popc(v.z) + __popc(v.w);
            }
            for (int m = 32; m >= 1; m >>= 1) ones += __shfl_xor(ones, m, 64);
            if (lane == 0) atomicAdd(&s_misc[1], ones);
            __syncthreads();
            stored = stored_proof(n, ny - s_misc[1]);
            // poorly compressible but not provably stored (the c3 noisy blocks): likely to bail out
            // at the first control word past 3/4 of the input, so try the prefix alone first
            prefix = !stored && n >= kPrefixMinLen && 100ull * (ny - s_misc[1]) < (uint64_t)kPrefixRepeatPct * ny;
            cmode = !stored && 100ull * (ny - s_misc[1]) < (uint64_t)kCompactPct * ny;
            if (stored) {  // quicklz.c:722-727 from the global copy of the input
                QLZX_TID_REFRESH();
                if ((((uintptr_t)dst) & 15u) == 0) {
                    // 16 B per thread per step, four steps' loads in flight before any store
                    // (one dependent load per step made the copy latency-bound: 70 K cycles)
                    const uint32_t tot = n + hdr, a0 = (hdr + 15u) & ~15u, a1 = tot & ~15u;
                    constexpr uint32_t K = 4;
                    for (uint32_t o0 = a0 + tid * 16; o0 < (spec ? a0 : a1); o0 += T * 16 * K) {  // spec: done
                        uint4 v[K];
#pragma unroll
                        for (uint32_t k = 0; k < K; k++) {
                            const uint32_t o = min(o0 + k * T * 16, a1 - 16);  // clamped: loads unconditional
                            const uint32_t *q = (const uint32_t *)(src + o - hdr);  // unaligned loads
                            v[k] = make_uint4(q[0], q[1], q[2], q[3]);
                        }
#pragma unroll
                        for (uint32_t k = 0; k < K; k++)
                            if (o0 + k * T * 16 < a1) *(uint4 *)(dst + o0 + k * T * 16) = v[k];
                    }
                    for (uint32_t o = hdr + tid; o < tot; o += T)
                        if (o < a0 || o >= a1) dst[o] = src[o - hdr];
                } else if ((((uintptr_t)dst) & 3u) == 0) {
                    const uint32_t tot = n + hdr, a0 = (hdr + 3u) & ~3u;
                    for (uint32_t o = a0 + tid * 4; o + 4 <= tot; o += T * 4)
                        *(uint32_t *)(dst + o) = *(const uint32_t *)(src + o - hdr);  // unaligned load
                    for (uint32_t o = hdr + tid; o < tot; o += T)
                        if (o < a0 || o >= (tot & ~3u)) dst[o] = src[o - hdr];
                } else {
                    for (uint32_t o = tid; o < n; o += T) dst[hdr + o] = src[o];
                }
                if (tid == 0) write_header(dst + zero_here(), hdr, false, (n + hdr) | zero_here(), n | zero_here());
            }
            __syncthreads();  // the bitmap region becomes s_in / s_l8
        }

        uint32_t csz = n + hdr;
        if (!stored) {
            // ---- 0. input -> LDS (zero padded for word over-reads) ----
            QLZX_TID_REFRESH();
            if ((((uintptr_t)src) & 15u) == 0) {
                for (uint32_t o = tid * 16; o < n; o += T * 16) {
                    if (o + 16 <= n) *(uint4 *)(s_in + o) = *(const uint4 *)(src + o);
                    else for (uint32_t k = o; k < n; k++) s_in[k] = src[k];
                }
            } else {
                for (uint32_t o = tid; o < n; o += T) s_in[o] = src[o];
            }
            for (uint32_t o = n + tid; o < ((n + 15u) & ~15u) + 48u; o += T) s_in[o] = 0;
            const uint32_t Pfull = n >= 11 ? n - 10 : 0;  // searched positions: 0 .. size-11 (quicklz.c:204)
            __syncthreads();
          // Pass 0 (prefix): only the positions below T + kPrefixMargin are sorted, matched and
          // parsed -- their candidates are earlier positions, so their best matches are exact --
          // and only the first bail-out test past T (quicklz.c:216-219, T = 3 (n >> 2)) is
          // evaluated.  If it fires the block is stored; otherwise (or if that test is not inside
          // the prefix) pass 1 does the whole block.
          for (;;) {
            const uint32_t P = prefix ? min(Pfull, 3u * (n >> 2) + kPrefixMargin) : Pfull;
            if (P) {
                PROF_MARK(1);  // 1: proof + input load
                QLZX_TID_REFRESH();
                // ---- 1. positions sorted by bucket, stable: LSD radix on the low 4 hash
                //         bits, then on the bucket group (hash >> 4) ----
#ifdef QLZX_PROFILE
                unsigned long long *subA = _pacc_sub, *subB = _pacc_sub + 8;
                subA[7] = subB[7] = __builtin_amdgcn_s_memtime();
#else
                unsigned long long *subA = nullptr, *subB = nullptr;
#endif
                bucket_sort<W, C::L8_B>(s_in, P, goff, gl, bst, s_scr, (uint32_t *)s_l8, s_wsum, subA, subB);

                PROF_MARK(2);  // 2: sort by bucket
                QLZX_TID_REFRESH();
                // ---- 2. best match per position, all positions in parallel ----
                // The candidates of the position at sorted index t are the d most recent
                // earlier positions of its bucket -- sorted indices t-1 .. t-d -- with
                // d = min(rank mod 256, 16) (u8 hash_counter, c > k bound, quicklz.c:316-331).
                // Longest wins, ties to the larger position (quicklz.c:344): scanning from
                // the most recent, a candidate must be strictly longer, and a match of the
                // full extension limit ends the scan.
                // The candidates of the wave's 64 consecutive sorted indices are the 16 entries
                // before the first and the wave's own: each list entry is loaded from global
                // memory once per wave-iteration into an 80-word LDS stage (s_scr is free between
                // the sort and the parse) and the 16 candidate reads per position are LDS reads
                // of consecutive words, not 16 global loads.
                // With kMatchStage = S > 1 a wave takes S consecutive steps (64 S entries)
                // at a time: their S + 1 list loads are issued together and waited for once.
                constexpr uint32_t S = kMatchStage, SW = 64 * S + 16;
                static_assert(C::SCR >= SW * W, "candidate stage");
                uint32_t *const stg0 = s_scr + wave * SW;
                auto best_matches = [&](auto compact) {
                  for (uint32_t tb = (tid - lane) * S; tb < P; tb += T * S) {  // wave-uniform
                    if (S > 1) {
                        uint32_t v[S];
#pragma unroll
                        for (uint32_t u = 0; u < S; u++) v[u] = tb + 64 * u + lane < P ? gl[tb + 64 * u + lane] : 0u;
                        const uint32_t halo = (lane < 16 && tb + lane >= 16) ? gl[tb + lane - 16] : 0u;
#pragma unroll
                        for (uint32_t u = 0; u < S; u++) stg0[16 + 64 * u + lane] = v[u];
                        if (lane < 16) stg0[lane] = halo;
                    }
                  for (uint32_t u = 0; u < S; u++) {  // wave-uniform
                    const uint32_t t0 = tb + 64 * u;
                    if (t0 >= P) break;
                    uint32_t *const stg = stg0 + 64 * u;
                    const uint32_t t = t0 + lane;
                    const bool act = t < P;
                    if (S == 1) {
                        const uint32_t self = act ? gl[t] : 0u;
                        const uint32_t halo = (lane < 16 && t0 + lane >= 16) ? gl[t0 + lane - 16] : 0u;
                        stg[16 + lane] = self;
                        if (lane < 16) stg[lane] = halo;
                    }
                    if (!act) continue;
                    const uint32_t self = stg[16 + lane];
                    const uint32_t p = self & 0xFFFFu;
                    const uint32_t rm = (t - (uint32_t)bst[hash12(fetch24(s_in, p))]) & 255u;
                    const uint32_t d = rm < 16u ? rm : 16u;
                    const uint32_t limit = min(255u, n - 4u - p);  // quicklz.c:310
                    // First pass: bytes 3..6 of every candidate against this position's, all
                    // LDS reads independent.  A mismatch there gives the exact length; the
                    // candidates equal through byte 6 ("long") are extended afterwards, most
                    // recent first -- they beat every short one, and ties stay with the more
                    // recent (larger) position.
                    const uint32_t P3 = ld32u(s_in, p + 3);
                    uint32_t best = 0, bpos = 0, longm = 0;
                    auto first = [&](uint32_t k, uint32_t q, bool ok) {
                        const uint32_t x = ld32u(s_in, q + 3) ^ P3;
                        const uint32_t m = min(x ? 3u + ((uint32_t)__builtin_ctz(x) >> 3) : 7u, limit);
                        if (ok && !x && limit > 7u) longm |= 1u << k;
                        else if (ok && m > best) {
                            best = m;
                            bpos = q;
                        }
                    };
                    // A candidate can match when it is in the bucket (k < d) with the same
                    // fetch[23:12] (same bucket + same fetch[23:12] = same 3 bytes) and
                    // o < src - MINOFFSET (q + 3 <= p): with fhs = fetch[23:12] << 16, the word
                    // c - fhs is q when the fetch bits agree and >= 2^16 otherwise, so one
                    // subtraction and one compare against p - 3 test both (no candidate at p < 3).
                    const uint32_t fhs = self & 0xFFFF0000u, lim3 = p - 3u;
                    const uint32_t dmask = p >= 3u ? (1u << d) - 1u : 0u;
                    if constexpr (decltype(compact)::value) {
                        uint32_t okm = 0;
#pragma unroll
                        for (uint32_t k = 0; k < 16; k++) {
                            const uint32_t c = stg[15u + lane - k];
                            okm |= (c - fhs <= lim3) ? 1u << k : 0u;
                        }
                        okm &= dmask;
                        if (__ballot((uint32_t)__popc(okm) > kMatchCompactMax) == 0ull) {  // wave-uniform
                            for (uint32_t t2 = okm; t2; t2 &= t2 - 1u) {  // set bits, most recent first
                                const uint32_t k = (uint32_t)__builtin_ctz(t2);
                                first(k, stg[15u + lane - k] & 0xFFFFu, true);
                            }
                        } else {
#pragma unroll
                            for (uint32_t k = 0; k < 16; k++) first(k, stg[15u + lane - k] & 0xFFFFu, (okm >> k) & 1u);
                        }
                    } else {
                        uint32_t cand[16];  // most recent first
#pragma unroll
                        for (uint32_t k = 0; k < 16; k++) cand[k] = stg[k < d ? 15u + lane - k : 16u + lane];
#pragma unroll
                        for (uint32_t k = 0; k < 16; k++)
                            first(k, cand[k] & 0xFFFFu, (((dmask >> k) & 1u) & (cand[k] - fhs <= lim3 ? 1u : 0u)) != 0u);
                    }
                    if (longm) best = 0;  // a long candidate always wins
                    while (longm && best < limit) {
                        const uint32_t k = (uint32_t)__builtin_ctz(longm);
                        longm &= longm - 1u;
                        const uint32_t q = stg[15u + lane - k] & 0xFFFFu;
                        uint32_t m = 7;
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
                        if (m > best) {
                            best = m;
                            bpos = q;
                        }
                    }
                    s_l8[p] = (uint8_t)best;  // 0 = literal, else 3..255
                    if (best) goff[p] = (uint16_t)(p - bpos);
                  }
                  }
                };
                if (cmode) best_matches(std::true_type{});
                else best_matches(std::false_type{});
            }
            __syncthreads();

            PROF_MARK(3);  // 3: best match per position
            QLZX_TID_REFRESH();
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
                if (round + 1 == kParseRounds) {
                    // Not converged: long matches carry the parse across many segments
                    // (runs, repeated stretches), one segment per round.  Such a parse has
                    // few items, so one lane walks it from the start in item steps.
                    uint64_t *sb = (uint64_t *)(s_scr + ((nseg + 1) & ~1u));
                    for (uint32_t k = tid; k < nseg; k += T) sb[k] = zero_here();
                    __syncthreads();
                    if (tid == 0) {
                        for (uint32_t p = 0; p < n;) {
                            sb[p >> 6] |= 1ull << (p & 63u);
                            const uint32_t L = p < P ? (uint32_t)s_l8[p] : 0u;
                            p += L ? L : 1u;
                        }
                    }
                    __syncthreads();
                    if (tid < nseg) bits = sb[tid];
                    break;
                }
            }

            PROF_MARK(4);  // 4: greedy parse
            QLZX_TID_REFRESH();
            // ---- 4. sizes, bail-out test, emission ----
            uint32_t items = 0, bytes = 0;
            uint32_t szc[4] = {0, 0, 0, 0};  // item sizes - 1, 2 bits per item of the segment (in order)
            if (tid < nseg) {
                items = __popcll(bits);
                // Literal items are one byte and leave their 2-bit size code 0, so only the match
                // items are visited: the segment's positions with a nonzero best length (64 bytes
                // of s_l8, a nonzero-byte mask per dword), below P, that are items.
                uint64_t nz = 0;
                const uint4 *l16 = (const uint4 *)(s_l8 + s0);  // s0 = 64 tid: 16-B aligned
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    const uint4 v = l16[q];
                    const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
                    for (int e = 0; e < 4; e++) {
                        const uint32_t w = w4[e];
                        const uint32_t hi = ((((w & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | w) & 0x80808080u) >> 7;
                        nz |= (uint64_t)((hi * 0x10204080u) >> 28) << (16 * q + 4 * e);  // bit b: byte b != 0
                    }
                }
                const uint32_t keep = P > s0 ? min(64u, P - s0) : 0u;  // positions >= P are never searched
                nz &= keep >= 64 ? ~0ull : ((1ull << keep) - 1ull);
                const uint64_t mm = bits & nz;
                bytes = items - (uint32_t)__popcll(mm);
                for (uint64_t t = mm; t;) {  // four matches per iteration: their offset loads overlap
                    uint32_t p4[4], L4[4], o4[4];
#pragma unroll
                    for (int u = 0; u < 4; u++) {
                        p4[u] = t ? s0 + (uint32_t)__builtin_ctzll(t) : 0xFFFFFFFFu;
                        t &= t - 1;
                        L4[u] = p4[u] != 0xFFFFFFFFu ? (uint32_t)s_l8[p4[u]] : 0u;
                        o4[u] = L4[u] ? (uint32_t)goff[p4[u]] : 0u;
                    }
#pragma unroll
                    for (int u = 0; u < 4; u++) {
                        if (p4[u] == 0xFFFFFFFFu) break;
                        uint32_t tk;
                        const uint32_t sz = token_of(L4[u], o4[u], tk);
                        const uint32_t j = (uint32_t)__popcll(bits & ((1ull << (p4[u] - s0)) - 1ull));  // item rank
                        bytes += sz;
                        szc[j >> 4] |= (sz - 1u) << (2 * (j & 15));
                    }
                }
            }
            uint64_t tot;
            const uint64_t exs = block_scan_excl<W>(((uint64_t)items << 32) | bytes, s_wsum, tot);
            const uint32_t I0 = (uint32_t)(exs >> 32), B0 = (uint32_t)exs;
            const uint32_t Itot = (uint32_t)(tot >> 32), Btot = (uint32_t)tot;
            int bail = 0;
            if (prefix) {
                // the first test past T, if the prefix holds it: min over threads of (p << 1 | fails)
                if (tid == 0) s_misc[2] = 0xFFFFFFFFu;
                __syncthreads();
                if (tid < nseg) {
                    // the segment's control-word items (global item index a multiple of 31): the
                    // r-th item sits at the r-th set bit of bits, after B0 + r + (its code sum) bytes
                    for (uint32_t idx = (I0 + 30u) / 31u * 31u; idx < I0 + items; idx += 31u) {
                        if (!idx) continue;
                        const uint32_t r = idx - I0, p = s0 + select64(bits, r);
                        if (p < P && p > 3u * (n >> 2)) {
                            const uint32_t op = 4u * (idx / 31u) + B0 + r + fields2_prefix(szc, r);
                            atomicMin(&s_misc[2], (p << 1) | (op > p - (p >> 5) ? 1u : 0u));
                            break;
                        }
                    }
                }
                __syncthreads();
                const uint32_t v = s_misc[2];
                __syncthreads();
                prefix = false;
                if (v == 0xFFFFFFFFu || !(v & 1u)) continue;  // not decided by the prefix: pass 1
                bail = 1;
            } else if (tid < nseg) {  // quicklz.c:216-219: at each new control word inside the main loop
                for (uint32_t idx = (I0 + 30u) / 31u * 31u; idx < I0 + items; idx += 31u) {
                    if (!idx) continue;
                    const uint32_t r = idx - I0, p = s0 + select64(bits, r);
                    if (p < P && p > 3u * (n >> 2)) {
                        const uint32_t op = 4u * (idx / 31u) + B0 + r + fields2_prefix(szc, r);
                        if (op > p - (p >> 5)) bail = 1;
                    }
                }
            }
            bail = __syncthreads_or(bail);
            if (bail) {  // stored block (quicklz.c:722-727)
                QLZX_TID_REFRESH();
                if ((((uintptr_t)dst) & 15u) == 0) {  // 16-B stores from the LDS copy of the input
                    const uint32_t tot = n + hdr, a0 = (hdr + 15u) & ~15u, a1 = tot & ~15u;
                    // a bail-out emits nothing before this point, so after a speculative copy
                    // only the edges are missing
                    for (uint32_t o = a0 + tid * 16; o < (spec && kBailSpec ? a0 : a1); o += T * 16) {
                        const uint32_t q = o - hdr;
                        *(uint4 *)(dst + o) = make_uint4(ld32u(s_in, q), ld32u(s_in, q + 4), ld32u(s_in, q + 8),
                                                         ld32u(s_in, q + 12));
                    }
                    for (uint32_t o = hdr + tid; o < tot; o += T)
                        if (o < a0 || o >= a1) dst[o] = s_in[o - hdr];
                } else {
                    for (uint32_t o = tid; o < n; o += T) dst[hdr + o] = s_in[o];
                }
                if (tid == 0) write_header(dst + zero_here(), hdr, false, (n + hdr) | zero_here(), n | zero_here());
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
                            uint8_t *o = dst + op;  // one address, immediate offsets
                            o[0] = (uint8_t)tk;
                            if (sz > 1) o[1] = (uint8_t)(tk >> 8);
                            if (sz > 2) o[2] = (uint8_t)(tk >> 16);
                            if (sz > 3) o[3] = (uint8_t)(tk >> 24);
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
                if (tid == 0) write_header(dst + zero_here(), hdr, true, core + hdr, n);
                csz = core + hdr;
            }
            break;
          }
        }

        PROF_MARK(5);  // 5: sizes/bail/emission (or stored copy)
        QLZX_TID_REFRESH();
        // ---- 5. fused CRC of the emitted value (store/crc32.go:61-68) ----
        if (crc_state && crc_out) {
            __syncthreads();  // emitted bytes visible to the whole workgroup
            uint32_t *t8 = (uint32_t *)s_l8;
            for (uint32_t k = tid; k < 8 * 256; k += T) t8[k] = g_crc_slice8[k];
            __syncthreads();
            const uint32_t nst = (csz + 4095) / 4096;
            for (uint32_t st = wave; st < nst; st += W) {
                const uint32_t len = min(4096u, csz - st * 4096);
                const uint32_t raw = wave_crc_raw(t8, dst + (size_t)st * 4096, len, lane);
                if (lane == 0) s_misc[4 + st] = raw;
            }
            __syncthreads();
            // Combine in one wave, every stripe at once: with L = the last stripe's length,
            //   raw = (state * x^(8*4096*(nst-1)) ^ XOR_{s<nst-1} raw_s * x^(8*4096*(nst-2-s))) * x^(8L)
            //         ^ raw_{nst-1}
            // (a stripe's CRC shifted over the bytes after it; the state over all of them).
            if (wave == 0) {
                // one GF(2) product per lane, operands selected (branches would run the lanes'
                // products one after another): lanes < nst - 1 the stripes, 63 the state, 62
                // x^(8L) for the last stripe's length L; then the one remaining product
                const uint32_t last = csz - (nst - 1) * 4096;  // 1..4096
                uint32_t a = 0, c = 0;
                if (lane + 1 < nst) a = g_crc_stripe[nst - 2 - lane], c = s_misc[4 + lane];
                if (lane == 63) a = g_crc_stripe[nst - 1], c = crc_state[i];
                if (lane == 62) a = g_crc_piece[last >> 6], c = g_crc_byte[last & 63];
                uint32_t v = gf2_mulmod(a, c);
                const uint32_t xp = last == 4096 ? g_crc_pow[12] : __shfl(v, 62, 64);
                if (lane == 62) v = 0;
                for (int m = 32; m >= 1; m >>= 1) v ^= __shfl_xor(v, m, 64);
                if (lane == 0) crc_out[i] = ~(gf2_mulmod(xp, v) ^ s_misc[4 + nst - 1]);
            }
        }
        PROF_MARK(6);  // 6: CRC
        if (tid == 0) {
            csize_out[i] = csz;
            if (status) status[i] = QLZX_OK;
        }
    }
#undef QLZX_TID_REFRESH
    PROF_FLUSH(2);
#ifdef QLZX_PROFILE
    if (g_prof && (threadIdx.x & 63) == 0)
        for (int _j = 0; _j < 16; _j++) atomicAdd(&g_prof[24 + _j], _pacc_sub[_j]);
#endif
}

inline bool encode_wg_enabled() { return true; }

inline uint32_t encode_wg_cap(uint32_t max_len) {
    if (max_len > QLZX_WG_MAX_LEN) max_len = QLZX_WG_MAX_LEN;
    return max_len <= 4096 ? 4096u : (max_len <= 16384 ? 16384u : 65536u);
}
// Persistent workgroups per class: LDS-bound residency x 256 CUs.
inline uint32_t encode_wg_slots(uint32_t cap) { return cap == 65536 ? 256u : (cap == 16384 ? 1024u : 2560u); }

inline size_t encode_wg_slot_bytes(uint32_t cap) {
    return cap == 4096 ? WgCfg<4096>::SLOT_BYTES : (cap == 16384 ? WgCfg<16384>::SLOT_BYTES : WgCfg<65536>::SLOT_BYTES);
}

// [ticket counter, 256 B][slot 0][slot 1]...
inline size_t encode_wg_ws_bytes(uint32_t n, uint32_t max_len) {
    const uint32_t cap = encode_wg_cap(max_len);
    const uint32_t slots = std::min<uint32_t>(std::max<uint32_t>(n, 1), encode_wg_slots(cap));
    return 256 + (size_t)slots * encode_wg_slot_bytes(cap);
}

inline int launch_encode_wg(const qlzx_blocks &b, uint32_t *csize, int32_t *status, const uint32_t *crc_state,
                            uint32_t *crc_out, uint32_t max_len, uint32_t flags, void *ws, hipStream_t s) {
    (void)flags;
    const uint32_t cap = encode_wg_cap(max_len);
    const uint32_t grid = std::min<uint32_t>(b.n, encode_wg_slots(cap));
    if (grid == 0) return 0;
    uint32_t *ticket = (uint32_t *)ws;
    uint8_t *w = (uint8_t *)ws + 256;
    hipError_t e = hipMemsetAsync(ticket, 0, sizeof(uint32_t), s);
    if (e != hipSuccess) return (int)e;
    if (cap == 4096)
        hipLaunchKernelGGL(k_encode_wg<4096>, dim3(grid), dim3(64), 0, s, b, csize, status, crc_state, crc_out, w,
                           ticket);
    else if (cap == 16384)
        hipLaunchKernelGGL(k_encode_wg<16384>, dim3(grid), dim3(256), 0, s, b, csize, status, crc_state, crc_out, w,
                           ticket);
    else
        hipLaunchKernelGGL(k_encode_wg<65536>, dim3(grid), dim3(1024), 0, s, b, csize, status, crc_state, crc_out, w,
                           ticket);
    return (int)hipGetLastError();
}

}  // namespace qlzx
