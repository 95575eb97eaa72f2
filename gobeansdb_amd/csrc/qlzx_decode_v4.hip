// qlzx_decode_v4.hip -- the batch decoder pair (dsize <= QLZX_FAST_MAX_DSIZE):
//
// K1 k_dec_parse6 (round 5)  one LANE per block: the serial control-word chain of
//     quicklz.c:513-671, one item STEP at a time (a literal run and the match that ends it, or a
//     control word), reading only control words and the first byte of each match token from a
//     per-lane LDS ring the lane refills itself.  The remaining control bits are kept with their
//     sentinel (cwr; 1 = group exhausted), so the item index is clz(cwr) and a literal run is
//     ctz(cwr): no per-item counters.  Emits one GroupRec {ip, cw, a, b} per control word (a, b:
//     bit-planes of token bytes - 1).
//
// K2 k_dec_chunk4  one WAVE per block, 64 items per batch and 256 output bytes per chunk:
//     * ITEM PHASE: token position from the GroupRec, branch-free token decode, DPP scan of the
//       output lengths; item i leaves ONE u32 key (d << 16 | off) in a 256-entry marker ring
//       at slot d (off = 0 for a literal, whose byte also goes to the output window);
//     * CHUNK PHASE: lane l owns bytes c + 4l .. c + 4l + 3.  The keys grow with d, so the
//       forward fill of "the item covering byte p" is a max-scan (in-lane max + DPP max across
//       lanes + the previous chunk's carry) and the source is s = p - (key & 0xffff) for match
//       and literal bytes alike.  In-chunk sources are chased by pointer jumping over the
//       chunk's own marker slots (free once read), then every byte is gathered from the 4 KiB
//       LDS window (or, when older than the window, from the block's output in HBM).
//     The batch loop is unrolled by two with two register sets for the prefetched GroupRec and
//     token dword, so no prefetched register is copied (and waited for) at a batch boundary.
//
// Checks C1-C5 are applied exactly as by the oracle (oracle/qlz_oracle.c:180-231).
#ifndef QLZX_SPLIT_K1  // 1 (release build): K1 lives in qlzx_k2.hip's unit, launched through launch_k1_parse6
#define QLZX_SPLIT_K1 0
#endif
namespace qlzx {

// ------------------------------------------------------------------------------- K1 ----
// K1 k_dec_parse6 (round 5): one LANE per block walks the serial control-word chain.  Each lane
// refills its own LDS ring: an iteration writes the rounds (32 B) loaded in the previous
// iteration into the lane's slots, issues plain global loads for up to two more rounds the ring
// has room for, then takes at most `kmax` steps.  Round 4's k_dec_parse4 moved every lane of a
// wave through the same round (one LDS-DMA per round into a wave-uniform slot) and looped until
// the lane with the most steps in that round was done: the wave paid max-over-lanes steps per
// round.  Here lanes drift apart in stream position and the wave pays kmax steps per iteration.
// c2 25.1-25.3 -> 24.7-24.9 ms at kmax 16; c4 346 -> 377 GiB/s at kmax 10
// (tools/gpu_r5lr3.sh, profiles/r05_k1_lane_ring_ab.txt).
#if (!defined(QLZX_K2_ONLY) && !QLZX_SPLIT_K1) || (defined(QLZX_K2_ONLY) && QLZX_SPLIT_K1)
// One wave's 64 blocks (lin = the block's place in the chunk), called by the kernel below.
__device__ __forceinline__ void k1_parse_wave(uint8_t *ring, uint32_t lane, uint32_t lin, const qlzx_blocks &b,
                                              const uint32_t *dst_cap, uint32_t *dsize_out, int32_t *status,
                                              uint32_t first, uint32_t count, BlkInfo *info, GroupRec *recs,
                                              uint32_t gmax, const uint32_t *order, uint32_t max_dsize,
                                              uint32_t kmax) {
    constexpr uint32_t S = kRingSlots;
    const bool inrange = lin < count;
    const uint32_t i = inrange ? (order ? order[lin] : first + lin) : first;

    int st = QLZX_OK;
    uint32_t kind = kBlkSkip, csize = 0, dsize = 0, hdr = 0, len = 0;
    const uint8_t *src = b.src + b.src_off[i];
    if (inrange) {
        len = b.src_len[i];
        st = classify_block(src, len, dst_cap ? dst_cap[i] : 0xffffffffu, max_dsize, kind, csize, dsize, hdr);
        if (st == QLZX_OK && kind == kBlkCompressed && dsize == 0) {  // oracle/qlz_oracle.c:197,228
            st = (csize == hdr || csize == hdr + 9) ? QLZX_OK : QLZX_E_CORRUPT;
            kind = kBlkSkip;
        }
    }
    const uintptr_t a0 = (uintptr_t)src;
    const uint8_t *gbase = (const uint8_t *)(a0 & ~(uintptr_t)15);
    const uint32_t shift = (uint32_t)(a0 & 15);
    const uint32_t span = (st == QLZX_OK && kind == kBlkCompressed) ? csize : 0;
    const uint32_t last16 = span ? (span + shift - 1) >> 4 : 0;
    const uint32_t nrounds = span ? (span + shift - 1) / kRoundBytes + 1 : 0;
    const bool parsing = inrange && span > 0;

    uint32_t ip = hdr, g = 0, cwr = 1, cwg = 0, ra = 0, rb = 0, rec_ip = 0;
    GroupRec *myrec = recs + (size_t)(inrange ? lin : 0) * gmax;
    bool done_parse = !parsing;

    // ring bookkeeping: rounds [0, rl) are in the lane's slots (round r in slot r % S), rounds
    // [rl, ri) are loaded into registers and go to the slots at the next iteration
    uint32_t rl = 0, ri = 0;
    // accept up to two rounds: a round r may overwrite round r - S only once the lane reads no
    // byte below round r - S + 1 (ring_rd32 reads the aligned dwords at and after its position)
    // rounds loaded per iteration (at most; the ring can take up to S - 1 rounds past the one
    // being read).  Three rounds per iteration were slower at every step budget (c2 25.3-26.2 vs
    // 24.7 ms, c5 517-543 vs 571 GiB/s: profiles/r05_k1_lane_ring_ab.txt)
    constexpr uint32_t M = 2;
    static_assert(M == 2 || M == 3, "rounds per iteration");
    auto accept = [&]() __attribute__((always_inline)) -> uint32_t {
        const uint32_t cap = ((ip + shift) & ~3u) / kRoundBytes + S - 1;  // last round the ring can take
        uint32_t n = 0;
#pragma unroll
        for (uint32_t k = 0; k < M; k++) n += (!done_parse && ri + k < nrounds && ri + k <= cap) ? 1u : 0u;
        return n;
    };
    // the M rounds from ri on (16-B pieces 2 ri ..), clamped into the stream; a lane taking fewer
    // rounds loads the stream's first piece instead (cached, never written)
    typedef uint32_t u4v __attribute__((ext_vector_type(4)));
    typedef const __attribute__((address_space(1))) u4v g_u4;
    const uintptr_t gaddr = (uintptr_t)gbase;  // integer -> global pointer: global_load, not flat
#define K1_LD(n, k, j) (*(g_u4 *)(gaddr + (size_t)((n) > (k) ? min(ri * kPieces + 2 * (k) + (j), last16) : 0u) * 16))
#define K1_LOAD(n, v0, v1, v2, v3, v4, v5)                                                        \
    do {                                                                                          \
        v0 = K1_LD(n, 0, 0), v1 = K1_LD(n, 0, 1), v2 = K1_LD(n, 1, 0), v3 = K1_LD(n, 1, 1);        \
        if (M >= 3) v4 = K1_LD(n, 2, 0), v5 = K1_LD(n, 2, 1);                                     \
        ri += (n);                                                                                \
    } while (0)
    // rounds rl .. rl + n - 1 into their slots
#define K1_STORE(n, v0, v1, v2, v3, v4, v5)                                                       \
    do {                                                                                          \
        /* an unconditional use: the loads land here in every lane, so no later reuse of their   \
           registers waits on a vmcnt that also counts the newer loads */                         \
        asm volatile("" ::"v"(v0.x), "v"(v0.y), "v"(v0.z), "v"(v0.w), "v"(v1.x), "v"(v1.y),        \
                     "v"(v1.z), "v"(v1.w), "v"(v2.x), "v"(v2.y), "v"(v2.z), "v"(v2.w), "v"(v3.x),  \
                     "v"(v3.y), "v"(v3.z), "v"(v3.w));                                             \
        if (M >= 3) asm volatile("" ::"v"(v4.x), "v"(v4.y), "v"(v4.z), "v"(v4.w), "v"(v5.x),      \
                                 "v"(v5.y), "v"(v5.z), "v"(v5.w));                                 \
        uint8_t *sl0 = ring + (((rl & (S - 1)) * kPieces) << 10) + lane * 16;                     \
        uint8_t *sl1 = ring + ((((rl + 1) & (S - 1)) * kPieces) << 10) + lane * 16;               \
        uint8_t *sl2 = ring + ((((rl + 2) & (S - 1)) * kPieces) << 10) + lane * 16;               \
        if ((n) >= 1) *(u4v *)sl0 = v0, *(u4v *)(sl0 + 1024) = v1;                                \
        if ((n) >= 2) *(u4v *)sl1 = v2, *(u4v *)(sl1 + 1024) = v3;                                \
        if (M >= 3 && (n) >= 3) *(u4v *)sl2 = v4, *(u4v *)(sl2 + 1024) = v5;                      \
        rl += (n);                                                                                \
    } while (0)
    // One step: a control word, or a literal run (ctz of the remaining control bits, no bytes
    // read), the match that ends it and, when the next item is a match whose first byte is in the
    // same dword, that one too.  Round 6 form (87 instead of 103 vector instructions per step,
    // same checks in the same order as round 5's select-based step, in git history): a lane that
    // cannot advance leaves the loop before anything is updated, the control-word and match cases
    // update through a branch each, and the second token's byte is taken with one alignbyte.
    // c2 time unchanged (23.77 vs 23.79 ms): K1's instructions cost c2 about half their issue
    // time (+32 per step: +0.42 ms), DESIGN.md §3.
    const uint32_t lane16 = lane << 4;
    auto rd32 = [&](uint32_t x) __attribute__((always_inline)) -> uint32_t {  // ring_rd32<S>(ring, x, lane)
        constexpr uint32_t PB = S * kPieces == 8 ? 3u : S * kPieces == 4 ? 2u : 4u;  // log2(pieces of 1 KiB)
        static_assert((1u << PB) == S * kPieces, "ring address below assumes 4, 8 or 16 pieces of 1 KiB");
        const uint32_t x4 = x + 4;
        const uint32_t a1 = (__builtin_amdgcn_ubfe(x, 4, PB) << 10) | ((x & 12u) | lane16);
        const uint32_t a2 = (__builtin_amdgcn_ubfe(x4, 4, PB) << 10) | ((x4 & 12u) | lane16);
        const uint32_t lo = *(const uint32_t *)(ring + a1);
        const uint32_t hi = *(const uint32_t *)(ring + a2);
        return __builtin_amdgcn_alignbyte(hi, lo, x);
    };
    // token bytes - 1 from the token's first byte (quicklz.c:579-610): 0, 1, 1, 2 by b & 3,
    // 3 when b & 127 == 3
    auto tlc = [](uint32_t b) __attribute__((always_inline)) -> uint32_t {
        return __builtin_amdgcn_ubfe(0x94u, (b & 3u) * 2, 2) + ((b & 127u) == 3u ? 1u : 0u);
    };
    auto steps = [&]() __attribute__((always_inline)) -> uint32_t {
        const uint32_t lim = rl * kRoundBytes - shift;  // stream bytes below lim are in the ring
        uint32_t k = 0;
        if (!done_parse) {
            for (;;) {  // per-lane loop, at most kmax steps
                const bool gb = cwr == 1;
                const uint32_t run = min((uint32_t)__builtin_ctz(cwr), csize - ip);
                const uint32_t q = ip + run;
                const uint32_t rest = cwr >> run;
                // a match at q (gb: rest == 1; a run cut by the stream end: q == csize)
                const bool hasm = (rest > 1u) & (q < csize);
                const uint32_t need = gb ? 4u : 1u;
                if (ip + need > csize) {  // the stream ends here (C1/C5 are K2's or the caller's)
                    done_parse = true;
                    break;
                }
                if ((gb | hasm) & (q + need > lim)) break;  // wait for the ring
                const uint32_t w = rd32(q + shift);
                const uint32_t e = tlc(w);
                const uint32_t q2 = q + e + 1, rest2 = rest >> 1;
                const bool hasm2 = hasm & (e < 3u) & ((rest2 & 1u) != 0) & (rest2 > 1u) & (q2 < csize) & (q2 < lim);
                const uint32_t e2 = hasm2 ? tlc(__builtin_amdgcn_alignbyte(0u, w, e + 1)) : 0u;
                const bool bad = (gb & (((int32_t)w >= 0) | (g >= gmax))) | (hasm & (q2 > csize)) |
                                 (hasm2 & (q2 + e2 + 1 > csize));
                if (bad) {
                    st = QLZX_E_CORRUPT;
                    done_parse = true;
                    break;
                }
                if (gb) {
                    // the record store is invisible to the compiler's vmcnt bookkeeping: counted, it
                    // made every wait before the step loop a vmcnt(0), i.e. a wait for the loads just
                    // issued (an unseen store only makes the compiler's later vmcnt(N) waits stricter)
                    if (g > 0) {
                        typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
                        const u32x4 rec = {rec_ip, cwg, ra, rb};
                        asm volatile("global_store_dwordx4 %0, %1, off" ::"v"(myrec + (g - 1)), "v"(rec) : "memory");
                    }
                    rec_ip = ip;
                    cwg = w;
                    g++;
                    ip += 4;
                    cwr = w;
                    ra = 0;
                    rb = 0;
                } else {
                    const uint32_t idx = __builtin_clz(cwr) + run;  // item index of the match
                    const uint32_t em = hasm ? e : 0u, e2m = hasm2 ? e2 : 0u;
                    ra |= ((em & 1u) | ((e2m & 1u) << 1)) << idx;
                    rb |= ((em >> 1) | (e2m & 2u)) << idx;
                    ip = q + em + e2m + (hasm ? 1u : 0u) + (hasm2 ? 1u : 0u);
                    cwr = rest >> ((hasm ? 1u : 0u) + (hasm2 ? 1u : 0u));
                }
                if (++k >= kmax) break;
            }
        }
        return k;
    };
#ifdef QLZX_PROFILE
    // profile build: outer iterations, wave step trips (max steps over lanes per iteration) and
    // lane steps (sum over lanes) per wave, in slot 0
    PROF_DECL
    auto k1prof = [&](uint32_t k) __attribute__((always_inline)) {
        uint32_t mx = k, sm = k;
        for (int o = 32; o >= 1; o >>= 1) {
            mx = max(mx, (uint32_t)__shfl_xor((int)mx, o));
            sm += (uint32_t)__shfl_xor((int)sm, o);
        }
        PROF_COUNT(0, 1);
        PROF_COUNT(1, mx);
        PROF_COUNT(2, sm);
    };
#define K1_STEPS() k1prof(steps())
#else
#define K1_STEPS() (void)steps()
#endif

    u4v pa0, pa1, pa2, pa3, pa4, pa5, pb0, pb1, pb2, pb3, pb4, pb5;
    uint32_t na = accept();
    K1_LOAD(na, pa0, pa1, pa2, pa3, pa4, pa5);
    uint32_t nb = 0;
    // Every iteration a lane either steps or lands a round, so csize + nrounds iterations finish
    // any stream; past that bound a lane stops as corrupt (a guard: the loop always ends).
    const uint32_t trip_cap = span + nrounds + 8;
    uint32_t trips = 0;
    auto guard = [&]() __attribute__((always_inline)) {
        trips++;
        if (!done_parse && trips > trip_cap) done_parse = true, st = QLZX_E_CORRUPT;
    };
    // two iterations per loop trip: register sets va / vb alternate, no copies of loaded data
    for (;;) {
        K1_STORE(na, pa0, pa1, pa2, pa3, pa4, pa5);
        nb = accept();
        K1_LOAD(nb, pb0, pb1, pb2, pb3, pb4, pb5);
        K1_STEPS();
        guard();
        if (__ballot(!done_parse) == 0) break;
        K1_STORE(nb, pb0, pb1, pb2, pb3, pb4, pb5);
        na = accept();
        K1_LOAD(na, pa0, pa1, pa2, pa3, pa4, pa5);
        K1_STEPS();
        guard();
        if (__ballot(!done_parse) == 0) break;
    }
#undef K1_LD
#undef K1_LOAD
#undef K1_STORE
#undef K1_STEPS
    if (parsing && st == QLZX_OK && g > 0) myrec[g - 1] = GroupRec{rec_ip, cwg, ra, rb};
    vm_sync();
#ifdef QLZX_PROFILE
    PROF_MARK(3);
    PROF_COUNT(4, 1);
    PROF_FLUSH(0);
#endif
    if (!inrange) return;
    if (st == QLZX_OK && kind == kBlkCompressed && (!done_parse || g == 0)) st = QLZX_E_CORRUPT;
    BlkInfo bi{0, 0, kind, dsize};
    if (st != QLZX_OK) {
        bi.kind = kBlkSkip;
        status[i] = st;
        if (dsize_out && st != kPending) dsize_out[i] = 0;
    } else if (kind == kBlkCompressed) {
        bi.ngroups = g;
        bi.nitems = (g - 1) * 31 + __builtin_clz(cwr);
    } else if (kind == kBlkSkip) {
        status[i] = QLZX_OK;
        if (dsize_out) dsize_out[i] = 0;
    }
    info[lin] = bi;
}

__global__ void __launch_bounds__(kParseWG) k_dec_parse6(qlzx_blocks b, const uint32_t *dst_cap, uint32_t *dsize_out,
                                                     int32_t *status, uint32_t first, uint32_t count, BlkInfo *info,
                                                     GroupRec *recs, uint32_t gmax, const uint32_t *order,
                                                     uint32_t max_dsize, uint32_t kmax) {
    constexpr uint32_t S = kRingSlots;
    __shared__ __attribute__((aligned(16))) uint8_t ring_all[(kParseWG / 64) * kRingWaveS<S>];
    const uint32_t lane = threadIdx.x & 63;
    uint8_t *ring = ring_all + (threadIdx.x >> 6) * kRingWaveS<S>;
    k1_parse_wave(ring, lane, blockIdx.x * kParseWG + threadIdx.x, b, dst_cap, dsize_out, status, first, count, info,
                  recs, gmax, order, max_dsize, kmax);
}
#endif  // QLZX_K2_ONLY

// ------------------------------------------------------------------------------- K2 ----
constexpr uint32_t kV4W = 4096;   // output window (LDS ring)
constexpr uint32_t kV4MR = 256;   // marker ring (u32 keys)
constexpr uint32_t kV4Bpl = 4;  // output bytes per lane per chunk
constexpr uint32_t kV4Chunk = 64 * kV4Bpl;      // 256 or 512 output bytes per chunk
static_assert(kV4Chunk <= kV4MR, "a chunk's pointer-jumping array lives in its marker slots");

template <uint32_t W = kV4W>
struct K2v4Lds {
    uint8_t win[W];
    uint32_t mk[kV4MR];
};

// Inclusive max over lanes 0..lane; DPP row shifts + row broadcasts.
__device__ __forceinline__ uint32_t v4_incl_max(uint32_t v) {
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false));
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false));
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false));
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false));
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false));
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false));
    return v;
}

template <uint32_t WIN>
__device__ __forceinline__ void dec_v4_block(K2v4Lds<WIN> &L, const uint8_t *src, uint8_t *dst, uint32_t csize,
                                             const BlkInfo bi, const GroupRec *rb, int32_t *status_i,
                                             uint32_t *dsize_i, uint32_t lane) {
    constexpr uint32_t W = WIN, MR = kV4MR, CH = kV4Chunk;
    const uint32_t dsize = bi.dsize;
    if (bi.kind == kBlkStored) {  // quicklz.c:808-811
        const uint32_t hdr = (src[0] & 2u) ? 9u : 3u;
        const uint8_t *s = src + hdr;
        uint32_t p0 = 0;
        if ((((uintptr_t)dst) & 15u) == 0) {
            p0 = dsize & ~15u;
            for (uint32_t p = lane * 16; p < p0; p += 1024) {
                const uint32_t *q = (const uint32_t *)(s + p);
                *(uint4 *)(dst + p) = make_uint4(q[0], q[1], q[2], q[3]);
            }
        }
        for (uint32_t p = p0 + lane; p < dsize; p += 64) dst[p] = s[p];
        if (lane == 0) { *status_i = QLZX_OK; if (dsize_i) *dsize_i = dsize; }
        return;
    }
    for (uint32_t q = lane * 4; q < MR; q += 256) *(uint4 *)(L.mk + q) = make_uint4(0, 0, 0, 0);

    const uint32_t nitems = bi.nitems;
    const uint32_t hdr = (src[0] & 2u) ? 9u : 3u;
    const uint32_t nb = (nitems + 63) / 64;
    const uint32_t tail_from = dsize > QLZX_TAIL ? dsize - 1 - QLZX_TAIL : 0;  // op >= this: tail (quicklz.c:503)

    // token position of item (c.g, c.k) and its dword address (clamped into the stream; lanes past
    // the last item read a clamped record and are masked by v where it matters)
    auto tok_pos = [&](const GroupRec &gr, const ItemCursor &c, uint32_t &p) -> uint32_t {
        const uint32_t low = (1u << c.k) - 1u;
        const uint32_t pos = gr.ip + 4 + c.k + __builtin_popcount(gr.a & low) + 2 * __builtin_popcount(gr.b & low);
        p = min(pos, csize - 4);
        return (pos & 0x7fffffffu) | (((gr.m >> c.k) & 1u) << 31);
    };
    const uint32_t glast = bi.ngroups - 1;
    // register sets: (posm, tok) of the batch being decoded and of the next; GroupRec of the
    // batch after the decoded one and of the one after that
    ItemCursor ck{lane / 31, lane % 31};
    uint32_t posmA, tokA, posmB = 0, tokB = 0;
    GroupRec grA, grB;
    {
        const GroupRec g0 = rb[min(ck.g, glast)];
        uint32_t tp;
        posmA = tok_pos(g0, ck, tp);
        tokA = *(const uint32_t *)(src + tp);
        ck.next();
        grB = rb[min(ck.g, glast)];
        grA = grB;
    }
    PROF_DECL
    uint32_t D = 0, bt = 0, c = 0, cin = 0;
    bool tail = false, complete = false, err = false;
    bool pend = false, mp = false;  // some lane's item / this lane's item waits for its marker slot
    uint32_t pd = 0, pkey = 0;
    uint32_t plit = 0;

    // one batch: decode (posm, tok), prefetch the next batch's token from gr_next into
    // (posm_n, tok_n) and the GroupRec after it into gr_nn
    auto batch = [&](uint32_t posm, uint32_t tok, const GroupRec &gr_next, uint32_t &posm_n, uint32_t &tok_n,
                     GroupRec &gr_nn) __attribute__((always_inline)) {
        if (pend) {  // a straddling batch's items not marked by a chunk yet (all start below c + CH)
            const bool wr = mp;
            if (wr) {
                L.mk[pd & (MR - 1)] = pkey;
                if (plit < 0x100u) L.win[pd & (W - 1)] = (uint8_t)plit;
            }
            pend = mp = false;
        }
        const bool v = bt * 64 + lane < nitems;
        {
            uint32_t tp;
            posm_n = tok_pos(gr_next, ck, tp);
            tok_n = *(const uint32_t *)(src + tp);
            ck.next();
            gr_nn = rb[min(ck.g, glast)];
        }
        const bool ism = v && (posm >> 31) != 0;
        const uint32_t pos = posm & 0x7fffffffu;
        const uint32_t t = tok >> (8 * (pos - min(pos, csize - 4)));  // the last tokens: dword clamped
        uint32_t off, mlen, tl;
        decode_tok_bf(t, off, mlen, tl);
        const uint32_t len = ism ? mlen : (v ? 1u : 0u);
        const uint32_t incl = wave_incl_scan(len);
        const uint32_t total = __builtin_amdgcn_readfirstlane(__builtin_amdgcn_readlane(incl, 63));
        const uint32_t d = D + incl - len;
        const bool live = v && d < dsize;
        bool bad, last = false;
        if (tail || D + total > tail_from) {
            tl = ism ? tl : 1u;
            const uint64_t tail_lanes = __ballot(live && !ism && d >= tail_from);
            const uint32_t tail_lane = tail ? 0u : ff1_or(tail_lanes, 64u);  // C4: no match after it
            tail = tail || tail_lanes != 0;
            const bool mok = off >= 3 && off <= d && d + len + 4 <= dsize && lane < tail_lane;  // C3, C4
            last = live && d + len == dsize;  // C5: the item completing dsize ends the stream
            const uint32_t ip_end = pos + tl;
            const bool eok = ip_end == csize || (ip_end < hdr + 9 && csize == hdr + 9);
            bad = live && ((ism && !mok) || (last && !eok));
        } else {
            bad = ism && (off < 3 || off > d);  // C3
        }
        if (__ballot(bad)) {
            err = true;
            return;
        }
        complete = __ballot(last) != 0;
        const uint32_t key = (d << 16) | (ism ? off : 0u);
        const bool wr = live && d < c + MR;
        if (wr) {
            L.mk[d & (MR - 1)] = key;
            // a match's own window slot holds a byte older than the far bound (d < c + MR) that no
            // gather reads before the chunk of d overwrites it: the byte can go there unconditionally
            L.win[d & (W - 1)] = (uint8_t)t;
        }
        mp = live && !wr;
        pend = __ballot(mp) != 0;
        pd = d;
        pkey = key;
        plit = ism ? 0x100u : (t & 0xffu);
        D = __builtin_amdgcn_readfirstlane(D + total);
        bt++;
        PROF_COUNT(5, 1);
    };

    // chunk phases while every item starting below c + 256 is known; true when the block is done
    auto chunks = [&]() __attribute__((always_inline)) -> bool {
        while (c < dsize && (complete || D >= c + CH)) {
            if (pend) {  // items of the last batch that start at or above c_prev + MR
                const bool wr = mp && pd < c + MR;
                if (wr) {
                    L.mk[pd & (MR - 1)] = pkey;
                    if (plit < 0x100u) L.win[pd & (W - 1)] = (uint8_t)plit;
                }
                mp = mp && !wr;
                pend = __ballot(mp) != 0;
            }
            constexpr uint32_t B = kV4Bpl;
            const uint32_t r0 = B * lane, p0 = c + r0;
            uint32_t *mkl = L.mk + ((c & (MR - 1)) + r0);
            uint32_t m[B];
#pragma unroll
            for (uint32_t h = 0; h < B; h += 4) {
                const uint4 q = *(const uint4 *)(mkl + h);
                m[h] = q.x, m[h + 1] = q.y, m[h + 2] = q.z, m[h + 3] = q.w;
            }
            uint32_t lmax = m[0];
#pragma unroll
            for (uint32_t j = 1; j < B; j++) lmax = max(lmax, m[j]);
            const uint32_t incl = v4_incl_max(lmax);
            uint32_t f = max(wave_shr1(incl), cin);
            cin = max(cin, (uint32_t)__builtin_amdgcn_readfirstlane(__builtin_amdgcn_readlane(incl, 63)));
            // sources relative to the chunk (rj = s - c mod 2^32): in-chunk sources of match bytes
            // are s in [c, p), i.e. rj < r0 + j unsigned (a literal has rj = r0 + j, a source
            // below c wraps above every in-chunk value), and the pointer jumping below compares
            // and indexes the chunk's slots with rj directly
            uint32_t rj[B];
            bool qa[B], anyq = false;
#pragma unroll
            for (uint32_t j = 0; j < B; j++) {
                f = max(f, m[j]);
                rj[j] = r0 + j - (f & 0xffffu);
                qa[j] = rj[j] < r0 + j;
                anyq = anyq || qa[j];
            }
            PROF_MARK(1);
            if (__ballot(anyq)) {
                // the chunk's marker slots are free once read: they hold each byte's current source
                uint32_t *spb = L.mk + (c & (MR - 1));
#pragma unroll
                for (uint32_t h = 0; h < B; h += 4) *(uint4 *)(mkl + h) = make_uint4(rj[h], rj[h + 1], rj[h + 2], rj[h + 3]);
                do {
                    uint32_t t[B];
#pragma unroll
                    for (uint32_t j = 0; j < B; j++) t[j] = spb[qa[j] ? rj[j] : r0 + j];
                    uint64_t anym = 0;
#pragma unroll
                    for (uint32_t j = 0; j < B; j++) {
                        // a byte whose source's source is outside the chunk or a literal is final
                        qa[j] = t[j] < rj[j];
                        anym |= __ballot(qa[j]);
                        rj[j] = t[j];
                    }
                    anyq = anym != 0;
#pragma unroll
                    for (uint32_t h = 0; h < B; h += 4)
                        *(uint4 *)(mkl + h) = make_uint4(rj[h], rj[h + 1], rj[h + 2], rj[h + 3]);
                    PROF_COUNT(7, 1);
                } while (anyq);

            }
            PROF_MARK(2);
            // far: s < lo  <=>  rj < lo - c as signed (lo - c = MR - W once the window is full,
            // else -c: nothing is below the block start)
            const int32_t lo_rel = c + MR > W ? (int32_t)MR - (int32_t)W : -(int32_t)c;
            uint32_t vb[B], sv[B];
#pragma unroll
            for (uint32_t j = 0; j < B; j++) {
                sv[j] = rj[j] + c;
                vb[j] = L.win[sv[j] & (W - 1)];
            }
            int32_t mn = (int32_t)rj[0];
#pragma unroll
            for (uint32_t j = 1; j < B; j++) mn = min(mn, (int32_t)rj[j]);
            const bool far = mn < lo_rel;
            const uint32_t lo = c + lo_rel;
            PROF_COUNT(6, __ballot(far) ? 1 : 0);  // chunks with a byte older than the window
            uint32_t w[B / 4];
            if (__ballot(far)) {
#pragma unroll
                for (uint32_t j = 0; j < B; j++)
                    if (sv[j] < lo) vb[j] = dst[sv[j]];
            }
#pragma unroll
            for (uint32_t h = 0; h < B / 4; h++)
                w[h] = vb[4 * h] | (vb[4 * h + 1] << 8) | (vb[4 * h + 2] << 16) | (vb[4 * h + 3] << 24);
            *(uint32_t *)(L.win + (p0 & (W - 1))) = w[0];
#pragma unroll
            for (uint32_t h = 0; h < B; h += 4) *(uint4 *)(mkl + h) = make_uint4(0, 0, 0, 0);  // slots of c + MR ..
            PROF_MARK(3);
            if (c + CH <= dsize) {
                *(uint32_t *)(dst + p0) = w[0];
            } else {
                for (uint32_t j = 0; j < B && p0 + j < dsize; j++) dst[p0 + j] = (uint8_t)(w[j >> 2] >> (8 * (j & 3)));
            }
            c += CH;
            PROF_MARK(4);
        }
        return c >= dsize;
    };

    for (;;) {
        if (bt >= nb) { err = true; break; }  // stream ended before dsize (check C5)
        batch(posmA, tokA, grB, posmB, tokB, grA);
        PROF_MARK(0);
        if (err || chunks()) break;
        if (bt >= nb) { err = true; break; }
        batch(posmB, tokB, grA, posmA, tokA, grB);
        PROF_MARK(0);
        if (err || chunks()) break;
    }
    vm_sync();
    PROF_FLUSH(1);
    if (lane == 0) {
        *status_i = err ? QLZX_E_CORRUPT : QLZX_OK;
        if (dsize_i) *dsize_i = err ? 0u : dsize;
    }
}

template <bool CRC, uint32_t WIN = kV4W>
__global__ void __launch_bounds__(64) k_dec_chunk4(qlzx_blocks b, uint32_t *dsize_out, int32_t *status,
                                                   uint32_t first, uint32_t count, const BlkInfo *info,
                                                   const GroupRec *recs, uint32_t gmax, const uint32_t *list,
                                                   const uint32_t *crc_state, const uint32_t *crc_expect,
                                                   uint32_t *crc_out) {
    __shared__ __attribute__((aligned(16))) K2v4Lds<WIN> L;
    const uint32_t bx = blockIdx.x;
    if (bx >= count) return;
    const uint32_t i = list ? list[bx] : first + bx;
    if constexpr (CRC) {
        static_assert(sizeof(K2v4Lds<WIN>) >= 4096, "the slicing-by-4 CRC tables fill 4 KiB of the window");
        const uint32_t lane = threadIdx.x;
        uint32_t *tab = (uint32_t *)&L;
        for (uint32_t e = lane * 4; e < 1024; e += 256) *(uint4 *)(tab + e) = *(const uint4 *)(g_crc_slice8 + e);
        __syncthreads();
        const uint32_t c = ~wave_crc_rep<4, 1>(tab, g_crc_mul, b.src + b.src_off[i], b.src_len[i],
                                                crc_state ? crc_state[i] : 0xffffffffu, lane);
        __syncthreads();
        if (lane == 0 && crc_out) crc_out[i] = c;
        if (crc_expect && c != crc_expect[i]) {
            if (lane == 0) {
                status[i] = QLZX_E_CRC;
                if (dsize_out) dsize_out[i] = 0;
            }
            return;
        }
    }
    const BlkInfo bi = info[bx];
    if (bi.kind == kBlkSkip) return;
    dec_v4_block(L, b.src + b.src_off[i], b.dst + b.dst_off[i], b.src_len[i], bi, recs + (size_t)bx * gmax,
                 status + i, dsize_out ? dsize_out + i : nullptr, threadIdx.x);
}

}  // namespace qlzx
