// qlzx_decode_v4.hip -- round-4 batch decoder pair (dsize <= QLZX_FAST_MAX_DSIZE):
//
// K1 k_dec_parse4  one LANE per block: the serial control-word chain of quicklz.c:513-671,
//     one item STEP at a time (a literal run and the match that ends it, or a control word),
//     reading only control words and the first byte of each match token.  The remaining
//     control bits are kept with their sentinel (cwr; 1 = group exhausted), so the item index
//     is clz(cwr) and a literal run is ctz(cwr): no per-item counters, no multi-match step.
//     Emits one GroupRec {ip, cw, a, b} per control word (a, b: bit-planes of token bytes - 1).
//
// K2 k_dec_chunk4  one WAVE per block, 64 items per batch and 256 output bytes per chunk:
//     * ITEM PHASE: token position from the GroupRec, branch-free token decode, DPP scan of the
//       output lengths; item i leaves ONE u32 key (d << 16 | off) in a 512-entry marker ring
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
#ifndef QLZX_K1_STRUCT
#define QLZX_K1_STRUCT 0
#endif
#ifndef QLZX_K1_LANELOOP  // K1's step loop as a per-lane loop instead of a ballot-tested one
#define QLZX_K1_LANELOOP 1
#endif
#ifndef QLZX_K2_JUMP_BALLOTS  // pointer jumping's loop test from per-byte ballots
#define QLZX_K2_JUMP_BALLOTS 1
#endif
#ifndef QLZX_K1_V4M2  // k_dec_parse4 takes a second match from the same dword, as k_dec_parse does
#define QLZX_K1_V4M2 1
#endif
#ifndef QLZX_K1_V4M3  // ... or up to three matches from an 8-byte window
#define QLZX_K1_V4M3 0
#endif
namespace qlzx {

// ------------------------------------------------------------------------------- K1 ----
__global__ void __launch_bounds__(kParseWG) k_dec_parse4(qlzx_blocks b, const uint32_t *dst_cap, uint32_t *dsize_out,
                                                     int32_t *status, uint32_t first, uint32_t count, BlkInfo *info,
                                                     GroupRec *recs, uint32_t gmax, const uint32_t *order,
                                                     uint32_t max_dsize) {
    __shared__ __attribute__((aligned(16))) uint8_t ring_all[(kParseWG / 64) * kRingWave];
    const uint32_t lane = threadIdx.x & 63;
    uint8_t *ring = ring_all + (threadIdx.x >> 6) * kRingWave;
    const uint32_t lin = blockIdx.x * kParseWG + threadIdx.x;
    const bool inrange = lin < count;
    const uint32_t i = inrange ? (order ? order[lin] : first + lin) : first;

    int st = QLZX_OK;
    uint32_t kind = kBlkSkip, csize = 0, dsize = 0, hdr = 0, len = 0;
    const uint8_t *src = b.src + b.src_off[i];
    if (inrange) {
        len = b.src_len[i];
        st = classify_block(src, len, dst_cap ? dst_cap[i] : 0xffffffffu, max_dsize, kind, csize, dsize, hdr);
        // a compressed stream of dsize 0 decodes to nothing: the oracle's loop never runs and C5
        // accepts csize == hdr or the 9-byte core minimum (oracle/qlz_oracle.c:197,228)
        if (st == QLZX_OK && kind == kBlkCompressed && dsize == 0) {
            st = (csize == hdr || csize == hdr + 9) ? QLZX_OK : QLZX_E_CORRUPT;
            kind = kBlkSkip;
        }
    }
    const uintptr_t a0 = (uintptr_t)src;
    const uint8_t *gbase = (const uint8_t *)(a0 & ~(uintptr_t)15);
    const uint32_t shift = (uint32_t)(a0 & 15);
    const uint32_t span = (st == QLZX_OK && kind == kBlkCompressed) ? csize : 0;
    const uint32_t last16 = span ? (span + shift - 1) >> 4 : 0;
    const uint32_t last_round = span ? (span + shift - 1) / kRoundBytes : 0;
    bool stream = inrange && span > 0;
    const bool parsing = stream;

    // parse state: ip = next stream byte; cwr = control bits not consumed yet, sentinel
    // included (1: the group is exhausted, the next step reads a control word)
    uint32_t ip = hdr, g = 0, cwr = 1, cwg = 0, ra = 0, rb = 0, rec_ip = 0;
    GroupRec *myrec = recs + (size_t)(inrange ? lin : 0) * gmax;
    bool done_parse = !parsing;

    PROF_DECL
    const uint8_t *dummy = (const uint8_t *)(((uintptr_t)b.src) & ~(uintptr_t)15);
    ring_issue(ring, gbase, dummy, 0, last16, stream);
    ring_issue(ring, gbase, dummy, 1, last16, stream && last_round >= 1);
    ring_issue(ring, gbase, dummy, 2, last16, stream && last_round >= 2);
    for (uint32_t r = 0;; r++) {
        if (__ballot(stream && r <= last_round) == 0) break;
        PROF_MARK(0);
#if QLZX_K1_ROUND == 64
        asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
#elif QLZX_K1_ROUND == 32
        asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
#else
        asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
#endif
        PROF_MARK(1);
        const bool act = stream && r <= last_round;
        const uint32_t lim = (r + 1) * kRoundBytes - shift;  // stream bytes below lim have landed
        if (act && !done_parse) {
#if QLZX_K1_STRUCT
            // structured steps: a lane leaves the loop when its bytes run out (it resumes next
            // round) or its stream ends; only active lanes update their state
            for (;;) {
#ifdef QLZX_PROFILE
                _pacc[6] += 1;
#endif
                const bool gb = cwr == 1;
                const uint32_t rem = csize - ip;
                uint32_t run = __builtin_ctz(cwr);
                run = run < rem ? run : rem;
                const uint32_t q = ip + run;
                const uint32_t rest = cwr >> run;
                const bool hasm = (rest != 1u) & ((rest & 1u) != 0) & (q < csize);  // gb: rest == 1
                if (ip + (gb ? 4u : 1u) > csize) { done_parse = true; break; }     // stream exhausted
                if ((gb | hasm) && q + (gb ? 4u : 1u) > lim) break;                 // wait for the next round
                const uint32_t w = ring_rd32(ring, q + shift, lane);
                const uint32_t ty = (w & 3u) + ((w & 127u) == 3u ? 1u : 0u);
                const uint32_t e = __builtin_amdgcn_ubfe(0x32110u, ty * 4, 4);  // token bytes - 1
                if (gb) {
                    if (((w >> 31) == 0) | (g >= gmax)) { st = QLZX_E_CORRUPT; done_parse = true; break; }  // C1
                    if (g > 0) myrec[g - 1] = GroupRec{rec_ip, cwg, ra, rb};
                    rec_ip = ip;
                    cwg = w;
                    cwr = w;
                    ra = 0;
                    rb = 0;
                    ip += 4;
                    g++;
                } else {
                    if (hasm & (q + e + 1 > csize)) { st = QLZX_E_CORRUPT; done_parse = true; break; }  // C2
                    const uint32_t kb = hasm ? 1u << (__builtin_clz(cwr) + run) : 0u;
                    ra |= (e & 1u) ? kb : 0u;
                    rb |= (e & 2u) ? kb : 0u;
                    ip = q + (hasm ? e + 1 : 0u);
                    cwr = rest >> (hasm ? 1 : 0);
                }
            }
#else
        bool go = true;
#if QLZX_K1_LANELOOP
        while (go) {  // per-lane loop: the exec mask carries go (no cross-lane op in the step)
#else
        while (__ballot(go)) {
#endif
#ifdef QLZX_PROFILE
            _pacc[5] += 1;
            if (go) _pacc[6] += 1;
#endif
            const bool gb = cwr == 1;
            const uint32_t rem = csize - ip;
            uint32_t run = __builtin_ctz(cwr);  // literals before the next match (or the sentinel)
            run = run < rem ? run : rem;
            const uint32_t q = ip + run;        // control word (gb) or the match token
            const uint32_t rest = cwr >> run;
            const bool hasm = !gb & (rest != 1u) & ((rest & 1u) != 0) & (q < csize);
            const bool end = ip + (gb ? 4u : 1u) > csize;
            const uint32_t need = gb ? 4u : 1u;
            const bool landed = q + need <= lim;
            const bool stepping = go & !end & ((gb | hasm) ? landed : true);
            const uint32_t w = ring_rd32(ring, q + shift, lane);
            const uint32_t ty = (w & 3u) + ((w & 127u) == 3u ? 1u : 0u);
            const uint32_t e = __builtin_amdgcn_ubfe(0x32110u, ty * 4, 4);  // token bytes - 1
#if QLZX_K1_V4M3
            // up to three matches per step from an 8-byte window at q (the tokens' first bytes)
            const uint32_t wh = ring_rd32(ring, q + 4 + shift, lane);
            const uint64_t W8 = ((uint64_t)wh << 32) | w;
            const uint32_t q2 = q + e + 1, rest2 = rest >> 1;
            const bool hasm2 = hasm & ((rest2 & 1u) != 0) & (rest2 != 1u) & (q2 < csize) & (q2 + 1 <= lim);
            const uint32_t t2 = (uint32_t)(W8 >> (8 * (e + 1)));
            const uint32_t ty2 = (t2 & 3u) + ((t2 & 127u) == 3u ? 1u : 0u);
            const uint32_t e2 = hasm2 ? __builtin_amdgcn_ubfe(0x32110u, ty2 * 4, 4) : 0u;
            const uint32_t q3 = q2 + e2 + 1, rest3 = rest2 >> 1;
            const bool hasm3 = hasm2 & ((rest3 & 1u) != 0) & (rest3 != 1u) & (q3 < csize) & (q3 + 1 <= lim) &
                               (e + e2 + 2 <= 7u);
            const uint32_t t3 = (uint32_t)(W8 >> (8 * ((e + e2 + 2) & 7u)));
            const uint32_t ty3 = (t3 & 3u) + ((t3 & 127u) == 3u ? 1u : 0u);
            const uint32_t e3 = hasm3 ? __builtin_amdgcn_ubfe(0x32110u, ty3 * 4, 4) : 0u;
            const bool bad = stepping & ((gb & (((w >> 31) == 0) | (g >= gmax))) | (hasm & (q2 > csize)) |
                                         (hasm2 & (q3 > csize)) | (hasm3 & (q3 + e3 + 1 > csize)));
#elif QLZX_K1_V4M2
            // a second match right after the first when its first byte is already in w
            const uint32_t q2 = q + e + 1, rest2 = rest >> 1;
            const bool hasm2 = hasm & (e < 3u) & ((rest2 & 1u) != 0) & (rest2 != 1u) & (q2 < csize) & (q2 + 1 <= lim);
            const uint32_t w2 = w >> (8 * ((e + 1) & 3u));
            const uint32_t ty2 = (w2 & 3u) + ((w2 & 127u) == 3u ? 1u : 0u);
            const uint32_t e2 = hasm2 ? __builtin_amdgcn_ubfe(0x32110u, ty2 * 4, 4) : 0u;
            const bool bad = stepping & ((gb & (((w >> 31) == 0) | (g >= gmax))) | (hasm & (q2 > csize)) |
                                         (hasm2 & (q2 + e2 + 1 > csize)));
#else
            const bool bad = stepping & ((gb & (((w >> 31) == 0) | (g >= gmax))) | (hasm & (q + e + 1 > csize)));
#endif
            if (stepping & gb & (g > 0)) myrec[g - 1] = GroupRec{rec_ip, cwg, ra, rb};
            st = bad ? QLZX_E_CORRUPT : st;
            const bool adv = stepping & !bad;
            const uint32_t kb = hasm ? 1u << (__builtin_clz(cwr) + run) : 0u;  // item index clz(cwr) + run
#if QLZX_K1_V4M3
            const uint32_t kb2 = hasm2 ? kb << 1 : 0u, kb3 = hasm3 ? kb << 2 : 0u;
            const uint32_t nip = gb ? ip + 4 : q + (hasm ? e + 1 : 0u) + (hasm2 ? e2 + 1 : 0u) + (hasm3 ? e3 + 1 : 0u);
            const uint32_t ncwr = gb ? w : (rest >> (hasm ? (hasm2 ? (hasm3 ? 3 : 2) : 1) : 0));
            const uint32_t nra = gb ? 0u : (ra | ((e & 1u) ? kb : 0u) | ((e2 & 1u) ? kb2 : 0u) | ((e3 & 1u) ? kb3 : 0u));
            const uint32_t nrb = gb ? 0u : (rb | ((e & 2u) ? kb : 0u) | ((e2 & 2u) ? kb2 : 0u) | ((e3 & 2u) ? kb3 : 0u));
#elif QLZX_K1_V4M2
            const uint32_t kb2 = hasm2 ? kb << 1 : 0u;
            const uint32_t nip = gb ? ip + 4 : q + (hasm ? e + 1 : 0u) + (hasm2 ? e2 + 1 : 0u);
            const uint32_t ncwr = gb ? w : (rest >> (hasm ? (hasm2 ? 2 : 1) : 0));
            const uint32_t nra = gb ? 0u : (ra | ((e & 1u) ? kb : 0u) | ((e2 & 1u) ? kb2 : 0u));
            const uint32_t nrb = gb ? 0u : (rb | ((e & 2u) ? kb : 0u) | ((e2 & 2u) ? kb2 : 0u));
#else
            const uint32_t nip = gb ? ip + 4 : q + (hasm ? e + 1 : 0u);
            const uint32_t ncwr = gb ? w : (rest >> (hasm ? 1 : 0));
            const uint32_t nra = gb ? 0u : (ra | ((e & 1u) ? kb : 0u));
            const uint32_t nrb = gb ? 0u : (rb | ((e & 2u) ? kb : 0u));
#endif
            rec_ip = (adv & gb) ? ip : rec_ip;
            cwg = (adv & gb) ? w : cwg;
            g += (adv & gb) ? 1u : 0u;
            ip = adv ? nip : ip;
            cwr = adv ? ncwr : cwr;
            ra = adv ? nra : ra;
            rb = adv ? nrb : rb;
            done_parse = done_parse | (go & (end | bad));
            go = adv;
        }
#endif
        }
        PROF_MARK(3);
        if (done_parse) stream = false;
        ring_issue(ring, gbase, dummy, r + 3, last16, stream && r + 3 <= last_round);
    }
    PROF_MARK(4);
    if (parsing && st == QLZX_OK && g > 0) myrec[g - 1] = GroupRec{rec_ip, cwg, ra, rb};
    PROF_FLUSH(0);
    vm_sync();
    if (!inrange) return;
    if (st == QLZX_OK && kind == kBlkCompressed && (!done_parse || g == 0)) st = QLZX_E_CORRUPT;
    BlkInfo bi{0, 0, kind, dsize};
    if (st != QLZX_OK) {
        bi.kind = kBlkSkip;
        status[i] = st;
        if (dsize_out && st != kPending) dsize_out[i] = 0;
    } else if (kind == kBlkCompressed) {
        bi.ngroups = g;
        bi.nitems = (g - 1) * 31 + __builtin_clz(cwr);  // items consumed in the last group
    } else if (kind == kBlkSkip) {  // dsize-0 compressed stream accepted above
        status[i] = QLZX_OK;
        if (dsize_out) dsize_out[i] = 0;
    }
    info[lin] = bi;
}

// ------------------------------------------------------------- K1 without the LDS ring ----
// k_dec_parse's step (a literal run and up to two matches, quicklz.c:513-671), reading each step's
// dword straight from the stream in global memory (L1/L2; a lane's bytes are sequential) instead
// of an LDS DMA ring: K1 then holds no LDS, so K2 of the previous chunk keeps its occupancy while
// K1 runs beside it (the 16 KiB ring per K1 wave displaced three K2 waves each).
__device__ __forceinline__ uint32_t g_rd32(const uint8_t *src, uint32_t q, uint32_t csize) {
    const uint32_t qa = q + 4 <= csize ? q : csize - 4;  // csize >= 7 for a compressed stream
    uint64_t a = (uint64_t)(uintptr_t)(src + qa);
    asm volatile("" : "+v"(a));  // a vector load (any byte address), never a scalar one
    return *(const uint32_t *)(uintptr_t)a >> (8 * (q - qa));
}
__global__ void __launch_bounds__(kParseWG) k_dec_parse_g(qlzx_blocks b, const uint32_t *dst_cap, uint32_t *dsize_out,
                                                      int32_t *status, uint32_t first, uint32_t count, BlkInfo *info,
                                                      GroupRec *recs, uint32_t gmax, const uint32_t *order,
                                                      uint32_t max_dsize) {
    const uint32_t lin = blockIdx.x * kParseWG + threadIdx.x;
    const bool inrange = lin < count;
    const uint32_t i = inrange ? (order ? order[lin] : first + lin) : first;
    int st = QLZX_OK;
    uint32_t kind = kBlkSkip, csize = 0, dsize = 0, hdr = 0;
    const uint8_t *src = b.src + b.src_off[i];
    if (inrange) {
        st = classify_block(src, b.src_len[i], dst_cap ? dst_cap[i] : 0xffffffffu, max_dsize, kind, csize, dsize, hdr);
        if (st == QLZX_OK && kind == kBlkCompressed && dsize == 0) {  // oracle/qlz_oracle.c:197,228
            st = (csize == hdr || csize == hdr + 9) ? QLZX_OK : QLZX_E_CORRUPT;
            kind = kBlkSkip;
        }
    }
    const bool parsing = inrange && st == QLZX_OK && kind == kBlkCompressed;
    uint32_t ip = hdr, g = 0, k = 31, cw = 0, m = 0, ra = 0, rb = 0, rec_ip = 0;
    GroupRec *myrec = recs + (size_t)(inrange ? lin : 0) * gmax;
    bool done_parse = !parsing, go = parsing;
    PROF_DECL
    while (__ballot(go)) {
#ifdef QLZX_PROFILE
        _pacc[5] += 1;
        if (go) _pacc[6] += 1;
#endif
        const bool gb = k == 31;
        const uint32_t kk = k & 31;
        const uint32_t cwk = cw >> kk;
        uint32_t run = __builtin_ctz(cwk | (1u << (31 - kk)));  // literals before the next match
        run = gb ? 0u : (run < csize - ip ? run : csize - ip);
        const uint32_t ipm = ip + run, km = kk + run;
        const bool hasm = !gb & (km < 31) & (ipm < csize);
        const bool end = ip + (gb ? 4u : 1u) > csize;
        const bool stepping = go & !end & (gb | (run > 0) | hasm);
        const uint32_t w = g_rd32(src, ipm, csize);
        const uint32_t ty = (w & 3u) + ((w & 127u) == 3u ? 1u : 0u);
        const uint32_t code = __builtin_amdgcn_ubfe(0x32110u, ty * 4, 4);
        const uint32_t ip2 = ipm + code + 1, k2 = km + 1;
        const uint32_t w2 = w >> (8 * ((code + 1) & 3));
        const bool mat2 = hasm & (code < 3) & (k2 < 31) & (((cw >> (k2 & 31)) & 1u) != 0) & (ip2 < csize);
        const uint32_t ty2 = (w2 & 3u) + ((w2 & 127u) == 3u ? 1u : 0u);
        const uint32_t code2 = __builtin_amdgcn_ubfe(0x32110u, ty2 * 4, 4);
        bool bad = stepping & ((gb & (((w >> 31) == 0) | (g >= gmax))) | (hasm & (ipm + code + 1 > csize)) |
                               (mat2 & (ip2 + code2 + 1 > csize)));
        if (stepping & gb & (g > 0)) myrec[g - 1] = GroupRec{rec_ip, m, ra, rb};
        st = bad ? QLZX_E_CORRUPT : st;
        const bool adv = stepping & !bad;
        const bool ag = adv & gb;
        const uint32_t bm = hasm ? (1u << (km & 31)) : 0u;
        const uint32_t bm2 = mat2 ? (1u << (k2 & 31)) : 0u;
        rec_ip = ag ? ip : rec_ip;
        cw = ag ? w : cw;
        g += ag ? 1u : 0u;
        ip += adv ? (gb ? 4u : run + (hasm ? code + 1 : 0u) + (mat2 ? code2 + 1 : 0u)) : 0u;
        k = adv ? (gb ? 0u : km + (hasm ? 1u : 0u) + (mat2 ? 1u : 0u)) : k;
        m = adv ? (gb ? 0u : m | bm | bm2) : m;
        ra = adv ? (gb ? 0u : ra | ((code & 1u) ? bm : 0u) | ((code2 & 1u) ? bm2 : 0u)) : ra;
        rb = adv ? (gb ? 0u : rb | ((code & 2u) ? bm : 0u) | ((code2 & 2u) ? bm2 : 0u)) : rb;
        done_parse = done_parse | (go & (end | bad | !stepping));
        go = adv;
    }
    PROF_MARK(3);
    if (parsing && st == QLZX_OK && g > 0) myrec[g - 1] = GroupRec{rec_ip, m, ra, rb};
    PROF_FLUSH(0);
    vm_sync();
    if (!inrange) return;
    if (st == QLZX_OK && kind == kBlkCompressed && (!done_parse || g == 0)) st = QLZX_E_CORRUPT;
    BlkInfo bi{0, 0, kind, dsize};
    if (st != QLZX_OK) {
        bi.kind = kBlkSkip;
        status[i] = st;
        if (dsize_out && st != kPending) dsize_out[i] = 0;
    } else if (kind == kBlkCompressed) {
        bi.ngroups = g;
        bi.nitems = (g - 1) * 31 + (k > 31 ? 31 : k);
    } else if (kind == kBlkSkip) {  // dsize-0 compressed stream accepted above
        status[i] = QLZX_OK;
        if (dsize_out) dsize_out[i] = 0;
    }
    info[lin] = bi;
}

// ------------------------------------------------------------------------------- K2 ----
#ifndef QLZX_K2_BPL
#define QLZX_K2_BPL 4
#endif
#ifndef QLZX_K2_ASM_STORE
#define QLZX_K2_ASM_STORE 0
#endif
#ifndef QLZX_K2_COUNTED  // chunk loop with its trip count computed at entry
#define QLZX_K2_COUNTED 0
#endif
#ifndef QLZX_K2_FARSEL  // literal window byte written for every item that marks (no nested branch)
#define QLZX_K2_FARSEL 1
#endif
#ifndef QLZX_K2_FARALL  // far loads issued by every lane of a chunk with far bytes
#define QLZX_K2_FARALL 0
#endif
#ifndef QLZX_K2_FARSPLIT
#define QLZX_K2_FARSPLIT 0
#endif
#ifndef QLZX_K2_PRIO  // wave priority of K2 (s_setprio) over the overlapped K1
#define QLZX_K2_PRIO 0
#endif
#ifndef QLZX_K2_EARLYFAR  // far loads issued before the pointer jumping: measured slower
#define QLZX_K2_EARLYFAR 0
#endif
#ifndef QLZX_K2_WIN
#define QLZX_K2_WIN 4096
#endif
#ifndef QLZX_K2_MR
#define QLZX_K2_MR 256
#endif
constexpr uint32_t kV4W = QLZX_K2_WIN;   // output window (LDS ring)
constexpr uint32_t kV4MR = QLZX_K2_MR;   // marker ring (u32 keys)
constexpr uint32_t kV4Bpl = QLZX_K2_BPL;        // output bytes per lane per chunk (4 or 8)
constexpr uint32_t kV4Chunk = 64 * kV4Bpl;      // 256 or 512 output bytes per chunk
static_assert(kV4Chunk <= kV4MR, "a chunk's pointer-jumping array lives in its marker slots");

struct K2v4Lds {
    uint8_t win[kV4W];
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

__device__ __forceinline__ void dec_v4_block(K2v4Lds &L, const uint8_t *src, uint8_t *dst, uint32_t csize,
                                             const BlkInfo bi, const GroupRec *rb, int32_t *status_i,
                                             uint32_t *dsize_i, uint32_t lane) {
    constexpr uint32_t W = kV4W, MR = kV4MR, CH = kV4Chunk;
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
    uint64_t pend = 0;
    uint32_t pd = 0, pkey = 0;
    uint32_t plit = 0;

    // one batch: decode (posm, tok), prefetch the next batch's token from gr_next into
    // (posm_n, tok_n) and the GroupRec after it into gr_nn
    auto batch = [&](uint32_t posm, uint32_t tok, const GroupRec &gr_next, uint32_t &posm_n, uint32_t &tok_n,
                     GroupRec &gr_nn) __attribute__((always_inline)) {
        if (pend) {  // a straddling batch's items not marked by a chunk yet (all start below c + CH)
            const bool wr = (pend >> lane) & 1u;
            if (wr) {
                L.mk[pd & (MR - 1)] = pkey;
                if (plit < 0x100u) L.win[pd & (W - 1)] = (uint8_t)plit;
            }
            pend = 0;
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
#if QLZX_K2_FARSEL
            // a match's own window slot holds a byte older than the far bound (d < c + MR) that no
            // gather reads before the chunk of d overwrites it: the byte can go there unconditionally
            L.win[d & (W - 1)] = (uint8_t)t;
#else
            if (!ism) L.win[d & (W - 1)] = (uint8_t)t;
#endif
        }
        pend = __ballot(live && !wr);
        pd = d;
        pkey = key;
        plit = ism ? 0x100u : (t & 0xffu);
        D = __builtin_amdgcn_readfirstlane(D + total);
        bt++;
#ifdef QLZX_PROFILE
        _pacc[5] += 1;
#endif
    };

    // chunk phases while every item starting below c + 256 is known; true when the block is done
    auto chunks = [&]() __attribute__((always_inline)) -> bool {
#if QLZX_K2_COUNTED
        // D does not move while chunks run: the number of ready chunks is known up front
        const uint32_t left = c < dsize ? (dsize - c + CH - 1) / CH : 0u;
        uint32_t nch = complete ? left : (D >= c + CH ? min((D - c) / CH, left) : 0u);
        nch = __builtin_amdgcn_readfirstlane(nch);
        for (; nch; nch--) {
#else
        while (c < dsize && (complete || D >= c + CH)) {
#endif
            if (pend) {  // items of the last batch that start at or above c_prev + MR
                const bool wr = ((pend >> lane) & 1u) && pd < c + MR;
                if (wr) {
                    L.mk[pd & (MR - 1)] = pkey;
                    if (plit < 0x100u) L.win[pd & (W - 1)] = (uint8_t)plit;
                }
                pend &= ~__ballot(wr);
            }
            constexpr uint32_t B = kV4Bpl;
            const uint32_t r0 = B * lane, p0 = c + r0;
            uint32_t *mkl = L.mk + ((c & (MR - 1)) + r0);
            uint32_t m[B], sv[B];
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
            bool qa[B], anyq = false;
#pragma unroll
            for (uint32_t j = 0; j < B; j++) {
                f = max(f, m[j]);
                sv[j] = p0 + j - (f & 0xffffu);
                // in-chunk sources of match bytes: s in [c, p)  <=>  s - c < p - c (unsigned)
                qa[j] = sv[j] - c < r0 + j;
                anyq = anyq || qa[j];
            }
            PROF_MARK(1);
            const uint32_t lo = c + MR > W ? c + MR - W : 0u;
#if QLZX_K2_EARLYFAR
            // bytes whose source is older than the window: their loads go out now and land while
            // the pointer jumping and the window gather run (sources that jumping changes are in
            // the chunk, so a byte is far here exactly when its final source is a direct far one)
            uint32_t fv[B];
            bool fd[B], anyfd = false;
#pragma unroll
            for (uint32_t j = 0; j < B; j++) {
                fd[j] = sv[j] < lo;
                anyfd = anyfd || fd[j];
                fv[j] = 0;
            }
            const bool farq = __ballot(anyfd) != 0;
            if (farq) {
#pragma unroll
                for (uint32_t j = 0; j < B; j++)
                    if (fd[j]) fv[j] = dst[sv[j]];
            }
#endif
            if (__ballot(anyq)) {
                // the chunk's marker slots are free once read: they hold each byte's current source
                uint32_t *spb = L.mk + (c & (MR - 1));
#pragma unroll
                for (uint32_t h = 0; h < B; h += 4) *(uint4 *)(mkl + h) = make_uint4(sv[h], sv[h + 1], sv[h + 2], sv[h + 3]);
                do {
                    uint32_t t[B];
#pragma unroll
                    for (uint32_t j = 0; j < B; j++) t[j] = spb[(qa[j] ? sv[j] : p0 + j) - c];
#if QLZX_K2_JUMP_BALLOTS
                    // the wave's "any byte still jumping" as an OR of per-byte ballots (scalar
                    // masks), not an OR of the lanes' bools (packed into a bit vector per lane)
                    uint64_t anym = 0;
#pragma unroll
                    for (uint32_t j = 0; j < B; j++) {
                        // a byte whose source's source is outside the chunk or a literal is final
                        qa[j] = t[j] - c < sv[j] - c;
                        anym |= __ballot(qa[j]);
                        sv[j] = t[j];
                    }
                    anyq = anym != 0;
#else
                    anyq = false;
#pragma unroll
                    for (uint32_t j = 0; j < B; j++) {
                        // a byte whose source's source is outside the chunk or a literal is final
                        qa[j] = t[j] - c < sv[j] - c;
                        anyq = anyq || qa[j];
                        sv[j] = t[j];
                    }
#endif
#pragma unroll
                    for (uint32_t h = 0; h < B; h += 4)
                        *(uint4 *)(mkl + h) = make_uint4(sv[h], sv[h + 1], sv[h + 2], sv[h + 3]);
#ifdef QLZX_PROFILE
                    _pacc[7] += 1;
#endif
#if QLZX_K2_JUMP_BALLOTS
                } while (anyq);
#else
                } while (__ballot(anyq));
#endif
            }
            PROF_MARK(2);
            uint32_t vb[B];
            bool far = false;
#pragma unroll
            for (uint32_t j = 0; j < B; j++) {
                vb[j] = L.win[sv[j] & (W - 1)];
#if QLZX_K2_EARLYFAR
                far = far || (sv[j] < lo && !fd[j]);  // reached a far source through the chunk
#else
                far = far || sv[j] < lo;
#endif
            }
#if QLZX_K2_EARLYFAR
            if (farq) {
#pragma unroll
                for (uint32_t j = 0; j < B; j++) vb[j] = fd[j] ? fv[j] : vb[j];
            }
#endif
#ifdef QLZX_PROFILE
#if QLZX_K2_EARLYFAR
            _pacc[6] += (__ballot(far) || farq) ? 1 : 0;  // chunks with a byte older than the window
#else
            _pacc[6] += __ballot(far) ? 1 : 0;  // chunks with a byte older than the window
#endif
#endif
            uint32_t w[B / 4];
#if QLZX_K2_FARSPLIT
            // the far loads' wait stays inside their branch: a chunk without far bytes does not
            // wait for the previous chunk's store and the prefetched loads at a merged vmcnt(0)
            if (__ballot(far)) {
#pragma unroll
                for (uint32_t j = 0; j < B; j++)
                    if (sv[j] < lo) vb[j] = dst[sv[j]];
#pragma unroll
                for (uint32_t h = 0; h < B / 4; h++) {
                    w[h] = vb[4 * h] | (vb[4 * h + 1] << 8) | (vb[4 * h + 2] << 16) | (vb[4 * h + 3] << 24);
                    asm volatile("" : "+v"(w[h]));
                }
            } else {
#pragma unroll
                for (uint32_t h = 0; h < B / 4; h++)
                    w[h] = vb[4 * h] | (vb[4 * h + 1] << 8) | (vb[4 * h + 2] << 16) | (vb[4 * h + 3] << 24);
            }
#else
#ifndef QLZX_EXP_NOFAR  // (timing experiment: far bytes read from the window, wrong output)
            if (__ballot(far)) {
#if QLZX_K2_FARALL
                // every lane loads (a lane without a far byte reads the block's first output byte, which
                // it ignores): no exec-mask branch per byte -- measured slower (27.2 vs 27.0 ms on c2):
                // the loads of lanes without far bytes cost more than the branches they save
                uint32_t x[B];
#pragma unroll
                for (uint32_t j = 0; j < B; j++) x[j] = dst[sv[j] < lo ? sv[j] : 0u];
                // one barrier over all loads keeps them out of per-byte branches and in flight together
#pragma unroll
                for (uint32_t h = 0; h < B; h += 4) asm volatile("" : "+v"(x[h]), "+v"(x[h + 1]), "+v"(x[h + 2]), "+v"(x[h + 3]));
#pragma unroll
                for (uint32_t j = 0; j < B; j++) vb[j] = sv[j] < lo ? x[j] : vb[j];
#else
#pragma unroll
                for (uint32_t j = 0; j < B; j++)
                    if (sv[j] < lo) vb[j] = dst[sv[j]];
#endif
            }
#endif
#pragma unroll
            for (uint32_t h = 0; h < B / 4; h++)
                w[h] = vb[4 * h] | (vb[4 * h + 1] << 8) | (vb[4 * h + 2] << 16) | (vb[4 * h + 3] << 24);
#endif
            if constexpr (B == 8) {
                *(uint2 *)(L.win + (p0 & (W - 1))) = make_uint2(w[0], w[1]);
            } else {
                *(uint32_t *)(L.win + (p0 & (W - 1))) = w[0];
            }
#pragma unroll
            for (uint32_t h = 0; h < B; h += 4) *(uint4 *)(mkl + h) = make_uint4(0, 0, 0, 0);  // slots of c + MR ..
            PROF_MARK(3);
            if (c + CH <= dsize) {
#if QLZX_K2_ASM_STORE
                // stored behind the compiler's back: with no store in its VM_CNT bookkeeping it waits
                // for a prefetched load with vmcnt(N) instead of draining every store first (vm_sync()
                // at the end of the block orders them before the status word)
#pragma unroll
                for (uint32_t h = 0; h < B / 4; h++)
                    asm volatile("global_store_dword %0, %1, off" ::"v"(dst + p0 + 4 * h), "v"(w[h]) : "memory");
#else
                if constexpr (B == 8) {
                    if ((((uintptr_t)dst) & 7u) == 0) *(uint2 *)(dst + p0) = make_uint2(w[0], w[1]);
                    else *(uint32_t *)(dst + p0) = w[0], *(uint32_t *)(dst + p0 + 4) = w[1];
                } else {
                    *(uint32_t *)(dst + p0) = w[0];
                }
#endif
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

template <bool CRC>
__global__ void __launch_bounds__(64) k_dec_chunk4(qlzx_blocks b, uint32_t *dsize_out, int32_t *status,
                                                   uint32_t first, uint32_t count, const BlkInfo *info,
                                                   const GroupRec *recs, uint32_t gmax, const uint32_t *list,
                                                   const uint32_t *crc_state, const uint32_t *crc_expect,
                                                   uint32_t *crc_out) {
    __shared__ __attribute__((aligned(16))) K2v4Lds L;
#if QLZX_K2_PRIO
    // K2 waves first when they share a SIMD with the next chunk's K1 (which has slack)
    __builtin_amdgcn_s_setprio(QLZX_K2_PRIO);
#endif
    const uint32_t bx = blockIdx.x;
    if (bx >= count) return;
    const uint32_t i = list ? list[bx] : first + bx;
    if constexpr (CRC) {
        static_assert(sizeof(K2v4Lds) >= 4096, "the slicing-by-4 CRC tables fill 4 KiB of the window");
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
