// qlzx_decode_v5.hip -- round-5 batch decoder pair for blocks with dsize <= kW5 (16 KiB).
//
// Budget (DESIGN.md §3 "Decode v5"): the round-4 pair spent 24.7 K wave-instructions per
// 16 KiB block (K1 6.6 K, K2 18.1 K); the chip issues about one wave64 VALU per SIMD per two
// cycles, so that count alone set a floor near 13 ms.  This pair is laid out for fewer
// instructions per output byte:
//
// K1 k_dec_parse5  one LANE per block, the serial control-word chain of quicklz.c:513-671
//     (a literal run, the match that ends it and a second match when its first byte is in the
//     same dword).  The stream is read with plain unaligned global loads: no LDS at all, so K1
//     waves fill the wave slots that K2's LDS-heavy waves leave free.  Emits one GroupRec
//     {ip, cw, a, b} per control word (a, b: bit-planes of token bytes - 1), as k_dec_parse4.
//
// K2 k_dec_chunk5  one WAVE per block; the WHOLE output (dsize <= 16 KiB) stays in LDS, so no
//     byte is ever read back from HBM (round 4: a 4 KiB ring, 76 % of chunks had a far byte):
//     * ITEM PHASE (64 items per batch, one per lane): token position from the GroupRec,
//       branch-free token decode, DPP scan of the lengths; item i leaves ONE key
//       d << 16 | off in the marker ring.  A literal's byte goes to a literal area right
//       below the window, and its key's "offset" points there (off = 512 + (d & ~511)), so
//       literal and match bytes are gathered alike and a literal is never an in-chunk source.
//     * CHUNK PHASE (512 output bytes, 8 per lane): forward max-fill of the keys (in-lane
//       max + one DPP max-scan per 512 bytes), z = r0 - off per byte, in-chunk sources
//       (z >= -j) chased by pointer jumping, then one ds_read_u8 per byte from the window
//       (address = window + c + z, the byte index folded into the instruction offset), one
//       8-byte LDS store and one 8-byte global store per lane.
//     Blocks with dsize > kW5 take the round-4 path (dec_v4_block) inside the same kernel.
//
// Checks C1-C5 are applied exactly as by the oracle (oracle/qlz_oracle.c:180-231).
namespace qlzx {

#ifndef QLZX_K5_WIN
#define QLZX_K5_WIN 16384
#endif
#ifndef QLZX_K1_M2  // K1 v5: a second match per step from the same dword
#define QLZX_K1_M2 1
#endif
constexpr uint32_t kW5 = QLZX_K5_WIN;  // output window = whole block (no wrap)
constexpr uint32_t kC5 = 512;          // output bytes per chunk (8 per lane)
constexpr uint32_t kMR5 = 512;         // marker ring (u32 keys) = one chunk
static_assert(kW5 % kC5 == 0, "chunks tile the window");

// ------------------------------------------------------------------------------- K1 ----
// Token bytes - 1 of a match token from its first byte (quicklz.c:579-610):
// (b & 3) == 0 -> 0, 1 or 2 -> 1, 3 -> 2, and (b & 127) == 3 -> 3.
__device__ __forceinline__ uint32_t tok_e(uint32_t w) {
    const uint32_t x = w & 3u;
    return x - (x >> 1) + ((w & 127u) == 3u ? 1u : 0u);
}

// unaligned loads from global memory (global_load, not flat: the address space is explicit)
typedef const __attribute__((address_space(1))) uint32_t g_u32;
typedef const __attribute__((address_space(1))) uint64_t g_u64;
typedef const __attribute__((address_space(1))) uint8_t g_u8;
__device__ __forceinline__ uint32_t g_ld32(const uint8_t *p) { return *(g_u32 *)p; }
__device__ __forceinline__ uint64_t g_ld64(const uint8_t *p) { return *(g_u64 *)p; }

__global__ void __launch_bounds__(kParseWG) k_dec_parse5(qlzx_blocks b, const uint32_t *dst_cap, uint32_t *dsize_out,
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
        // the first control word must fit (C1); also keeps the clamped loads below inside the stream
        if (st == QLZX_OK && kind == kBlkCompressed && csize < hdr + 4) st = QLZX_E_CORRUPT;
    }
    const bool parsing = inrange && st == QLZX_OK && kind == kBlkCompressed;
    // ip = next stream byte; cwr = control bits not consumed yet with their sentinel (1: the
    // group is exhausted and the next step reads a control word); item index = clz(cwr)
    uint32_t ip = hdr, g = 0, cwr = 1, cwg = 0, ra = 0, rb = 0, rec_ip = 0;
    const uint32_t cs4 = parsing ? csize - 4 : 0;
    GroupRec *myrec = recs + (size_t)(inrange ? lin : 0) * gmax;
    bool done = !parsing, go = parsing;
    while (go) {  // per-lane loop: no cross-lane operation in the step
        const bool gb = cwr == 1;
        const uint32_t rem = csize - ip;
        uint32_t run = __builtin_ctz(cwr);  // literals before the next match (0 when gb)
        run = run < rem ? run : rem;
        const uint32_t q = ip + run;        // control word (gb) or the match token
        const uint32_t rest = cwr >> run;
        const bool end = ip + (gb ? 4u : 1u) > csize;
        const uint32_t qa = q < cs4 ? q : cs4;
        const uint32_t w = g_ld32(src + qa) >> (8 * (q - qa));
        const bool hasm = !gb & (rest != 1u) & ((rest & 1u) != 0) & (q < csize);
        const uint32_t e = tok_e(w);
#if QLZX_K1_M2
        const uint32_t q2 = q + e + 1, rest2 = rest >> 1;
        const bool hasm2 = hasm & (e < 3u) & ((rest2 & 1u) != 0) & (rest2 != 1u) & (q2 < csize);
        const uint32_t e2 = hasm2 ? tok_e(w >> (8 * (e + 1))) : 0u;
        const bool bad = !end & ((gb & (((w >> 31) == 0) | (g >= gmax))) | (hasm & (q2 > csize)) |
                                 (hasm2 & (q2 + e2 + 1 > csize)));
#else
        const bool bad = !end & ((gb & (((w >> 31) == 0) | (g >= gmax))) | (hasm & (q + e + 1 > csize)));
#endif
        if (end | bad) {
            st = bad ? QLZX_E_CORRUPT : st;
            done = !bad;
            go = false;
            break;
        }
        if (gb) {
            if (g > 0) myrec[g - 1] = GroupRec{rec_ip, cwg, ra, rb};
            rec_ip = ip;
            cwg = w;
            cwr = w;
            ra = 0;
            rb = 0;
            ip += 4;
            g++;
        } else {
            const uint32_t kb = hasm ? 1u << __builtin_clz(rest) : 0u;  // item index clz(rest)
#if QLZX_K1_M2
            const uint32_t kb2 = hasm2 ? kb << 1 : 0u;
            ra |= ((e & 1u) ? kb : 0u) | ((e2 & 1u) ? kb2 : 0u);
            rb |= ((e & 2u) ? kb : 0u) | ((e2 & 2u) ? kb2 : 0u);
            ip = q + (hasm ? e + 1 : 0u) + (hasm2 ? e2 + 1 : 0u);
            cwr = rest >> (hasm ? (hasm2 ? 2 : 1) : 0);
#else
            ra |= (e & 1u) ? kb : 0u;
            rb |= (e & 2u) ? kb : 0u;
            ip = q + (hasm ? e + 1 : 0u);
            cwr = rest >> (hasm ? 1 : 0);
#endif
        }
    }
    if (parsing && st == QLZX_OK && g > 0) myrec[g - 1] = GroupRec{rec_ip, cwg, ra, rb};
    vm_sync();
    if (!inrange) return;
    if (st == QLZX_OK && kind == kBlkCompressed && (!done || g == 0)) st = QLZX_E_CORRUPT;
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

// ------------------------------------------------------------------------------- K2 ----
struct K5Lds {
    uint8_t lit[kMR5];  // literal bytes of the items in the marker ring, at d & (kMR5 - 1)
    uint8_t win[kW5];   // output bytes 0 .. dsize - 1
    uint32_t mk[kMR5];  // keys d << 16 | off at d & (kMR5 - 1); pointer-jumping scratch
};
// the literal area sits right below the window, so a literal key's offset kMR5 + (d & ~(kMR5-1))
// sends window + d - off to lit + (d & (kMR5 - 1))
static_assert(offsetof(K5Lds, win) == offsetof(K5Lds, lit) + kMR5, "literal area below the window");

#ifndef QLZX_K5_FULL  // 1: whole-block window (dec_v5_block); 0: ring window (dec_v5r_block)
#define QLZX_K5_FULL 0
#endif

__device__ __forceinline__ uint32_t lit_off(uint32_t d) { return kMR5 + (d & ~(kMR5 - 1)); }

// blocks with dsize <= kW5 and csize >= 16 (compressed): see the file comment.
// Items: batch bt covers groups 4 bt .. 4 bt + 3; lane l takes items k0 = 2 (l & 15) and k0 + 1
// of group 4 bt + (l >> 4), so a lane reads one GroupRec and one 8-byte token window, and the
// second item's token starts right after the first (same group: k0 + 1 <= 31, item 31 absent).
__device__ __forceinline__ void dec_v5_block(K5Lds &L, const uint8_t *src, uint8_t *dst, uint32_t csize,
                                             const BlkInfo bi, const GroupRec *rb, int32_t *status_i,
                                             uint32_t *dsize_i, uint32_t lane) {
    constexpr uint32_t MR = kMR5, CH = kC5;
    const uint32_t dsize = bi.dsize;
    for (uint32_t q = lane * 4; q < MR; q += 256) *(uint4 *)(L.mk + q) = make_uint4(0, 0, 0, 0);

    const uint32_t nitems = bi.nitems, ngroups = bi.ngroups;
    const uint32_t hdr = (src[0] & 2u) ? 9u : 3u;
    const uint32_t nbt = (ngroups + 3) / 4;
    const uint32_t tail_from = dsize > QLZX_TAIL ? dsize - 1 - QLZX_TAIL : 0;  // op >= this: tail (quicklz.c:503)
    const uint32_t cs8 = csize - 8;
    const uint32_t glast = ngroups - 1;
    const uint32_t gl = lane >> 4, k0 = 2 * (lane & 15);
    const uint32_t low0 = (1u << k0) - 1u;

    // token window of this lane's first item in group g: W = stream bytes pos0 .. pos0 + 7 (zeros
    // past csize); mm = match bits of items k0, k0 + 1 (bits 0, 1) | the window's byte shift << 8
    auto tok_fetch = [&](const GroupRec &gr, uint32_t &pos0, uint32_t &mm, uint64_t &W) __attribute__((always_inline)) {
        pos0 = gr.ip + 4 + k0 + __builtin_popcount(gr.a & low0) + 2 * __builtin_popcount(gr.b & low0);
        mm = __builtin_amdgcn_ubfe(gr.m, k0, 2);
        const uint32_t pa = min(pos0, cs8);
        W = g_ld64(src + pa);
        mm |= (pos0 - pa) << 8;  // byte shift of the window, applied when it has landed
    };
    uint32_t pos0A, mmA, pos0B = 0, mmB = 0;
    uint64_t WA, WB = 0;
    GroupRec grA, grB;
    {
        const GroupRec g0 = rb[min(gl, glast)];
        tok_fetch(g0, pos0A, mmA, WA);
        grB = rb[min(4 + gl, glast)];
        grA = grB;
    }
    uint32_t D = 0, bt = 0, c = 0, cin = 0;
    bool tail = false, complete = false, err = false;
    // items that did not fit the marker ring when decoded (d >= c + MR), at most two per lane
    bool pp0 = false, pp1 = false, anyp = false;
    uint32_t pd0 = 0, pk0 = 0, pl0 = 0, pd1 = 0, pk1 = 0, pl1 = 0;
    const uint32_t r0 = lane * 8;
    uint8_t *const win = L.win;
    uint32_t *const mkl = L.mk + r0;

    auto flush_pend = [&]() __attribute__((always_inline)) {
        const bool w0 = pp0 && pd0 < c + MR, w1 = pp1 && pd1 < c + MR;
        if (w0) L.mk[pd0 & (MR - 1)] = pk0, L.lit[pd0 & (MR - 1)] = (uint8_t)pl0;
        if (w1) L.mk[pd1 & (MR - 1)] = pk1, L.lit[pd1 & (MR - 1)] = (uint8_t)pl1;
        pp0 = pp0 && !w0;
        pp1 = pp1 && !w1;
        anyp = __ballot(pp0 || pp1) != 0;
    };

    auto batch = [&](uint32_t pos0, uint32_t mm, uint64_t W, const GroupRec &gr_next, uint32_t &pos0_n,
                     uint32_t &mm_n, uint64_t &W_n, GroupRec &gr_nn) __attribute__((always_inline)) {
        if (anyp) flush_pend();
        const uint32_t g = 4 * bt + gl;
        const uint32_t i0 = 31 * g + k0;
        const bool v0 = i0 < nitems, v1 = i0 + 1 < nitems && k0 < 30;
        tok_fetch(gr_next, pos0_n, mm_n, W_n);
        gr_nn = rb[min(4 * bt + 8 + gl, glast)];
        W >>= 8 * (mm >> 8);
        const bool ism0 = v0 && (mm & 1u), ism1 = v1 && (mm & 2u);
        const uint32_t t0 = (uint32_t)W;
        uint32_t off0, ml0, tl0, off1, ml1, tl1;
        decode_tok_bf(t0, off0, ml0, tl0);
        tl0 = ism0 ? tl0 : 1u;
        const uint32_t t1 = (uint32_t)(W >> (8 * tl0));
        decode_tok_bf(t1, off1, ml1, tl1);
        const uint32_t len0 = ism0 ? ml0 : (v0 ? 1u : 0u);
        const uint32_t len1 = ism1 ? ml1 : (v1 ? 1u : 0u);
        const uint32_t sum = len0 + len1;
        const uint32_t incl = wave_incl_scan(sum);
        const uint32_t total = __builtin_amdgcn_readfirstlane(__builtin_amdgcn_readlane(incl, 63));
        const uint32_t d0 = D + incl - sum, d1 = d0 + len0;
        const bool live0 = v0 && d0 < dsize, live1 = v1 && d1 < dsize;
        bool bad, last = false;
        if (tail || D + total > tail_from) {
            tl1 = ism1 ? tl1 : 1u;
            const bool tl0l = live0 && !ism0 && d0 >= tail_from, tl1l = live1 && !ism1 && d1 >= tail_from;
            const uint64_t tail_lanes = __ballot(tl0l || tl1l);
            const uint32_t tail_lane = ff1_or(tail_lanes, 64u);  // C4: no match after the first tail literal
            const bool after0 = tail || lane > tail_lane, after1 = after0 || (lane == tail_lane && tl0l);
            tail = tail || tail_lanes != 0;
            const bool mok0 = off0 >= 3 && off0 <= d0 && d0 + len0 + 4 <= dsize && !after0;  // C3, C4
            const bool mok1 = off1 >= 3 && off1 <= d1 && d1 + len1 + 4 <= dsize && !after1;
            const bool last0 = live0 && d0 + len0 == dsize, last1 = live1 && d1 + len1 == dsize;
            last = last0 || last1;  // C5: the item completing dsize ends the stream
            const uint32_t ip_end = pos0 + tl0 + (last1 ? tl1 : 0u);
            const bool eok = ip_end == csize || (ip_end < hdr + 9 && csize == hdr + 9);
            bad = (live0 && ism0 && !mok0) || (live1 && ism1 && !mok1) || (last && !eok);
        } else {
            bad = (ism0 && (off0 < 3 || off0 > d0)) || (ism1 && (off1 < 3 || off1 > d1));  // C3
        }
        if (__ballot(bad)) {
            err = true;
            return;
        }
        complete = __ballot(last) != 0;
        const uint32_t key0 = (d0 << 16) | (ism0 ? off0 : lit_off(d0));
        const uint32_t key1 = (d1 << 16) | (ism1 ? off1 : lit_off(d1));
        const bool wr0 = live0 && d0 < c + MR, wr1 = live1 && d1 < c + MR;
        if (wr0) L.mk[d0 & (MR - 1)] = key0, L.lit[d0 & (MR - 1)] = (uint8_t)t0;  // a match's slot is never read
        if (wr1) L.mk[d1 & (MR - 1)] = key1, L.lit[d1 & (MR - 1)] = (uint8_t)t1;
        pp0 = live0 && !wr0;
        pp1 = live1 && !wr1;
        pd0 = d0, pk0 = key0, pl0 = t0, pd1 = d1, pk1 = key1, pl1 = t1;
        anyp = __ballot(pp0 || pp1) != 0;
        D = __builtin_amdgcn_readfirstlane(D + total);
        bt++;
    };

    // chunk phases while every item starting below c + CH is known; true when the block is done
    auto chunks = [&]() __attribute__((always_inline)) -> bool {
        while (c < dsize && (complete || D >= c + CH)) {
            if (anyp) flush_pend();
            uint32_t m[8];
            {
                const uint4 q0 = *(const uint4 *)(mkl), q1 = *(const uint4 *)(mkl + 4);
                m[0] = q0.x, m[1] = q0.y, m[2] = q0.z, m[3] = q0.w, m[4] = q1.x, m[5] = q1.y, m[6] = q1.z, m[7] = q1.w;
            }
            *(uint4 *)(mkl) = make_uint4(0, 0, 0, 0);  // slots of c + MR ..
            *(uint4 *)(mkl + 4) = make_uint4(0, 0, 0, 0);
            const uint32_t lmax = max(max(max(m[0], m[1]), max(m[2], m[3])), max(max(m[4], m[5]), max(m[6], m[7])));
            const uint32_t incl = v4_incl_max(lmax);
            uint32_t f = max(wave_shr1(incl), cin);
            cin = max(cin, (uint32_t)__builtin_amdgcn_readfirstlane(__builtin_amdgcn_readlane(incl, 63)));
            // source of byte c + r0 + j: window + P + j with P = c + r0 - off (a literal's lands in
            // the literal area below the window)
            const int P0 = (int)(c + r0);
            int S[8];
            uint32_t omin = 0xffffu;
#pragma unroll
            for (uint32_t j = 0; j < 8; j++) {
                f = max(f, m[j]);
                S[j] = P0 - (int)(f & 0xffffu);
                omin = min(omin, f & 0xffffu);
            }
            uint32_t vb[8];
#pragma unroll
            for (uint32_t j = 0; j < 8; j++) vb[j] = win[S[j] + (int)j];
            uint32_t w0 = vb[0] | (vb[1] << 8) | (vb[2] << 16) | (vb[3] << 24);
            uint32_t w1 = vb[4] | (vb[5] << 8) | (vb[6] << 16) | (vb[7] << 24);
            *(uint2 *)(win + P0) = make_uint2(w0, w1);
            // a source inside this chunk (off <= r0 + j) read a byte of this chunk: gather again
            // until nothing changes (the sources form a DAG, so the fixed point is the output)
            if (__ballot(omin <= r0 + 7)) {
                bool ch;
                do {
#pragma unroll
                    for (uint32_t j = 0; j < 8; j++) vb[j] = win[S[j] + (int)j];
                    const uint32_t n0 = vb[0] | (vb[1] << 8) | (vb[2] << 16) | (vb[3] << 24);
                    const uint32_t n1 = vb[4] | (vb[5] << 8) | (vb[6] << 16) | (vb[7] << 24);
                    ch = __ballot(n0 != w0 || n1 != w1) != 0;
                    w0 = n0, w1 = n1;
                    *(uint2 *)(win + P0) = make_uint2(w0, w1);
                } while (ch);
            }
            if (c + CH <= dsize) {
                if ((((uintptr_t)dst) & 7u) == 0) *(uint2 *)(dst + P0) = make_uint2(w0, w1);
                else *(uint32_t *)(dst + P0) = w0, *(uint32_t *)(dst + P0 + 4) = w1;
            } else {
                for (uint32_t j = 0; j < 8 && c + r0 + j < dsize; j++)
                    dst[c + r0 + j] = (uint8_t)((j < 4 ? w0 : w1) >> (8 * (j & 3)));
            }
            c += CH;
        }
        return c >= dsize;
    };

    for (;;) {
        if (bt >= nbt) { err = true; break; }  // stream ended before dsize (check C5)
        batch(pos0A, mmA, WA, grB, pos0B, mmB, WB, grA);
        if (err || chunks()) break;
        if (bt >= nbt) { err = true; break; }
        batch(pos0B, mmB, WB, grA, pos0A, mmA, WA, grB);
        if (err || chunks()) break;
    }
    vm_sync();
    if (lane == 0) {
        *status_i = err ? QLZX_E_CORRUPT : QLZX_OK;
        if (dsize_i) *dsize_i = err ? 0u : dsize;
    }
}

// ------------------------------------------------------------ K2, ring window ----
// The same item and chunk phases over a kWr-byte ring window (8-9 KiB of LDS per wave instead of
// 19 KiB, so 3x the waves per CU).  Differences from dec_v5_block:
// * a literal's byte goes to its own ring slot and its key's offset is 0 (own slot);
// * a byte whose source is older than the valid ring window [c + CH - kWr, c) (the slots of the
//   chunk being gathered are overwritten by its passes) is "far": it is read once from the
//   block's output in HBM (final there) into a per-lane staging slot and gathered from there;
// * ring addresses wrap; a 16-byte mirror after the ring keeps the 8 byte reads of a lane
//   contiguous.
#ifndef QLZX_K5_RING
#define QLZX_K5_RING 4096
#endif
constexpr uint32_t kWr = QLZX_K5_RING;
struct K5rLds {
    uint8_t win[kWr + 16];  // ring + mirror of slots 0..15
    uint32_t mk[kMR5];
    uint8_t far[kC5];       // far bytes of the chunk, 8 per lane
};

__device__ __forceinline__ void dec_v5r_block(K5rLds &L, const uint8_t *src, uint8_t *dst, uint32_t csize,
                                              const BlkInfo bi, const GroupRec *rb, int32_t *status_i,
                                              uint32_t *dsize_i, uint32_t lane) {
    constexpr uint32_t MR = kMR5, CH = kC5, W = kWr;
    const uint32_t dsize = bi.dsize;
    for (uint32_t q = lane * 4; q < MR; q += 256) *(uint4 *)(L.mk + q) = make_uint4(0, 0, 0, 0);

    const uint32_t nitems = bi.nitems, ngroups = bi.ngroups;
    const uint32_t hdr = (src[0] & 2u) ? 9u : 3u;
    const uint32_t nbt = (ngroups + 3) / 4;
    const uint32_t tail_from = dsize > QLZX_TAIL ? dsize - 1 - QLZX_TAIL : 0;  // op >= this: tail (quicklz.c:503)
    const uint32_t cs8 = csize - 8;
    const uint32_t glast = ngroups - 1;
    const uint32_t gl = lane >> 4, k0 = 2 * (lane & 15);
    const uint32_t low0 = (1u << k0) - 1u;

    auto tok_fetch = [&](const GroupRec &gr, uint32_t &pos0, uint32_t &mm, uint64_t &Wd) __attribute__((always_inline)) {
        pos0 = gr.ip + 4 + k0 + __builtin_popcount(gr.a & low0) + 2 * __builtin_popcount(gr.b & low0);
        mm = __builtin_amdgcn_ubfe(gr.m, k0, 2);
        const uint32_t pa = min(pos0, cs8);
        Wd = g_ld64(src + pa);
        mm |= (pos0 - pa) << 8;
    };
    // two batches in flight: at batch b the tokens of b + 1 and b + 2 and the GroupRecs of b + 3
    // and b + 4 are loading (register sets A/B alternate between even and odd batches)
    uint32_t pos0A, mmA, pos0B, mmB;
    uint64_t WA, WB;
    GroupRec grA, grB;
    {
        const GroupRec g0 = rb[min(gl, glast)], g1 = rb[min(4 + gl, glast)];
        tok_fetch(g0, pos0A, mmA, WA);
        tok_fetch(g1, pos0B, mmB, WB);
        grA = rb[min(8 + gl, glast)];
        grB = rb[min(12 + gl, glast)];
    }
    uint32_t touch = 0;  // far sources touched ahead (into L2); consumed at the end of the block
    uint32_t D = 0, bt = 0, c = 0, cin = 0;
    bool tail = false, complete = false, err = false;
    bool pp0 = false, pp1 = false, anyp = false;
    uint32_t pd0 = 0, pk0 = 0, pl0 = 0, pd1 = 0, pk1 = 0, pl1 = 0;
    const uint32_t r0 = lane * 8;
    uint8_t *const win = L.win;
    uint32_t *const mkl = L.mk + r0;

    PROF_DECL
    auto flush_pend = [&]() __attribute__((always_inline)) {
        const bool w0 = pp0 && pd0 < c + MR, w1 = pp1 && pd1 < c + MR;
        if (w0) L.mk[pd0 & (MR - 1)] = pk0, win[pd0 & (W - 1)] = (uint8_t)pl0;
        if (w1) L.mk[pd1 & (MR - 1)] = pk1, win[pd1 & (W - 1)] = (uint8_t)pl1;
        pp0 = pp0 && !w0;
        pp1 = pp1 && !w1;
        anyp = __ballot(pp0 || pp1) != 0;
    };

    auto batch = [&](uint32_t &pos0r, uint32_t &mmr, uint64_t &Wr, GroupRec &gr) __attribute__((always_inline)) {
        if (anyp) flush_pend();
        const uint32_t g = 4 * bt + gl;
        const uint32_t i0 = 31 * g + k0;
        const bool v0 = i0 < nitems, v1 = i0 + 1 < nitems && k0 < 30;
        const uint32_t pos0 = pos0r, mm = mmr;
        uint64_t Wd = Wr;
        tok_fetch(gr, pos0r, mmr, Wr);          // tokens of batch bt + 2
        gr = rb[min(4 * bt + 16 + gl, glast)];  // GroupRecs of batch bt + 4
        Wd >>= 8 * (mm >> 8);
        const bool ism0 = v0 && (mm & 1u), ism1 = v1 && (mm & 2u);
        const uint32_t t0 = (uint32_t)Wd;
        uint32_t off0, ml0, tl0, off1, ml1, tl1;
        decode_tok_bf(t0, off0, ml0, tl0);
        tl0 = ism0 ? tl0 : 1u;
        const uint32_t t1 = (uint32_t)(Wd >> (8 * tl0));
        decode_tok_bf(t1, off1, ml1, tl1);
        const uint32_t len0 = ism0 ? ml0 : (v0 ? 1u : 0u);
        const uint32_t len1 = ism1 ? ml1 : (v1 ? 1u : 0u);
        const uint32_t sum = len0 + len1;
        const uint32_t incl = wave_incl_scan(sum);
        const uint32_t total = __builtin_amdgcn_readfirstlane(__builtin_amdgcn_readlane(incl, 63));
        const uint32_t d0 = D + incl - sum, d1 = d0 + len0;
        const bool live0 = v0 && d0 < dsize, live1 = v1 && d1 < dsize;
        bool bad, last = false;
        if (tail || D + total > tail_from) {
            tl1 = ism1 ? tl1 : 1u;
            const bool tl0l = live0 && !ism0 && d0 >= tail_from, tl1l = live1 && !ism1 && d1 >= tail_from;
            const uint64_t tail_lanes = __ballot(tl0l || tl1l);
            const uint32_t tail_lane = ff1_or(tail_lanes, 64u);  // C4: no match after the first tail literal
            const bool after0 = tail || lane > tail_lane, after1 = after0 || (lane == tail_lane && tl0l);
            tail = tail || tail_lanes != 0;
            const bool mok0 = off0 >= 3 && off0 <= d0 && d0 + len0 + 4 <= dsize && !after0;  // C3, C4
            const bool mok1 = off1 >= 3 && off1 <= d1 && d1 + len1 + 4 <= dsize && !after1;
            const bool last0 = live0 && d0 + len0 == dsize, last1 = live1 && d1 + len1 == dsize;
            last = last0 || last1;  // C5: the item completing dsize ends the stream
            const uint32_t ip_end = pos0 + tl0 + (last1 ? tl1 : 0u);
            const bool eok = ip_end == csize || (ip_end < hdr + 9 && csize == hdr + 9);
            bad = (live0 && ism0 && !mok0) || (live1 && ism1 && !mok1) || (last && !eok);
        } else {
            bad = (ism0 && (off0 < 3 || off0 > d0)) || (ism1 && (off1 < 3 || off1 > d1));  // C3
        }
        if (__ballot(bad)) {
            err = true;
            return;
        }
        complete = __ballot(last) != 0;
        const uint32_t key0 = (d0 << 16) | (ism0 ? off0 : 0u);
        const uint32_t key1 = (d1 << 16) | (ism1 ? off1 : 0u);
        {
            // a match whose source will be older than the ring window: touch it now, so the chunk
            // phase's far load hits L2 (unconditional loads: a conditional one would be waited on)
            const bool f0 = live0 && ism0 && off0 + 2 * CH > W, f1 = live1 && ism1 && off1 + 2 * CH > W;
            touch ^= *(g_u8 *)(dst + (f0 ? d0 - off0 : 0u));
            touch ^= *(g_u8 *)(dst + (f1 ? d1 - off1 : 0u));
        }
        const bool wr0 = live0 && d0 < c + MR, wr1 = live1 && d1 < c + MR;
        // a literal's byte goes to its own slot; a match's own slot holds a byte older than the valid
        // window (d < c + MR), so its token byte may go there too
        if (wr0) L.mk[d0 & (MR - 1)] = key0, win[d0 & (W - 1)] = (uint8_t)t0;
        if (wr1) L.mk[d1 & (MR - 1)] = key1, win[d1 & (W - 1)] = (uint8_t)t1;
        pp0 = live0 && !wr0;
        pp1 = live1 && !wr1;
        pd0 = d0, pk0 = key0, pl0 = t0, pd1 = d1, pk1 = key1, pl1 = t1;
        anyp = __ballot(pp0 || pp1) != 0;
        D = __builtin_amdgcn_readfirstlane(D + total);
        bt++;
#ifdef QLZX_PROFILE
        _pacc[5] += 1;
#endif
        PROF_MARK(0);
    };

    auto chunks = [&]() __attribute__((always_inline)) -> bool {
        while (c < dsize && (complete || D >= c + CH)) {
            if (anyp) flush_pend();
            uint32_t m[8];
            {
                const uint4 q0 = *(const uint4 *)(mkl), q1 = *(const uint4 *)(mkl + 4);
                m[0] = q0.x, m[1] = q0.y, m[2] = q0.z, m[3] = q0.w, m[4] = q1.x, m[5] = q1.y, m[6] = q1.z, m[7] = q1.w;
            }
            *(uint4 *)(mkl) = make_uint4(0, 0, 0, 0);
            *(uint4 *)(mkl + 4) = make_uint4(0, 0, 0, 0);
            const uint32_t lmax = max(max(max(m[0], m[1]), max(m[2], m[3])), max(max(m[4], m[5]), max(m[6], m[7])));
            const uint32_t incl = v4_incl_max(lmax);
            uint32_t f = max(wave_shr1(incl), cin);
            cin = max(cin, (uint32_t)__builtin_amdgcn_readfirstlane(__builtin_amdgcn_readlane(incl, 63)));
            const int P0 = (int)(c + r0);
            const int lo = (int)(c + CH) - (int)W;  // sources below lo are far
            const uint32_t own = P0 & (W - 1);      // this lane's ring slots
            int S[8];
            uint32_t A[8];
            uint64_t farm = 0;
            bool lfar = false, lin = false;
#pragma unroll
            for (uint32_t j = 0; j < 8; j++) {
                f = max(f, m[j]);
                S[j] = P0 - (int)(f & 0xffffu);  // source of byte P0 + j is S + j (own slot: a literal)
                A[j] = (uint32_t)S[j] & (W - 1);
                const bool fj = S[j] + (int)j < lo;
                farm |= __ballot(fj);
                lfar = lfar || fj;
                lin = lin || (S[j] + (int)j >= (int)c && S[j] != P0);  // a source in this chunk
            }
            PROF_MARK(1);
            if (farm) {
#ifdef QLZX_PROFILE
                _pacc[7] += 1;
#endif
                // far bytes: once from the output in HBM to the lane's staging slot, gathered there
                // (all eight loads in flight before one wait: a lane's non-far bytes read dst[0],
                // final since c >= kWr - CH whenever a far byte exists)
                const uint32_t fs = (uint32_t)(L.far + r0 - win);
                if (lfar) {
                    uint32_t fv[8];
#pragma unroll
                    for (uint32_t j = 0; j < 8; j++) {
                        const bool fj = S[j] + (int)j < lo;
                        fv[j] = *(g_u8 *)(dst + (fj ? S[j] + (int)j : 0));
                        A[j] = fj ? fs : A[j];
                    }
                    *(uint2 *)(L.far + r0) = make_uint2(fv[0] | (fv[1] << 8) | (fv[2] << 16) | (fv[3] << 24),
                                                        fv[4] | (fv[5] << 8) | (fv[6] << 16) | (fv[7] << 24));
                }
            }
            PROF_MARK(2);
            uint32_t vb[8];
#pragma unroll
            for (uint32_t j = 0; j < 8; j++) vb[j] = win[A[j] + j];
            uint32_t w0 = vb[0] | (vb[1] << 8) | (vb[2] << 16) | (vb[3] << 24);
            uint32_t w1 = vb[4] | (vb[5] << 8) | (vb[6] << 16) | (vb[7] << 24);
            const bool mirror = (c & (W - 1)) == 0;  // lane 0's slots 0..7 are mirrored at W..W+7
            *(uint2 *)(win + own) = make_uint2(w0, w1);
            if (mirror && lane == 0) *(uint2 *)(win + W) = make_uint2(w0, w1);
            // lanes with a source in this chunk gather again until nothing changes (the sources
            // form a DAG, so the fixed point is the output; see dec_v5_block)
            PROF_MARK(3);
            if (__ballot(lin)) {
                bool ch;
                do {
#ifdef QLZX_PROFILE
                    _pacc[6] += 1;
#endif
                    bool mine = false;
                    if (lin) {
#pragma unroll
                        for (uint32_t j = 0; j < 8; j++) vb[j] = win[A[j] + j];
                        const uint32_t n0 = vb[0] | (vb[1] << 8) | (vb[2] << 16) | (vb[3] << 24);
                        const uint32_t n1 = vb[4] | (vb[5] << 8) | (vb[6] << 16) | (vb[7] << 24);
                        mine = n0 != w0 || n1 != w1;
                        w0 = n0, w1 = n1;
                        *(uint2 *)(win + own) = make_uint2(w0, w1);
                        if (mirror && lane == 0) *(uint2 *)(win + W) = make_uint2(w0, w1);
                    }
                    ch = __ballot(mine) != 0;
                } while (ch);
            }
            if (c + CH <= dsize) {
                if ((((uintptr_t)dst) & 7u) == 0) *(uint2 *)(dst + P0) = make_uint2(w0, w1);
                else *(uint32_t *)(dst + P0) = w0, *(uint32_t *)(dst + P0 + 4) = w1;
            } else {
                for (uint32_t j = 0; j < 8 && c + r0 + j < dsize; j++)
                    dst[c + r0 + j] = (uint8_t)((j < 4 ? w0 : w1) >> (8 * (j & 3)));
            }
            c += CH;
            PROF_MARK(4);
        }
        return c >= dsize;
    };

    for (;;) {
        if (bt >= nbt) { err = true; break; }  // stream ended before dsize (check C5)
        batch(pos0A, mmA, WA, grA);
        if (err || chunks()) break;
        if (bt >= nbt) { err = true; break; }
        batch(pos0B, mmB, WB, grB);
        if (err || chunks()) break;
    }
    asm volatile("" ::"v"(touch));
    vm_sync();
    PROF_FLUSH(1);
    if (lane == 0) {
        *status_i = err ? QLZX_E_CORRUPT : QLZX_OK;
        if (dsize_i) *dsize_i = err ? 0u : dsize;
    }
}

template <bool CRC>
__global__ void __launch_bounds__(64) k_dec_chunk5(qlzx_blocks b, uint32_t *dsize_out, int32_t *status,
                                                   uint32_t first, uint32_t count, const BlkInfo *info,
                                                   const GroupRec *recs, uint32_t gmax, const uint32_t *list,
                                                   const uint32_t *crc_state, const uint32_t *crc_expect,
                                                   uint32_t *crc_out) {
#if QLZX_K5_FULL
    __shared__ __attribute__((aligned(16))) union { K5Lds v5; K2v4Lds v4; } L;
#else
    __shared__ __attribute__((aligned(16))) union { K5rLds v5; K2v4Lds v4; } L;
#endif
    const uint32_t bx = blockIdx.x;
    if (bx >= count) return;
    const uint32_t i = list ? list[bx] : first + bx;
    if constexpr (CRC) {
        const uint32_t lane = threadIdx.x;
        uint32_t *tab = (uint32_t *)L.v5.win;
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
    const uint8_t *src = b.src + b.src_off[i];
    uint8_t *dst = b.dst + b.dst_off[i];
#if QLZX_K5_FULL
    if (bi.kind == kBlkCompressed && bi.dsize <= kW5 && b.src_len[i] >= 16)
        dec_v5_block(L.v5, src, dst, b.src_len[i], bi, recs + (size_t)bx * gmax, status + i,
                     dsize_out ? dsize_out + i : nullptr, threadIdx.x);
#else
    if (bi.kind == kBlkCompressed && bi.dsize <= 65536 && b.src_len[i] >= 16)
        dec_v5r_block(L.v5, src, dst, b.src_len[i], bi, recs + (size_t)bx * gmax, status + i,
                     dsize_out ? dsize_out + i : nullptr, threadIdx.x);
#endif
    else  // stored blocks and dsize > kW5
        dec_v4_block(L.v4, src, dst, b.src_len[i], bi, recs + (size_t)bx * gmax, status + i,
                     dsize_out ? dsize_out + i : nullptr, threadIdx.x);
}

}  // namespace qlzx
