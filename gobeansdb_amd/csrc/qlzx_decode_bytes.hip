// qlzx_decode_bytes.hip -- K2 "byte-parallel": one WAVE per block, output produced 256 bytes
// (one CHUNK) at a time, 4 bytes per lane, each byte gathered from the position it copies.
//
// K1 (k_dec_parse, qlzx_decode_wave.hip) still walks the serial control-word chain and emits
// one GroupRec per control word.  This kernel replaced the item-per-lane K2 of rounds 1-2
// (k_dec_blocks, removed in round 3), whose cost was the per-item 16-B masked copies and their
// readiness sub-rounds (≈580 instructions per 64 items).  Here the work per output
// byte is a gather:
//
//   ITEM PHASE (64 items per batch, one per lane; quicklz.c:513-671 restated item-parallel):
//     token position from the GroupRec (ip + 4 + k + popc(a & low(k)) + 2 popc(b & low(k))),
//     branch-free token decode, DPP scan of the output lengths -> start d of every item,
//     checks C3-C5.  Every item leaves ONE u16 marker at its start in a marker
//     ring (the match offset, or 1 for a literal) and a literal also leaves its byte in the
//     output window.  Nothing else is copied here.
//
//   CHUNK PHASE (bytes [c, c + 256), lane l owns c + 4l .. c + 4l + 3):
//     1. read the lane's four markers, forward-fill them (in-lane selects + a DPP max-scan of
//        "last marker" across lanes + the previous chunk's carry): every byte p now knows the
//        offset of the item covering it, so its source is s = p - off (s = p for a literal);
//     2. sources inside this chunk (a match whose offset is < 256) are chased by pointer
//        jumping over a per-chunk u16 array (log2 of the chain depth rounds; 0 for ~90 % of
//        the chunks of text);
//     3. gather: a source at or above c + MR - W is in the LDS window, an older one is read
//        back from the block's destination in HBM, where every finished chunk was stored;
//     4. the lane's dword goes to the window and, as one coalesced 256-B wave store, to HBM.
//
// LDS: the output ring win[W] (position p at p & (W-1)), the marker ring mk[MR] (u16 per
// output position, zero = no item starts here) and the chunk pointer array (256 x u16).
// Items may only mark positions below c + MR, so a literal write never lands on a window slot
// a chunk still reads: the slot of d < c + MR holds d - W < c + MR - W, which is "far" for
// chunk c and every later one.  Markers are cleared as a chunk reads them.
#include "qlzx_device.h"

namespace qlzx {

constexpr uint32_t kChunk = 256;        // output bytes per chunk phase (4 per lane)
constexpr uint16_t kMkLit = 1;          // marker of a literal (match offsets are >= 3, check C3)
constexpr uint16_t kSpLit = 0xFFFFu;    // pointer-array entry of a literal byte (no source)

template <uint32_t W, uint32_t MR>
struct K2bLds {
    uint8_t win[W];
    uint16_t mk[MR];
    uint16_t sp[kChunk];
};

// Inclusive max over lanes 0..lane (DPP row shifts + row broadcasts).
__device__ __forceinline__ uint32_t wave_incl_max(uint32_t v) {
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false));  // row_shr:1
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false));  // row_shr:2
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false));  // row_shr:4
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false));  // row_shr:8
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false));  // row_bcast:15
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false));  // row_bcast:31
    return v;
}
// Value of lane - 1 (0 in lane 0): DPP wave_shr:1.
__device__ __forceinline__ uint32_t wave_shr1(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x138, 0xf, 0xf, false);
}

// One block by one wave (lane = 0..63): src/csize its stream, dst its output, bi/rb what K1
// (or the solo parse, qlzx_decode_solo.hip) found; the block's status and size go to
// *status_i / *dsize_i.  kind is kBlkStored or kBlkCompressed.
template <uint32_t W, uint32_t MR>
__device__ __forceinline__ void dec_bytes_block(K2bLds<W, MR> &L, const uint8_t *src, uint8_t *dst,
                                                uint32_t csize, const BlkInfo bi, const GroupRec *rb,
                                                int32_t *status_i, uint32_t *dsize_i, uint32_t lane) {
    static_assert(W >= 2 * MR && MR >= kChunk && (W & (W - 1)) == 0 && (MR & (MR - 1)) == 0, "ring sizes");
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
    for (uint32_t q = lane * 16; q < MR * 2; q += 1024) *(uint4 *)((uint8_t *)L.mk + q) = make_uint4(0, 0, 0, 0);

    const uint32_t nitems = bi.nitems;
    const uint32_t hdr = (src[0] & 2u) ? 9u : 3u;
    const uint32_t nb = (nitems + 63) / 64;
    const uint32_t tail_from = dsize > QLZX_TAIL ? dsize - 1 - QLZX_TAIL : 0;  // op >= this: tail (quicklz.c:503)

    // ---- prefetch pipeline: the GroupRec of batch bt+1 and the token dword of batch bt are in
    // registers (loaded while batch bt-1 was decoded; plain loads, so the compiler waits for them)
    ItemCursor c1{lane / 31, lane % 31};  // item coordinates of batch bt+1 once the prologue ran
    auto load_rec = [&](const ItemCursor &c, bool v) -> GroupRec { return rb[v ? c.g : 0u]; };
    auto tok_pos = [&](const GroupRec &gr, const ItemCursor &c, bool v, uint32_t &p) -> uint32_t {
        const uint32_t low = (1u << c.k) - 1u;
        const uint32_t pos = gr.ip + 4 + c.k + __builtin_popcount(gr.a & low) + 2 * __builtin_popcount(gr.b & low);
        p = v ? (pos + 4 <= csize ? pos : csize - 4) : 0u;
        return v ? (pos | (((gr.m >> c.k) & 1u) << 31)) : 0u;
    };
    uint32_t posm0, tok0, tp;
    {
        const bool v0 = lane < nitems;
        const GroupRec g0 = load_rec(c1, v0);
        posm0 = tok_pos(g0, c1, v0, tp);
        tok0 = *(const uint32_t *)(src + tp);  // unaligned dword (unaligned access mode)
    }
    c1.next();
    GroupRec gr1 = load_rec(c1, 64 + lane < nitems);
    PROF_DECL
    uint32_t D = 0;          // output start of the next batch's first item
    uint32_t bt = 0;         // next batch to decode
    bool tail = false, complete = dsize == 0, err = false;
    uint64_t pend = 0;       // lanes of the held batch whose marker is not written yet
    uint32_t pd = 0, pmk = 0;  // held item: start d, marker | literal byte << 16
    uint32_t cin = 0;        // marker carried into the next chunk (the last item start before it)
    for (uint32_t c = 0; c < dsize; c += kChunk) {
        // ---- item phase: every item starting before c + kChunk gets its marker ----
        for (;;) {
            if (pend == 0) {
                if (complete || D >= c + kChunk) break;
                if (bt >= nb) { err = true; break; }  // stream ended before dsize (check C5)
                const bool v = bt * 64 + lane < nitems;
                // prefetch: token of batch bt+1 (its GroupRec is in gr1), GroupRec of batch bt+2
                const bool v1 = (bt + 1) * 64 + lane < nitems;
                const uint32_t posm1 = tok_pos(gr1, c1, v1, tp);
                const uint32_t tok1 = *(const uint32_t *)(src + tp);
                c1.next();
                gr1 = load_rec(c1, (bt + 2) * 64 + lane < nitems);
                // decode batch bt
                const bool ism = (posm0 >> 31) != 0;
                const uint32_t pos = posm0 & 0x7fffffffu;
                const uint32_t t = pos + 4 <= csize ? tok0 : tok0 >> (8 * (pos + 4 - csize));
                uint32_t off, mlen, tl;
                decode_tok_bf(t, off, mlen, tl);
                const uint32_t len = ism ? mlen : (v ? 1u : 0u);
                tl = ism ? tl : 1u;
                const uint32_t incl = wave_incl_scan(len);
                const uint32_t total = __builtin_amdgcn_readfirstlane(__builtin_amdgcn_readlane(incl, 63));
                const uint32_t d = D + incl - len;
                // checks C3-C5 on the live items (those that start before dsize).  Until the batch
                // reaches the tail (the last 11 bytes) every item ends <= dsize - 11, so only
                // 3 <= off <= d (C3) can fail there.
                const bool live = v && d < dsize;
                bool bad, last = false;
                if (tail || D + total > tail_from) {
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
                if (__ballot(bad)) { err = true; break; }
                complete = __ballot(last) != 0;
                pend = __ballot(live);
                pd = d;
                pmk = (ism ? off : kMkLit) | ((t & 0xffu) << 16);
                D = __builtin_amdgcn_readfirstlane(D + total);
                posm0 = posm1;
                tok0 = tok1;
                bt++;
#ifdef QLZX_PROFILE
                _pacc[5] += 1;  // batches decoded
#endif
            }
            // markers (and literal bytes) of the held items that start below c + MR
            const bool wr = ((pend >> lane) & 1u) && pd < c + MR;
            const uint64_t wm = __ballot(wr);
            if (wr) {
                L.mk[pd & (MR - 1)] = (uint16_t)pmk;
                if ((pmk & 0xffffu) == kMkLit) L.win[pd & (W - 1)] = (uint8_t)(pmk >> 16);
            }
            pend &= ~wm;
#ifdef QLZX_PROFILE
            _pacc[6] += 1;  // marker passes
#endif
            if (pend) break;  // the rest start at or above c + MR >= c + kChunk
        }
        if (err) break;
        PROF_MARK(0);  // 0: item phase
        // ---- chunk phase: bytes p_j = c + 4 lane + j ----
        const uint32_t p0 = c + 4 * lane;
        uint16_t *mkl = L.mk + ((c & (MR - 1)) + 4 * lane);
        const uint2 mw = *(const uint2 *)mkl;
        *(uint2 *)mkl = make_uint2(0, 0);  // cleared for position c + MR .. (read above: LDS is in order)
        const uint32_t m0 = mw.x & 0xffffu, m1 = mw.x >> 16, m2 = mw.y & 0xffffu, m3 = mw.y >> 16;
        const uint32_t mlast = m3 ? m3 : (m2 ? m2 : (m1 ? m1 : m0));
        const uint32_t sc = wave_incl_max(mlast ? (((lane + 1) << 16) | mlast) : 0u);
        const uint32_t ex = wave_shr1(sc);
        const uint32_t f0 = m0 ? m0 : (ex ? (ex & 0xffffu) : cin);
        const uint32_t f1 = m1 ? m1 : f0, f2 = m2 ? m2 : f1, f3 = m3 ? m3 : f2;
        {
            const uint32_t e63 = __builtin_amdgcn_readlane(sc, 63);
            cin = __builtin_amdgcn_readfirstlane(e63 ? (e63 & 0xffffu) : cin);
        }
        uint32_t s0 = f0 == kMkLit ? p0 : p0 - f0;
        uint32_t s1 = f1 == kMkLit ? p0 + 1 : p0 + 1 - f1;
        uint32_t s2 = f2 == kMkLit ? p0 + 2 : p0 + 2 - f2;
        uint32_t s3 = f3 == kMkLit ? p0 + 3 : p0 + 3 - f3;
        PROF_MARK(1);  // 1: markers + fill
        // ---- sources inside this chunk: pointer jumping ----
        bool q0 = f0 != kMkLit && s0 >= c, q1 = f1 != kMkLit && s1 >= c;
        bool q2 = f2 != kMkLit && s2 >= c, q3 = f3 != kMkLit && s3 >= c;
        if (__ballot(q0 || q1 || q2 || q3)) {
            uint16_t *spl = L.sp + 4 * lane;
            auto ent = [](uint32_t f, uint32_t s) -> uint32_t { return f == kMkLit ? (uint32_t)kSpLit : s & 0xffffu; };
            *(uint2 *)spl = make_uint2(ent(f0, s0) | (ent(f1, s1) << 16), ent(f2, s2) | (ent(f3, s3) << 16));
            do {
                // a byte whose source reached a literal keeps it; else it takes its source's source.
                // All four reads go out before any is used (one LDS round trip per round); a byte
                // that is not jumping reads its own entry.
                const uint32_t t0 = L.sp[(q0 ? s0 : p0) - c], t1 = L.sp[(q1 ? s1 : p0 + 1) - c];
                const uint32_t t2 = L.sp[(q2 ? s2 : p0 + 2) - c], t3 = L.sp[(q3 ? s3 : p0 + 3) - c];
                auto jump = [&](bool &q, uint32_t &s, uint32_t t) {
                    const bool lit = t == kSpLit;
                    s = q && !lit ? t : s;
                    q = q && !lit && t >= c;
                };
                jump(q0, s0, t0), jump(q1, s1, t1), jump(q2, s2, t2), jump(q3, s3, t3);
                *(uint2 *)spl = make_uint2(ent(f0, s0) | (ent(f1, s1) << 16), ent(f2, s2) | (ent(f3, s3) << 16));
#ifdef QLZX_PROFILE
                _pacc[7] += 1;  // pointer-jumping rounds
#endif
            } while (__ballot(q0 || q1 || q2 || q3));
        }
        PROF_MARK(2);  // 2: pointer jumping
        // ---- gather: window (LDS) or, below c + MR - W, the block's output in HBM ----
        const uint32_t lo = c + MR > W ? c + MR - W : 0u;
        uint32_t v0 = L.win[s0 & (W - 1)], v1 = L.win[s1 & (W - 1)];
        uint32_t v2 = L.win[s2 & (W - 1)], v3 = L.win[s3 & (W - 1)];
        if (__ballot(s0 < lo || s1 < lo || s2 < lo || s3 < lo)) {
            if (s0 < lo) v0 = dst[s0];
            if (s1 < lo) v1 = dst[s1];
            if (s2 < lo) v2 = dst[s2];
            if (s3 < lo) v3 = dst[s3];
        }
        const uint32_t w = v0 | (v1 << 8) | (v2 << 16) | (v3 << 24);
        *(uint32_t *)(L.win + (p0 & (W - 1))) = w;
        PROF_MARK(3);  // 3: gather
        if (c + kChunk <= dsize) {
            *(uint32_t *)(dst + p0) = w;  // 256 B per wave instruction (unaligned access mode)
        } else {
            for (uint32_t j = 0; j < 4 && p0 + j < dsize; j++) dst[p0 + j] = (uint8_t)(w >> (8 * j));
        }
        PROF_MARK(4);  // 4: store
    }
    vm_sync();
    PROF_FLUSH(1);
    if (lane == 0) {
        *status_i = err ? QLZX_E_CORRUPT : QLZX_OK;
        if (dsize_i) *dsize_i = err ? 0u : dsize;
    }
}

// CRC: the record CRC (store/datafile.go:161-168) is verified first, over all src_len bytes from
// crc_state (or ~0), with the slicing-by-4 tables in the 4 KiB window (wave_crc_rep<4, true>; the
// byte table four times over, QLZX_K2_CRC_S4=0, measured ~1 % slower on c2 + CRC) and the g_crc_mul
// tables read from global memory; a mismatch sets QLZX_E_CRC and nothing is decoded.
#ifndef QLZX_K2_CRC_S4
#define QLZX_K2_CRC_S4 1
#endif
template <uint32_t W, uint32_t MR, bool CRC>
__global__ void __launch_bounds__(64) k_dec_bytes(qlzx_blocks b, uint32_t *dsize_out, int32_t *status,
                                                  uint32_t first, uint32_t count, const BlkInfo *info,
                                                  const GroupRec *recs, uint32_t gmax, const uint32_t *list,
                                                  const uint32_t *crc_state, const uint32_t *crc_expect,
                                                  uint32_t *crc_out) {
    __shared__ __attribute__((aligned(16))) K2bLds<W, MR> L;
    const uint32_t bx = blockIdx.x;  // workspace slot
    if (bx >= count) return;
    const uint32_t i = list ? list[bx] : first + bx;  // block
    if constexpr (CRC) {
        static_assert(W >= 4096, "the 4-fold CRC table fills 4 KiB of the window");
        const uint32_t lane = threadIdx.x;
        uint32_t *tab = (uint32_t *)L.win;
#if QLZX_K2_CRC_S4
        for (uint32_t e = lane * 4; e < 1024; e += 256)
            *(uint4 *)(tab + e) = *(const uint4 *)(g_crc_slice8 + e);
#else
        for (uint32_t e = lane; e < 256; e += 64) {
            const uint32_t v = g_crc_table[e];
            *(uint4 *)(tab + 4 * e) = make_uint4(v, v, v, v);
        }
#endif
        __syncthreads();
        const uint32_t c = ~wave_crc_rep<4, QLZX_K2_CRC_S4>(tab, g_crc_mul, b.src + b.src_off[i], b.src_len[i],
                                                             crc_state ? crc_state[i] : 0xffffffffu, lane);
        __syncthreads();  // the window is the decode's again
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
    dec_bytes_block<W, MR>(L, b.src + b.src_off[i], b.dst + b.dst_off[i], b.src_len[i], bi,
                           recs + (size_t)bx * gmax, status + i, dsize_out ? dsize_out + i : nullptr, threadIdx.x);
}

}  // namespace qlzx
