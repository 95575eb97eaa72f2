// qlzx_decode_wave.hip -- fast batched level-3 decoder for blocks with
// dsize <= QLZX_FAST_MAX_DSIZE (the 4-64 KiB values of the BASELINE configs).
//
// Two kernels per chunk of blocks:
//
// K1 k_dec_parse  one LANE per block.  Walks the serial control-word/token
//     chain of quicklz.c:513-671 once -- reading only control words and the
//     first byte of each match token (its length) -- computes the record CRC
//     of store/datafile.go:66-76 over the compressed bytes (slicing-by-8), and
//     emits one 16-B record per control-word group:
//       ip  stream offset of the group's control word
//       m   match mask (bit k = item k is a match)
//       a,b bit-planes of (token bytes - 1) per match item (token length 1..4)
//     Input arrives in rounds: every lane's next 64-B chunk is DMA'd
//     (global_load_lds) into the same ring slot, one round ahead, so the M0
//     base is wave-uniform and no register waits on in-flight loads.  A lane
//     parses until it runs out of landed bytes, so rounds self-align by bytes.
//
// K2 k_dec_blocks one WAVE per block, the whole output block resident in LDS.
//     Items are decoded 64 at a time, one per lane.  Item k of group g sits at
//       ip + 4 + k + popc(a & low(k)) + 2 popc(b & low(k)),
//     so no serial walk is needed.  Group records (two batches ahead) and
//     token bytes (one batch ahead) are DMA'd into LDS while the current batch
//     resolves.  Per batch: decode tokens, DPP-scan output lengths, validate
//     (checks C1-C5), write literals, then copy matches in
//     sub-rounds: a match is copied once every source byte it needs lies below
//     the first pending match (the lowest pending match is always ready, so
//     every sub-round makes progress).  The finished block leaves LDS in
//     16-B-per-lane coalesced stores.
#include "qlzx_device.h"

#ifndef QLZX_FAST_MAX_DSIZE
#define QLZX_FAST_MAX_DSIZE 65536
#endif

namespace qlzx {

struct BlkInfo {
    uint32_t ngroups;
    uint32_t nitems;
    uint32_t kind;  // 0 skip (error / general path), 1 stored, 2 compressed
    uint32_t dsize;
};
struct GroupRec {
    uint32_t ip, m, a, b;
};

constexpr int32_t kPending = -1;  // status of blocks left to the general path
constexpr uint32_t kBlkSkip = 0, kBlkStored = 1, kBlkCompressed = 2;
constexpr uint32_t kParseWG = 256;
constexpr uint32_t kChunkBlocks = 131072;  // >= 256 CUs x 8 waves x 64 lanes: K1 fills the chip
constexpr uint32_t kRoundBytes = 64;          // bytes DMA'd per lane per round (4 x 16 B)
constexpr uint32_t kRingSlots = 4;            // rounds resident per lane: r-1, r, r+1, r+2 (issuing)
constexpr uint32_t kRingWave = kRingSlots * kRoundBytes * 64;  // 16 KiB per wave

__host__ __device__ inline uint32_t groups_max(uint32_t max_dsize) { return max_dsize / 31u + 2u; }

inline bool decode_wave_enabled() { return true; }

inline size_t decode_wave_ws_bytes(uint32_t n, uint32_t max_dsize) {
    const uint32_t md = max_dsize > QLZX_FAST_MAX_DSIZE ? QLZX_FAST_MAX_DSIZE : max_dsize;
    const uint32_t c = n < kChunkBlocks ? (n ? n : 1) : kChunkBlocks;
    return (((size_t)c * sizeof(BlkInfo) + 255) & ~(size_t)255) + (size_t)c * groups_max(md) * sizeof(GroupRec) +
           256;
}

// ------------------------------------------------------------------ K1 ----
// Ring layout per wave: [slot][piece 0..3][lane][16 B]; stream byte p of a lane
// (q = p + shift, shift = src & 15) lives in round q/64, slot (q/64) % 4,
// piece (q/16) % 4, byte q % 16.
__device__ __forceinline__ uint32_t ring_off(uint32_t q, uint32_t lane) {
    return ((((q >> 6) & (kRingSlots - 1)) * 4 + ((q >> 4) & 3)) * 64 + lane) * 16 + (q & 15);
}
__device__ __forceinline__ uint32_t ring_rd32(const uint8_t *ring, uint32_t q, uint32_t lane) {
    const uint32_t qa = q & ~3u;
    const uint32_t lo = *(const uint32_t *)(ring + ring_off(qa, lane));
    const uint32_t hi = *(const uint32_t *)(ring + ring_off(qa + 4, lane));
    return __builtin_amdgcn_alignbyte(hi, lo, q & 3u);
}

// DMA round r (q in [64r, 64r+64)) of every lane into its ring slot.  All
// lanes always issue exactly 4 DMAs per round (inactive lanes fetch a dummy
// chunk of the source buffer's first bytes into their own, unused, slot) so
// that "s_waitcnt vmcnt(4)" means exactly "every round but the newest landed".
__device__ __forceinline__ void ring_issue(uint8_t *ring_wave, const uint8_t *gbase, const uint8_t *dummy,
                                           uint32_t r, uint32_t last16, bool active) {
#pragma unroll
    for (uint32_t j = 0; j < 4; j++) {
        const uint32_t c16 = r * 4 + j;
        const uint8_t *g = (active && c16 <= last16) ? gbase + (size_t)c16 * 16 : dummy;
        dma16(g, lds_addr(ring_wave + ((r & (kRingSlots - 1)) * 4 + j) * 1024));
    }
}

template <bool CRC>
__global__ void __launch_bounds__(kParseWG) k_dec_parse(qlzx_blocks b, const uint32_t *dst_cap,
                                                         uint32_t *dsize_out, int32_t *status,
                                                         const uint32_t *crc_state, const uint32_t *crc_expect,
                                                         uint32_t *crc_out, uint32_t first, uint32_t count,
                                                         BlkInfo *info, GroupRec *recs, uint32_t gmax) {
    __shared__ __attribute__((aligned(16))) uint8_t ring_all[(kParseWG / 64) * kRingWave];
    __shared__ uint32_t tab[CRC ? 8 * 256 : 1];
    if (CRC) {
        for (uint32_t t = threadIdx.x; t < 8 * 256; t += kParseWG) tab[t] = g_crc_slice8[t];
        __syncthreads();
    }
    const uint32_t lane = threadIdx.x & 63;
    uint8_t *ring = ring_all + (threadIdx.x >> 6) * kRingWave;
    const uint32_t li = blockIdx.x * kParseWG + threadIdx.x;
    const bool inrange = li < count;
    const uint32_t i = first + (inrange ? li : 0);

    int st = QLZX_OK;
    uint32_t kind = kBlkSkip, csize = 0, dsize = 0, hdr = 0, len = 0;
    const uint8_t *src = b.src + b.src_off[i];
    if (inrange) {
        len = b.src_len[i];
        if (len < 3) st = QLZX_E_HEADER;
        else {
            hdr = (src[0] & 2u) ? 9u : 3u;
            if (len < hdr) st = QLZX_E_HEADER;
            else {
                const Header h = parse_header(src);
                csize = h.csize;
                dsize = h.dsize;
                if (h.csize != len) st = QLZX_E_SIZE_COMPRESSED;
                else if (h.level != 3) st = QLZX_E_LEVEL;
                else if (dst_cap && h.dsize > dst_cap[i]) st = QLZX_E_DST_CAP;
                else if (h.dsize > QLZX_FAST_MAX_DSIZE) st = kPending;  // general path owns it
                else if (!h.compressed) {
                    if (csize >= hdr + dsize) kind = kBlkStored;
                    else st = QLZX_E_CORRUPT;
                } else kind = kBlkCompressed;
            }
        }
    }
    const uintptr_t a = (uintptr_t)src;
    const uint8_t *gbase = (const uint8_t *)(a & ~(uintptr_t)15);
    const uint32_t shift = (uint32_t)(a & 15);
    // bytes to stream: all `len` bytes when the CRC is wanted, else the compressed stream
    const uint32_t span = (CRC && inrange) ? len : ((st == QLZX_OK && kind == kBlkCompressed) ? csize : 0);
    const uint32_t last16 = span ? (span + shift - 1) >> 4 : 0;
    const uint32_t last_round = span ? (span + shift - 1) / kRoundBytes : 0;
    bool stream = inrange && span > 0;
    const bool parsing = stream && st == QLZX_OK && kind == kBlkCompressed;

    // parse state
    uint32_t ip = hdr, g = 0, k = 31, cw = 0, m = 0, ra = 0, rb = 0, rec_ip = 0;
    GroupRec *myrec = recs + (size_t)(inrange ? li : 0) * gmax;
    uint32_t crc = (CRC && inrange && crc_state) ? crc_state[i] : 0xffffffffu;
    bool done_parse = !parsing;

    const uint8_t *dummy = (const uint8_t *)(((uintptr_t)b.src) & ~(uintptr_t)15);
    ring_issue(ring, gbase, dummy, 0, last16, stream);
    ring_issue(ring, gbase, dummy, 1, last16, stream && last_round >= 1);
    for (uint32_t r = 0;; r++) {
        if (__ballot(stream && r <= last_round) == 0) break;
        // rounds <= r landed once at most the newest round's 4 DMAs are in flight
        asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        const bool act = stream && r <= last_round;
        if (CRC && act) {  // CRC of this round's bytes, in stream order
            const uint32_t q0 = r * kRoundBytes, q1 = q0 + kRoundBytes;
            const uint32_t lo = q0 > shift ? q0 : shift, hi = (q1 < span + shift) ? q1 : span + shift;
            uint32_t q = lo;
            while (q < hi && (q & 7u)) { crc = crc_byte(tab, crc, ring[ring_off(q, lane)]); q++; }
            while (q + 8 <= hi) {
                const uint32_t w0 = *(const uint32_t *)(ring + ring_off(q, lane));
                const uint32_t w1 = *(const uint32_t *)(ring + ring_off(q + 4, lane));
                crc = crc_slice8(tab, crc, w0, w1);
                q += 8;
            }
            while (q < hi) { crc = crc_byte(tab, crc, ring[ring_off(q, lane)]); q++; }
        }
        // parse while the bytes the next step reads have landed (stream pos < lim)
        const uint32_t lim = (r + 1) * kRoundBytes - shift;
        bool go = act && !done_parse;
        while (__ballot(go)) {
            if (!go) continue;
            if (k == 31) {  // group boundary: control word (quicklz.c:517-525)
                if (ip + 4 > csize) { done_parse = true; go = false; continue; }  // stream ends
                if (ip + 4 > lim) { go = false; continue; }
                if (g > 0) myrec[g - 1] = GroupRec{rec_ip, m, ra, rb};
                if (g >= gmax) { st = QLZX_E_CORRUPT; done_parse = true; go = false; continue; }
                rec_ip = ip;
                cw = ring_rd32(ring, ip + shift, lane);
                if (!(cw >> 31)) { st = QLZX_E_CORRUPT; done_parse = true; go = false; continue; }  // C1
                ip += 4;
                k = 0; m = 0; ra = 0; rb = 0;
                g++;
                continue;
            }
            if (ip >= csize) { done_parse = true; go = false; continue; }
            if ((cw >> k) & 1u) {  // match: only the token's first byte (its length) is needed
                if (ip + 1 > lim) { go = false; continue; }
                const uint32_t tl = token_bytes(ring[ring_off(ip + shift, lane)]);
                if (ip + tl > csize) { st = QLZX_E_CORRUPT; done_parse = true; go = false; continue; }  // C2/C5
                m |= 1u << k;
                ra |= ((tl - 1) & 1u) << k;
                rb |= ((tl - 1) >> 1) << k;
                ip += tl;
                k++;
            } else {  // literal run to the next match bit or the group end (no bytes read)
                uint32_t run = __builtin_ctz((cw >> k) | (1u << (31 - k)));
                if (run > csize - ip) run = csize - ip;
                ip += run;
                k += run;
            }
        }
        if (!CRC && done_parse) stream = false;  // nothing left to read for this lane
        // round r+2 reuses the slot of round r-2 (consumed: every lane is past 64 (r-1))
        ring_issue(ring, gbase, dummy, r + 2, last16, stream && r + 2 <= last_round);
    }
    if (parsing && st == QLZX_OK && g > 0) myrec[g - 1] = GroupRec{rec_ip, m, ra, rb};
    vm_sync();
    if (!inrange) return;
    if (st == QLZX_OK && kind == kBlkCompressed && (!done_parse || g == 0)) st = QLZX_E_CORRUPT;
    if (CRC) {
        const uint32_t c = ~crc;
        if (crc_out) crc_out[i] = c;
        if (crc_expect && c != crc_expect[i]) st = QLZX_E_CRC;  // store/datafile.go:161-168: before decode
    }
    BlkInfo bi{0, 0, kind, dsize};
    if (st != QLZX_OK) {
        bi.kind = kBlkSkip;
        status[i] = st;
        if (dsize_out && st != kPending) dsize_out[i] = 0;
    } else if (kind == kBlkCompressed) {
        bi.ngroups = g;
        bi.nitems = (g - 1) * 31 + (k > 31 ? 31 : k);
    }
    info[li] = bi;
}

// ------------------------------------------------------------------ K2 ----
// Read 16 bytes starting at LDS byte p.
__device__ __forceinline__ void lds_get16(const uint8_t *out, uint32_t p, uint32_t w[4]) {
    const uint32_t *s = (const uint32_t *)(out + (p & ~3u));
    const uint32_t pa = p & 3u;
    const uint32_t x0 = s[0], x1 = s[1], x2 = s[2], x3 = s[3], x4 = s[4];
    w[0] = __builtin_amdgcn_alignbyte(x1, x0, pa);
    w[1] = __builtin_amdgcn_alignbyte(x2, x1, pa);
    w[2] = __builtin_amdgcn_alignbyte(x3, x2, pa);
    w[3] = __builtin_amdgcn_alignbyte(x4, x3, pa);
}

// mem = (mem & ~mask) | val in one LDS instruction (val pre-masked).
__device__ __forceinline__ void lds_mskor(uint32_t *addr, uint32_t mask, uint32_t val) {
    const uint32_t a = (uint32_t)(uintptr_t)addr;
    asm volatile("ds_mskor_b32 %0, %1, %2" ::"v"(a), "v"(mask), "v"(val) : "memory");
}

// Store n (1..16) bytes held in w[0..3] at LDS byte q; bytes outside [q, q+n) untouched.
__device__ __forceinline__ void lds_put16(uint8_t *out, uint32_t q, const uint32_t w[4], uint32_t n) {
    const uint32_t qa = q & 3u;
    uint32_t *d = (uint32_t *)(out + (q & ~3u));
    uint32_t o[5];
    o[0] = w[0] << (8 * qa);
    o[1] = qa ? __builtin_amdgcn_alignbyte(w[1], w[0], 4 - qa) : w[1];
    o[2] = qa ? __builtin_amdgcn_alignbyte(w[2], w[1], 4 - qa) : w[2];
    o[3] = qa ? __builtin_amdgcn_alignbyte(w[3], w[2], 4 - qa) : w[3];
    o[4] = qa ? (w[3] >> (8 * (4 - qa))) : 0u;
    const uint32_t end = qa + n;
#pragma unroll
    for (uint32_t j = 0; j < 5; j++) {
        const int lo = (int)qa - (int)(4 * j), hi = (int)end - (int)(4 * j);
        const uint32_t blo = lo < 0 ? 0u : (lo > 4 ? 4u : (uint32_t)lo);
        const uint32_t bhi = hi < 0 ? 0u : (hi > 4 ? 4u : (uint32_t)hi);
        if (bhi > blo) {
            const uint32_t mask = (bhi == 4 ? 0xffffffffu : ((1u << (8 * bhi)) - 1u)) & ~((1u << (8 * blo)) - 1u);
            if (mask == 0xffffffffu) d[j] = o[j];
            else lds_mskor(d + j, mask, o[j] & mask);
        }
    }
}

template <uint32_t MAXD>
struct K2Lds {
    uint8_t out[MAXD + 32];
    GroupRec rec[3][64];     // per-lane group record of batches b, b+1, b+2 (slot = batch % 3)
    uint32_t tok[2][2][64];  // per-lane token dwords (lo, hi) of batches b, b+1 (slot = batch % 2)
};

// DMA the group record of item I = 64 bt + lane into rec slot bt % 3.
__device__ __forceinline__ void issue_rec(GroupRec (*rec)[64], const GroupRec *rb, uint32_t bt, uint32_t nitems,
                                          uint32_t lane) {
    const uint32_t I = bt * 64 + lane;
    if (I < nitems) dma16(rb + I / 31, lds_addr(&rec[bt % 3][0]));
}

// From the landed record of batch bt, DMA the two dwords holding item bytes [pos, pos+4).
__device__ __forceinline__ void issue_tok(const GroupRec *recslot, uint32_t (*tok)[64], const uint8_t *src,
                                          uint32_t csize, uint32_t bt, uint32_t nitems, uint32_t lane) {
    const uint32_t I = bt * 64 + lane;
    if (I < nitems) {
        const GroupRec gr = recslot[lane];
        const uint32_t k = I - (I / 31) * 31, low = (1u << k) - 1u;
        const uint32_t pos = gr.ip + 4 + k + __builtin_popcount(gr.a & low) + 2 * __builtin_popcount(gr.b & low);
        const uintptr_t aa = ((uintptr_t)(src + pos)) & ~(uintptr_t)3;
        dma4((const void *)aa, lds_addr(&tok[0][0]));
        if (aa + 4 < (uintptr_t)(src + csize)) dma4((const void *)(aa + 4), lds_addr(&tok[1][0]));
    }
}

// Inclusive prefix sum over the 64 lanes with DPP (row shifts + row broadcasts).
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, true);   // row_shr:1
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, true);   // row_shr:2
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, true);   // row_shr:4
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, true);   // row_shr:8
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false);  // row_bcast:15
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false);  // row_bcast:31
    return v;
}

template <uint32_t MAXD>
__global__ void __launch_bounds__(64) k_dec_blocks(qlzx_blocks b, uint32_t *dsize_out, int32_t *status,
                                                   uint32_t first, uint32_t count, const BlkInfo *info,
                                                   const GroupRec *recs, uint32_t gmax) {
    __shared__ __attribute__((aligned(16))) K2Lds<MAXD> L;
    const uint32_t lane = threadIdx.x;
    const uint32_t li = blockIdx.x;
    if (li >= count) return;
    const uint32_t i = first + li;
    const BlkInfo bi = info[li];
    if (bi.kind == kBlkSkip) return;
    const uint8_t *src = b.src + b.src_off[i];
    uint8_t *dst = b.dst + b.dst_off[i];
    const uint32_t dsize = bi.dsize;
    if (bi.kind == kBlkStored) {  // quicklz.c:808-811
        const uint32_t hdr = (src[0] & 2u) ? 9u : 3u;
        for (uint32_t p = lane; p < dsize; p += 64) dst[p] = src[hdr + p];
        if (lane == 0) { status[i] = QLZX_OK; if (dsize_out) dsize_out[i] = dsize; }
        return;
    }
    uint8_t *out = L.out;
    const GroupRec *rb = recs + (size_t)li * gmax;
    const uint32_t nitems = bi.nitems;
    const uint32_t csize = b.src_len[i];
    const uint32_t hdr = (src[0] & 2u) ? 9u : 3u;
    const uint32_t nb = (nitems + 63) / 64;
    const uint32_t tail_from = dsize > QLZX_TAIL ? dsize - 1 - QLZX_TAIL : 0;  // op >= this: tail (quicklz.c:503)
    // prologue: records of batches 0 and 1, then the tokens of batch 0
    issue_rec(L.rec, rb, 0, nitems, lane);
    issue_rec(L.rec, rb, 1, nitems, lane);
    vm_sync();
    issue_tok(L.rec[0], L.tok[0], src, csize, 0, nitems, lane);
    vm_sync();
    uint32_t D = 0;
    bool bad = false, tail = false, complete = dsize == 0;
    for (uint32_t bt = 0; bt < nb && !complete && !bad; bt++) {
        // invariant: rec[bt], rec[bt+1], tok[bt] landed.  Read this batch's state first.
        const uint32_t I = bt * 64 + lane;
        const bool valid = I < nitems;
        const GroupRec gr = L.rec[bt % 3][lane];
        const uint32_t tlo = L.tok[bt & 1][0][lane], thi = L.tok[bt & 1][1][lane];
        lds_sync();
        // prefetch: tokens of bt+1 (its records landed), records of bt+2
        if (bt + 1 < nb) issue_tok(L.rec[(bt + 1) % 3], L.tok[(bt + 1) & 1], src, csize, bt + 1, nitems, lane);
        if (bt + 2 < nb) issue_rec(L.rec, rb, bt + 2, nitems, lane);

        const uint32_t k = I - (I / 31) * 31, low = (1u << k) - 1u;
        const bool is_match = valid && ((gr.m >> k) & 1u);
        const uint32_t pos = gr.ip + 4 + k + __builtin_popcount(gr.a & low) + 2 * __builtin_popcount(gr.b & low);
        const uint32_t t = __builtin_amdgcn_alignbyte(thi, tlo, (uint32_t)(((uintptr_t)(src + pos)) & 3u));
        uint32_t off = 0, len = valid ? 1u : 0u, tl = 1;
        if (is_match) tl = decode_token(t, off, len);
        const uint32_t incl = wave_incl_scan(len);
        const uint32_t d = D + incl - len;
        const uint32_t total = __builtin_amdgcn_readlane(incl, 63);
        // ---- checks C2-C5 on the live items (those that start before dsize) ----
        const bool live = valid && d < dsize;
        const bool lit_tail = live && !is_match && d >= tail_from;
        const uint64_t tail_lanes = __ballot(lit_tail);
        const uint32_t tail_lane = tail ? 0u : (tail_lanes ? (uint32_t)__builtin_ctzll(tail_lanes) : 64u);  // C4
        bool ok = true;
        if (live && is_match)  // C3, and C4: no match after the first tail literal
            ok = off >= 3 && off <= d && d + len + 4 <= dsize && lane < tail_lane;
        if (live && d + len == dsize) {  // the item that completes dsize: C5
            const uint32_t ip_end = pos + tl;
            ok = ok && (ip_end == csize || (ip_end < hdr + 9 && csize == hdr + 9));
        }
        if (__ballot(live && !ok)) { bad = true; break; }
        tail = tail || tail_lanes != 0;
        complete = __ballot(live && d + len == dsize) != 0;
        if (live && !is_match) out[d] = (uint8_t)t;
        bool done = !(live && is_match);
        const uint32_t s = d - off;
        const uint32_t send = (s + len < d) ? s + len : d;
        const bool bytewise = off < 16 && off < len;
        for (;;) {
            lds_sync();
            const uint64_t pend = __ballot(!done);
            if (!pend) break;
            const uint32_t du = __builtin_amdgcn_readlane(d, (uint32_t)__builtin_ctzll(pend));
            if (!done && send <= du) {
                if (bytewise) {
                    uint32_t j2 = 0;
                    for (uint32_t j = 0; j < len; j++) {
                        out[d + j] = out[s + j2];
                        j2 = (j2 + 1 == off) ? 0 : j2 + 1;
                    }
                } else {
                    for (uint32_t c = 0; c < len; c += 16) {
                        uint32_t w[4];
                        lds_get16(out, s + c, w);
                        lds_put16(out, d + c, w, len - c < 16 ? len - c : 16);
                        if (off < len) lds_sync();
                    }
                }
                done = true;
            }
        }
        D += total;
        vm_sync();  // prefetches of bt+1 / bt+2 landed (issued before the resolve)
    }
    vm_sync();
    lds_sync();
    if (bad || !complete) {
        if (lane == 0) { status[i] = QLZX_E_CORRUPT; if (dsize_out) dsize_out[i] = 0; }
        return;
    }
    // write the block out: 16 B per lane, 1 KiB per wave instruction
    const bool a16 = (((uintptr_t)dst) & 15u) == 0;
    for (uint32_t p = lane * 16; p < dsize; p += 1024) {
        if (p + 16 <= dsize && a16) {
            *(uint4 *)(dst + p) = *(const uint4 *)(out + p);
        } else {
            const uint32_t e = p + 16 < dsize ? p + 16 : dsize;
            for (uint32_t q = p; q < e; q++) dst[q] = out[q];
        }
    }
    if (lane == 0) {
        status[i] = QLZX_OK;
        if (dsize_out) dsize_out[i] = dsize;
    }
}

inline int launch_decode_wave(const qlzx_blocks &b, const uint32_t *dst_cap, uint32_t *dsize,
                              int32_t *status, const uint32_t *crc_state, const uint32_t *crc_expect,
                              uint32_t *crc_out, uint32_t max_dsize, void *ws, size_t ws_bytes,
                              hipStream_t s) {
    (void)ws_bytes;
    const uint32_t md = max_dsize > QLZX_FAST_MAX_DSIZE ? QLZX_FAST_MAX_DSIZE : max_dsize;
    const uint32_t gmax = groups_max(md);
    const uint32_t chunk = b.n < kChunkBlocks ? b.n : kChunkBlocks;
    BlkInfo *info = (BlkInfo *)ws;
    GroupRec *recs = (GroupRec *)((uint8_t *)ws + (((size_t)chunk * sizeof(BlkInfo) + 255) & ~(size_t)255));
    const bool crc = crc_state || crc_expect || crc_out;
    for (uint32_t first = 0; first < b.n; first += chunk) {
        const uint32_t cnt = b.n - first < chunk ? b.n - first : chunk;
        if (crc)
            hipLaunchKernelGGL(k_dec_parse<true>, dim3((cnt + kParseWG - 1) / kParseWG), dim3(kParseWG), 0, s, b,
                               dst_cap, dsize, status, crc_state, crc_expect, crc_out, first, cnt, info, recs, gmax);
        else
            hipLaunchKernelGGL(k_dec_parse<false>, dim3((cnt + kParseWG - 1) / kParseWG), dim3(kParseWG), 0, s, b,
                               dst_cap, dsize, status, crc_state, crc_expect, crc_out, first, cnt, info, recs, gmax);
        if (md <= 16384)
            hipLaunchKernelGGL(k_dec_blocks<16384>, dim3(cnt), dim3(64), 0, s, b, dsize, status, first, cnt, info,
                               recs, gmax);
        else
            hipLaunchKernelGGL(k_dec_blocks<QLZX_FAST_MAX_DSIZE>, dim3(cnt), dim3(64), 0, s, b, dsize, status, first,
                               cnt, info, recs, gmax);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return (int)e;
    }
    return 0;
}

}  // namespace qlzx
