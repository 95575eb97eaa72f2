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
constexpr uint32_t kParseWG = 64;          // K1 workgroup: one wave (LDS per wave bounds occupancy)
constexpr uint32_t kChunkBlocks = 131072;  // >= 256 CUs x 8 waves x 64 lanes: K1 fills the chip
constexpr uint32_t kRoundBytes = 64;          // bytes DMA'd per lane per round (4 x 16 B)
constexpr uint32_t kRingSlots = 3;            // rounds resident per lane: r, r+1 (landing), r+2 (issuing)
constexpr uint32_t kRingWave = kRingSlots * kRoundBytes * 64;  // 12 KiB per wave
constexpr uint32_t kTokSlots = 4;  // K2 token prefetch slots (batch % 4)
constexpr uint32_t kRecSlots = 7;  // K2 group-record prefetch slots (batch % 7)

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
// (q = p + shift, shift = src & 15) lives in round q/64, slot (q/64) % 3,
// piece (q/16) % 4, byte q % 16.
__device__ __forceinline__ uint32_t ring_off(uint32_t q, uint32_t lane) {
    return ((((q >> 6) % kRingSlots) * 4 + ((q >> 4) & 3)) * 64 + lane) * 16 + (q & 15);
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
        dma16(g, lds_addr(ring_wave + ((r % kRingSlots) * 4 + j) * 1024));
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

    PROF_DECL
    const uint8_t *dummy = (const uint8_t *)(((uintptr_t)b.src) & ~(uintptr_t)15);
    ring_issue(ring, gbase, dummy, 0, last16, stream);
    ring_issue(ring, gbase, dummy, 1, last16, stream && last_round >= 1);
    for (uint32_t r = 0;; r++) {
        if (__ballot(stream && r <= last_round) == 0) break;
        // rounds <= r landed once at most the newest round's 4 DMAs are in flight
        PROF_MARK(0);
        asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        PROF_MARK(1);  // 1: waiting for the round's DMA
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
        PROF_MARK(2);  // 2: CRC
        // parse while the bytes the next step reads have landed (stream pos < lim)
        const uint32_t lim = (r + 1) * kRoundBytes - shift;
        bool go = act && !done_parse;
        while (__ballot(go)) {
#ifdef QLZX_PROFILE
            _pacc[5] += 1;
            if (go) _pacc[6] += 1;
#endif
            // one step = a control word (k == 31) or one item: a match token or a
            // literal run.  Straight-line selects; only the record store branches.
            const bool gb = k == 31;
            const uint32_t bit = gb ? 0u : ((cw >> k) & 1u);
            const uint32_t need = gb ? 4u : bit;          // bytes this step reads at ip
            const bool end = gb ? (ip + 4 > csize) : (ip >= csize);
            const bool wait = !end && ip + need > lim;
            const bool stepping = go && !end && !wait;
            const uint32_t w = ring_rd32(ring, ip + shift, lane);  // cword or token (unused for literals)
            const uint32_t code = ((w & 3u) == 0) ? 0u : ((w & 3u) != 3u) ? 1u : ((w & 127u) != 3u) ? 2u : 3u;
            uint32_t run = __builtin_ctz((cw >> (k & 31)) | (1u << (31 - (k & 31))));
            if (run > csize - ip) run = csize - ip;
            const bool rec_out = stepping && gb && g > 0;
            const GroupRec prev{rec_ip, m, ra, rb};
            if (rec_out) myrec[g - 1] = prev;
            const bool sentinel_bad = stepping && gb && !(w >> 31);
            const bool trunc_bad = stepping && bit && ip + code + 1 > csize;
            const bool gmax_bad = stepping && gb && g >= gmax;
            if (sentinel_bad || trunc_bad || gmax_bad) st = QLZX_E_CORRUPT;  // C1 / C2 / C5
            const bool bad = sentinel_bad || trunc_bad || gmax_bad;
            const bool adv = stepping && !bad;
            const uint32_t kk = k & 31;
            if (adv) {
                if (gb) {
                    rec_ip = ip; cw = w; ip += 4; k = 0; m = 0; ra = 0; rb = 0; g++;
                } else {
                    m |= bit << kk;
                    ra |= (bit & code) << kk;
                    rb |= (bit & (code >> 1)) << kk;
                    ip += bit ? code + 1 : run;
                    k += bit ? 1u : run;
                }
            }
            if (go && (end || bad)) done_parse = true;
            go = adv;
        }
        PROF_MARK(3);  // 3: parse
        if (!CRC && done_parse) stream = false;  // nothing left to read for this lane
        // round r+2 reuses the slot of round r-2 (consumed: every lane is past 64 (r-1))
        ring_issue(ring, gbase, dummy, r + 2, last16, stream && r + 2 <= last_round);
    }
    PROF_MARK(4);  // 4: DMA issue + loop overhead
    if (parsing && st == QLZX_OK && g > 0) myrec[g - 1] = GroupRec{rec_ip, m, ra, rb};
    PROF_FLUSH(0);
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

template <uint32_t MAXD>
struct K2Lds {
    uint8_t front[16];       // lets a match's first source dword start up to 4 B before out[0]
    uint8_t out[MAXD + 32];
    uint32_t tok[kTokSlots][64];     // per-lane token dword of batches b..b+3
    GroupRec rec[kRecSlots][4];      // records of the <= 4 groups of batches b..b+6
};

// Every K2 iteration issues exactly 2 DMA instructions (1 token dword + 1
// record), with dummy addresses for lanes/batches past the end, so that
// "s_waitcnt vmcnt(4)" at the end of iteration bt means "everything issued up
// to iteration bt-2 has landed".  Iteration bt issues the tokens of bt+3 and
// the records of bt+6, so both have two whole iterations to arrive.
__device__ __forceinline__ void issue_rec(GroupRec (*rec)[4], const GroupRec *rb, uint32_t bt, uint32_t ngroups,
                                          uint32_t lane) {
    const uint32_t g = (bt * 64) / 31 + lane;
    if (lane < 4) dma16(g < ngroups ? (const void *)(rb + g) : (const void *)rb, lds_addr(&rec[bt % kRecSlots][0]));
}
// Item position: cword at gr.ip, then k items of which popc(a)+2popc(b) extra token bytes.
__device__ __forceinline__ uint32_t item_pos(const GroupRec &gr, uint32_t k) {
    const uint32_t low = (1u << k) - 1u;
    return gr.ip + 4 + k + __builtin_popcount(gr.a & low) + 2 * __builtin_popcount(gr.b & low);
}
// The 4 stream bytes at min(pos, csize - 4) (unaligned dword DMA; csize >= 7
// for a compressed level-3 stream, so the read stays inside the block).
__device__ __forceinline__ void issue_tok(const GroupRec *recslot, uint32_t *tok, const uint8_t *src,
                                          uint32_t csize, uint32_t bt, uint32_t nitems, uint32_t lane) {
    const uint32_t I = bt * 64 + lane;
    uint32_t p = 0;
    if (I < nitems) {
        const uint32_t g = I / 31;
        p = item_pos(recslot[g - (bt * 64) / 31], I - g * 31);
        p = p + 4 <= csize ? p : csize - 4;
    }
    dma4(src + p, lds_addr(tok));
}

// Byte mask of bytes [lo, hi) of one dword (lo, hi clamped to [0, 4]).
__device__ __forceinline__ uint32_t dw_mask(int lo, int hi) {
    lo = lo < 0 ? 0 : (lo > 4 ? 4 : lo);
    hi = hi < 0 ? 0 : (hi > 4 ? 4 : hi);
    if (hi <= lo) return 0u;
    const uint32_t h = hi == 4 ? 0xffffffffu : ((1u << (8 * hi)) - 1u);
    return h & ~((1u << (8 * lo)) - 1u);
}

// One 16-byte copy step, prepared once per batch: destination dword j (at
// qa + 4j) takes the source bytes at qa + 4j - off, i.e. alignbyte(x[j+1], x[j], sh)
// over the aligned source dwords x[] starting at xa.
struct Copy16 {
    uint32_t qa, mk[5];
    int xa;
    uint32_t sh;
    __device__ __forceinline__ void prep(uint32_t q, uint32_t off, uint32_t n) {
        qa = q & ~3u;
        const int sa = (int)qa - (int)off;  // >= -4: out[] has a 16-B front pad
        xa = sa & ~3;
        sh = (uint32_t)sa & 3u;
        const int lo = (int)(q & 3u), hi = lo + (int)n;
        mk[0] = dw_mask(lo, hi);
        mk[1] = dw_mask(lo - 4, hi - 4);
        mk[2] = dw_mask(lo - 8, hi - 8);
        mk[3] = dw_mask(lo - 12, hi - 12);
        mk[4] = dw_mask(lo - 16, hi - 16);
    }
    __device__ __forceinline__ void run(uint8_t *out) const {
        const uint32_t *x = (const uint32_t *)(out + xa);
        const uint32_t x0 = x[0], x1 = x[1], x2 = x[2], x3 = x[3], x4 = x[4], x5 = x[5];
        uint32_t *dw = (uint32_t *)(out + qa);
        if (mk[0]) lds_mskor(dw + 0, mk[0], __builtin_amdgcn_alignbyte(x1, x0, sh) & mk[0]);
        if (mk[1]) lds_mskor(dw + 1, mk[1], __builtin_amdgcn_alignbyte(x2, x1, sh) & mk[1]);
        if (mk[2]) lds_mskor(dw + 2, mk[2], __builtin_amdgcn_alignbyte(x3, x2, sh) & mk[2]);
        if (mk[3]) lds_mskor(dw + 3, mk[3], __builtin_amdgcn_alignbyte(x4, x3, sh) & mk[3]);
        if (mk[4]) lds_mskor(dw + 4, mk[4], __builtin_amdgcn_alignbyte(x5, x4, sh) & mk[4]);
    }
};

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
    const uint32_t nitems = bi.nitems, ngroups = bi.ngroups;
    const uint32_t csize = b.src_len[i];
    const uint32_t hdr = (src[0] & 2u) ? 9u : 3u;
    const uint32_t nb = (nitems + 63) / 64;
    const uint32_t tail_from = dsize > QLZX_TAIL ? dsize - 1 - QLZX_TAIL : 0;  // op >= this: tail (quicklz.c:503)
    // prologue: records of batches 0..5, then the tokens of batches 0..2
    for (uint32_t j = 0; j < 6; j++) issue_rec(L.rec, rb, j, ngroups, lane);
    vm_sync();
    for (uint32_t j = 0; j < 3; j++) issue_tok(L.rec[j], L.tok[j], src, csize, j, nitems, lane);
    vm_sync();
    PROF_DECL
    uint32_t D = 0;
    bool bad = false, tail = false, complete = dsize == 0;
    for (uint32_t bt = 0; bt < nb && !complete && !bad; bt++) {
        // invariant: tok[bt..bt+2] and rec[bt..bt+5] landed.  Read this batch's state first.
        const uint32_t I = bt * 64 + lane;
        const bool valid = I < nitems;
        const uint32_t g = I / 31;
        const GroupRec gr = L.rec[bt % kRecSlots][valid ? g - (bt * 64) / 31 : 0];
        const uint32_t tw = L.tok[bt % kTokSlots][lane];
        lds_sync();
        PROF_MARK(0);  // 0: batch state reads
        // prefetch: tokens of bt+3 (its records landed), records of bt+6
        issue_tok(L.rec[(bt + 3) % kRecSlots], L.tok[(bt + 3) % kTokSlots], src, csize, bt + 3, nitems, lane);
        issue_rec(L.rec, rb, bt + 6, ngroups, lane);
        PROF_MARK(1);  // 1: prefetch issue
        const uint32_t k = I - g * 31;
        const bool is_match = valid && ((gr.m >> k) & 1u);
        const uint32_t pos = item_pos(gr, k);
        const uint32_t t = pos + 4 <= csize ? tw : tw >> (8 * (pos + 4 - csize));
        uint32_t off = 0, len = valid ? 1u : 0u, tl = 1;
        if (is_match) tl = decode_token(t, off, len);
        const uint32_t incl = wave_incl_scan(len);
        const uint32_t d = D + incl - len;
        const uint32_t total = __builtin_amdgcn_readlane(incl, 63);
        // ---- checks C2-C5 on the live items (those that start before dsize) ----
        const bool live = valid && d < dsize;
        const uint64_t tail_lanes = __ballot(live && !is_match && d >= tail_from);
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
        PROF_MARK(2);  // 2: decode + scan + checks
        if (live && !is_match) out[d] = (uint8_t)t;
        // ---- matches: copy in sub-rounds ----
        const bool mlive = live && is_match;
        bool done = !mlive;
        const uint32_t s = d - off;
        const uint32_t send = (s + len < d) ? s + len : d;
        const uint32_t end = d + len;
        const bool bytewise = off < 16 && off < len;
        Copy16 cp;
        cp.prep(d, off, len < 16 ? len : 16);
        for (;;) {
            lds_sync();
            uint64_t pend = __ballot(!done);
            if (!pend) break;
            // the first three pending matches bound three gaps whose bytes are all final
            const uint32_t u0 = (uint32_t)__builtin_ctzll(pend);
            pend &= pend - 1;
            const uint32_t u1 = pend ? (uint32_t)__builtin_ctzll(pend) : u0;
            pend &= pend - 1;
            const uint32_t u2 = pend ? (uint32_t)__builtin_ctzll(pend) : u1;
            const uint32_t d0 = __builtin_amdgcn_readlane(d, u0), e0 = __builtin_amdgcn_readlane(end, u0);
            const uint32_t d1 = u1 != u0 ? __builtin_amdgcn_readlane(d, u1) : 0xffffffffu;
            const uint32_t e1 = __builtin_amdgcn_readlane(end, u1);
            const uint32_t d2 = u2 != u1 ? __builtin_amdgcn_readlane(d, u2) : 0xffffffffu;
            const bool ready = !done && (send <= d0 || (s >= e0 && send <= d1) || (u1 != u0 && s >= e1 && send <= d2));
            if (ready) {
                if (bytewise) {
                    uint32_t j2 = 0;
                    for (uint32_t j = 0; j < len; j++) {
                        out[d + j] = out[s + j2];
                        j2 = (j2 + 1 == off) ? 0 : j2 + 1;
                    }
                } else {
                    cp.run(out);
                    for (uint32_t c = 16; c < len; c += 16) {  // long matches, chunk by chunk
                        if (off < len) lds_sync();
                        Copy16 c2;
                        c2.prep(d + c, off, len - c < 16 ? len - c : 16);
                        c2.run(out);
                    }
                }
                done = true;
            }
        }
        PROF_MARK(3);  // 3: match sub-rounds
        D += total;
        asm volatile("s_waitcnt vmcnt(4)" ::: "memory");  // DMAs of iterations <= bt-1 landed
        PROF_MARK(4);  // 4: waiting for prefetch
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
    PROF_MARK(5);  // 5: write-out
    PROF_FLUSH(1);
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
