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
// K2 k_dec_blocks one WAVE per block; output goes through a sliding LDS window of
//     kWin bytes (older output is flushed to HBM and read back from there by
//     "far" matches).  Items are decoded 64 at a time, one per lane.  Item k of
//     group g sits at
//       ip + 4 + k + popc(a & low(k)) + 2 popc(b & low(k)),
//     so no serial walk is needed.  Group records (kRecAhead batches ahead) and
//     token dwords (kTokAhead batches ahead) are DMA'd into LDS while the
//     current batch resolves.  Per batch: decode tokens, DPP-scan output lengths,
//     validate (checks C1-C5), write literals, then copy matches in
//     sub-rounds: a match is copied once none of the lanes producing its source
//     bytes is pending (the lowest pending match is always ready, so every
//     sub-round makes progress).  The finished block leaves LDS in
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
constexpr uint32_t kMaxDevices = 64;  // per-device side streams of the launcher
constexpr uint32_t kBlkSkip = 0, kBlkStored = 1, kBlkCompressed = 2;
// K1 workgroup: one wave (the 16 KiB LDS ring per wave bounds occupancy); with the CRC,
// four waves share one 8 KiB slicing-by-8 table (8 waves/CU instead of 6)
template <bool CRC>
constexpr uint32_t kParseWG = CRC ? 256 : 64;
#ifndef QLZX_CHUNK_BLOCKS
#define QLZX_CHUNK_BLOCKS 131072
#endif
constexpr uint32_t kChunkBlocks = QLZX_CHUNK_BLOCKS;  // >= 256 CUs x 8 waves x 64 lanes: K1 fills the chip
#ifndef QLZX_K1_ROUND
#define QLZX_K1_ROUND 64
#endif
constexpr uint32_t kRoundBytes = QLZX_K1_ROUND;  // bytes DMA'd per lane per round (16 B pieces)
constexpr uint32_t kPieces = kRoundBytes / 16;
constexpr uint32_t kRingSlots = 4;            // rounds resident per lane: r-1..r (read), r+1..r+2 (landing)
constexpr uint32_t kRingWave = kRingSlots * kRoundBytes * 64;  // 16 KiB per wave at 64-B rounds
#ifndef QLZX_K2_WIN
#define QLZX_K2_WIN 4096
#endif
constexpr uint32_t kWin = QLZX_K2_WIN;          // K2 LDS history window (bytes)
#ifndef QLZX_K2_SLACK
#define QLZX_K2_SLACK 1  // round 2: 1 beats 3 (c2 39.1 vs 39.9 ms, c5 482.6 vs 455 GiB/s)
#endif
constexpr uint32_t kK2Slack = QLZX_K2_SLACK;  // K2: iterations a prefetch DMA has to land
constexpr uint32_t kTokAhead = kK2Slack + 1;   // tokens of batch bt + kTokAhead issued in iteration bt
constexpr uint32_t kRecAhead = 2 * kTokAhead;  // records of batch bt + kRecAhead issued in iteration bt
constexpr uint32_t kTokSlots = kTokAhead;      // batches bt .. bt+kTokAhead-1 (bt+kTokAhead reuses bt's slot)
constexpr uint32_t kRecSlots = kTokAhead + 1;  // batches bt+kTokAhead .. bt+kRecAhead
constexpr uint32_t kSubMax = 64 * 32;          // K2 sub-batch output bound: the 64-word item-start bitmap
#ifndef QLZX_K2_VMWAIT
#define QLZX_K2_VMWAIT (2 * QLZX_K2_SLACK)  // two DMA instructions per iteration
#endif
static_assert(QLZX_K2_VMWAIT == 2 * QLZX_K2_SLACK,
              "K2 waits for the DMAs of iterations <= bt - slack: two per iteration");

__host__ __device__ inline uint32_t groups_max(uint32_t max_dsize) { return max_dsize / 31u + 2u; }

inline size_t rec_bytes_max(uint32_t md) { return (size_t)groups_max(md) * sizeof(GroupRec); }

inline size_t decode_wave_ws_bytes(uint32_t n, uint32_t max_dsize) {
    const uint32_t md = max_dsize > QLZX_FAST_MAX_DSIZE ? QLZX_FAST_MAX_DSIZE : max_dsize;
    const uint32_t c = n < kChunkBlocks ? (n ? n : 1) : kChunkBlocks;
    return (((size_t)c * sizeof(BlkInfo) + 255) & ~(size_t)255) +
           ((((size_t)c * rec_bytes_max(md)) + 255) & ~(size_t)255) +
           ((((size_t)n * sizeof(uint32_t)) + 255) & ~(size_t)255) +              // block order, whole call
           1024 + 256;                                                            // order aux
}

// ---------------------------------------------------------- block order ----
// K1 runs one lane per block, so a wave lasts as long as its longest stream: with mixed
// 4-64 KiB values (c4, c5) most lanes would idle behind one 64 KiB block.  Two small
// kernels list ALL blocks of the call by compressed size, smallest first (counting sort on
// len / 512, 128 classes), and the chunks are cut from that list: K1 and K2 of chunk c take
// blocks list[c * chunk ..] and index their workspace by the place in the chunk.  So a K1
// wave's lanes have similar lengths, and K1(c+1), whose blocks are at most a class longer,
// hides under K2(c), whose chunk has as many blocks; the first, exposed K1 parses the
// smallest blocks.  Order within a class is arbitrary: outputs are indexed by the block.
// aux (zeroed before k_order_count): [0,128) class counts, [128,256) class cursors.
// One-wave workgroups (16 blocks per lane), launched before the first K1: a kernel queued
// between two K1s on the side stream delayed K1(c+1) until K2(c) had filled the CUs, and a
// 1024-thread workgroup waited for a whole CU to drain; both serialised K1 behind K2.
constexpr uint32_t kOrderClasses = 128, kOrderWG = 64, kOrderEPT = 16, kOrderPerWG = kOrderWG * kOrderEPT;
constexpr uint32_t kOrderAux = 2 * kOrderClasses;
__device__ __forceinline__ uint32_t order_class(uint32_t len) {
    const uint32_t c = len >> 9;
    return c < kOrderClasses - 1 ? c : kOrderClasses - 1;
}
__global__ void __launch_bounds__(kOrderWG) k_order_count(const uint32_t *src_len, uint32_t n, uint32_t *aux) {
    __shared__ uint32_t h[kOrderClasses];
    const uint32_t tid = threadIdx.x, i0 = blockIdx.x * kOrderPerWG + tid;
    for (uint32_t k = tid; k < kOrderClasses; k += kOrderWG) h[k] = 0;
    __syncthreads();
    uint32_t len[kOrderEPT];
#pragma unroll
    for (uint32_t e = 0; e < kOrderEPT; e++) {
        const uint32_t i = i0 + e * kOrderWG;
        len[e] = i < n ? src_len[i] : 0u;
    }
#pragma unroll
    for (uint32_t e = 0; e < kOrderEPT; e++)
        if (i0 + e * kOrderWG < n) atomicAdd(&h[order_class(len[e])], 1u);
    __syncthreads();
    for (uint32_t k = tid; k < kOrderClasses; k += kOrderWG)
        if (h[k]) atomicAdd(&aux[k], h[k]);
}
__global__ void __launch_bounds__(kOrderWG) k_order_scatter(const uint32_t *src_len, uint32_t n, uint32_t *aux,
                                                           uint32_t *list) {
    __shared__ uint32_t start[kOrderClasses], lc[kOrderClasses];
    const uint32_t tid = threadIdx.x, i0 = blockIdx.x * kOrderPerWG + tid;
    for (uint32_t k = tid; k < kOrderClasses; k += kOrderWG) start[k] = aux[k], lc[k] = 0;
    __syncthreads();
    if (tid == 0) {  // exclusive scan of the class counts (128 LDS words)
        uint32_t acc = 0;
        for (uint32_t k = 0; k < kOrderClasses; k++) {
            const uint32_t v = start[k];
            start[k] = acc;
            acc += v;
        }
    }
    uint32_t c[kOrderEPT], r[kOrderEPT];
#pragma unroll
    for (uint32_t e = 0; e < kOrderEPT; e++) {
        const uint32_t i = i0 + e * kOrderWG;
        c[e] = i < n ? order_class(src_len[i]) : 0u;
    }
#pragma unroll
    for (uint32_t e = 0; e < kOrderEPT; e++)
        r[e] = (i0 + e * kOrderWG < n) ? atomicAdd(&lc[c[e]], 1u) : 0u;  // rank in this workgroup's class
    __syncthreads();
    for (uint32_t k = tid; k < kOrderClasses; k += kOrderWG)
        if (lc[k]) start[k] += atomicAdd(&aux[kOrderClasses + k], lc[k]);
    __syncthreads();
#pragma unroll
    for (uint32_t e = 0; e < kOrderEPT; e++)
        if (i0 + e * kOrderWG < n) list[start[c[e]] + r[e]] = i0 + e * kOrderWG;
}

// ------------------------------------------------------------------ K1 ----
// Header checks of one block of `len` bytes (quicklz.c:780-811 and the batch API's bounds):
// the status, and for QLZX_OK its kind (kBlkStored / kBlkCompressed), sizes and header length.
__device__ __forceinline__ int classify_block(const uint8_t *src, uint32_t len, uint32_t cap, uint32_t max_dsize,
                                              uint32_t &kind, uint32_t &csize, uint32_t &dsize, uint32_t &hdr) {
    kind = kBlkSkip;
    if (len < 3) return QLZX_E_HEADER;
    hdr = (src[0] & 2u) ? 9u : 3u;
    if (len < hdr) return QLZX_E_HEADER;
    const Header h = parse_header(src);
    csize = h.csize;
    dsize = h.dsize;
    if (h.csize != len) return QLZX_E_SIZE_COMPRESSED;
    if (h.level != 3) return QLZX_E_LEVEL;
    if (h.dsize > cap) return QLZX_E_DST_CAP;
    if (h.dsize > max_dsize) return QLZX_E_MAX_DSIZE;     // the caller's bound is wrong
    if (h.dsize > QLZX_FAST_MAX_DSIZE) return kPending;  // general path owns it
    if (!h.compressed) {
        if (csize < hdr + dsize) return QLZX_E_CORRUPT;
        kind = kBlkStored;
    } else {
        kind = kBlkCompressed;
    }
    return QLZX_OK;
}

// Ring layout per wave: [slot][piece 0..3][lane][16 B]; stream byte p of a lane
// (q = p + shift, shift = src & 15) lives in round q/64, slot (q/64) % 4,
// piece (q/16) % 4, byte q % 16 -- i.e. at ((q/16) % 16) * 1 KiB + lane * 16 + q % 16.
__device__ __forceinline__ uint32_t ring_off(uint32_t q, uint32_t lane) {
    return (((q >> 4) & (kPieces * kRingSlots - 1)) << 10) | (lane << 4) | (q & 15u);
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
// that "s_waitcnt vmcnt(8)" means exactly "every round but the newest two landed".
__device__ __forceinline__ void ring_issue(uint8_t *ring_wave, const uint8_t *gbase, const uint8_t *dummy,
                                           uint32_t r, uint32_t last16, bool active) {
#pragma unroll
    for (uint32_t j = 0; j < kPieces; j++) {
        const uint32_t c16 = r * kPieces + j;
        const uint8_t *g = (active && c16 <= last16) ? gbase + (size_t)c16 * 16 : dummy;
        dma16(g, lds_addr(ring_wave + ((r & (kRingSlots - 1)) * kPieces + j) * 1024));
    }
}

template <bool CRC>
__global__ void __launch_bounds__(kParseWG<CRC>) k_dec_parse(qlzx_blocks b, const uint32_t *dst_cap,
                                                         uint32_t *dsize_out, int32_t *status,
                                                         const uint32_t *crc_state, const uint32_t *crc_expect,
                                                         uint32_t *crc_out, uint32_t first, uint32_t count,
                                                         BlkInfo *info, GroupRec *recs, uint32_t gmax,
                                                         const uint32_t *order, uint32_t max_dsize) {
    __shared__ __attribute__((aligned(16))) uint8_t ring_all[(kParseWG<CRC> / 64) * kRingWave];
    __shared__ uint32_t tab[CRC ? 8 * 256 : 1];
    if (CRC) {
        for (uint32_t t = threadIdx.x; t < 8 * 256; t += kParseWG<CRC>) tab[t] = g_crc_slice8[t];
        __syncthreads();
    }
    const uint32_t lane = threadIdx.x & 63;
    uint8_t *ring = ring_all + (threadIdx.x >> 6) * kRingWave;
    const uint32_t lin = blockIdx.x * kParseWG<CRC> + threadIdx.x;
    const bool inrange = lin < count;
    // block: the lin-th of the chunk's list (or of the call, in order); workspace slot: lin
    const uint32_t i = inrange ? (order ? order[lin] : first + lin) : first;

    int st = QLZX_OK;
    uint32_t kind = kBlkSkip, csize = 0, dsize = 0, hdr = 0, len = 0;
    const uint8_t *src = b.src + b.src_off[i];
    if (inrange) {
        len = b.src_len[i];
        st = classify_block(src, len, dst_cap ? dst_cap[i] : 0xffffffffu, max_dsize, kind, csize, dsize, hdr);
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
    GroupRec *myrec = recs + (size_t)(inrange ? lin : 0) * gmax;
    uint32_t crc = (CRC && inrange && crc_state) ? crc_state[i] : 0xffffffffu;
    bool done_parse = !parsing;

    PROF_DECL
    const uint8_t *dummy = (const uint8_t *)(((uintptr_t)b.src) & ~(uintptr_t)15);
    ring_issue(ring, gbase, dummy, 0, last16, stream);
    ring_issue(ring, gbase, dummy, 1, last16, stream && last_round >= 1);
    ring_issue(ring, gbase, dummy, 2, last16, stream && last_round >= 2);
    for (uint32_t r = 0;; r++) {
        if (__ballot(stream && r <= last_round) == 0) break;
        // rounds <= r landed once at most the newest two rounds' 8 DMAs are in flight
        PROF_MARK(0);
#if QLZX_K1_ROUND == 64
        asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
#elif QLZX_K1_ROUND == 32
        asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
#else
#error "QLZX_K1_ROUND: 32 or 64"
#endif
        PROF_MARK(1);  // 1: waiting for the round's DMA
        const bool act = stream && r <= last_round;
        // CRC of this round's bytes [cq, chi), in stream order.  It is interleaved with the parse
        // steps below (one 8-byte slicing step per parse iteration) and finished after them: the
        // parse is a serial chain per lane, and the CRC steps fill its dependency bubbles instead
        // of running ahead of it on the critical path.
        uint32_t cq = 0, chi = 0;
        if (CRC && act) {
            const uint32_t q0 = r * kRoundBytes, q1 = q0 + kRoundBytes;
            cq = q0 > shift ? q0 : shift;
            chi = (q1 < span + shift) ? q1 : span + shift;
        }
        auto crc_step = [&]() {
            if (cq < chi) {
                if (!(cq & 7u) && cq + 8 <= chi) {
                    const uint32_t w0 = *(const uint32_t *)(ring + ring_off(cq, lane));
                    const uint32_t w1 = *(const uint32_t *)(ring + ring_off(cq + 4, lane));
                    crc = crc_slice8(tab, crc, w0, w1);
                    cq += 8;
                } else {
                    crc = crc_byte(tab, crc, ring[ring_off(cq, lane)]);
                    cq++;
                }
            }
        };
        PROF_MARK(2);  // 2: CRC
        // parse while the bytes the next step reads have landed (stream pos < lim)
        const uint32_t lim = (r + 1) * kRoundBytes - shift;
        bool go = act && !done_parse;
        while (__ballot(go)) {
#ifdef QLZX_PROFILE
            _pacc[5] += 1;
            if (go) _pacc[6] += 1;
#endif
            if (CRC) crc_step();
            // one step = a control word (k == 31), or a literal run (possibly empty)
            // followed by the match that ends it.  Straight-line selects; only the
            // record store branches.
            const bool gb = k == 31;
            const uint32_t kk = k & 31;
            const uint32_t cwk = cw >> kk;
            uint32_t run = __builtin_ctz(cwk | (1u << (31 - kk)));             // literals before the next match
            run = gb ? 0u : (run < csize - ip ? run : csize - ip);
            const uint32_t ipm = ip + run, km = kk + run;                       // the match after the run
            const bool hasm = !gb & (km < 31) & (ipm < csize);
            const bool end = ip + (gb ? 4u : 1u) > csize;                       // stream exhausted
            const bool landed = ipm + (gb ? 4u : 1u) <= lim;                    // bytes this step reads
            const bool mat = hasm & landed;
            const bool stepping = go & !end & (gb ? landed : (run > 0) | mat);
            const uint32_t w = ring_rd32(ring, ipm + shift, lane);  // cword, or the match token
            const uint32_t ty = (w & 3u) + ((w & 127u) == 3u ? 1u : 0u);
            const uint32_t code = __builtin_amdgcn_ubfe(0x32110u, ty * 4, 4);  // token bytes - 1
            // a second match right after it when its first byte is already in w
            const uint32_t ip2 = ipm + code + 1, k2 = km + 1;
            const uint32_t w2 = w >> (8 * ((code + 1) & 3));
            const bool mat2 = mat & (code < 3) & (k2 < 31) & (((cw >> (k2 & 31)) & 1u) != 0) & (ip2 < csize) &
                              (ip2 + 1 <= lim);
            const uint32_t ty2 = (w2 & 3u) + ((w2 & 127u) == 3u ? 1u : 0u);
            const uint32_t code2 = __builtin_amdgcn_ubfe(0x32110u, ty2 * 4, 4);
            bool bad = stepping & ((gb & (((w >> 31) == 0) | (g >= gmax))) |  // C1, group bound
                                   (mat & (ipm + code + 1 > csize)) |        // C2
                                   (mat2 & (ip2 + code2 + 1 > csize)));
            if (stepping & gb & (g > 0)) myrec[g - 1] = GroupRec{rec_ip, m, ra, rb};
            st = bad ? QLZX_E_CORRUPT : st;
            const bool adv = stepping & !bad;
            const bool ag = adv & gb;
            const uint32_t bm = mat ? (1u << (km & 31)) : 0u;
            const uint32_t bm2 = mat2 ? (1u << (k2 & 31)) : 0u;
            rec_ip = ag ? ip : rec_ip;
            cw = ag ? w : cw;
            g += ag ? 1u : 0u;
            ip += adv ? (gb ? 4u : run + (mat ? code + 1 : 0u) + (mat2 ? code2 + 1 : 0u)) : 0u;
            k = adv ? (gb ? 0u : km + (mat ? 1u : 0u) + (mat2 ? 1u : 0u)) : k;
            m = adv ? (gb ? 0u : m | bm | bm2) : m;
            ra = adv ? (gb ? 0u : ra | ((code & 1u) ? bm : 0u) | ((code2 & 1u) ? bm2 : 0u)) : ra;
            rb = adv ? (gb ? 0u : rb | ((code & 2u) ? bm : 0u) | ((code2 & 2u) ? bm2 : 0u)) : rb;
            done_parse = done_parse | (go & (end | bad));
            go = adv;
        }
        if (CRC)
            while (__ballot(cq < chi)) crc_step();  // the rest of the round's CRC
        PROF_MARK(3);  // 3: parse
        if (!CRC && done_parse) stream = false;  // nothing left to read for this lane
        // round r+3 reuses the slot of round r-1 (consumed: round r+1 reads only rounds r, r+1)
        ring_issue(ring, gbase, dummy, r + 3, last16, stream && r + 3 <= last_round);
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
    info[lin] = bi;
}

// ------------------------------------------------------------------ K2 ----
// mem = (mem & ~mask) | val in one LDS instruction (val pre-masked); OFF = byte
// offset folded into the instruction (one address register for a whole copy).
template <uint32_t OFF = 0>
__device__ __forceinline__ void lds_mskor(uint32_t *addr, uint32_t mask, uint32_t val) {
    const uint32_t a = (uint32_t)(uintptr_t)addr;
    asm volatile("ds_mskor_b32 %0, %1, %2 offset:%3" ::"v"(a), "v"(mask), "v"(val), "i"(OFF) : "memory");
}

// K2 shared memory: prefetch slots, then the output window.  Output position
// p lives at win[p - base] for p in [base, base + W); older output has been
// flushed to the block's destination in HBM ("window").
template <uint32_t W>
struct K2Lds {
    uint8_t pad[16];                 // a source dword may start 4 B before win[0]
    uint8_t win[W + 32];             // reads run <= 24 B past a write; win[W + 24] = literal dummy
    GroupRec rec[kRecSlots][4];      // records of the <= 4 groups of batches bt+kTokAhead .. bt+kRecAhead
    uint32_t tok[kTokSlots][64];     // per-lane token dword of batches bt .. bt+kTokAhead-1
};  // the window first: copy addresses fit the DS instructions' immediate offsets

// Every K2 iteration issues exactly 2 DMA instructions (1 token dword + 1
// record), with dummy addresses for lanes/batches past the end, so that
// "s_waitcnt vmcnt(2 * kK2Slack)" at the end of iteration bt means "everything
// issued up to iteration bt - kK2Slack has landed".  Iteration bt issues the
// tokens of bt + kTokAhead and the records of bt + kRecAhead, so both have
// kK2Slack whole iterations to arrive.  Slack 1 (the default since round 2) keeps 640 B less
// LDS and two fewer in-flight batch registers per wave than slack 3 and measured faster on
// c2 (39.1 vs 39.9 ms, interleaved runs) and c5 (482.6 vs 455 GiB/s): the wave issues about
// a whole iteration of work between a DMA and its use, which covers the DMA at this occupancy.
template <bool DMA = true>
__device__ __forceinline__ void issue_rec(GroupRec *slot, const GroupRec *rb, uint32_t g0, uint32_t ngroups,
                                          uint32_t lane) {
    const uint32_t g = g0 + lane;
    if (DMA && lane < 4) dma16(g < ngroups ? (const void *)(rb + g) : (const void *)rb, lds_addr(slot));
}

// Per-lane coordinates of item I = 64 bt + lane: group g = I / 31, index k = I % 31.
// Advanced by one batch (64 = 2 * 31 + 2) without a division.
struct ItemCursor {
    uint32_t g, k;
    __device__ __forceinline__ void next() {
        k += 2;
        const bool wrap = k >= 31;
        k = wrap ? k - 31 : k;
        g += wrap ? 3 : 2;
    }
};

// Token prefetch for one batch: returns pos | is_match << 31 for the lane's item
// (0 past the last item) and DMAs the 4 stream bytes at min(pos, csize - 4)
// (unaligned dword DMA; csize >= 7 for a compressed level-3 stream, so the read
// stays inside the block).  Item position: control word at gr.ip, then k items
// with popc(a) + 2 popc(b) extra token bytes before item k.
__device__ __forceinline__ GroupRec tok_rec(const GroupRec *recslot, uint32_t g0, const ItemCursor &c, bool valid) {
    return recslot[valid ? c.g - g0 : 0];
}
template <bool DMA = true>
__device__ __forceinline__ uint32_t issue_tok(const GroupRec &gr, const ItemCursor &c, bool valid, uint32_t *tok,
                                              const uint8_t *src, uint32_t csize, uint32_t *pout = nullptr) {
    const uint32_t low = (1u << c.k) - 1u;
    const uint32_t pos = gr.ip + 4 + c.k + __builtin_popcount(gr.a & low) + 2 * __builtin_popcount(gr.b & low);
    const uint32_t p = valid ? (pos + 4 <= csize ? pos : csize - 4) : 0u;
    if (DMA) dma4(src + p, lds_addr(tok));
    if (pout) *pout = p;
    return valid ? (pos | (((gr.m >> c.k) & 1u) << 31)) : 0u;
}

// Branch-free level-3 token decode (quicklz.c:579-610).  Token type
// ty = (t & 3) + ((t & 127) == 3) selects per-type bit fields from packed tables:
//   ty 0: 1 B, off = t[2:8),  len 3          ty 1: 2 B, off = t[2:16), len 3
//   ty 2: 2 B, off = t[6:16), len = t[2:6)+3  ty 3: 3 B, off = t[7:24), len = t[2:7)+2
//   ty 4: 4 B, off = t[15:32), len = t[7:15)+3
__device__ __forceinline__ void decode_tok_bf(uint32_t t, uint32_t &off, uint32_t &len, uint32_t &tl) {
    const uint32_t ty = (t & 3u) + ((t & 127u) == 3u ? 1u : 0u);
    const uint32_t f4 = ty * 4, f6 = ty * 6;
    const uint32_t osh = __builtin_amdgcn_ubfe(0xF7622u, f4, 4);
    const uint32_t ow = __builtin_amdgcn_ubfe((6u) | (14u << 6) | (10u << 12) | (17u << 18) | (17u << 24), f6, 6);
    const uint32_t lsh = __builtin_amdgcn_ubfe(0x72200u, f4, 4);
    const uint32_t lw = __builtin_amdgcn_ubfe(0x85400u, f4, 4);
    const uint32_t la = __builtin_amdgcn_ubfe(0x32333u, f4, 4);
    tl = __builtin_amdgcn_ubfe(0x43221u, f4, 4);
    off = __builtin_amdgcn_ubfe(t, osh, ow);
    len = __builtin_amdgcn_ubfe(t, lsh, lw) + la;
}

// Byte masks of bytes [lo, lo + n) (lo < 4, n <= 16) over five dwords.
struct Copy16 {
    uint32_t qa, sh, mk[5];
    int xa;
    __device__ __forceinline__ void prep(uint32_t q, uint32_t off, uint32_t n) {
        const uint32_t lo = q & 3u;
        qa = q - lo;
        const int sa = (int)qa - (int)off;  // >= -4: out[] has a 16-B front pad
        xa = sa & ~3;
        sh = (uint32_t)sa & 3u;
        const int H = 8 * (int)(lo + n);
#pragma unroll
        for (int j = 0; j < 5; j++) {
            int sj = 32 * (j + 1) - H;
            sj = sj < 0 ? 0 : (sj > 32 ? 32 : sj);
            mk[j] = (uint32_t)(0xffffffffull >> sj);
        }
        mk[0] &= 0xffffffffu << (8 * lo);
    }
    // source dwords already in registers (far matches: y[] from HBM)
    __device__ __forceinline__ void run_y(uint8_t *out, const uint32_t y[5]) const {
        uint32_t *dw = (uint32_t *)(out + qa);
        lds_mskor<0>(dw, mk[0], y[0] & mk[0]);
        lds_mskor<4>(dw, mk[1], y[1] & mk[1]);
        lds_mskor<8>(dw, mk[2], y[2] & mk[2]);
        lds_mskor<12>(dw, mk[3], y[3] & mk[3]);
        lds_mskor<16>(dw, mk[4], y[4] & mk[4]);
    }
    __device__ __forceinline__ void run(uint8_t *out) const {
        const uint32_t *x = (const uint32_t *)(out + xa);
        const uint32_t x0 = x[0], x1 = x[1], x2 = x[2], x3 = x[3], x4 = x[4], x5 = x[5];
        uint32_t *dw = (uint32_t *)(out + qa);
        lds_mskor<0>(dw, mk[0], __builtin_amdgcn_alignbyte(x1, x0, sh) & mk[0]);
        lds_mskor<4>(dw, mk[1], __builtin_amdgcn_alignbyte(x2, x1, sh) & mk[1]);
        lds_mskor<8>(dw, mk[2], __builtin_amdgcn_alignbyte(x3, x2, sh) & mk[2]);
        lds_mskor<12>(dw, mk[3], __builtin_amdgcn_alignbyte(x4, x3, sh) & mk[3]);
        lds_mskor<16>(dw, mk[4], __builtin_amdgcn_alignbyte(x5, x4, sh) & mk[4]);
    }
};

// Match sub-rounds when every pending match takes the plain 16-B copy (no byte or chunked
// path): per sub-round, ready = pending & no pending lane in `need`, copied under exec = ready.
// The compiled form of this loop spent ~37 of its ~55 instructions per sub-round on turning
// per-lane bools into masks and back; here the pending set stays in two SGPRs and the
// readiness test is three VALU.  The lowest pending lane's `need` holds only lanes below it
// (need lies inside [owner(s), owner(send - 1)], send <= d), so every sub-round copies at least
// that lane and the loop ends.  LDS operations of a wave execute in issue order, so a
// sub-round's reads observe the previous sub-round's ds_mskor writes.
__device__ __forceinline__ void subrounds_plain(uint64_t pend, uint64_t need, const Copy16 &cp, uint8_t *win) {
    uint32_t plo = (uint32_t)pend, phi = (uint32_t)(pend >> 32);
    const uint32_t nlo = (uint32_t)need, nhi = (uint32_t)(need >> 32);
    const uint32_t xaddr = (uint32_t)(uintptr_t)(win + cp.xa), qaddr = (uint32_t)(uintptr_t)(win + cp.qa);
    uint64_t sv;
    uint32_t st, t, x0, x1, x2, x3, x4, x5;
    asm volatile(
        "s_mov_b64 %[sv], exec\n"
        "1:\n"
        "v_and_b32 %[t], %[plo], %[nlo]\n"
        "v_and_or_b32 %[t], %[phi], %[nhi], %[t]\n"
        "v_cmp_eq_u32 vcc, 0, %[t]\n"
        "s_and_b32 vcc_lo, vcc_lo, %[plo]\n"
        "s_and_b32 vcc_hi, vcc_hi, %[phi]\n"
        "s_andn2_b32 %[plo], %[plo], vcc_lo\n"
        "s_andn2_b32 %[phi], %[phi], vcc_hi\n"
        "s_mov_b64 exec, vcc\n"
        "ds_read_b32 %[x0], %[xa]\n"
        "ds_read_b32 %[x1], %[xa] offset:4\n"
        "ds_read_b32 %[x2], %[xa] offset:8\n"
        "ds_read_b32 %[x3], %[xa] offset:12\n"
        "ds_read_b32 %[x4], %[xa] offset:16\n"
        "ds_read_b32 %[x5], %[xa] offset:20\n"
        "s_waitcnt lgkmcnt(4)\n"
        "v_alignbyte_b32 %[t], %[x1], %[x0], %[sh]\n"
        "v_and_b32 %[t], %[t], %[m0]\n"
        "ds_mskor_b32 %[qa], %[m0], %[t]\n"
        "s_waitcnt lgkmcnt(4)\n"
        "v_alignbyte_b32 %[x0], %[x2], %[x1], %[sh]\n"
        "v_and_b32 %[x0], %[x0], %[m1]\n"
        "ds_mskor_b32 %[qa], %[m1], %[x0] offset:4\n"
        "s_waitcnt lgkmcnt(4)\n"
        "v_alignbyte_b32 %[x1], %[x3], %[x2], %[sh]\n"
        "v_and_b32 %[x1], %[x1], %[m2]\n"
        "ds_mskor_b32 %[qa], %[m2], %[x1] offset:8\n"
        "s_waitcnt lgkmcnt(4)\n"
        "v_alignbyte_b32 %[x2], %[x4], %[x3], %[sh]\n"
        "v_and_b32 %[x2], %[x2], %[m3]\n"
        "ds_mskor_b32 %[qa], %[m3], %[x2] offset:12\n"
        "s_waitcnt lgkmcnt(4)\n"
        "v_alignbyte_b32 %[x3], %[x5], %[x4], %[sh]\n"
        "v_and_b32 %[x3], %[x3], %[m4]\n"
        "ds_mskor_b32 %[qa], %[m4], %[x3] offset:16\n"
        "s_mov_b64 exec, %[sv]\n"
        "s_or_b32 %[st], %[plo], %[phi]\n"
        "s_cbranch_scc1 1b\n"
        : [sv] "=&s"(sv), [plo] "+s"(plo), [phi] "+s"(phi), [st] "=&s"(st), [t] "=&v"(t), [x0] "=&v"(x0),
          [x1] "=&v"(x1), [x2] "=&v"(x2), [x3] "=&v"(x3), [x4] "=&v"(x4), [x5] "=&v"(x5)
        : [nlo] "v"(nlo), [nhi] "v"(nhi), [xa] "v"(xaddr), [qa] "v"(qaddr), [sh] "v"(cp.sh), [m0] "v"(cp.mk[0]),
          [m1] "v"(cp.mk[1]), [m2] "v"(cp.mk[2]), [m3] "v"(cp.mk[3]), [m4] "v"(cp.mk[4])
        : "vcc", "scc", "memory");
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

// Lane owning byte D + r of the sub-batch (r < kSubMax): starts at or before r, minus one.
__device__ __forceinline__ uint32_t owner_of(const uint32_t *bm, uint32_t bex, uint32_t r) {
    const uint32_t w = bm[r >> 5];
    const uint32_t below = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((r >> 5) << 2), (int)bex);
    return below + __builtin_popcount(w & ((2u << (r & 31)) - 1u)) - 1u;
}

__device__ __forceinline__ uint32_t ff1_or(uint64_t m, uint32_t dflt) {
    return m ? (uint32_t)__builtin_ctzll(m) : dflt;
}

// Far source (below the window): the five destination-aligned dwords
// y[j] = bytes [a0 + 4j, a0 + 4j + 4) of the block's output in HBM, a0 = s - lo
// (lo = the destination's byte offset in its dword, whose lo leading bytes the
// caller masks off; callers guarantee s >= lo), as unaligned dword loads straight into y
// (no shuffle), so nothing waits on them until the first sub-round.  A far source ends
// below base, so the 20-B read stays inside the block while base + 20 <= dsize (no
// per-dword clamp); otherwise far lanes take the byte path.
// Five dword loads from opaque offsets: merged loads need aligned register tuples (66 VGPRs).
// While the window base is within 20 B of the block's end, far lanes take the byte path instead
// (c2 38.09 -> 37.79 ms against a per-dword clamp).
__device__ __forceinline__ void far_load20_fast(const uint8_t *dst, uint32_t a0, uint32_t y[5]) {
#pragma unroll
    for (int j = 0; j < 5; j++) {
        uint32_t a = a0 + 4 * j;
        asm volatile("" : "+v"(a));
        y[j] = *(const uint32_t *)(dst + a);
    }
}

template <uint32_t W>
__global__ void __launch_bounds__(64) k_dec_blocks(qlzx_blocks b, uint32_t *dsize_out, int32_t *status,
                                                   uint32_t first, uint32_t count, const BlkInfo *info,
                                                   const GroupRec *recs, uint32_t gmax, const uint32_t *list) {
    static_assert(W % 2048 == 0 && W >= 2048, "window: a multiple of 2 KiB (slides by W/2)");
    __shared__ __attribute__((aligned(16))) K2Lds<W> L;
    const uint32_t lane = threadIdx.x;
    const uint32_t bx = blockIdx.x;  // workspace slot
    if (bx >= count) return;
    const uint32_t i = list ? list[bx] : first + bx;  // block
    const BlkInfo bi = info[bx];
    if (bi.kind == kBlkSkip) return;
    const uint8_t *src = b.src + b.src_off[i];
    uint8_t *dst = b.dst + b.dst_off[i];
    const uint32_t dsize = bi.dsize;
    if (bi.kind == kBlkStored) {  // quicklz.c:808-811
        const uint32_t hdr = (src[0] & 2u) ? 9u : 3u;
        const uint8_t *s = src + hdr;
        uint32_t p0 = 0;
        if ((((uintptr_t)dst) & 15u) == 0) {
            // 16 B per lane: four unaligned dword loads (unaligned access mode, as in far_load20),
            // one aligned 16-B store; 1 KiB per wave instruction
            p0 = dsize & ~15u;
            for (uint32_t p = lane * 16; p < p0; p += 1024) {
                const uint32_t *q = (const uint32_t *)(s + p);
                *(uint4 *)(dst + p) = make_uint4(q[0], q[1], q[2], q[3]);
            }
        }
        for (uint32_t p = p0 + lane; p < dsize; p += 64) dst[p] = s[p];
        if (lane == 0) { status[i] = QLZX_OK; if (dsize_out) dsize_out[i] = dsize; }
        return;
    }
    uint8_t *win = L.win;
    const GroupRec *rb = recs + (size_t)bx * gmax;
    const uint32_t nitems = bi.nitems, ngroups = bi.ngroups;
    const uint32_t csize = b.src_len[i];
    const uint32_t hdr = (src[0] & 2u) ? 9u : 3u;
    const uint32_t nb = (nitems + 63) / 64;
    const uint32_t tail_from = dsize > QLZX_TAIL ? dsize - 1 - QLZX_TAIL : 0;  // op >= this: tail (quicklz.c:503)
    const bool a16 = (((uintptr_t)dst) & 15u) == 0;

    // prologue: records of batches 0..3, the tokens of batches 0..3 (which read
    // those records), then the records of batches 4..7 (slots 4, 0, 1, 2)
    for (uint32_t j = 0; j < kTokAhead; j++) issue_rec(L.rec[j], rb, (j * 64) / 31, ngroups, lane);
    vm_sync();
    ItemCursor cur{lane / 31, lane % 31};  // item coordinates of the next batch to issue
    uint32_t pm[kTokAhead];
#pragma unroll
    for (uint32_t j = 0; j < kTokAhead; j++) {
        const bool v = j * 64 + lane < nitems;
        pm[j] = issue_tok(tok_rec(L.rec[j], (j * 64) / 31, cur, v), cur, v, L.tok[j], src, csize);
        cur.next();
    }
    for (uint32_t j = kTokAhead; j < kRecAhead; j++) issue_rec(L.rec[j % kRecSlots], rb, (j * 64) / 31, ngroups, lane);
    vm_sync();
    PROF_DECL
    uint32_t D = 0;                   // output bytes of all earlier items
    uint32_t base = 0;                // window start (multiple of W/2)
    bool err = false;                 // per-lane: a check failed on this lane's item
    bool tail = false, complete = dsize == 0;
    // slot counters: tokens of bt (read) and bt+kTokAhead (issue); records of bt+kTokAhead (read)
    // and bt+kRecAhead (issue)
    uint32_t ts = 0, rs4 = kTokAhead % kRecSlots, rs8 = kRecAhead % kRecSlots;
    for (uint32_t bt = 0; bt < nb && !complete; bt++) {
        // this batch's token dword, and the record the prefetch of batch bt+kTokAhead needs;
        // both reads complete before that prefetch reuses this batch's token slot
        const uint32_t tw = L.tok[ts][lane];
        const bool v4 = (bt + kTokAhead) * 64 + lane < nitems;
        const GroupRec gr4 = tok_rec(L.rec[rs4], ((bt + kTokAhead) * 64) / 31, cur, v4);
        lds_sync();
        const uint32_t posm = pm[0];
#pragma unroll
        for (uint32_t j = 0; j + 1 < kTokAhead; j++) pm[j] = pm[j + 1];
        // the token DMA of batch bt+kTokAhead goes out at the end of the iteration: until then
        // this batch's token slot holds the item-start bitmap of the sub-batches
        uint32_t tokp;
        pm[kTokAhead - 1] = issue_tok<false>(gr4, cur, v4, nullptr, src, csize, &tokp);
        cur.next();
        uint32_t *const bm = L.tok[ts];
        GroupRec *const rslot8 = L.rec[rs8];
        ts = ts == kTokSlots - 1 ? 0 : ts + 1;
        rs4 = rs4 == kRecSlots - 1 ? 0 : rs4 + 1;
        rs8 = rs8 == kRecSlots - 1 ? 0 : rs8 + 1;
        PROF_MARK(1);  // 1: prefetch issue
        const bool valid = bt * 64 + lane < nitems;
        const bool ism = (posm >> 31) != 0;
        const uint32_t pos = posm & 0x7fffffffu;
        const uint32_t t = pos + 4 <= csize ? tw : tw >> (8 * (pos + 4 - csize));
        uint32_t off, mlen, tl;
        decode_tok_bf(t, off, mlen, tl);
        const uint32_t len0 = ism ? mlen : (valid ? 1u : 0u);
        tl = ism ? tl : 1u;
        // ---- sub-batches: normally one; more when the batch's output overflows the window ----
        uint32_t lo_lane = 0;
        bool more = true;
        while (more) {
            const uint32_t sub0 = lo_lane;  // first lane of this sub-batch
            const bool act = lane >= lo_lane;
            const uint32_t len = act ? len0 : 0u;
            uint32_t incl = wave_incl_scan(len);
            uint32_t total = __builtin_amdgcn_readfirstlane(__builtin_amdgcn_readlane(incl, 63));
            if (D + total > base + W && D - base >= W / 2) {
                // slide: flush win[0, W/2) to HBM, move the rest down, base += W/2
                for (uint32_t q = lane * 16; q < W / 2; q += 1024) {
                    const uint4 v = *(const uint4 *)(win + q);
                    if (a16) *(uint4 *)(dst + base + q) = v;
                    else for (uint32_t k = 0; k < 16; k++) dst[base + q + k] = win[q + k];
                }
                for (uint32_t q = lane * 16; q < D - base - W / 2; q += 1024)
                    *(uint4 *)(win + q) = *(const uint4 *)(win + W / 2 + q);
                base = __builtin_amdgcn_readfirstlane(base + W / 2);
            }
            const uint32_t d = D + incl - len;
            // this sub-batch: the active lanes whose output fits the window (a prefix)
            const bool fits = d + len <= base + W && d + len <= D + kSubMax;
            const uint64_t outm = __ballot(act && len && !fits);
            const uint32_t cut = outm ? (uint32_t)__builtin_ctzll(outm) : 64u;
            const bool in = act && lane < cut;
            more = cut < 64;
            lo_lane = __builtin_amdgcn_readfirstlane(cut);
            const uint32_t stotal = cut < 64 ? __builtin_amdgcn_readlane(incl - len, cut) : total;
            // far sources (below the window, already in HBM): load them first, use them in the first sub-round
            const uint32_t s = d - off;
            const bool far = s < base;
            // byte / chunked path; also every far source while the window base is within 20 B
            // of the block's end (wave-uniform, rare), so far_load20_fast never reads past dsize
            const bool nearend = base + 20 > dsize;
            const bool spec = off < len || len > 16 || (far && (s + len > base || s < 3 || nearend));
            // only read under fc, which implies fload: no zero fill, whose register writes made
            // the compiler wait (vmcnt) for every load still in flight, prefetch DMAs included
            uint32_t fy[5];
            const bool fload = in && valid && ism && far && !spec;
            if (__ballot(fload)) {
                // a far source ends below base: its 20-B read stays inside the block unless the
                // window base is within 20 B of the end (then those lanes are spec)
                if (fload) far_load20_fast(dst, s - (d & 3u), fy);
            }
            // ---- checks C2-C5 on the live items (those that start before dsize) ----
            const bool live = in && valid && d < dsize;
            const uint64_t tail_lanes = __ballot(live && !ism && d >= tail_from);
            const uint32_t tail_lane = tail ? 0u : ff1_or(tail_lanes, 64u);  // C4: no match after it
            tail = tail || tail_lanes != 0;
            const bool mok = off >= 3 && off <= d && d + len + 4 <= dsize && lane < tail_lane;  // C3, C4
            const bool last = live && d + len == dsize;  // C5: the item completing dsize ends the stream
            const uint32_t ip_end = pos + tl;
            const bool eok = ip_end == csize || (ip_end < hdr + 9 && csize == hdr + 9);
            const bool bad = live && ((ism && !mok) || (last && !eok));
            err = err || bad;
            complete = __ballot(last) != 0;
            if (complete) more = false;
            PROF_MARK(2);  // 2: decode + scan + checks
            // literals (non-literal lanes store to an unused byte past the window)
            win[(live && !ism) ? d - base : W + 24] = (uint8_t)t;
            PROF_MARK(0);  // 0: literal stores
            // ---- matches: which in-sub-batch lanes each match's source needs ----
            // Bit r of the bitmap bm marks an item starting at D + r.  The lane owning
            // byte D + r is sub0 + (#starts at or before r) - 1; a match needs the lanes owning
            // [max(s, D), send): the contiguous lane range [la, lb].
            const uint32_t rs = d - D;  // < kSubMax for `in` lanes
            bm[lane] = 0;
            if (in && len) __hip_atomic_fetch_or(&bm[rs >> 5], 1u << (rs & 31), __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_WORKGROUP);
            // other lanes' ORs land in this lane's word: a compiler barrier so the read is
            // not folded into the lane's own store (the wave's LDS ops run in issue order)
            asm volatile("" ::: "memory");
            const uint32_t bw = bm[lane];
            const uint32_t bpc = __builtin_popcount(bw);
            const uint32_t bex = wave_incl_scan(bpc) - bpc;  // starts in words below `lane`
            const uint32_t send = (s + len < d) ? s + len : d;
            const bool dep = in && ism && send > D;
            const uint32_t qa = (dep && s > D) ? s - D : 0u, qb = dep ? send - 1 - D : 0u;
            // lanes below sub0 (earlier sub-batches) own nothing here; every later valid lane
            // has len > 0, so the k-th start belongs to lane sub0 + k
            const uint32_t la = sub0 + owner_of(bm, bex, qa), lb = sub0 + owner_of(bm, bex, qb);
            const uint64_t need = dep ? ((~0ull << la) & (~0ull >> (63 - lb))) : 0ull;
            // ---- matches: copy in sub-rounds ----
            bool done = !(live && ism && !bad);
            const uint32_t n16 = len < 16 ? len : 16;
            Copy16 cp;
            cp.prep(d - base, off, n16);
            PROF_MARK(6);  // 6: bitmap, owner lookups, need mask, copy masks
            // far matches (source in HBM, below the window) depend on no lane of this batch:
            // copy them before the sub-rounds, so the loop needs no source select
            {
                const bool fc = !done && far && !spec;
                if (__ballot(fc)) {
                    if (fc) cp.run_y(win, fy);
                }
                done = done || fc;
            }
            PROF_MARK(7);  // 7: far copies (waits for the far loads)
            uint64_t pend = __ballot(!done);
            const bool spec_any = __ballot(!done && spec) != 0;  // rare: skip its test per sub-round
            if (!spec_any) {  // every pending match takes the 16-B copy: the hand-scheduled loop
                if (pend) subrounds_plain(pend, need, cp, win);
                pend = 0;
            }
            while (pend) {
                // exact: every byte of the source is final once none of the lanes owning it is pending
                const bool ready = !done & ((need & pend) == 0);
                if (ready && !spec) cp.run(win);
                if (spec_any && __ballot(ready && spec)) {
                    if (ready && spec) {
                        if (far || (off < 16 && off < len)) {
                            // byte by byte, in order (short-period overlap, or a source in HBM)
                            for (uint32_t j = 0; j < len; j++) {
                                const uint32_t sp = s + j;  // = d + j - off: earlier bytes of this copy included
                                const uint8_t v = sp < base ? dst[sp] : win[sp - base];
                                win[d + j - base] = v;
                            }
                        } else {  // 16-B chunks, in issue order (so an overlapping source sees earlier chunks)
                            for (uint32_t c = 0; c < len; c += 16) {
                                Copy16 c2;
                                c2.prep(d + c - base, off, len - c < 16 ? len - c : 16);
                                c2.run(win);
                            }
                        }
                    }
                }
                done = done || ready;
                // no lgkmcnt wait: a wave's LDS operations execute in issue order, so the
                // next sub-round's reads observe these writes
                pend = __ballot(!done);
            }
            PROF_MARK(3);  // 3: match sub-rounds
            D = __builtin_amdgcn_readfirstlane(D + stotal);
            if (__ballot(err)) { more = false; complete = false; }
        }
        if (__ballot(err)) break;
        // the records of batch bt+kRecAhead, issued after this iteration's far loads were consumed:
        // a DMA issued before them is in the in-order vmcnt queue ahead of them, so the far-load
        // wait would also wait for it (c2: 41.0-41.4 -> 39.7-40.2 ms with the fy change above)
        issue_rec(rslot8, rb, ((bt + kRecAhead) * 64) / 31, ngroups, lane);
        dma4(src + tokp, lds_addr(bm));  // tokens of batch bt+kTokAhead into the slot bt used (bitmap done)
        // DMAs of iterations <= bt - kK2Slack have landed
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(QLZX_K2_VMWAIT) : "memory");
        PROF_MARK(4);  // 4: waiting for prefetch
    }
    vm_sync();
    lds_sync();
    PROF_FLUSH(1);
    if (__ballot(err) || !complete) {
        if (lane == 0) { status[i] = QLZX_E_CORRUPT; if (dsize_out) dsize_out[i] = 0; }
        return;
    }
    // write the rest of the block out: 16 B per lane, 1 KiB per wave instruction
    for (uint32_t p = base + lane * 16; p < dsize; p += 1024) {
        if (p + 16 <= dsize && a16) {
            *(uint4 *)(dst + p) = *(const uint4 *)(win + (p - base));
        } else {
            const uint32_t e = p + 16 < dsize ? p + 16 : dsize;
            for (uint32_t q = p; q < e; q++) dst[q] = win[q - base];
        }
    }
    PROF_MARK(5);  // 5: write-out (not flushed: stamps of the loop only)
    if (lane == 0) {
        status[i] = QLZX_OK;
        if (dsize_out) dsize_out[i] = dsize;
    }
}

}  // namespace qlzx
#include "qlzx_decode_bytes.hip"
namespace qlzx {

#ifndef QLZX_K2B_WIN
#define QLZX_K2B_WIN 4096
#endif
#ifndef QLZX_K2B_MR
#define QLZX_K2B_MR 256
#endif
constexpr uint32_t kWinB = QLZX_K2B_WIN, kMarkRing = QLZX_K2B_MR;

}  // namespace qlzx
#include "qlzx_decode_solo.hip"
namespace qlzx {

inline int launch_decode_wave(const qlzx_blocks &b, const uint32_t *dst_cap, uint32_t *dsize,
                              int32_t *status, const uint32_t *crc_state, const uint32_t *crc_expect,
                              uint32_t *crc_out, uint32_t max_dsize, void *ws, size_t ws_bytes,
                              hipStream_t s) {
    const uint32_t md = max_dsize > QLZX_FAST_MAX_DSIZE ? QLZX_FAST_MAX_DSIZE : max_dsize;
    const uint32_t gmax = groups_max(md);
    const uint32_t chunk = b.n < kChunkBlocks ? b.n : kChunkBlocks;
    const size_t o_rec = ((size_t)chunk * sizeof(BlkInfo) + 255) & ~(size_t)255;
    const size_t one = decode_wave_ws_bytes(b.n, max_dsize);
    const size_t o_list = o_rec + ((((size_t)chunk * rec_bytes_max(md)) + 255) & ~(size_t)255);
    const size_t o_aux = o_list + ((((size_t)b.n * sizeof(uint32_t)) + 255) & ~(size_t)255);
    const bool sort = chunk > 64;
    // two workspace halves when the caller gave room for them: K1 of chunk c+1 runs on a
    // side stream while K2 of chunk c runs on `s` (K1 is latency-bound at low occupancy)
    const bool overlap = ws_bytes >= 2 * one && b.n > chunk;
    // per host thread (the batch API is re-entrant like the reference) and per device: the
    // side stream and events are created on the device that owns `s`
    struct Side {
        hipStream_t st = nullptr;
        hipEvent_t k1[2], k2[2];
    };
    thread_local Side sides[kMaxDevices];
    hipStream_t side = nullptr;
    hipEvent_t *ev_k1 = nullptr, *ev_k2 = nullptr;
    if (overlap) {
        int dev = 0, cur = 0;
        if (s) {
            hipDevice_t hd;
            if (hipStreamGetDevice(s, &hd) != hipSuccess) return (int)hipErrorInvalidResourceHandle;
            dev = (int)hd;
        } else if (hipGetDevice(&dev) != hipSuccess) {
            return (int)hipErrorNoDevice;
        }
        if (dev < 0 || dev >= (int)kMaxDevices) return (int)hipErrorInvalidDevice;
        Side &sd = sides[dev];
        if (!sd.st) {
            (void)hipGetDevice(&cur);
            if (cur != dev) (void)hipSetDevice(dev);
            hipError_t e = hipStreamCreateWithFlags(&sd.st, hipStreamNonBlocking);
            for (int j = 0; j < 2 && e == hipSuccess; j++) {
                e = hipEventCreateWithFlags(&sd.k1[j], hipEventDisableTiming);
                if (e == hipSuccess) e = hipEventCreateWithFlags(&sd.k2[j], hipEventDisableTiming);
            }
            if (cur != dev) (void)hipSetDevice(cur);
            if (e != hipSuccess) return (int)e;
        }
        side = sd.st;
        ev_k1 = sd.k1;
        ev_k2 = sd.k2;
    }
    const bool crc = crc_state || crc_expect || crc_out;
    if (overlap) (void)hipEventRecord(ev_k2[1], s), (void)hipStreamWaitEvent(side, ev_k2[1], 0);
    if (sort) {  // block order of the whole call, ahead of the first K1 (workspace half 0)
        hipStream_t s1 = overlap ? side : s;
        uint32_t *aux = (uint32_t *)((uint8_t *)ws + o_aux);
        (void)hipMemsetAsync(aux, 0, kOrderAux * sizeof(uint32_t), s1);
        const dim3 g((b.n + kOrderPerWG - 1) / kOrderPerWG);
        hipLaunchKernelGGL(k_order_count, g, dim3(kOrderWG), 0, s1, b.src_len, b.n, aux);
        hipLaunchKernelGGL(k_order_scatter, g, dim3(kOrderWG), 0, s1, b.src_len, b.n, aux,
                           (uint32_t *)((uint8_t *)ws + o_list));
    }
    uint32_t c = 0;
    for (uint32_t first = 0; first < b.n; first += chunk, c++) {
        const uint32_t cnt = b.n - first < chunk ? b.n - first : chunk;
        uint8_t *w = (uint8_t *)ws + (overlap ? (c & 1) * one : 0);
        BlkInfo *info = (BlkInfo *)w;
        GroupRec *recs = (GroupRec *)(w + o_rec);
        uint32_t *order = sort ? (uint32_t *)((uint8_t *)ws + o_list) + first : nullptr;
        hipStream_t s1 = overlap ? side : s;
        if (overlap && c >= 2) (void)hipStreamWaitEvent(side, ev_k2[c & 1], 0);  // K2(c-2) freed this half
        const dim3 g1c((cnt + kParseWG<true> - 1) / kParseWG<true>), g1((cnt + kParseWG<false> - 1) / kParseWG<false>);
        if (crc)
            hipLaunchKernelGGL((k_dec_parse<true>), g1c, dim3(kParseWG<true>), 0, s1, b, dst_cap, dsize, status,
                               crc_state, crc_expect, crc_out, first, cnt, info, recs, gmax, order, max_dsize);
        else
            hipLaunchKernelGGL((k_dec_parse<false>), g1, dim3(kParseWG<false>), 0, s1, b, dst_cap, dsize, status,
                               crc_state, crc_expect, crc_out, first, cnt, info, recs, gmax, order, max_dsize);
        if (overlap) (void)hipEventRecord(ev_k1[c & 1], side), (void)hipStreamWaitEvent(s, ev_k1[c & 1], 0);
        // one kernel for every block size: the LDS window slides over longer blocks
#ifdef QLZX_K2_ITEMS
        hipLaunchKernelGGL(k_dec_blocks<kWin>, dim3(cnt), dim3(64), 0, s, b, dsize, status, first, cnt, info, recs,
                           gmax, (const uint32_t *)order);
#else
        hipLaunchKernelGGL((k_dec_bytes<kWinB, kMarkRing>), dim3(cnt), dim3(64), 0, s, b, dsize, status, first, cnt,
                           info, recs, gmax, (const uint32_t *)order);
#endif
        if (overlap) (void)hipEventRecord(ev_k2[c & 1], s);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return (int)e;
    }
    return 0;
}

}  // namespace qlzx
