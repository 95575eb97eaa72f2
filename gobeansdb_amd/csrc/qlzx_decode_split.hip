// qlzx_decode_split.hip -- K2 of the fast decoder, split into an item phase and a match
// phase (DESIGN.md §3 "K2: item phase + match phase").  One wave per block, dsize <= 64 KiB.
//
// The level-3 decode loop of quicklz.c:513-671 does two kinds of work per item: a literal
// byte goes to the output at once, a match copies earlier output.  Only the matches depend on
// each other, so this kernel separates them:
//
//   item phase (IP)   64 items per batch, one per lane.  Item k of group g sits at
//                     ip + 4 + k + popc(a & low(k)) + 2 popc(b & low(k)) (the K1 group record),
//                     its token is read from an LDS ring holding the compressed stream, a DPP
//                     scan places it in the output, checks C3-C5 run, literals are written to
//                     the LDS output window and matches are appended to a match ring in order.
//   match phase (MP)  64 matches per step, one per lane.  A coverage bitmap of the step's own
//                     outputs tells each match whether its source is final (no byte of it is
//                     produced by another match of the step); ready matches copy, the rest are
//                     written back to the front of the ring and retried in the next step with
//                     the new matches behind them.  The first match of a step is always ready.
//
// Per block this issues a fraction of the instructions of the item-per-lane sub-round loop
// (k_dec_blocks): literals never enter the match machinery, and a step copies each match once.
//
// Streams: the compressed bytes arrive by LDS DMA in 256-B chunks (4-chunk ring), the group
// records in 16-group chunks (2-chunk ring).  An iteration issues what the next batch needs
// and the next iteration starts with `s_waitcnt vmcnt(0)`: with 20+ waves per CU the wave
// has spent thousands of cycles elsewhere by then, so the wait rarely stalls.
// The output window holds output [base, base + W); older output has been flushed to the
// block's destination in HBM, and matches reading it ("far") load it back from there.
#include "qlzx_device.h"

namespace qlzx {

constexpr uint32_t kSpChunk = 256;               // stream DMA chunk: 64 lanes x 4 B
constexpr uint32_t kSpRing = 4 * kSpChunk;       // stream ring bytes
constexpr uint32_t kSpRecChunk = 16;             // groups per record DMA (64 lanes x 4 B)
constexpr uint32_t kSpRecRing = 2 * kSpRecChunk; // groups resident
constexpr uint32_t kSpMq = 256;                  // match ring entries (two IP batches + carries)
constexpr uint32_t kSpCov = 2048;                // coverage bitmap reach (64 words)
constexpr uint32_t kMaxDevices = 64;             // per-device side streams of the launcher
#ifndef QLZX_SP_WIN
#define QLZX_SP_WIN 4096
#endif
constexpr uint32_t kSpWin = QLZX_SP_WIN;         // output window (bytes)

template <uint32_t W>
struct SplitLds {
    uint8_t pad[16];                  // a source dword may start 4 B before win[0]
    uint8_t win[W + 32];              // reads run <= 24 B past a write; win[W + 24] = literal dummy
    uint8_t srng[kSpRing];            // compressed stream ring (16-B aligned)
    GroupRec rrng[kSpRecRing];        // group record ring
    uint32_t mqd[kSpMq + 1];          // match ring: d | off << 16; [kSpMq] = dummy slot
    uint8_t mql[kSpMq + 4];           // match ring: len - 3
    uint32_t cov[66];                 // coverage bitmap of a match step (+2 words of slack)
};

// y[j] = bytes [a0 + 4j, a0 + 4j + 4) of the block's output in HBM (a0 = s - (d & 3), s >= d & 3),
// five destination-aligned dwords for Copy16::run_y (bytes past the needed ones are masked off).
__device__ __forceinline__ void sp_far20(const uint8_t *dst, uint32_t a0, uint32_t dsize, uint32_t y[5]) {
    far_load20(dst, a0, dsize, y);
}

// A copy the one-shot 16-B path cannot do: longer than 16 B, overlapping its own output with
// a period < 16, or reading HBM (far) output.  Done in pieces in output order, so every piece's
// source is final when it is read:
//  * a period-`off` overlap copies off, off, 2 off, 4 off ... bytes (source = the bytes just
//    written) until pieces reach 16 B;
//  * a far source is loaded 20 B at a time from HBM; a piece straddling `base` takes its HBM
//    part first and its window part second.
__device__ __forceinline__ void sp_copy_long(uint8_t *win, const uint8_t *dst, uint32_t d, uint32_t off,
                                             uint32_t len, uint32_t base, uint32_t dsize) {
    uint32_t c = 0;
    while (c < len) {
        // source offset: a multiple of the period that is at most c (and off itself at c = 0)
        const uint32_t per = off >= 16u ? off : (c < off ? off : off * (c / off));
        uint32_t n = len - c;
        n = n < 16u ? n : 16u;
        n = n < per ? n : per;
        const uint32_t dp = d + c, sp = dp - per;
        Copy16 cp;
        cp.prep(dp - base, per, n);
        if (sp < base && sp < (dp & 3u)) {  // HBM source too close to the block start for sp_far20
            for (uint32_t j = 0; j < n; j++) win[dp + j - base] = sp + j < base ? dst[sp + j] : win[sp + j - base];
        } else if (sp + n <= base) {  // all in HBM
            uint32_t y[5];
            sp_far20(dst, sp - (dp & 3u), dsize, y);
            cp.run_y(win, y);
        } else if (sp >= base) {  // all in the window
            cp.run(win);
        } else {  // straddles base: HBM bytes first, then the window part
            uint32_t y[5];
            sp_far20(dst, sp - (dp & 3u), dsize, y);
            const uint32_t k = base - sp;  // bytes from HBM
            Copy16 a;
            a.prep(dp - base, per, k);
            a.run_y(win, y);
            Copy16 b;
            b.prep(dp + k - base, per, n - k);
            b.run(win);
        }
        c += n;
    }
}

#ifdef QLZX_PROFILE
#define SP_PROF_ARGS , unsigned long long *_mp
#define SP_PROF_PASS , _mp
#define SP_T0 unsigned long long _mt = __builtin_amdgcn_s_memtime();
#define SP_T(ph)                                                    \
    do {                                                            \
        const unsigned long long _n = __builtin_amdgcn_s_memtime(); \
        _mp[ph] += _n - _mt;                                        \
        _mt = _n;                                                   \
    } while (0)
#define SP_CNT(ph, v) (_mp[ph] += (v))
#else
#define SP_PROF_ARGS
#define SP_PROF_PASS
#define SP_T0
#define SP_T(ph) \
    do {         \
    } while (0)
#define SP_CNT(ph, v) \
    do {              \
    } while (0)
#endif

// Wave-uniform value: tells the compiler it lives in an SGPR (loop-carried state that it
// would otherwise keep in VGPRs, turning uniform branches into exec-mask bookkeeping).
__device__ __forceinline__ uint32_t uni(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }

__device__ __forceinline__ uint32_t lane_rank(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// Bits [b, b + min(k, 64 - b)) of a bitmap word pair (b < 32, k >= 1): the 64-bit mask.
__device__ __forceinline__ uint64_t bits64(uint32_t b, uint32_t k) {
    const uint32_t kk = k < 64u - b ? k : 64u - b;
    return (~0ull >> (64u - kk)) << b;
}

// One match-phase step over the ring entries [hq, hq + min(64, tq - hq)).  Returns the new
// head: ready matches are copied into the window; the others are written back, in order,
// just before the first entry the step did not take.  The common case is straight-line code:
// matches of <= 33 B touch two bitmap words, copies of <= 16 B take one Copy16; longer,
// overlapping and far copies go to sp_copy_long behind a wave-uniform test.
template <uint32_t W>
__device__ __forceinline__ uint32_t sp_mp_step(SplitLds<W> &L, uint32_t hq, uint32_t tq, uint32_t base,
                                               uint8_t *dst, uint32_t dsize, uint32_t lane SP_PROF_ARGS) {
    SP_T0
    const uint32_t n = uni(tq - hq < 64u ? tq - hq : 64u);
    const bool valid = lane < n;
    const uint32_t ei = (hq + lane) & (kSpMq - 1);
    const uint32_t e = L.mqd[ei], el = L.mql[ei];
    const uint32_t d = e & 0xffffu, off = e >> 16, len = el + 3u;
    const uint32_t d0 = uni(d);
    const uint32_t rel = d - d0;
    // lanes whose output ends past the bitmap's reach form a suffix: carried, not covered
    const bool fitb = valid && rel + len <= kSpCov;
    // ---- coverage bitmap: bit r = byte d0 + r is produced by a match of this step ----
    L.cov[lane] = 0;
    {
        const uint64_t m = fitb ? bits64(rel & 31u, len) : 0ull;
        const uint32_t w = fitb ? rel >> 5 : 64u;  // words 64, 65: never read with a non-zero mask
        __hip_atomic_fetch_or(&L.cov[w], (uint32_t)m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        __hip_atomic_fetch_or(&L.cov[w + 1], (uint32_t)(m >> 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    if (__ballot(fitb && (rel & 31u) + len > 64u)) {  // long match (rare): the words past the first two
        if (fitb && (rel & 31u) + len > 64u) {
            for (uint32_t r = (rel & ~31u) + 64u; r < rel + len; r += 32u) {
                const uint32_t k = rel + len - r;
                __hip_atomic_fetch_or(&L.cov[r >> 5], k >= 32u ? 0xffffffffu : (1u << k) - 1u, __ATOMIC_RELAXED,
                                      __HIP_MEMORY_SCOPE_WORKGROUP);
            }
        }
    }
    // other lanes' ORs land in the words read below: keep the reads after them
    asm volatile("" ::: "memory");
    SP_T(0);
    // ---- readiness: no byte of the source [s, se) is produced by a match of this step ----
    const uint32_t s = d - off;
    const uint32_t se = (s + len < d) ? s + len : d;  // an overlapping copy reads its own earlier bytes
    const bool need = fitb && se > d0;
    const uint32_t r0 = (s > d0 ? s : d0) - d0, span = se - d0 - r0;
    bool ready;
    {
        const uint32_t w = need ? r0 >> 5 : 64u;
        const uint64_t x = (uint64_t)L.cov[w] | ((uint64_t)L.cov[w + 1] << 32);
        const uint64_t mm = need ? bits64(r0 & 31u, span) : 0ull;
        ready = fitb && (x & mm) == 0;
    }
    if (__ballot(ready && need && (r0 & 31u) + span > 64u)) {  // long source (rare): the words past the first two
        if (ready && need && (r0 & 31u) + span > 64u) {
            for (uint32_t r = (r0 & ~31u) + 64u; r < r0 + span; r += 32u) {
                const uint32_t k = r0 + span - r;
                const uint32_t m = k >= 32u ? 0xffffffffu : (1u << k) - 1u;
                if (L.cov[r >> 5] & m) ready = false;
            }
        }
    }
    SP_T(1);
    // ---- copy the ready matches ----
    uint8_t *win = L.win;
    const bool spec = off < len || len > 16u || s < base;  // overlapping, long or far: in pieces
    Copy16 cp;
    cp.prep(d - base, off, len);
    if (ready && !spec) cp.run(win);
    SP_T(3);
    if (__ballot(ready && spec)) {
        if (ready && spec) sp_copy_long(win, dst, d, off, len, base, dsize);
        SP_CNT(7, 1);
    }
    SP_T(4);
    // ---- carry the others to the front of the unprocessed part of the ring ----
    const uint64_t cm = __ballot(valid && !ready);
    const uint32_t nd = (uint32_t)__builtin_popcountll(cm);
    const uint32_t slot = (valid && !ready) ? ((hq + n - nd + lane_rank(cm)) & (kSpMq - 1)) : kSpMq;
    L.mqd[slot] = e;
    L.mql[slot] = (uint8_t)el;
    SP_T(5);
    SP_CNT(6, 1);
    return uni(hq + n - nd);
}

// Flush output [base, nb) of the window to HBM and move [nb, D) down to win[0].
template <uint32_t W>
__device__ __forceinline__ void sp_slide(SplitLds<W> &L, uint8_t *dst, bool a16, uint32_t base, uint32_t nb,
                                         uint32_t D, uint32_t lane) {
    uint8_t *win = L.win;
    const uint32_t fl = nb - base;  // multiple of 16
    for (uint32_t q = lane * 16; q < fl; q += 1024) {
        const uint4 v = *(const uint4 *)(win + q);
        if (a16) *(uint4 *)(dst + base + q) = v;
        else for (uint32_t k = 0; k < 16; k++) dst[base + q + k] = win[q + k];
    }
    // every lane has read its flush bytes before any lane overwrites them (in-order LDS)
    for (uint32_t q = lane * 16; q < D - nb; q += 1024) {
        const uint4 v = *(const uint4 *)(win + fl + q);
        *(uint4 *)(win + q) = v;
    }
}

#ifndef QLZX_SP_WAVES_PER_EU
#define QLZX_SP_WAVES_PER_EU 6
#endif
template <uint32_t W>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(QLZX_SP_WAVES_PER_EU)))
k_dec_split(qlzx_blocks b, uint32_t *dsize_out, int32_t *status, uint32_t first, uint32_t count,
            const BlkInfo *info, const GroupRec *recs, uint32_t gmax, const uint32_t *list) {
    static_assert(W % 2048 == 0 && W >= 2048, "window: a multiple of 2 KiB");
    __shared__ __attribute__((aligned(16))) SplitLds<W> L;
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
    const uint32_t tail_from = dsize > QLZX_TAIL ? dsize - 1 - QLZX_TAIL : 0;  // op >= this: tail (quicklz.c:503)
    const bool a16 = (((uintptr_t)dst) & 15u) == 0;
    const bool a4 = (((uintptr_t)dst) & 3u) == 0;

    // stream bytes: ring coordinate q = p + shift (gbase = src rounded down to 4)
    const uint8_t *gbase = (const uint8_t *)(((uintptr_t)src) & ~(uintptr_t)3);
    const uint32_t shift = (uint32_t)(((uintptr_t)src) & 3u);
    const uint32_t last_sc = (csize + shift - 1) >> 8;                   // last stream chunk
    const uint32_t last_rc = ngroups ? (ngroups - 1) / kSpRecChunk : 0;  // last record chunk
    // per-lane DMA sources: the lane's dword of the next stream / record chunk (clamped to
    // the block's first dword past its end)
    const uint32_t lane_s = lane * 4, lane_r = lane * 4;
    const uint32_t s_lim = ((csize + shift + 3) & ~3u) - 4;  // last dword of the stream
    const uint32_t r_lim = ngroups * (uint32_t)sizeof(GroupRec) - 4;
    auto issue_stream = [&](uint32_t c) {  // chunk c into slot c % 4
        const uint32_t o = c * kSpChunk + lane_s;
        dma4(gbase + (o <= s_lim ? o : s_lim), lds_addr(L.srng + (c & 3u) * kSpChunk));
    };
    auto issue_rec = [&](uint32_t r) {  // chunk r (16 groups, all lanes) into slot r % 2
        const uint32_t o = r * (kSpRecChunk * (uint32_t)sizeof(GroupRec)) + lane_r;
        dma4((const uint8_t *)rb + (o <= r_lim ? o : r_lim), lds_addr(&L.rrng[(r & 1u) * kSpRecChunk]));
    };
    // prologue: the whole stream ring and record ring
#pragma unroll
    for (uint32_t c = 0; c < kSpRing / kSpChunk; c++)
        if (c <= last_sc) issue_stream(c);
    issue_rec(0);
    if (last_rc >= 1) issue_rec(1);
    uint32_t sc_next = kSpRing / kSpChunk, rc_next = 2;
    vm_sync();

    PROF_DECL
#ifdef QLZX_PROFILE
    unsigned long long _mp[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#endif
    ItemCursor cur{lane / 31, lane % 31};
    uint32_t D = 0;           // output bytes of all items before the batch
    uint32_t base = 0;        // window start
    uint32_t hq = 0, tq = 0;  // match ring head / tail
    bool err = false, tail = false, complete = dsize == 0;
    // every match step retires at least its first entry, so nitems + 1 steps always suffice;
    // the budget only guarantees the wave terminates whatever the stream holds
    uint32_t budget = nitems + 1;
    // Far matches (source entirely below the window, <= 16 B) are the item phase's own: their
    // 24 source bytes are loaded from HBM when the item is decoded and written into the window
    // at the top of the next iteration, when the wait there has covered the loads.  The match
    // phase of an iteration takes only entries of earlier batches (after those writes), so
    // every far match is in place before a match that reads it is copied.
    bool farp = false;  // this lane holds a far match not yet written
    uint32_t fx0 = 0, fx1 = 0, fx2 = 0, fx3 = 0, fx4 = 0, fx5 = 0, fdn = 0;  // fdn: d | len << 16 | sh << 24
    auto far_write = [&]() {
        if (__ballot(farp)) {
            if (farp) {
                const uint32_t fd = fdn & 0xffffu, fn = (fdn >> 16) & 0xffu, fsh = fdn >> 24;
                Copy16 cp;
                cp.prep(fd - base, 0, fn);
                uint32_t y[5];
                y[0] = __builtin_amdgcn_alignbyte(fx1, fx0, fsh);
                y[1] = __builtin_amdgcn_alignbyte(fx2, fx1, fsh);
                y[2] = __builtin_amdgcn_alignbyte(fx3, fx2, fsh);
                y[3] = __builtin_amdgcn_alignbyte(fx4, fx3, fsh);
                y[4] = __builtin_amdgcn_alignbyte(fx5, fx4, fsh);
                cp.run_y(win, y);
            }
            farp = false;
        }
    };
    auto drain = [&]() {  // finish every pending match (far ones included)
        vm_sync();
        far_write();
        while (tq != hq && budget) {
            hq = sp_mp_step(L, hq, tq, base, dst, dsize, lane SP_PROF_PASS);
            budget--;
        }
        if (tq != hq) err = true;  // unreachable: every step retires its first entry
    };
    const uint32_t nb = (nitems + 63) / 64;
    for (uint32_t bt = 0; bt < nb && !complete && !err; bt++) {
        vm_sync();  // the previous iteration's DMAs and far loads have landed
        PROF_MARK(0);
        far_write();
        const uint32_t tq_prev = tq;  // the match phase of this iteration takes entries of earlier batches
        // ---- item phase: decode 64 items ----
        const uint32_t I = bt * 64 + lane;
        const bool valid = I < nitems;
        const GroupRec gr = L.rrng[cur.g & (kSpRecRing - 1)];
        const uint32_t low = (1u << cur.k) - 1u;
        const uint32_t pos = gr.ip + 4 + cur.k + __builtin_popcount(gr.a & low) + 2 * __builtin_popcount(gr.b & low);
        const bool ism = valid && ((gr.m >> cur.k) & 1u);
        const uint32_t q = pos + shift, qa = q & ~3u;
        const uint32_t w0 = *(const uint32_t *)(L.srng + (qa & (kSpRing - 1)));
        const uint32_t w1 = *(const uint32_t *)(L.srng + ((qa + 4) & (kSpRing - 1)));
        const uint32_t t = __builtin_amdgcn_alignbyte(w1, w0, q & 3u);
        uint32_t off, mlen, tl;
        decode_tok_bf(t, off, mlen, tl);
        const uint32_t len0 = valid ? (ism ? mlen : 1u) : 0u;
        tl = ism ? tl : 1u;
        PROF_MARK(1);
        // ---- place, check and emit the items of lanes [lo, cut): normally one pass over all ----
        uint32_t lo_lane = 0;
        bool more = true;
        for (uint32_t pass = 0; more && pass <= 64; pass++) {  // each pass takes >= 1 lane
            const bool act = lane >= lo_lane;
            const uint32_t len = act ? len0 : 0u;
            const uint32_t incl = wave_incl_scan(len);
            const uint32_t total = uni(__builtin_amdgcn_readlane(incl, 63));
            uint32_t cut = 64u;
            if (D + total > base + W) {  // rare: the batch's output overflows the window
                drain();
                if (err) break;
                const uint32_t nbase = uni(base + ((D - base) / (W / 2)) * (W / 2));  // flush whole halves below D
                if (nbase > base) {
                    sp_slide(L, dst, a16, base, nbase, D, lane);
                    base = nbase;
                }
                const uint64_t outm = __ballot(act && len && D + incl > base + W);
                cut = uni(outm ? (uint32_t)__builtin_ctzll(outm) : 64u);
            }
            const uint32_t d = D + incl - len;
            const bool in = act && lane < cut;
            more = cut < 64u;
            lo_lane = cut;
            const uint32_t stotal = cut < 64u ? uni(__builtin_amdgcn_readlane(incl - len, cut)) : total;
            // ---- checks C3-C5 on the live items (those that start before dsize) ----
            const bool live = in && valid && d < dsize;
            const uint64_t tail_lanes = __ballot(live && !ism && d >= tail_from);
            const uint32_t tail_lane = tail ? 0u : ff1_or(tail_lanes, 64u);  // C4: no match after it
            tail = tail || tail_lanes != 0;
            const bool mok = off >= 3 && off <= d && d + len + 4 <= dsize && lane < tail_lane;  // C3, C4
            const bool last = live && d + len == dsize;  // C5: the item completing dsize ends the stream
            const uint32_t ip_end = pos + tl;
            const bool eok = ip_end == csize || (ip_end < hdr + 9 && csize == hdr + 9);
            const bool bad = live && ((ism && !mok) || (last && !eok));
            err = __ballot(bad) != 0;
            complete = __ballot(last) != 0;
            if (err) break;
            // literals (other lanes store to an unused byte past the window)
            win[(live && !ism) ? d - base : W + 24] = (uint8_t)t;
            // far matches: load their source now, write it next iteration (far_write)
            const uint32_t s = d - off, lo = d & 3u, a0 = s - lo, a0a = a0 & ~3u;
#ifdef QLZX_SP_EXP_NOFAR  // experiment: far matches dropped (wrong bytes; timing only)
            const bool isfar = false;
            const bool dropfar = live && ism && s < base;
#else
            const bool isfar = live && ism && a4 && len <= 16u && s + len <= base && s >= lo && a0a + 24u <= dsize;
            const bool dropfar = false;
#endif
            if (isfar) {
                const uint4 v = *(const uint4 *)(dst + a0a);
                const uint2 v2 = *(const uint2 *)(dst + a0a + 16);
                fx0 = v.x, fx1 = v.y, fx2 = v.z, fx3 = v.w, fx4 = v2.x, fx5 = v2.y;
                fdn = d | (len << 16) | ((a0 & 3u) << 24);
                farp = true;
            }
            // the other matches: appended to the ring in item order
            const bool app = live && ism && !isfar && !dropfar;
            const uint64_t am = __ballot(app);
            const uint32_t slot = app ? ((tq + lane_rank(am)) & (kSpMq - 1)) : kSpMq;
            L.mqd[slot] = d | (off << 16);
            L.mql[slot] = (uint8_t)(len - 3u);
            tq = uni(tq + (uint32_t)__builtin_popcountll(am));
            D = uni(D + stotal);
            if (complete) more = false;
        }
        if (more) err = true;  // unreachable: every pass takes at least one lane
        if (err) break;
        PROF_MARK(2);
        // ---- match phase: the matches of earlier batches, 64 at a time (the far loads just
        // issued get this phase to land); a drain above may have taken hq past tq_prev ----
#ifdef QLZX_SP_EXP_NOMP  // experiment: no match phase (wrong bytes; timing only)
        hq = tq_prev;
#endif
        while (hq + 64u <= tq_prev && budget) {
            hq = sp_mp_step(L, hq, tq_prev, base, dst, dsize, lane SP_PROF_PASS);
            budget--;
        }
        PROF_MARK(3);
        // ---- prefetch for the next batch: it lands by the wait at the top of the next iteration ----
        {
            // stream: keep 512 B past the next batch's first item issued (a batch reads <= 268 B),
            // in ring slots whose chunk lies wholly below that item
            const uint32_t qn = uni(__builtin_amdgcn_readlane(pos + tl, 63)) + shift;
            while (sc_next <= last_sc && sc_next < (qn >> 8) + kSpRing / kSpChunk && sc_next * kSpChunk < qn + 512u) {
                issue_stream(sc_next);
                sc_next++;
            }
            // records: the next batch reads groups gn .. gn + 3; a chunk's slot is free once the
            // chunk two back is wholly below gn
            const uint32_t gn = ((bt + 1) * 64) / 31;
            if (rc_next <= last_rc && (gn + 3) / kSpRecChunk >= rc_next) {
                issue_rec(rc_next);
                rc_next++;
            }
        }
        cur.next();
        PROF_MARK(4);
    }
    if (!err && complete) drain();
    vm_sync();
    lds_sync();
    PROF_FLUSH(2);
#ifdef QLZX_PROFILE
    if (g_prof && lane == 0)
        for (int _j = 0; _j < 8; _j++) atomicAdd(&g_prof[3 * 8 + _j], _mp[_j]);
#endif
    if (err || !complete) {
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
    if (lane == 0) {
        status[i] = QLZX_OK;
        if (dsize_out) dsize_out[i] = dsize;
    }
}

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
    static const bool sort_env = [] {  // QLZX_BLOCK_ORDER=0: chunk order (experiments)
        const char *e = getenv("QLZX_BLOCK_ORDER");
        return !(e && e[0] == '0');
    }();
    const bool sort = sort_env && chunk > 64;
    // two workspace halves when the caller gave room for them: K1 of chunk c+1 runs on a
    // side stream while K2 of chunk c runs on `s` (K1 is latency-bound at low occupancy)
    static const bool overlap_env = [] {  // QLZX_K1_OVERLAP=0: serial K1/K2 (experiments)
        const char *e = getenv("QLZX_K1_OVERLAP");
        return !(e && e[0] == '0');
    }();
    const bool overlap = overlap_env && ws_bytes >= 2 * one && b.n > chunk;
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
    // QLZX_K2=split: the item-phase/match-phase kernel (k_dec_split, DESIGN.md §4 "Round 2:
    // the split K2"); default: the item-per-lane kernel k_dec_blocks, which measured faster
    // (read per call so tests can run both kernels in one process)
    const int k2mode = (int)k2_mode();
    const bool seq = k2mode == kK2Seq;
    const uint32_t mcap = seq_mcap(md);
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
        if (crc && seq)
            hipLaunchKernelGGL((k_dec_parse<true, true>), g1c, dim3(kParseWG<true>), 0, s1, b, dst_cap, dsize, status,
                               crc_state, crc_expect, crc_out, first, cnt, info, recs, gmax, order, max_dsize, mcap);
        else if (seq)
            hipLaunchKernelGGL((k_dec_parse<false, true>), g1, dim3(kParseWG<false>), 0, s1, b, dst_cap, dsize, status,
                               crc_state, crc_expect, crc_out, first, cnt, info, recs, gmax, order, max_dsize, mcap);
        else if (crc)
            hipLaunchKernelGGL((k_dec_parse<true>), g1c, dim3(kParseWG<true>), 0, s1, b, dst_cap, dsize, status,
                               crc_state, crc_expect, crc_out, first, cnt, info, recs, gmax, order, max_dsize, 0u);
        else
            hipLaunchKernelGGL((k_dec_parse<false>), g1, dim3(kParseWG<false>), 0, s1, b, dst_cap, dsize, status,
                               crc_state, crc_expect, crc_out, first, cnt, info, recs, gmax, order, max_dsize, 0u);
        if (overlap) (void)hipEventRecord(ev_k1[c & 1], side), (void)hipStreamWaitEvent(s, ev_k1[c & 1], 0);
#ifndef QLZX_EXP_K2_EXTRA_LDS
#define QLZX_EXP_K2_EXTRA_LDS 0  // experiments: extra dynamic LDS per WG to lower occupancy
#endif
        // one kernel for every block size: the LDS window slides over longer blocks
        if (seq)
            hipLaunchKernelGGL(k_dec_seq<kSeqWin>, dim3(cnt), dim3(64), 0, s, b, dsize, status, first, cnt, info,
                               (const uint32_t *)recs, mcap, (const uint32_t *)order);
        else if (k2mode == 0)
            hipLaunchKernelGGL(k_dec_blocks<kWin>, dim3(cnt), dim3(64), QLZX_EXP_K2_EXTRA_LDS, s, b, dsize, status,
                               first, cnt, info, recs, gmax, (const uint32_t *)order);
        else
            hipLaunchKernelGGL(k_dec_split<kSpWin>, dim3(cnt), dim3(64), 0, s, b, dsize, status, first, cnt, info,
                               recs, gmax, (const uint32_t *)order);
        if (overlap) (void)hipEventRecord(ev_k2[c & 1], s);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return (int)e;
    }
    if (seq)  // blocks K1<SEQ> left to the general kernel (a literal run over kSeqRunMax items)
        hipLaunchKernelGGL(k_dec_lane8, dim3((b.n + 255) / 256), dim3(256), 0, s, b, dst_cap, dsize, status,
                           crc_state, crc_expect, crc_out, kLane8Pending);
    return 0;
}

}  // namespace qlzx
