// qlzx_decode_seq.hip -- K2 with one SEQUENCE per lane (QLZX_K2=seq).
//
// k_dec_blocks decodes 64 items per batch, one per lane; two thirds of the items of a text
// block are single literal bytes, so most lanes carry one output byte per batch.  Here a lane
// owns a sequence: the literal run before a match plus the match (quicklz.c:513-671 emits
// exactly this shape), so a batch covers ~2.9 items and ~7 output bytes per lane on c2.
//
// K1 (k_dec_parse<CRC, true>) writes one u32 per match, I | X << 16 (item index; token bytes
// beyond the first of all earlier matches).  For sequence j (match j, or the terminal
// literal run when j = nmatch):
//   literal run  items I_{j-1}+1 .. I_j-1, L = I_j - I_{j-1} - 1 <= kSeqRunMax,
//                item x at stream hdr + 4 (x / 31 + 1) + x + X_j (the run's items share X_j)
//   match        token at hdr + 4 (I_j / 31 + 1) + I_j + X_j
//   output       the run at D_j = I_{j-1} + 1 - j + sum_{i<j} mlen_i, the match right after it
// I_{j-1} comes from the lane below (DPP wave_shr:1, the previous batch's last I in lane 0).
//
// Per batch: token decode (DMA'd kTokAhead batches ahead, as in K2), one DPP scan of the
// sequence lengths, checks C3-C5 (C1/C2 are K1's), literal runs from the compressed stream
// (20-B register loads issued with the far-match loads, 16-B chunks that stop at control
// words), then the matches in sub-rounds with K2's exact readiness (item-start bitmap,
// owner lanes; a match never waits for its own literal run, which is written first).
// Window, far matches, sub-batches and the write-out are K2's.
#include "qlzx_device.h"

namespace qlzx {

#ifndef QLZX_SQ_WAVES_PER_EU
#define QLZX_SQ_WAVES_PER_EU 1
#endif

template <uint32_t W>
struct SeqLds {
    uint8_t pad[16];
    uint8_t win[W + 32];
    uint32_t rec[kRecSlots][64];   // match records of batches bt+kTokAhead .. bt+kRecAhead
    uint32_t tok[kTokSlots][64];   // token dwords of batches bt .. bt+kTokAhead-1 (then the bitmap)
};

__device__ __forceinline__ uint32_t seq_tokpos(uint32_t hdr, uint32_t I, uint32_t X) {
    return hdr + 4u * (I / 31u + 1u) + I + X;
}

// lane l gets v of lane l-1; lane 0 gets `carry`
__device__ __forceinline__ uint32_t wave_shr1(uint32_t v, uint32_t carry) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)carry, (int)v, 0x138, 0xf, 0xf, false);
}

// Five source-aligned dwords y[j] = stream bytes [a0 + 4j, a0 + 4j + 4) of a literal chunk,
// never reading at or past lim (csize): a dword that would is loaded at lim - 4, and
// stream_fix20 (called where y is used, so the loads stay in flight until then) shifts it
// down, so its bytes below lim stay exact (the chunk's bytes all are) and the rest read 0.
// Every load is unconditional: a select that skips an unneeded load becomes a branch per
// dword, each waiting for the load before it.
__device__ __forceinline__ void stream_load20(const uint8_t *src, uint32_t a0, uint32_t lim, uint32_t y[5]) {
#pragma unroll
    for (int j = 0; j < 5; j++) {
        const uint32_t a = a0 + 4 * j;
        y[j] = *(const uint32_t *)(src + (a + 4 > lim ? lim - 4 : a));
    }
}
__device__ __forceinline__ void stream_fix20(uint32_t a0, uint32_t lim, uint32_t y[5]) {
#pragma unroll
    for (int j = 0; j < 5; j++) {
        const uint32_t a = a0 + 4 * j;
        const uint32_t over = a + 4 > lim ? a + 4 - lim : 0u;  // bytes past lim
        y[j] = (y[j] >> (8 * (over < 3u ? over : 3u))) & (over >= 4u ? 0u : 0xFFFFFFFFu);
    }
}

// One batch's records into its slot (1 dword DMA per lane; dummy address past nmatch).
__device__ __forceinline__ void issue_mrec(uint32_t *slot, const uint32_t *mrec, uint32_t b0, uint32_t nmatch,
                                           uint32_t lane) {
    const uint32_t j = b0 + lane;
    dma4(j < nmatch ? (const void *)(mrec + j) : (const void *)mrec, lds_addr(slot));
}

// Record word -> (I, X) of sequence jj; the terminal sequence (jj == nmatch) has I = nitems.
struct SeqRec {
    uint32_t I, X;
    bool ism;
};
__device__ __forceinline__ SeqRec seq_rec(uint32_t rw, uint32_t jj, uint32_t nmatch, uint32_t nitems,
                                          uint32_t xtot) {
    SeqRec r;
    r.ism = jj < nmatch;
    r.I = r.ism ? (rw & 0xFFFFu) : nitems;
    r.X = r.ism ? (rw >> 16) : xtot;
    return r;
}

constexpr uint32_t kSeqWin = 4096;  // k_dec_seq's own window (independent of QLZX_K2_WIN)

template <uint32_t W>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(QLZX_SQ_WAVES_PER_EU)))
k_dec_seq(qlzx_blocks b, uint32_t *dsize_out, int32_t *status, uint32_t first, uint32_t count,
          const BlkInfo *info, const uint32_t *mrec_all, uint32_t mcap, const uint32_t *list) {
    static_assert(W % 2048 == 0 && W >= 2048, "window: a multiple of 2 KiB (slides by W/2)");
    static_assert(kSeqRunMax + 258 <= W / 2 && kSeqRunMax + 258 <= kSubMax, "a sequence fits half the window");
    __shared__ __attribute__((aligned(16))) SeqLds<W> L;
    const uint32_t lane = threadIdx.x;
    const uint32_t bx = blockIdx.x;
    if (bx >= count) return;
    const uint32_t i = list ? list[bx] : first + bx;
    const BlkInfo bi = info[bx];
    const uint32_t kind = bi.kind & 0xFFu;
    if (kind == kBlkSkip) return;
    const uint8_t *src = b.src + b.src_off[i];
    uint8_t *dst = b.dst + b.dst_off[i];
    const uint32_t dsize = bi.dsize;
    if (kind == kBlkStored) {  // quicklz.c:808-811
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
    const uint32_t *mrec = mrec_all + (size_t)bx * mcap;
    const uint32_t nmatch = bi.ngroups, nitems = bi.nitems, xtot = bi.kind >> 8;
    const uint32_t csize = b.src_len[i];
    const uint32_t hdr = (src[0] & 2u) ? 9u : 3u;
    const uint32_t nb = (nmatch + 1 + 63) / 64;  // sequences: nmatch matches + the terminal run
    const uint32_t tail_from = dsize > QLZX_TAIL ? dsize - 1 - QLZX_TAIL : 0;
    const bool a16 = (((uintptr_t)dst) & 15u) == 0;

    // prologue: records of batches 0..kTokAhead-1, their tokens, then the records of
    // batches kTokAhead..kRecAhead-1
    for (uint32_t j = 0; j < kTokAhead; j++) issue_mrec(L.rec[j], mrec, j * 64, nmatch, lane);
    vm_sync();
    uint32_t pm[kTokAhead];  // record word of each in-flight batch (tokens DMA'd)
#pragma unroll
    for (uint32_t j = 0; j < kTokAhead; j++) {
        const uint32_t rw = L.rec[j][lane];
        const SeqRec r = seq_rec(rw, j * 64 + lane, nmatch, nitems, xtot);
        const uint32_t p = seq_tokpos(hdr, r.I, r.X);
        dma4(src + (r.ism ? (p + 4 <= csize ? p : csize - 4) : 0u), lds_addr(L.tok[j]));
        pm[j] = rw;
    }
    for (uint32_t j = kTokAhead; j < kRecAhead; j++) issue_mrec(L.rec[j % kRecSlots], mrec, j * 64, nmatch, lane);
    vm_sync();
    PROF_DECL
    uint32_t D = 0, base = 0;
    uint32_t Iprev_carry = 0xFFFFFFFFu;  // I of the sequence before this batch (-1 at the start)
    bool err = false, tail = false, complete = dsize == 0;
    uint32_t ts = 0, rs4 = kTokAhead % kRecSlots, rs8 = kRecAhead % kRecSlots;
    for (uint32_t bt = 0; bt < nb && !complete; bt++) {
        const uint32_t tw = L.tok[ts][lane];
        // the records of batch bt+kTokAhead: their token DMA goes out at the end of the iteration
        const uint32_t rw4 = L.rec[rs4][lane];
        lds_sync();
        const uint32_t rw = pm[0];
#pragma unroll
        for (uint32_t j = 0; j + 1 < kTokAhead; j++) pm[j] = pm[j + 1];
        pm[kTokAhead - 1] = rw4;
        uint32_t *const bm = L.tok[ts];
        uint32_t *const rslot8 = L.rec[rs8];
        ts = ts == kTokSlots - 1 ? 0 : ts + 1;
        rs4 = rs4 == kRecSlots - 1 ? 0 : rs4 + 1;
        rs8 = rs8 == kRecSlots - 1 ? 0 : rs8 + 1;
        PROF_MARK(1);
        const uint32_t jj = bt * 64 + lane;
        const bool valid = jj <= nmatch;
        const SeqRec r = seq_rec(rw, jj, nmatch, nitems, xtot);
        const uint32_t Iprev = wave_shr1(r.I, Iprev_carry);
        Iprev_carry = __builtin_amdgcn_readfirstlane(__builtin_amdgcn_readlane(r.I, 63));
        const uint32_t nlit = valid ? r.I - Iprev - 1u : 0u;  // K1: <= kSeqRunMax
        const bool ism = valid && r.ism;
        const uint32_t pos = seq_tokpos(hdr, r.I, r.X);
        const uint32_t t = pos + 4 <= csize ? tw : tw >> (8 * (pos + 4 - csize));
        uint32_t off, mlen, tl;
        decode_tok_bf(t, off, mlen, tl);
        mlen = ism ? mlen : 0u;
        const uint32_t len0 = nlit + mlen;
        // ---- sub-batches: normally one; more when the batch's output overflows the window ----
        uint32_t lo_lane = 0;
        bool more = true;
        while (more) {
#ifdef QLZX_PROFILE
            _pacc[7] += 1;  // sub-batches
#endif
            const uint32_t sub0 = lo_lane;
            const bool act = lane >= lo_lane;
            const uint32_t len = act ? len0 : 0u;
            const uint32_t incl = wave_incl_scan(len);
            const uint32_t total = __builtin_amdgcn_readfirstlane(__builtin_amdgcn_readlane(incl, 63));
            if (D + total > base + W && D - base >= W / 2) {  // slide: flush win[0, W/2)
                for (uint32_t q = lane * 16; q < W / 2; q += 1024) {
                    const uint4 v = *(const uint4 *)(win + q);
                    if (a16) *(uint4 *)(dst + base + q) = v;
                    else for (uint32_t k = 0; k < 16; k++) dst[base + q + k] = win[q + k];
                }
                for (uint32_t q = lane * 16; q < D - base - W / 2; q += 1024)
                    *(uint4 *)(win + q) = *(const uint4 *)(win + W / 2 + q);
                base = __builtin_amdgcn_readfirstlane(base + W / 2);
            }
            const uint32_t dl = D + incl - len;  // the literal run's output position
            const uint32_t d = dl + nlit;         // the match's
            const bool fits = dl + len <= base + W && dl + len <= D + kSubMax;
            const uint64_t outm = __ballot(act && len && !fits);
            const uint32_t cut = outm ? (uint32_t)__builtin_ctzll(outm) : 64u;
            const bool in = act && lane < cut;
            more = cut < 64;
            lo_lane = __builtin_amdgcn_readfirstlane(cut);
            const uint32_t stotal = cut < 64 ? __builtin_amdgcn_readlane(incl - len, cut) : total;
            // ---- loads: far match sources (below the window) and the first literal chunk ----
            const uint32_t s = d - off;
            const bool far = s < base;
            const bool spec = off < mlen || mlen > 16 || (far && (s + mlen > base || s < 3));
            const bool live = in && valid && dl < dsize;       // the sequence starts before dsize
            const bool mlive = live && ism && d < dsize;        // its match does
            const bool fload = mlive && far && !spec;
            uint32_t fy[5];
            // first literal chunk: items Iprev+1 .. up to 16 bytes, not past the group's end
            const uint32_t x0 = Iprev + 1u;
            const uint32_t lp0 = seq_tokpos(hdr, x0, r.X);
            const uint32_t c0 = min(min(nlit, 16u), 31u - x0 % 31u);
            const bool lload = live && nlit > 0;
            uint32_t ly[5];
#ifdef QLZX_SQ_EXP_NOLIT  // experiment: no literal loads (wrong bytes; timing only)
            ly[0] = ly[1] = ly[2] = ly[3] = ly[4] = lp0;
#else
            if (__ballot(lload)) {
                if (lload) stream_load20(src, lp0 - (dl & 3u), csize, ly);
            }
#endif
            // far loads after the literal loads: the literal phase, which runs first, then waits
            // only for its own loads (vmcnt is in order)
#ifdef QLZX_SQ_EXP_NOFAR  // experiment: no far loads (wrong bytes; timing only)
            fy[0] = fy[1] = fy[2] = fy[3] = fy[4] = s;
#else
            if (__ballot(fload)) {
                if (fload) far_load20(dst, s - (d & 3u), dsize, fy);
            }
#endif
            // ---- checks C3-C5 ----
            // C4: a literal at op >= dsize - 11 starts the tail; no match may follow it
            const uint64_t tail_lanes = __ballot(live && nlit > 0 && d - 1u >= tail_from);
            const uint32_t tail_lane = tail ? 0u : ff1_or(tail_lanes, 64u);
            tail = tail || tail_lanes != 0;
            const bool mok = off >= 3 && off <= d && d + mlen + 4 <= dsize && lane < tail_lane;  // C3, C4
            // C5: the item completing dsize ends the stream: a literal of the run, or the match
            const bool lit_last = live && nlit > 0 && dl < dsize && d >= dsize;
            const bool m_last = mlive && d + mlen == dsize;
            const uint32_t xl = x0 + (dsize - 1u - dl);  // the completing literal's item
            const uint32_t ip_end = m_last ? pos + tl : seq_tokpos(hdr, xl, r.X) + 1u;
            const bool last = lit_last || m_last;
            const bool eok = ip_end == csize || (ip_end < hdr + 9 && csize == hdr + 9);
            const bool bad = (mlive && !mok) || (last && !eok);
            err = err || bad;
            complete = __ballot(last) != 0;
            if (complete) more = false;
            PROF_MARK(2);
            // ---- literal runs ----
            {
                uint32_t rem = lload ? nlit : 0u;
                if (__ballot(rem)) {
                    if (rem) {
                        stream_fix20(lp0 - (dl & 3u), csize, ly);
                        Copy16 cl;
                        cl.prep(dl - base, 0u, c0);
                        cl.run_y(win, ly);
                    }
                    uint32_t x = x0 + c0, o = dl + c0;
                    rem = rem > c0 ? rem - c0 : 0u;
                    while (__ballot(rem)) {  // long runs and runs across a control word (rare)
                        if (rem) {
                            const uint32_t c = min(min(rem, 16u), 31u - x % 31u);
                            uint32_t y[5];
                            const uint32_t a0 = seq_tokpos(hdr, x, r.X) - (o & 3u);
                            stream_load20(src, a0, csize, y);
                            stream_fix20(a0, csize, y);
                            Copy16 cl;
                            cl.prep(o - base, 0u, c);
                            cl.run_y(win, y);
                            x += c;
                            o += c;
                            rem -= c;
                        }
                    }
                }
            }
            // ---- matches: which in-sub-batch lanes each match's source needs ----
            const uint32_t rs = dl - D;
            bm[lane] = 0;
            if (in && len) __hip_atomic_fetch_or(&bm[rs >> 5], 1u << (rs & 31), __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_WORKGROUP);
            asm volatile("" ::: "memory");
            const uint32_t bw = bm[lane];
            const uint32_t bpc = __builtin_popcount(bw);
            const uint32_t bex = wave_incl_scan(bpc) - bpc;
            const uint32_t send = (s + mlen < d) ? s + mlen : d;
            const bool dep = in && ism && send > D;
            const uint32_t qa = (dep && s > D) ? s - D : 0u, qb = dep ? send - 1 - D : 0u;
            const uint32_t la = sub0 + owner_of(bm, bex, qa), lb = sub0 + owner_of(bm, bex, qb);
            // its own literal run is already written: never wait for the own lane
            const uint64_t need = dep ? ((~0ull << la) & (~0ull >> (63 - lb)) & ~(1ull << lane)) : 0ull;
            bool done = !(mlive && !bad);
            const uint32_t n16 = mlen < 16 ? mlen : 16;
            Copy16 cp;
            cp.prep(d - base, off, n16);
            {
                const bool fc = !done && far && !spec;
                if (__ballot(fc)) {
                    if (fc) cp.run_y(win, fy);
                }
                done = done || fc;
            }
            uint64_t pend = __ballot(!done);
            const bool spec_any = __ballot(!done && spec) != 0;
            while (pend) {
#ifdef QLZX_PROFILE
                _pacc[6] += 1;  // sub-rounds
#endif
                const bool ready = !done & ((need & pend) == 0);
                if (ready && !spec) cp.run(win);
                if (spec_any && __ballot(ready && spec)) {
                    if (ready && spec) {
                        if (far || (off < 16 && off < mlen)) {
                            for (uint32_t j = 0; j < mlen; j++) {
                                const uint32_t sp = s + j;
                                const uint8_t v = sp < base ? dst[sp] : win[sp - base];
                                win[d + j - base] = v;
                            }
                        } else {
                            for (uint32_t c = 0; c < mlen; c += 16) {
                                Copy16 c2;
                                c2.prep(d + c - base, off, mlen - c < 16 ? mlen - c : 16);
                                c2.run(win);
                            }
                        }
                    }
                }
                done = done || ready;
                pend = __ballot(!done);
            }
            // the register loads of this sub-batch are consumed on every path (a path that
            // skipped them would leave them pending into the next sub-batch, whose first
            // writes to these registers would then wait for them behind newer loads)
            asm volatile("" ::"v"(ly[0]), "v"(ly[1]), "v"(ly[2]), "v"(ly[3]), "v"(ly[4]), "v"(fy[0]), "v"(fy[1]),
                         "v"(fy[2]), "v"(fy[3]), "v"(fy[4]));
            PROF_MARK(3);
            D = __builtin_amdgcn_readfirstlane(D + stotal);
            if (__ballot(err)) { more = false; complete = false; }
        }
        if (__ballot(err)) break;
        // prefetch: records of batch bt+kRecAhead, tokens of batch bt+kTokAhead (into the slot
        // this batch used for its bitmap); issued after this iteration's register loads were used
        issue_mrec(rslot8, mrec, (bt + kRecAhead) * 64, nmatch, lane);
        {
            const uint32_t j4 = (bt + kTokAhead) * 64 + lane;
            const SeqRec r4 = seq_rec(pm[kTokAhead - 1], j4, nmatch, nitems, xtot);
            const uint32_t p4 = seq_tokpos(hdr, r4.I, r4.X);
            dma4(src + ((r4.ism && j4 <= nmatch) ? (p4 + 4 <= csize ? p4 : csize - 4) : 0u), lds_addr(bm));
        }
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(QLZX_K2_VMWAIT) : "memory");
        PROF_MARK(4);
    }
    vm_sync();
    lds_sync();
    PROF_FLUSH(1);
    if (__ballot(err) || !complete) {
        if (lane == 0) { status[i] = QLZX_E_CORRUPT; if (dsize_out) dsize_out[i] = 0; }
        return;
    }
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

}  // namespace qlzx
