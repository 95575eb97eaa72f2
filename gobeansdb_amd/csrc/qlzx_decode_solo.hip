// qlzx_decode_solo.hip -- the latency path for ONE level-3 block (the single-call drop-ins
// qlz_decompress / qlzx_decompress1, called once per GET by store/item.go:167).
//
// The batch decoder parses with one LANE per block (K1) and decodes with one WAVE per block
// (K2b): right when 131072 blocks share the chip, but a lone 64 KiB block then walks ~2,100
// control-word groups on one lane and ~16,000 items on one wave.  Here one 1024-thread
// workgroup does the whole block, every phase position-parallel:
//
//   PARSE (the control-word chain, quicklz.c:513-530 and the token forms of 579-610)
//   1. code[x]  = token bytes - 1 if a match token started at stream byte x (2 bits each);
//   2. delta[x] = length of the control-word group that WOULD start at x (4 + 31 items), at
//                 every x at once: a speculative parse, each thread walking the match bits of
//                 the dword at x and adding code[] of each match token.  0 (no shortcut) for a
//                 dword without bit 31 (check C1) and for x within 128 B of the end, where a
//                 group may run past the stream;  j2[x] = delta[x] + delta[x + delta[x]];
//   3. one lane follows hdr -> hdr + j2[hdr] -> ... (two groups per LDS read) and lists the
//      group starts; a group without a shortcut is parsed byte by byte there as K1 parses it
//      (qlzx_decode_wave.hip k_dec_parse: checks C1, C2, the group bound, the item count);
//   4. the GroupRec {ip, m, a, b} of every listed group, in parallel.
//   DECODE (quicklz.c:531-671 restated output-parallel, as K2b does per chunk)
//   5. items: each thread decodes a contiguous run of items (token from its GroupRec), a
//      block-wide scan of the output lengths gives every item its start d; checks C3-C5;
//      the item leaves a u16 marker at d (match offset, or 1 for a literal, whose byte goes
//      straight to the destination);
//   6. fill: thread t owns output bytes [64 t, 64 t + 64): its markers are forward-filled
//      (block max-scan for the carry) into the SOURCE position of every byte (itself for a
//      literal byte, p - offset for a match byte);
//   7. pointer jumping s[p] <- s[s[p]] over the whole block until every byte points at a
//      literal (log2 of the longest copy chain rounds);
//   8. gather: out[p] = out[s[p]] (the literal bytes written in 5).
// Status and output equal K1 + K2b's on the same stream (tests/test_gpu_solo.py).
namespace qlzx {

constexpr uint32_t kSoloWG = 1024;
constexpr uint32_t kSoloMaxCsize = 65536;            // LDS: 2-bit codes + delta + j2 per stream byte
constexpr uint32_t kSoloOwn = 64;                    // output bytes per thread: kSoloWG * 64 = 64 KiB
constexpr uint32_t kSoloGmax = QLZX_FAST_MAX_DSIZE / 31 + 2;
constexpr uint32_t kSoloIT = 16;                     // items per thread per decode round
static_assert(kSoloWG * kSoloOwn >= QLZX_FAST_MAX_DSIZE, "one output run per thread");
constexpr uint32_t kSoloLit = 1;                     // marker of a literal (match offsets are >= 3)

struct SoloLds {
    union {
        struct {
            uint32_t code[kSoloMaxCsize / 16];
            uint8_t delta[kSoloMaxCsize];
            uint8_t j2[kSoloMaxCsize];              // delta of two groups - 69 (1..187), 0: none
            uint32_t glist[kSoloGmax];
        } p;
        uint16_t s[QLZX_FAST_MAX_DSIZE];            // markers, then source positions
    };
    uint32_t wsum[kSoloWG / 64];
    uint32_t ngroups, klast;
    int32_t st;
    uint32_t bad, tail_idx, max_match, done;
};

__device__ __forceinline__ uint32_t tok_code(uint32_t t) {  // token bytes - 1 from its first byte
    const uint32_t ty = (t & 3u) + ((t & 127u) == 3u ? 1u : 0u);
    return __builtin_amdgcn_ubfe(0x32110u, ty * 4, 4);
}
// An unaligned dword of the stream.  The address is pinned to VGPRs: where it is wave-uniform
// (the chain walk starts at hdr) the compiler would otherwise emit a scalar load, which drops
// the address's low two bits; vector loads take any byte address (unaligned access mode).
__device__ __forceinline__ uint32_t ld_dword(const uint8_t *p) {
    uint64_t a = (uint64_t)(uintptr_t)p;
    asm volatile("" : "+v"(a));
    return *(const uint32_t *)(uintptr_t)a;
}
__device__ __forceinline__ uint32_t code_at(const uint32_t *code, uint32_t x) {
    return __builtin_amdgcn_ubfe(code[x >> 4], 2 * (x & 15u), 2);
}
__device__ __forceinline__ uint32_t u16_get(const uint32_t *v, uint32_t j) { return (v[j >> 1] >> (16 * (j & 1))) & 0xffffu; }
__device__ __forceinline__ void u16_set(uint32_t *v, uint32_t j, uint32_t x) {
    v[j >> 1] = (j & 1) ? ((v[j >> 1] & 0xffffu) | (x << 16)) : ((v[j >> 1] & 0xffff0000u) | x);
}

// Exclusive prefix sum (or max) over the workgroup; `all` = the sum (max) of every thread.
// wsum: 16 words of LDS, free again after the caller's next barrier.
template <bool MAX>
__device__ __forceinline__ uint32_t block_excl(uint32_t v, uint32_t *wsum, uint32_t &all) {
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint32_t incl = MAX ? wave_incl_max(v) : wave_incl_scan(v);
    if (lane == 63) wsum[w] = incl;
    __syncthreads();
    uint32_t below = 0, tot = 0;
#pragma unroll
    for (uint32_t j = 0; j < kSoloWG / 64; j++) {
        const uint32_t x = wsum[j];
        if (MAX) {
            below = j < w ? max(below, x) : below;
            tot = max(tot, x);
        } else {
            below += j < w ? x : 0u;
            tot += x;
        }
    }
    all = tot;
    if (MAX) return max(below, wave_shr1(incl));
    return below + incl - v;
}

#ifdef QLZX_PROFILE  // phase stamps of thread 0 into profile slot 2 (tools/solo_prof.py)
#define SOLO_T0 unsigned long long _st = __builtin_amdgcn_s_memtime();
#define SOLO_STAMP(k)                                                        \
    do {                                                                     \
        if (tid == 0 && g_prof) {                                            \
            const unsigned long long _n = __builtin_amdgcn_s_memtime();       \
            atomicAdd(&g_prof[16 + (k)], (k) == 7 ? 1ull : _n - _st);       \
            _st = _n;                                                        \
        }                                                                    \
    } while (0)
#else
#define SOLO_T0
#define SOLO_STAMP(k) \
    do {              \
    } while (0)
#endif

// The whole block by one 1024-thread workgroup; *status / *dsize_out are written by thread 0
// (global or LDS words).  Every return is workgroup-uniform.
__device__ __forceinline__ void solo_decode(SoloLds &L, const uint8_t *src, uint32_t len, uint8_t *dst,
                                            uint32_t dst_cap, uint32_t max_dsize, GroupRec *recs, int32_t *status,
                                            uint32_t *dsize_out) {
    const uint32_t tid = threadIdx.x;
    SOLO_T0
    uint32_t kind, csize = 0, dsize = 0, hdr = 0;
    const int st0 = classify_block(src, len, dst_cap, max_dsize, kind, csize, dsize, hdr);
    if (st0 != QLZX_OK) {  // the host routes only blocks <= QLZX_FAST_MAX_DSIZE here: no kPending
        if (tid == 0) *status = st0, *dsize_out = 0;
        return;
    }
    if (kind == kBlkStored) {  // quicklz.c:808-811
        for (uint32_t p = tid; p < dsize; p += kSoloWG) dst[p] = src[hdr + p];
        if (tid == 0) *status = QLZX_OK, *dsize_out = dsize;
        return;
    }
    const bool al16 = ((uintptr_t)src & 15u) == 0;
    // ---- 1. token codes, 16 stream bytes per word ----
    for (uint32_t w = tid; w < (csize + 15) / 16; w += kSoloWG) {
        uint32_t v = 0;
        if (al16 && 16 * w + 16 <= csize) {
            const uint4 q = *(const uint4 *)(src + 16 * w);
            const uint32_t d4[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
            for (uint32_t j = 0; j < 16; j++) v |= tok_code(d4[j >> 2] >> (8 * (j & 3))) << (2 * j);
        } else {
            for (uint32_t j = 0; j < 16 && 16 * w + j < csize; j++) v |= tok_code(src[16 * w + j]) << (2 * j);
        }
        L.p.code[w] = v;
    }
    __syncthreads();
    SOLO_STAMP(0);
    // ---- 2. speculative group length at every stream byte (next candidate's dword in flight) ----
    {
        uint32_t x = hdr + tid;
        uint32_t cwn = x + 128 <= csize ? ld_dword(src + x) : 0u;
        for (; x < csize; x += kSoloWG) {
            const uint32_t cw = cwn;
            cwn = x + kSoloWG + 128 <= csize ? ld_dword(src + x + kSoloWG) : 0u;
            uint32_t d = 0;
            if (cw >> 31) {  // C1; cw = 0 within 128 B of the end (no shortcut there)
                uint32_t mrem = cw & 0x7fffffffu, extra = 0;
                const uint32_t base = x + 4;
                while (mrem) {
                    extra += code_at(L.p.code, base + __builtin_ctz(mrem) + extra);
                    mrem &= mrem - 1;
                }
                d = 35 + extra;
            }
            L.p.delta[x] = (uint8_t)d;
        }
    }
    __syncthreads();
    for (uint32_t x = hdr + tid; x < csize; x += kSoloWG) {
        const uint32_t d1 = L.p.delta[x];
        const uint32_t d2 = d1 && x + d1 < csize ? L.p.delta[x + d1] : 0u;
        L.p.j2[x] = (uint8_t)(d2 ? d1 + d2 - 69 : 0u);
    }
    __syncthreads();
    SOLO_STAMP(1);
    // ---- 3. the group chain (one lane); K1's byte-level parse where there is no shortcut ----
    if (tid == 0) {
        const uint32_t gmax = groups_max(max_dsize < QLZX_FAST_MAX_DSIZE ? max_dsize : QLZX_FAST_MAX_DSIZE);
        uint32_t x = hdr, g = 0, klast = 31;
        int st = QLZX_OK;
        for (;;) {
            if (x + 4 > csize) break;  // stream exhausted at a control word
            const uint32_t j = L.p.j2[x], d = L.p.delta[x];
            if (j && g + 2 <= gmax) {  // two whole groups
                L.p.glist[g] = x;
                L.p.glist[g + 1] = x + d;
                g += 2;
                x += j + 69;
                continue;
            }
            if (g >= gmax) { st = QLZX_E_CORRUPT; break; }
            L.p.glist[g++] = x;
            if (d) { x += d; continue; }
            const uint32_t cw = ld_dword(src + x);
            if (!(cw >> 31)) { st = QLZX_E_CORRUPT; break; }  // C1
            uint32_t p = x + 4, k = 0;
            for (; k < 31 && p < csize; k++) {
                const uint32_t c = ((cw >> k) & 1u) ? code_at(L.p.code, p) : 0u;
                if (p + c + 1 > csize) { st = QLZX_E_CORRUPT; break; }  // C2
                p += c + 1;
            }
            if (st != QLZX_OK) break;
            if (k < 31) { klast = k; break; }  // the stream ends inside this group
            x = p;
        }
        if (st == QLZX_OK && g == 0) st = QLZX_E_CORRUPT;  // no control word
        L.ngroups = g;
        L.klast = klast;
        L.st = st;
        L.bad = 0;
        L.tail_idx = 0xffffffffu;
        L.max_match = 0;
        L.done = 0;
    }
    __syncthreads();
    SOLO_STAMP(2);
    const uint32_t ng = L.ngroups, klast = L.klast;
    if (L.st != QLZX_OK) {
        if (tid == 0) *status = L.st, *dsize_out = 0;
        return;
    }
    // ---- 4. GroupRecs of the listed groups (the last one holds klast items) ----
    for (uint32_t g = tid; g < ng; g += kSoloWG) {
        const uint32_t x = L.p.glist[g];
        const uint32_t cw = ld_dword(src + x);
        const uint32_t nk = g + 1 == ng ? klast : 31u;
        uint32_t mrem = cw & ((1u << nk) - 1u), extra = 0, a = 0, bb = 0;
        const uint32_t m = mrem;
        while (mrem) {
            const uint32_t k = __builtin_ctz(mrem);
            const uint32_t c = code_at(L.p.code, x + 4 + k + extra);
            a |= (c & 1u) << k;
            bb |= (c >> 1) << k;
            extra += c;
            mrem &= mrem - 1;
        }
        recs[g] = GroupRec{x, m, a, bb};
    }
    __threadfence();  // the records are read back by other waves below
    __syncthreads();
    SOLO_STAMP(3);
    // ---- 5. items: thread tid decodes items [I0, I1), kSoloIT per round ----
    const uint32_t nitems = (ng - 1) * 31 + klast;
    const uint32_t per = (nitems + kSoloWG - 1) / kSoloWG;
    const uint32_t I0 = min(tid * per, nitems), I1 = min(I0 + per, nitems);
    const uint32_t tail_from = dsize > QLZX_TAIL ? dsize - 1 - QLZX_TAIL : 0;  // op >= this: tail (quicklz.c:503)
    struct Item {
        uint32_t off, len, tl, pos, lit;
        bool ism;
    };
    auto decode_round = [&](uint32_t I, Item (&it)[kSoloIT]) {
        const uint32_t g0 = I / 31;  // a round of <= 16 items spans at most two groups
        const GroupRec r0 = recs[g0], r1 = recs[g0 + 1 < ng ? g0 + 1 : g0];
        uint32_t tok[kSoloIT];
#pragma unroll
        for (uint32_t j = 0; j < kSoloIT; j++) {
            const uint32_t Ij = I + j, k0 = I - 31 * g0 + j;
            const bool second = k0 >= 31;
            const uint32_t k = second ? k0 - 31 : k0;
            const uint32_t ip = second ? r1.ip : r0.ip, m = second ? r1.m : r0.m;
            const uint32_t a = second ? r1.a : r0.a, b = second ? r1.b : r0.b;
            const uint32_t low = (1u << k) - 1u;
            const uint32_t pos = ip + 4 + k + __builtin_popcount(a & low) + 2 * __builtin_popcount(b & low);
            it[j].pos = pos;
            it[j].ism = Ij < I1 && ((m >> k) & 1u) != 0;
            tok[j] = ld_dword(src + (Ij < I1 && pos + 4 <= csize ? pos : csize - 4));
        }
#pragma unroll
        for (uint32_t j = 0; j < kSoloIT; j++) {
            const uint32_t pos = it[j].pos;
            const uint32_t t = pos + 4 <= csize ? tok[j] : tok[j] >> (8 * (pos + 4 - csize));
            uint32_t off, mlen, tl;
            decode_tok_bf(t, off, mlen, tl);
            it[j].off = off;
            it[j].len = it[j].ism ? mlen : (I + j < I1 ? 1u : 0u);
            it[j].tl = it[j].ism ? tl : 1u;
            it[j].lit = t & 0xffu;
        }
    };
    uint32_t mysum = 0;
    for (uint32_t I = I0; I < I1; I += kSoloIT) {
        Item it[kSoloIT];
        decode_round(I, it);
#pragma unroll
        for (uint32_t j = 0; j < kSoloIT; j++) mysum += it[j].len;
    }
    // markers: clear the output range (the parse tables are dead: glist was read in 4)
    for (uint32_t q = tid; q < (dsize + 7) / 8; q += kSoloWG) *(uint4 *)(L.s + 8 * q) = make_uint4(0, 0, 0, 0);
    uint32_t total;
    uint32_t d = block_excl<false>(mysum, L.wsum, total);
    __syncthreads();  // markers cleared, wsum read
    {
        bool bad = false, complete = false;
        uint32_t tail_idx = 0xffffffffu, max_match = 0;
        for (uint32_t I = I0; I < I1; I += kSoloIT) {
            Item it[kSoloIT];
            decode_round(I, it);
#pragma unroll
            for (uint32_t j = 0; j < kSoloIT; j++) {
                const Item &e = it[j];
                if (I + j < I1 && d < dsize) {  // live
                    // C3 (3 <= off <= d) and a match ending >= 4 bytes before dsize (C4)
                    if (e.ism && (e.off < 3 || e.off > d || d + e.len + 4 > dsize)) bad = true;
                    if (!e.ism && d >= tail_from) tail_idx = min(tail_idx, I + j);  // C4: the tail
                    if (e.ism) max_match = I + j;
                    if (d + e.len == dsize) {  // C5: the item completing dsize ends the stream
                        complete = true;
                        const uint32_t ip_end = e.pos + e.tl;
                        if (!(ip_end == csize || (ip_end < hdr + 9 && csize == hdr + 9))) bad = true;
                    }
                    L.s[d] = (uint16_t)(e.ism ? e.off : kSoloLit);
                    if (!e.ism) dst[d] = (uint8_t)e.lit;
                }
                d += e.len;
            }
        }
        if (bad) L.bad = 1;
        if (complete) L.done = 1;
        if (tail_idx != 0xffffffffu) atomicMin(&L.tail_idx, tail_idx);
        if (max_match) atomicMax(&L.max_match, max_match);
    }
    __threadfence();  // literal bytes, read back by other threads in 8
    __syncthreads();
    SOLO_STAMP(4);
    {
        // a failed check; no item completing dsize (C5); a match after the first tail literal (C4)
        const bool corrupt = dsize > 0 && (L.bad || !L.done || (L.tail_idx != 0xffffffffu && L.max_match > L.tail_idx));
        if (corrupt || dsize == 0) {
#ifdef QLZX_SOLO_DEBUG
            if (tid == 0 && corrupt)
                *status = 100 + (L.bad ? 1 : 0) + (L.done ? 2 : 0) + (L.tail_idx != 0xffffffffu ? 4 : 0) +
                          (L.max_match > L.tail_idx ? 8 : 0), *dsize_out = 0;
            else
#endif
            if (tid == 0) *status = corrupt ? QLZX_E_CORRUPT : QLZX_OK, *dsize_out = 0;
            return;
        }
    }
    // ---- 6. fill: markers -> source position of every byte of [p0, p0 + 64) ----
    const uint32_t p0 = tid * kSoloOwn;
    uint32_t sv[kSoloOwn / 2];  // two u16 per register
    uint32_t lastp = 0;         // 1 + position of the run's last marker, 0: none
    if (p0 < dsize) {
#pragma unroll
        for (uint32_t q = 0; q < kSoloOwn / 8; q++) {
            const uint4 v = *(const uint4 *)(L.s + p0 + 8 * q);
            sv[4 * q] = v.x, sv[4 * q + 1] = v.y, sv[4 * q + 2] = v.z, sv[4 * q + 3] = v.w;
        }
#pragma unroll
        for (uint32_t j = 0; j < kSoloOwn; j++) lastp = u16_get(sv, j) ? p0 + j + 1 : lastp;
    }
    uint32_t unused;
    const uint32_t prevp = block_excl<true>(lastp, L.wsum, unused);
    uint32_t f = prevp ? L.s[prevp - 1] : kSoloLit;  // position 0 always has a marker
    __syncthreads();  // every carry read before the runs are rewritten
    if (p0 < dsize) {
#pragma unroll
        for (uint32_t j = 0; j < kSoloOwn; j++) {
            const uint32_t p = p0 + j, m = u16_get(sv, j);
            f = m ? m : f;
            u16_set(sv, j, (f == kSoloLit || p >= dsize) ? p : p - f);
        }
#pragma unroll
        for (uint32_t q = 0; q < kSoloOwn / 8; q++)
            *(uint4 *)(L.s + p0 + 8 * q) = make_uint4(sv[4 * q], sv[4 * q + 1], sv[4 * q + 2], sv[4 * q + 3]);
    }
    __syncthreads();
    SOLO_STAMP(5);
    // ---- 7. pointer jumping until every byte's source is a literal (s[s] == s) ----
    // Entries are rewritten while others read them; any value read is an earlier link of the
    // same chain, so a stale read only costs a round.
    for (;;) {
        bool ch = false;
        if (p0 < dsize) {
#pragma unroll
            for (uint32_t h = 0; h < kSoloOwn; h += 32) {  // 32 reads in flight (a literal reads itself)
                uint32_t t[32];
#pragma unroll
                for (uint32_t j = 0; j < 32; j++) t[j] = L.s[u16_get(sv, h + j)];
#pragma unroll
                for (uint32_t j = 0; j < 32; j++) {
                    const bool jump = t[j] != u16_get(sv, h + j);
                    if (jump) u16_set(sv, h + j, t[j]);
                    ch = ch || jump;
                }
            }
            if (ch) {
#pragma unroll
                for (uint32_t q = 0; q < kSoloOwn / 8; q++)
                    *(uint4 *)(L.s + p0 + 8 * q) = make_uint4(sv[4 * q], sv[4 * q + 1], sv[4 * q + 2], sv[4 * q + 3]);
            }
        }
        if (!__syncthreads_or(ch)) break;
    }
    SOLO_STAMP(6);
    // ---- 8. gather the run's bytes from the literals and store them ----
    if (p0 < dsize) {
        const uint32_t n = min(kSoloOwn, dsize - p0);
        uint32_t out[kSoloOwn / 4];
#pragma unroll
        for (uint32_t q = 0; q < kSoloOwn / 4; q++) out[q] = 0;
#pragma unroll
        for (uint32_t j = 0; j < kSoloOwn; j++) out[j >> 2] |= (uint32_t)dst[j < n ? u16_get(sv, j) : 0u] << (8 * (j & 3));
        if (n == kSoloOwn && (((uintptr_t)dst) & 15u) == 0) {
#pragma unroll
            for (uint32_t q = 0; q < kSoloOwn / 16; q++)
                *(uint4 *)(dst + p0 + 16 * q) = make_uint4(out[4 * q], out[4 * q + 1], out[4 * q + 2], out[4 * q + 3]);
        } else {
            for (uint32_t j = 0; j < n; j++) dst[p0 + j] = (uint8_t)(out[j >> 2] >> (8 * (j & 3)));
        }
    }
    if (tid == 0) *status = QLZX_OK, *dsize_out = dsize;
    SOLO_STAMP(7);
}

}  // namespace qlzx
