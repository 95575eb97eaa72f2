// qlzx_decode_small.hip -- the single-call latency path for small blocks (stream <= 17 KiB,
// output <= 32 KiB: the 4-16 KiB values of a GET, store/item.go:167), all in LDS.
//
// The general latency path (qlzx_decode_solo.hip) keeps its parse tables for a 64 KiB stream in
// LDS and reads the stream, its GroupRecs and the literal bytes from HBM; most of its 16 KiB call
// is load latency and one lane's 85-step chain walk.  Here the whole stream, the parse tables,
// the records, the markers and the literal bytes live in LDS, and the walk is log-depth:
//
//   0. the stream is staged into LDS (zero past csize) straight from the request's slot;
//   1. info[x] for every stream byte x: the outcome of parsing a control-word group at x --
//      FULL (its 31 items fit: info = group length 35..128), END k (the stream ends before
//      item k: the last group), BAD (no bit 31, check C1; a token past the end, check C2).
//      Every x whose dword has bit 31 parses its group at once (candidates listed first, for balance);
//   2. jump tables by pointer doubling: J2, J4, J8, J16 (u16 next-group position, 0: none);
//   3. one lane hops J16 to list every 16th group start, then steps the last groups by info;
//      threads expand each hop's 15 inner group starts in parallel;
//   4. GroupRecs {ip, m, a, b}, then items, markers, fill, pointer jumping and gather exactly as
//      qlzx_decode_solo.hip steps 4-8 (the checks C3-C5 included), with the literal bytes and
//      sources in LDS and the result written once to the destination (the caller's slot).
// Statuses and bytes equal the batch decoder's (K1 + K2, qlzx_decode_v4.hip) on the same stream,
// dsize-0 rule included (tests/test_gpu_solo.py).
namespace qlzx {

constexpr uint32_t kSmC = 17408;                 // stream bytes (csize bound of this path)
constexpr uint32_t kSmD = 32768;                 // output bytes (dsize bound)
constexpr uint32_t kSmG = kSmD / 31 + 2;         // groups_max(kSmD)
constexpr uint32_t kSmOwn = 16;                  // output bytes per thread per segment
constexpr uint32_t kSmSeg = kSmD / (kSoloWG * kSmOwn);  // 2 segments of 16 KiB
constexpr uint32_t kSmIT = 8;                    // items per thread per decode round
constexpr uint32_t kSmEnd = 0xA0, kSmBad = 0xFF;  // info codes besides FULL (35..128)
#ifndef QLZX_SM_PAIR  // step 1b takes a second match token per step when its code is in the same dword
#define QLZX_SM_PAIR 1
#endif
static_assert(kSmC % 16 == 0 && kSmC + 64 < 65536, "u16 positions");

struct SmallLds {
    uint32_t src[(kSmC + 64) / 4];  // the stream, zero from csize on
    uint8_t cb[kSmC + 64];          // token bytes - 1 of a match token at each byte; 4: it runs past csize (C2)
    uint16_t glist[kSmG + 16];
    union {
        struct {
            uint8_t info[kSmC + 64];
            uint16_t ja[kSmC + 64], jb[kSmC + 64];
        } p;
        struct {
            GroupRec recs[kSmG];
            uint16_t s[kSmD];       // markers, then source positions
            uint8_t out[kSmD];      // literal bytes at their output positions
        } d;
    };
    uint32_t wsum[2][kSoloWG / 64];
    uint32_t ngroups, klast, nhops, cursor;
    int32_t st;
    uint32_t bad, tail_idx, max_match, done;
};

#ifdef QLZX_PROFILE  // phase stamps of thread 0 into profile slots 24..31 (tools/solo_prof.py)
#define SM_STAMP(k)                                                          \
    do {                                                                     \
        if (tid == 0 && g_prof) {                                            \
            const unsigned long long _n = __builtin_amdgcn_s_memtime();       \
            atomicAdd(&g_prof[24 + (k)], (k) == 7 ? 1ull : _n - _st);       \
            _st = _n;                                                        \
        }                                                                    \
    } while (0)
#define SM_SUB(k)  /* sub-phase stamps into the general path's slots 16.. (unused here) */ \
    do {                                                                     \
        if (tid == 0 && g_prof) atomicAdd(&g_prof[16 + (k)], __builtin_amdgcn_s_memtime() - _st); \
    } while (0)
#else
#define SM_STAMP(k) \
    do {            \
    } while (0)
#define SM_SUB(k) \
    do {          \
    } while (0)
#endif

__device__ __forceinline__ uint32_t sm_dword(const SmallLds &L, uint32_t x) {  // unaligned dword
    const uint32_t w = x >> 2;
    return __builtin_amdgcn_alignbyte(L.src[w + 1], L.src[w], x & 3u);
}
__device__ __forceinline__ bool sm_full(uint32_t e) { return e >= 35u && e <= 128u; }

// Returns false (workgroup-uniform) when the block is not for this path: the caller then runs
// the general latency path on the same request.  src: `len` bytes, 16-B aligned with 16 bytes of
// slack readable past len; dst: dsize bytes (16-B stores when it is 16-B aligned).
__device__ __forceinline__ bool small_decode(SmallLds &L, const uint8_t *src, uint32_t len, uint8_t *dst,
                                             uint32_t dst_cap, uint32_t max_dsize, int32_t *status,
                                             uint32_t *dsize_out) {
    const uint32_t tid = threadIdx.x;
    if (len > kSmC || (((uintptr_t)src) & 15u)) return false;
    SOLO_T0
    // ---- 0. stage the stream (and 64 zero bytes past it) ----
    for (uint32_t o = tid * 16; o < ((len + 15) & ~15u) + 64; o += kSoloWG * 16) {
        uint4 q = make_uint4(0, 0, 0, 0);
        if (o < len) {
            q = *(const uint4 *)(src + o);
            if (o + 16 > len) {  // bytes past len are slack: zero them
                uint32_t w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
                for (uint32_t j = 0; j < 4; j++) {
                    const int keep = (int)len - (int)(o + 4 * j);
                    w[j] = keep >= 4 ? w[j] : keep <= 0 ? 0u : (w[j] & ((1u << (8 * keep)) - 1u));
                }
                q = make_uint4(w[0], w[1], w[2], w[3]);
            }
        }
        *(uint4 *)(L.src + o / 4) = q;
        const uint32_t w4[4] = {q.x, q.y, q.z, q.w};
        uint32_t cw4[4];
#pragma unroll
        for (uint32_t j = 0; j < 4; j++) {
            cw4[j] = 0;
#pragma unroll
            for (uint32_t b = 0; b < 4; b++) {
                const uint32_t x = o + 4 * j + b, c = tok_code(w4[j] >> (8 * b));
                cw4[j] |= (x + c + 1 > len ? 4u : c) << (8 * b);
            }
        }
        *(uint4 *)(L.cb + o) = make_uint4(cw4[0], cw4[1], cw4[2], cw4[3]);
    }
    __syncthreads();
    SM_SUB(0);
    const uint8_t *sb = (const uint8_t *)L.src;
    uint32_t kind, csize = 0, dsize = 0, hdr = 0;
    const int st0 = classify_block(sb, len, dst_cap, max_dsize, kind, csize, dsize, hdr);
    if (st0 == QLZX_OK && kind == kBlkCompressed && dsize > kSmD) return false;
    if (st0 != QLZX_OK) {
        if (tid == 0) *status = st0, *dsize_out = 0;
        return true;
    }
    if (kind == kBlkStored) {  // quicklz.c:808-811
        if ((((uintptr_t)dst) & 3u) == 0) {
            for (uint32_t p = tid * 4; p < dsize; p += kSoloWG * 4) {
                const uint32_t w = sm_dword(L, hdr + p);
                if (p + 4 <= dsize) *(uint32_t *)(dst + p) = w;
                else for (uint32_t j = 0; p + j < dsize; j++) dst[p + j] = (uint8_t)(w >> (8 * j));
            }
        } else {
            for (uint32_t p = tid; p < dsize; p += kSoloWG) dst[p] = sb[hdr + p];
        }
        if (tid == 0) *status = QLZX_OK, *dsize_out = dsize;
        return true;
    }
    if (dsize == 0) {  // nothing to decode: C5 accepts csize == hdr or the 9-byte minimum (oracle/qlz_oracle.c:197,228)
        if (tid == 0) *status = (csize == hdr || csize == hdr + 9) ? QLZX_OK : QLZX_E_CORRUPT, *dsize_out = 0;
        return true;
    }
    SM_SUB(1);
    // ---- 1. the group that would start at every stream byte x (x + 4 <= csize) ----
    // 1a. candidates: bytes whose dword has bit 31 (the rest fail C1), listed in ja for balance
    uint32_t ncand, cnt = 0;
    for (uint32_t x = hdr + tid; x + 4 <= csize; x += kSoloWG) {
        const bool c = (sb[x + 3] >> 7) != 0;
        if (!c) L.p.info[x] = (uint8_t)kSmBad;
        cnt += c ? 1u : 0u;
    }
    if (tid == 0) L.cursor = kSoloWG;
    uint32_t w = block_excl<false>(cnt, L.wsum[1], ncand);
    for (uint32_t x = hdr + tid; x + 4 <= csize; x += kSoloWG)
        if (sb[x + 3] >> 7) L.p.ja[w++] = (uint16_t)x;
    __syncthreads();
    SM_SUB(2);
    // 1b. parse the group at every candidate (one dependent LDS read per match token).  All
    //     lanes stay busy: a lane whose chain ends takes the next unparsed candidate from a
    //     shared cursor, and a step is a handful of VALU ops (codes from cb, C2 folded in).
    {
        uint32_t i = tid, x = 0, x4 = 0, lim = 0, mrem = 0, ex = 0, c = 0;
        auto start = [&]() {
            x = L.p.ja[i];
            x4 = x + 4;
            lim = csize - x4;
            mrem = sm_dword(L, x) & 0x7fffffffu;
            ex = 0;
            c = 0;
        };
        if (i < ncand) start();
        while (i < ncand) {
            const uint32_t kend = lim - ex;  // the item index that would start at csize
            const uint32_t k = min((uint32_t)__builtin_ctz(mrem | 0x80000000u), 30u);  // no match left: 30
            bool fin = kend <= k || !mrem;   // ends before the next match / item 31, or FULL
            if (!fin) {
#if QLZX_SM_PAIR
                // the codes of 4 bytes from this token's: a next match whose first byte is among
                // them (its code sits k2 - k + c bytes on) is taken in the same step
                const uint32_t a = x4 + k + ex;
                const uint32_t *cbw = (const uint32_t *)L.cb;
                const uint32_t w = __builtin_amdgcn_alignbyte(cbw[(a >> 2) + 1], cbw[a >> 2], a & 3u);
                c = w & 0xffu;
                fin = c > 3;  // C2
                if (!fin) {
                    ex += c;
                    mrem &= mrem - 1;
                    const uint32_t k2 = min((uint32_t)__builtin_ctz(mrem | 0x80000000u), 30u);
                    const uint32_t d = k2 - k + c;
                    if (lim - ex > k2 && mrem != 0 && d <= 3) {
                        c = (w >> (8 * d)) & 0xffu;
                        fin = c > 3;  // C2
                        ex += fin ? 0u : c;
                        mrem &= fin ? mrem : mrem - 1;
                    }
                }
#else
                c = L.cb[x4 + k + ex];
                fin = c > 3;  // C2
                ex += fin ? 0u : c;
                mrem &= fin ? mrem : mrem - 1;
#endif
            }
            if (fin) {
                const uint32_t ke = lim - ex;
                L.p.info[x] = (uint8_t)(c > 3 ? kSmBad : ke <= min((uint32_t)__builtin_ctz(mrem | 0x80000000u), 30u) ? kSmEnd + ke : 35 + ex);
                i = atomicAdd(&L.cursor, 1u);
                if (i < ncand) start();
            }
        }
    }
    __syncthreads();
    SM_STAMP(0);
    // ---- 2. J2 .. J16 (next position after 2^k whole groups; 0: a non-FULL group on the way) ----
    for (uint32_t x = hdr + tid; x <= csize; x += kSoloWG) {
        uint32_t j = 0;
        if (x + 4 <= csize) {
            const uint32_t e1 = L.p.info[x];
            if (sm_full(e1) && x + e1 + 4 <= csize) {
                const uint32_t e2 = L.p.info[x + e1];
                if (sm_full(e2)) j = x + e1 + e2;
            }
        }
        L.p.ja[x] = (uint16_t)j;
    }
    __syncthreads();
    for (uint32_t r = 0; r < 3; r++) {  // J4 -> jb, J8 -> ja, J16 -> jb
        const uint16_t *a = (r & 1) ? L.p.jb : L.p.ja;
        uint16_t *b = (r & 1) ? L.p.ja : L.p.jb;
        for (uint32_t x = hdr + tid; x <= csize; x += kSoloWG) {
            const uint32_t j = a[x];
            b[x] = j ? a[j] : (uint16_t)0;
        }
        __syncthreads();
    }
    SM_STAMP(1);
    // ---- 3. the group chain: J16 hops, then single groups to the end ----
    if (tid == 0) {
        const uint32_t md = min(min(max_dsize, dsize), (uint32_t)QLZX_FAST_MAX_DSIZE);
        const uint32_t gmax = groups_max(md);  // a valid stream has <= groups_max(dsize) groups
        uint32_t x = hdr, g = 0, klast = 31;
        int st = QLZX_OK;
        while (x + 4 <= csize && g + 16 <= gmax) {
            const uint32_t j = L.p.jb[x];
            if (!j) break;
            L.glist[g] = (uint16_t)x;
            g += 16;
            x = j;
        }
        L.nhops = g / 16;
        for (;;) {
            if (x + 4 > csize) break;  // stream exhausted at a control word
            if (g >= gmax) { st = QLZX_E_CORRUPT; break; }
            const uint32_t e = L.p.info[x];
            L.glist[g++] = (uint16_t)x;
            if (sm_full(e)) { x += e; continue; }
            if (e == kSmBad) { st = QLZX_E_CORRUPT; break; }  // C1 / C2
            klast = e - kSmEnd;  // the stream ends inside this group
            break;
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
    const uint32_t ng = L.ngroups, klast = L.klast;
    if (L.st != QLZX_OK) {
        if (tid == 0) *status = L.st, *dsize_out = 0;
        return true;
    }
    if (tid < L.nhops) {  // the 15 groups inside hop tid
        uint32_t x = L.glist[16 * tid];
#pragma unroll
        for (uint32_t k = 1; k < 16; k++) {
            x += L.p.info[x];
            L.glist[16 * tid + k] = (uint16_t)x;
        }
    }
    __syncthreads();
    SM_STAMP(2);
    // ---- 4. GroupRecs (the last group holds klast items); markers cleared ----
    for (uint32_t g = tid; g < ng; g += kSoloWG) {
        const uint32_t x = L.glist[g];
        const uint32_t cw = sm_dword(L, x);
        const uint32_t nk = g + 1 == ng ? klast : 31u;
        uint32_t mrem = cw & ((1u << nk) - 1u), extra = 0, a = 0, bb = 0;
        const uint32_t m = mrem;
        while (mrem) {
            const uint32_t k = __builtin_ctz(mrem);
            const uint32_t c = L.cb[x + 4 + k + extra];  // <= 3: the walk checked C2
            a |= (c & 1u) << k;
            bb |= (c >> 1) << k;
            extra += c;
            mrem &= mrem - 1;
        }
        L.d.recs[g] = GroupRec{x, m, a, bb};
    }
    for (uint32_t q = tid; q < (dsize + 7) / 8; q += kSoloWG) *(uint4 *)(L.d.s + 8 * q) = make_uint4(0, 0, 0, 0);
    __syncthreads();
    SM_STAMP(3);
    // ---- 5. items: thread tid decodes items [I0, I1), kSmIT per round ----
    const uint32_t nitems = (ng - 1) * 31 + klast;
    const uint32_t per = (nitems + kSoloWG - 1) / kSoloWG;
    const uint32_t I0 = min(tid * per, nitems), I1 = min(I0 + per, nitems);
    const uint32_t tail_from = dsize > QLZX_TAIL ? dsize - 1 - QLZX_TAIL : 0;  // op >= this: tail (quicklz.c:503)
    struct Item {
        uint32_t off, len, tl, pos, lit;
        bool ism;
    };
    auto decode_round = [&](uint32_t I, Item (&it)[kSmIT]) {
        const uint32_t g0 = I / 31;  // a round of <= 8 items spans at most two groups
        const GroupRec r0 = L.d.recs[g0], r1 = L.d.recs[g0 + 1 < ng ? g0 + 1 : g0];
        uint32_t tok[kSmIT];
#pragma unroll
        for (uint32_t j = 0; j < kSmIT; j++) {
            const uint32_t Ij = I + j, k0 = I - 31 * g0 + j;
            const bool second = k0 >= 31;
            const uint32_t k = second ? k0 - 31 : k0;
            const uint32_t ip = second ? r1.ip : r0.ip, m = second ? r1.m : r0.m;
            const uint32_t a = second ? r1.a : r0.a, b = second ? r1.b : r0.b;
            const uint32_t low = (1u << k) - 1u;
            const uint32_t pos = ip + 4 + k + __builtin_popcount(a & low) + 2 * __builtin_popcount(b & low);
            it[j].pos = pos;
            it[j].ism = Ij < I1 && ((m >> k) & 1u) != 0;
            tok[j] = sm_dword(L, Ij < I1 && pos < csize ? pos : 0u);  // zero bytes past csize
        }
#pragma unroll
        for (uint32_t j = 0; j < kSmIT; j++) {
            const uint32_t t = tok[j];
            uint32_t off, mlen, tl;
            decode_tok_bf(t, off, mlen, tl);
            it[j].off = off;
            it[j].len = it[j].ism ? mlen : (I + j < I1 ? 1u : 0u);
            it[j].tl = it[j].ism ? tl : 1u;
            it[j].lit = t & 0xffu;
        }
    };
    bool bad = false, complete = false;
    uint32_t tail_idx = 0xffffffffu, max_match = 0;
    auto emit = [&](const Item (&it)[kSmIT], uint32_t I, uint32_t &d) {  // checks + markers of a round
#pragma unroll
        for (uint32_t j = 0; j < kSmIT; j++) {
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
                L.d.s[d] = (uint16_t)(e.ism ? e.off : kSoloLit);
                if (!e.ism) L.d.out[d] = (uint8_t)e.lit;
            }
            d += e.len;
        }
    };
    uint32_t total;
    if (per <= kSmIT) {  // one round per thread: its items stay in registers between the passes
        Item it[kSmIT];
        decode_round(I0, it);
        uint32_t mysum = 0;
#pragma unroll
        for (uint32_t j = 0; j < kSmIT; j++) mysum += it[j].len;
        uint32_t d = block_excl<false>(mysum, L.wsum[0], total);
        emit(it, I0, d);
    } else {
        uint32_t mysum = 0;
        for (uint32_t I = I0; I < I1; I += kSmIT) {
            Item it[kSmIT];
            decode_round(I, it);
#pragma unroll
            for (uint32_t j = 0; j < kSmIT; j++) mysum += it[j].len;
        }
        uint32_t d = block_excl<false>(mysum, L.wsum[0], total);
        for (uint32_t I = I0; I < I1; I += kSmIT) {
            Item it[kSmIT];
            decode_round(I, it);
            emit(it, I, d);
        }
    }
    {
        // one LDS update per wave (1024 same-address atomics would serialise)
        const bool l0 = (tid & 63) == 0;
        const bool wbad = __ballot(bad) != 0, wdone = __ballot(complete) != 0;
        tail_idx = ~(uint32_t)__builtin_amdgcn_readlane((int)wave_incl_max(~tail_idx), 63);
        max_match = (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_max(max_match), 63);
        if (l0 && wbad) L.bad = 1;
        if (l0 && wdone) L.done = 1;
        if (l0 && tail_idx != 0xffffffffu) atomicMin(&L.tail_idx, tail_idx);
        if (l0 && max_match) atomicMax(&L.max_match, max_match);
    }
    __syncthreads();
    SM_STAMP(4);
    // a failed check; no item completing dsize (C5); a match after the first tail literal (C4)
    if (L.bad || !L.done || (L.tail_idx != 0xffffffffu && L.max_match > L.tail_idx)) {
        if (tid == 0) *status = QLZX_E_CORRUPT, *dsize_out = 0;
        return true;
    }
    // ---- 6. fill: markers -> source position of every byte of the thread's runs ----
    // (one u32 per byte in registers; the u16 LDS array is read and written 16 B at a time)
    const uint32_t nseg = (dsize + kSoloWG * kSmOwn - 1) / (kSoloWG * kSmOwn);
    uint32_t sv[kSmSeg][kSmOwn];
    uint32_t lastp[kSmSeg];
    auto ld16 = [&](uint32_t p0, uint32_t (&v)[kSmOwn]) {
#pragma unroll
        for (uint32_t q = 0; q < kSmOwn / 8; q++) {
            const uint4 w = *(const uint4 *)(L.d.s + p0 + 8 * q);
            const uint32_t w4[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
            for (uint32_t h = 0; h < 4; h++) v[8 * q + 2 * h] = w4[h] & 0xffffu, v[8 * q + 2 * h + 1] = w4[h] >> 16;
        }
    };
    auto st16 = [&](uint32_t p0, const uint32_t (&v)[kSmOwn]) {
#pragma unroll
        for (uint32_t q = 0; q < kSmOwn / 8; q++)
            *(uint4 *)(L.d.s + p0 + 8 * q) = make_uint4(v[8 * q] | (v[8 * q + 1] << 16), v[8 * q + 2] | (v[8 * q + 3] << 16),
                                                        v[8 * q + 4] | (v[8 * q + 5] << 16), v[8 * q + 6] | (v[8 * q + 7] << 16));
    };
#pragma unroll
    for (uint32_t z = 0; z < kSmSeg; z++) {
        const uint32_t p0 = z * kSoloWG * kSmOwn + tid * kSmOwn;
        lastp[z] = 0;
        if (p0 < dsize) {
            ld16(p0, sv[z]);
#pragma unroll
            for (uint32_t j = 0; j < kSmOwn; j++) lastp[z] = sv[z][j] ? p0 + j + 1 : lastp[z];
        }
    }
    uint32_t all0, all1, fz[kSmSeg];
    const uint32_t prev0 = block_excl<true>(lastp[0], L.wsum[0], all0);
    uint32_t prev1 = 0;
    if (nseg > 1) prev1 = max(block_excl<true>(lastp[1], L.wsum[1], all1), all0);
    fz[0] = prev0 ? L.d.s[prev0 - 1] : kSoloLit;  // position 0 always has a marker
    fz[1] = prev1 ? L.d.s[prev1 - 1] : kSoloLit;
    __syncthreads();  // every carry read before the runs are rewritten
#pragma unroll
    for (uint32_t z = 0; z < kSmSeg; z++) {
        const uint32_t p0 = z * kSoloWG * kSmOwn + tid * kSmOwn;
        if (p0 < dsize) {
            uint32_t f = fz[z];
#pragma unroll
            for (uint32_t j = 0; j < kSmOwn; j++) {
                const uint32_t p = p0 + j;
                f = sv[z][j] ? sv[z][j] : f;
                sv[z][j] = (f == kSoloLit || p >= dsize) ? p : p - f;
            }
            st16(p0, sv[z]);
        }
    }
    __syncthreads();
    SM_STAMP(5);
    // ---- 7. pointer jumping until every byte's source is a literal (s[s] == s) ----
    // Entries are rewritten while others read them; any value read is an earlier link of the
    // same chain, so a stale read only costs a round.  A run with no jump in a round is final
    // (every source it read is a literal) and drops out.
    bool fin[kSmSeg];
#pragma unroll
    for (uint32_t z = 0; z < kSmSeg; z++) fin[z] = z * kSoloWG * kSmOwn + tid * kSmOwn >= dsize;
    for (;;) {
        bool ch = false;
#pragma unroll
        for (uint32_t z = 0; z < kSmSeg; z++) {
            const uint32_t p0 = z * kSoloWG * kSmOwn + tid * kSmOwn;
            if (!fin[z]) {
                uint32_t t[kSmOwn];
                bool cz = false;
#pragma unroll
                for (uint32_t j = 0; j < kSmOwn; j++) t[j] = L.d.s[sv[z][j]];
#pragma unroll
                for (uint32_t j = 0; j < kSmOwn; j++) {
                    cz = cz || t[j] != sv[z][j];
                    sv[z][j] = t[j];
                }
                if (cz) st16(p0, sv[z]);
                fin[z] = !cz;
                ch = ch || cz;
            }
        }
        if (!__syncthreads_or(ch)) break;
    }
    SM_STAMP(6);
    // ---- 8. gather the runs' bytes from the literals and store them once ----
    const bool al16 = (((uintptr_t)dst) & 15u) == 0;
#pragma unroll
    for (uint32_t z = 0; z < kSmSeg; z++) {
        const uint32_t p0 = z * kSoloWG * kSmOwn + tid * kSmOwn;
        if (p0 < dsize) {
            const uint32_t n = min(kSmOwn, dsize - p0);
            uint32_t o[kSmOwn / 4];
#pragma unroll
            for (uint32_t q = 0; q < kSmOwn / 4; q++) o[q] = 0;
#pragma unroll
            for (uint32_t j = 0; j < kSmOwn; j++) o[j >> 2] |= (uint32_t)L.d.out[sv[z][j]] << (8 * (j & 3));
            if (n == kSmOwn && al16) {
                *(uint4 *)(dst + p0) = make_uint4(o[0], o[1], o[2], o[3]);
            } else {
                for (uint32_t j = 0; j < n; j++) dst[p0 + j] = (uint8_t)(o[j >> 2] >> (8 * (j & 3)));
            }
        }
    }
    if (tid == 0) *status = QLZX_OK, *dsize_out = dsize;
    SM_STAMP(7);
    return true;
}

// One block: the small path when it takes the block, else the general latency path
// (qlzx_decode_solo.hip).
__global__ void __launch_bounds__(kSoloWG) k_dec_solo(const uint8_t *src, uint32_t len, uint8_t *dst,
                                                     uint32_t dst_cap, uint32_t max_dsize, GroupRec *recs,
                                                     int32_t *status, uint32_t *dsize_out) {
    __shared__ __attribute__((aligned(16))) union {
        SoloLds solo;
        SmallLds small;
    } U;
    if (small_decode(U.small, src, len, dst, dst_cap, max_dsize, status, dsize_out)) return;
    solo_decode(U.solo, src, len, dst, dst_cap, max_dsize, recs, status, dsize_out);
}

// One block (len stream bytes at src, dsize <= QLZX_FAST_MAX_DSIZE, len <= kSoloMaxCsize):
// recs = kSoloGmax GroupRecs of workspace; status / dsize_out = one device word each.
inline int launch_decode_solo(const uint8_t *src, uint32_t len, uint8_t *dst, uint32_t dst_cap,
                              uint32_t max_dsize, GroupRec *recs, int32_t *status, uint32_t *dsize_out,
                              hipStream_t s) {
    hipLaunchKernelGGL(k_dec_solo, dim3(1), dim3(kSoloWG), 0, s, src, len, dst, dst_cap, max_dsize, recs,
                       status, dsize_out);
    return (int)hipGetLastError();
}

}  // namespace qlzx
