// qlzx_decode_wave.hip -- fast batched level-3 decoder for blocks with
// dsize <= QLZX_FAST_MAX_DSIZE (the 4-64 KiB values of BASELINE configs).
//
// Two kernels per chunk of blocks:
//
// K1 k_dec_parse  one LANE per block.  Walks the serial control-word/token
//     chain of quicklz.c:513-671 once, validates every bound (the checks of
//     qlzx_decode_lane.hip), and emits one 16-B record per control-word group:
//       ip  stream offset of the group's control word
//       m   effective match mask (bit k = item k is a match; tail literals 0)
//       a,b bit-planes of (token bytes - 1) per match item (token length 1..4)
//     With the bit-planes, item k's stream offset is a popcount away:
//       ip + 4 + k + popc(a & low(k)) + 2 popc(b & low(k)),
//     so K2 needs no serial walk.  Input is read through a per-lane register
//     window of 16-B aligned loads prefetched two chunks ahead (no LDS, so K1
//     runs at full occupancy).
//
// K2 k_dec_blocks one WAVE per block, the whole output block resident in LDS.
//     Items are decoded 64 at a time, one per lane: locate, read token,
//     exclusive-scan the output lengths, write literals, then copy matches in
//     sub-rounds.  A match is copied once every source byte it needs lies
//     below the first still-pending match of the batch (sources always precede
//     the destination, so the lowest pending match is always ready).  The
//     finished block leaves LDS in 16-B-per-lane coalesced stores.
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

constexpr uint32_t kBlkSkip = 0, kBlkStored = 1, kBlkCompressed = 2;
constexpr uint32_t kParseWG = 256;
constexpr uint32_t kChunkBlocks = 16384;

__host__ __device__ inline uint32_t groups_max(uint32_t max_dsize) { return max_dsize / 31u + 2u; }

inline bool decode_wave_enabled() { return true; }

inline size_t decode_wave_ws_bytes(uint32_t n, uint32_t max_dsize) {
    const uint32_t md = max_dsize > QLZX_FAST_MAX_DSIZE ? QLZX_FAST_MAX_DSIZE : max_dsize;
    const uint32_t c = n < kChunkBlocks ? (n ? n : 1) : kChunkBlocks;
    return (size_t)c * sizeof(BlkInfo) + (size_t)c * groups_max(md) * sizeof(GroupRec) + 256;
}

// ------------------------------------------------------------------ K1 ----
// Per-lane input window in registers: cur (16 B) + nxt (16 B) landed, far (16 B)
// in flight, all 16-B aligned absolute chunks of this lane's block.  Reads of
// up to 4 bytes at stream position p always fall inside cur..nxt[0] because the
// window is advanced before every read; the far chunk has two chunks of
// reading to land.  Chunks past the one holding the last byte are never
// fetched, so no load crosses the block's last 16-B chunk.
struct LaneWin {
    const uint8_t *gbase;  // 16-B aligned
    uint32_t shift, last, wchunk;
    uint32_t cur[4], nxt[4], far[4];

    __device__ __forceinline__ void fetch(uint32_t c, uint32_t w[4]) const {
        if (c <= last) {
            const uint4 v = *(const uint4 *)(gbase + (size_t)c * 16);
            w[0] = v.x; w[1] = v.y; w[2] = v.z; w[3] = v.w;
        }
    }
    __device__ __forceinline__ void init(const uint8_t *src, uint32_t csize) {
        const uintptr_t a = (uintptr_t)src;
        gbase = (const uint8_t *)(a & ~(uintptr_t)15);
        shift = (uint32_t)(a & 15);
        last = (csize + shift - 1) >> 4;
        wchunk = 0;
        fetch(0, cur); fetch(1, nxt); fetch(2, far);
    }
    __device__ __forceinline__ void advance_to(uint32_t p) {
        const uint32_t c = (p + shift) >> 4;
        while (wchunk < c) {
#pragma unroll
            for (int j = 0; j < 4; j++) { cur[j] = nxt[j]; nxt[j] = far[j]; }
            wchunk++;
            fetch(wchunk + 2, far);
        }
    }
    __device__ __forceinline__ uint32_t rd_u32(uint32_t p) {
        advance_to(p);
        const uint32_t o = (p + shift) & 15u, i0 = o >> 2;
        const uint32_t lo = (i0 & 2) ? ((i0 & 1) ? cur[3] : cur[2]) : ((i0 & 1) ? cur[1] : cur[0]);
        const uint32_t hi = (i0 == 3) ? nxt[0] : ((i0 & 2) ? cur[3] : ((i0 & 1) ? cur[2] : cur[1]));
        return __builtin_amdgcn_alignbyte(hi, lo, o & 3u);
    }
};

__global__ void __launch_bounds__(kParseWG) k_dec_parse(qlzx_blocks b, const uint32_t *dst_cap,
                                                         uint32_t *dsize_out, int32_t *status,
                                                         uint32_t first, uint32_t count, BlkInfo *info,
                                                         GroupRec *recs, uint32_t gmax) {
    const uint32_t li = blockIdx.x * kParseWG + threadIdx.x;
    if (li >= count) return;
    const uint32_t i = first + li;
    int st = QLZX_OK;
    uint32_t kind = kBlkSkip, csize = 0, dsize = 0, hdr = 0;
    const uint8_t *src = b.src + b.src_off[i];
    const uint32_t len = b.src_len[i];
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
            else if (h.dsize > QLZX_FAST_MAX_DSIZE) kind = kBlkSkip;  // general path owns it
            else if (!h.compressed) {
                if (csize >= hdr + dsize) kind = kBlkStored;
                else st = QLZX_E_CORRUPT;
            } else kind = kBlkCompressed;
        }
    }
    uint32_t g = 0, k = 31;
    if (st == QLZX_OK && kind == kBlkCompressed) {
        LaneWin w;
        w.init(src, csize);
        uint32_t ip = hdr, op = 0, cw = 0, m = 0, ra = 0, rb = 0, rec_ip = 0;
        const int64_t lit_end = (int64_t)dsize - 1 - QLZX_TAIL;
        GroupRec *myrec = recs + (size_t)li * gmax;
        for (;;) {
            if (k == 31) {  // group boundary: control word (quicklz.c:517-525)
                if (g > 0) myrec[g - 1] = GroupRec{rec_ip, m, ra, rb};
                if (g >= gmax || ip + 4 > csize) { st = QLZX_E_CORRUPT; break; }
                rec_ip = ip;
                cw = w.rd_u32(ip);
                if (!(cw >> 31)) { st = QLZX_E_CORRUPT; break; }  // sentinel bit (quicklz.c:221)
                ip += 4;
                k = 0; m = 0; ra = 0; rb = 0;
                g++;
            }
            if ((cw >> k) & 1u) {  // match token
                if (ip >= csize) { st = QLZX_E_CORRUPT; break; }
                uint32_t t = w.rd_u32(ip);
                const uint32_t tl = token_bytes(t & 0xffu);
                if (ip + tl > csize) { st = QLZX_E_CORRUPT; break; }
                if (tl < 4) t &= (1u << (8 * tl)) - 1u;
                uint32_t off, ml;
                decode_token(t, off, ml);
                if (off < 3 || off > op || (uint64_t)op + ml + 4 > dsize) { st = QLZX_E_CORRUPT; break; }
                m |= 1u << k;
                ra |= ((tl - 1) & 1u) << k;
                rb |= ((tl - 1) >> 1) << k;
                ip += tl;
                op += ml;
                k++;
            } else {  // literal run to the next match bit or the group end
                const uint32_t run = __builtin_ctz((cw >> k) | (1u << (31 - k)));
                const int64_t normal = lit_end - (int64_t)op;  // literals at op < dsize-11
                const uint32_t n1 = normal <= 0 ? 0u : (normal < (int64_t)run ? (uint32_t)normal : run);
                if (ip + n1 > csize) { st = QLZX_E_CORRUPT; break; }
                ip += n1; op += n1; k += n1;
                if (n1 < run) {  // tail loop (quicklz.c:645-668): literals to the end
                    const uint32_t rem = dsize - op;
                    const uint32_t c1 = rem < 31 - k ? rem : 31 - k;
                    ip += c1; op += c1; k += c1;
                    while (op < dsize && g < gmax) {
                        myrec[g - 1] = GroupRec{rec_ip, m, ra, rb};
                        rec_ip = ip;
                        ip += 4;  // control word skipped unread (quicklz.c:649-653)
                        const uint32_t c = dsize - op < 31 ? dsize - op : 31;
                        ip += c; op += c; k = c;
                        m = 0; ra = 0; rb = 0;
                        g++;
                    }
                    if (op < dsize || ip > csize) st = QLZX_E_CORRUPT;
                    else myrec[g - 1] = GroupRec{rec_ip, m, ra, rb};
                    break;
                }
            }
        }
    }
    BlkInfo bi{0, 0, kind, dsize};
    if (st != QLZX_OK) {
        bi.kind = kBlkSkip;
        status[i] = st;
        if (dsize_out) dsize_out[i] = 0;
    } else if (kind == kBlkCompressed) {
        bi.ngroups = g;
        bi.nitems = (g - 1) * 31 + k;
    }
    info[li] = bi;
}

// ------------------------------------------------------------------ K2 ----
template <uint32_t MAXD>
struct DecodeLds {
    uint8_t out[MAXD];
    GroupRec grp[4];  // records of the groups touched by the current batch (<= 4 for 64 items)
};

__device__ __forceinline__ void lds_mskor(uint32_t *addr, uint32_t mask, uint32_t val) {
    // mem = (mem & ~mask) | val  (atomic byte-masked write, val pre-masked)
    __hip_atomic_fetch_and(addr, ~mask, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    __hip_atomic_fetch_or(addr, val, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// Store `n` (<= 16) bytes held in w[0..3] (byte 0 = w[0] & 0xff) at LDS byte q.
__device__ __forceinline__ void lds_put16(uint8_t *out, uint32_t q, const uint32_t w[4], uint32_t n) {
    const uint32_t qa = q & 3u;
    uint32_t *d = (uint32_t *)(out + (q & ~3u));
    // shift the 16 bytes left by qa into 5 destination words
    uint32_t o[5];
    o[0] = w[0] << (8 * qa);
    o[1] = qa ? __builtin_amdgcn_alignbyte(w[1], w[0], 4 - qa) : w[1];
    o[2] = qa ? __builtin_amdgcn_alignbyte(w[2], w[1], 4 - qa) : w[2];
    o[3] = qa ? __builtin_amdgcn_alignbyte(w[3], w[2], 4 - qa) : w[3];
    o[4] = qa ? (w[3] >> (8 * (4 - qa))) : 0u;
    const uint32_t end = qa + n;  // byte index (relative to q & ~3) one past the last
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

// Read 16 bytes starting at LDS byte p (p + 19 < buffer size or padded).
__device__ __forceinline__ void lds_get16(const uint8_t *out, uint32_t p, uint32_t w[4]) {
    const uint32_t *s = (const uint32_t *)(out + (p & ~3u));
    const uint32_t pa = p & 3u;
    uint32_t x0 = s[0], x1 = s[1], x2 = s[2], x3 = s[3], x4 = s[4];
    w[0] = __builtin_amdgcn_alignbyte(x1, x0, pa);
    w[1] = __builtin_amdgcn_alignbyte(x2, x1, pa);
    w[2] = __builtin_amdgcn_alignbyte(x3, x2, pa);
    w[3] = __builtin_amdgcn_alignbyte(x4, x3, pa);
}

template <uint32_t MAXD>
__global__ void __launch_bounds__(64) k_dec_blocks(qlzx_blocks b, uint32_t *dsize_out, int32_t *status,
                                                   uint32_t first, uint32_t count, const BlkInfo *info,
                                                   const GroupRec *recs, uint32_t gmax) {
    constexpr uint32_t kPad = 32;
    __shared__ __attribute__((aligned(16))) uint8_t lds_raw[1][MAXD + kPad];
    __shared__ GroupRec grp_lds[1][4];
    const uint32_t lane = threadIdx.x & 63, wv = 0;
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
    uint8_t *out = lds_raw[wv];
    GroupRec *grp = grp_lds[wv];
    const GroupRec *rb = recs + (size_t)li * gmax;
    const uint32_t nitems = bi.nitems;
    uint32_t D = 0;
    for (uint32_t I0 = 0; I0 < nitems; I0 += 64) {
        // records of the (at most 4) groups this batch touches
        const uint32_t g0 = I0 / 31;
        if (lane < 4 && g0 + lane < bi.ngroups) grp[lane] = rb[g0 + lane];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        const uint32_t I = I0 + lane;
        const bool valid = I < nitems;
        const uint32_t g = I / 31, k = I - g * 31;
        const GroupRec gr = grp[valid ? g - g0 : 0];
        const uint32_t low = (1u << k) - 1u;
        const bool is_match = valid && ((gr.m >> k) & 1u);
        const uint32_t pos = gr.ip + 4 + k + __builtin_popcount(gr.a & low) + 2 * __builtin_popcount(gr.b & low);
        uint32_t t = 0;
        if (valid) {  // token or literal byte (a token's bytes lie inside csize: checked by K1)
            const uint8_t *p = src + pos;
            t = p[0];
            if (is_match) t |= ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
        }
        uint32_t off = 0, len = valid ? 1u : 0u;
        if (is_match) decode_token(t, off, len);
        // exclusive scan of output lengths
        uint32_t incl = len;
#pragma unroll
        for (int sh = 1; sh < 64; sh <<= 1) {
            const uint32_t v = __shfl_up(incl, sh, 64);
            if (lane >= (uint32_t)sh) incl += v;
        }
        const uint32_t d = D + incl - len;
        const uint32_t total = __shfl(incl, 63, 64);
        if (valid && !is_match) out[d] = (uint8_t)t;
        bool done = !is_match;
        const uint32_t s = d - off;
        const uint32_t send = (s + len < d) ? s + len : d;
        const bool bytewise = is_match && off < 16 && off < len;
        for (;;) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            const uint64_t pend = __ballot(!done);
            if (!pend) break;
            const uint32_t u = __builtin_ctzll(pend);
            const uint32_t du = __shfl(d, u, 64);
            const bool ready = !done && send <= du;
            if (ready) {
                if (bytewise) {
                    for (uint32_t j = 0; j < len; j++) out[d + j] = out[s + (j % off)];
                } else {
                    for (uint32_t c = 0; c < len; c += 16) {
                        uint32_t w[4];
                        lds_get16(out, s + c, w);
                        const uint32_t n = len - c < 16 ? len - c : 16;
                        lds_put16(out, d + c, w, n);
                        if (off < len) __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
                    }
                }
                done = true;
            }
        }
        D += total;
    }
    // write the block out: 16 B per lane, 1 KiB per wave instruction
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
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
        status[i] = D == dsize ? QLZX_OK : QLZX_E_CORRUPT;
        if (dsize_out) dsize_out[i] = D == dsize ? dsize : 0;
    }
}

inline int launch_decode_wave(const qlzx_blocks &b, const uint32_t *dst_cap, uint32_t *dsize,
                              int32_t *status, const uint32_t *crc_state, const uint32_t *crc_expect,
                              uint32_t *crc_out, uint32_t max_dsize, void *ws, size_t ws_bytes,
                              hipStream_t s) {
    (void)crc_state; (void)crc_expect; (void)crc_out; (void)ws_bytes;
    const uint32_t md = max_dsize > QLZX_FAST_MAX_DSIZE ? QLZX_FAST_MAX_DSIZE : max_dsize;
    const uint32_t gmax = groups_max(md);
    const uint32_t chunk = b.n < kChunkBlocks ? b.n : kChunkBlocks;
    BlkInfo *info = (BlkInfo *)ws;
    GroupRec *recs = (GroupRec *)((uint8_t *)ws + (((size_t)chunk * sizeof(BlkInfo) + 255) & ~(size_t)255));
    for (uint32_t first = 0; first < b.n; first += chunk) {
        const uint32_t cnt = b.n - first < chunk ? b.n - first : chunk;
        hipLaunchKernelGGL(k_dec_parse, dim3((cnt + kParseWG - 1) / kParseWG), dim3(kParseWG), 0, s, b, dst_cap,
                           dsize, status, first, cnt, info, recs, gmax);
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
