// qlzx_decode_huge.hip -- level-3 decode of ONE large block (dsize > QLZX_FAST_MAX_DSIZE, up to
// BodyMax = 50 MiB, config/mc_config.go:7) by the whole GPU, every phase data-parallel.
//
// The batch decoder parses with one lane per block (K1); for a 50 MiB value that lane would walk
// ~400 K control-word groups serially.  Here (N = csize, M = dsize, quicklz.c:513-671):
//   1. code[x]  2-bit token length code of every stream byte;
//   2. delta[x] length of the control-word group that WOULD start at x (speculative parse at
//      every byte; 0 = no shortcut: no sentinel (C1) or within 128 B of the end);
//   3. J_k[x]   the stream offset 2^k groups on (k = 1..8, u16, 0 = not all shortcuts), built
//      level by level from J_{k-1};
//   4. one lane walks the chain from the header with the largest valid jump at each step and
//      lists segments {start, first group, 2^k}; groups without a shortcut (the last ones, or a
//      corrupt stream) are parsed byte by byte there, with K1's checks (C1, C2, group bound);
//   5. the segments are expanded into the group list (one lane per segment);
//   6. per group: the output length of its items; 7. exclusive scan over groups;
//   8. per item: checks C3-C5 (oracle/qlz_oracle.c:180-231) and, for every output byte, its
//      source (itself for a literal, p - offset for a match byte) plus the literal bytes;
//   9. pointer jumping s[p] <- s[s[p]] until every byte points at a literal (log2 of the
//      deepest copy chain rounds); 10. gather: out[p] = lit[s[p]].
// The record CRC (store/datafile.go:161-168) is one wave per 16 KiB segment of the stream plus
// a GF(2) shift-combine, verified before decoding as readRecordAt does.
// The host drives the phases (it knows N and M), so a batch holding such values synchronises
// once per value; values over 64 KiB are rare (the batch path owns the 4-64 KiB ones).
namespace qlzx {

constexpr uint32_t kHugeLevels = 8;            // jump tables J_1 .. J_8 (256 groups per jump)
constexpr uint32_t kHugeSeg = 16u << 10;       // CRC segment
constexpr uint32_t kHugeGrid = 2048, kHugeWG = 256;

struct HugeCtl {
    uint32_t ngroups, nseg, klast, st;
    uint32_t bad, done, tail_idx, max_match;
    uint32_t crc;
    uint32_t pad[7];
    uint32_t changed[64];  // pointer-jumping rounds
};
struct HugeSeg {
    uint32_t x, g, cnt, pad;
};

__host__ __device__ inline uint64_t huge_nmax(uint64_t m) { return m + m / 2 + 64; }  // csize bound (4 B per 3 + cw)
__host__ __device__ inline uint64_t huge_gmax(uint64_t m) { return m / 31 + 2; }

struct HugeWs {  // carved out of one workspace
    HugeCtl *ctl;
    uint32_t *code;
    uint8_t *delta;
    uint16_t *J;      // kHugeLevels x nmax
    HugeSeg *seg;
    uint32_t *glist, *glen;
    uint32_t *src;    // per output byte
    uint8_t *lit;
    uint32_t *scrc;   // CRC per segment
};

inline size_t huge_ws_layout(uint64_t m, uint8_t *base, HugeWs *w) {
    const uint64_t n = huge_nmax(m), g = huge_gmax(m) + 64;
    size_t o = 0;
    auto take = [&](size_t bytes) { uint8_t *p = base ? base + o : nullptr; o += (bytes + 255) & ~(size_t)255; return p; };
    HugeWs h;
    h.ctl = (HugeCtl *)take(sizeof(HugeCtl));
    h.code = (uint32_t *)take((n / 16 + 8) * 4);
    h.delta = take(n + 256);
    h.J = (uint16_t *)take((size_t)kHugeLevels * (n + 256) * 2);
    h.seg = (HugeSeg *)take(g * sizeof(HugeSeg));
    h.glist = (uint32_t *)take(g * 4);
    h.glen = (uint32_t *)take(g * 4);
    h.src = (uint32_t *)take(m * 4 + 64);
    h.lit = take(m + 64);
    h.scrc = (uint32_t *)take((n / kHugeSeg + 8) * 4);
    if (w) *w = h;
    return o;
}

__device__ __forceinline__ uint32_t hg_ld32(const uint8_t *p) { return *(const uint32_t *)p; }  // unaligned mode
__device__ __forceinline__ uint32_t hg_code(const uint32_t *code, uint32_t x) {
    return __builtin_amdgcn_ubfe(code[x >> 4], 2 * (x & 15u), 2);
}
__device__ __forceinline__ uint32_t hg_tokcode(uint32_t b) {
    const uint32_t ty = (b & 3u) + ((b & 127u) == 3u ? 1u : 0u);
    return __builtin_amdgcn_ubfe(0x32110u, ty * 4, 4);
}

__global__ void __launch_bounds__(kHugeWG) k_h_codes(const uint8_t *src, uint32_t n, uint32_t *code) {
    for (uint32_t w = blockIdx.x * kHugeWG + threadIdx.x; w < (n + 15) / 16; w += gridDim.x * kHugeWG) {
        uint32_t v = 0;
        if (16 * w + 16 <= n) {
            const uint32_t d0 = hg_ld32(src + 16 * w), d1 = hg_ld32(src + 16 * w + 4);
            const uint32_t d2 = hg_ld32(src + 16 * w + 8), d3 = hg_ld32(src + 16 * w + 12);
            const uint32_t d4[4] = {d0, d1, d2, d3};
#pragma unroll
            for (uint32_t j = 0; j < 16; j++) v |= hg_tokcode(d4[j >> 2] >> (8 * (j & 3))) << (2 * j);
        } else {
            for (uint32_t j = 0; j < 16 && 16 * w + j < n; j++) v |= hg_tokcode(src[16 * w + j]) << (2 * j);
        }
        code[w] = v;
    }
}

__global__ void __launch_bounds__(kHugeWG) k_h_delta(const uint8_t *src, uint32_t n, uint32_t hdr, const uint32_t *code,
                                                  uint8_t *delta) {
    for (uint32_t x = blockIdx.x * kHugeWG + threadIdx.x; x < n + 256; x += gridDim.x * kHugeWG) {
        uint32_t d = 0;
        if (x >= hdr && x + 128 <= n) {
            const uint32_t cw = hg_ld32(src + x);
            if (cw >> 31) {  // C1
                uint32_t mrem = cw & 0x7fffffffu, extra = 0;
                while (mrem) {
                    extra += hg_code(code, x + 4 + __builtin_ctz(mrem) + extra);
                    mrem &= mrem - 1;
                }
                d = 35 + extra;
            }
        }
        delta[x] = (uint8_t)d;
    }
}

// J_1 from delta, J_k from J_{k-1}: two valid jumps compose, any invalid one gives 0
__global__ void __launch_bounds__(kHugeWG) k_h_jump1(const uint8_t *delta, uint32_t n, uint16_t *J1) {
    for (uint32_t x = blockIdx.x * kHugeWG + threadIdx.x; x < n + 256; x += gridDim.x * kHugeWG) {
        const uint32_t a = delta[x];
        const uint32_t b = a && x + a < n ? delta[x + a] : 0u;
        J1[x] = (uint16_t)(b ? a + b : 0u);
    }
}
__global__ void __launch_bounds__(kHugeWG) k_h_jumpk(const uint16_t *Jp, uint32_t n, uint16_t *Jk) {
    for (uint32_t x = blockIdx.x * kHugeWG + threadIdx.x; x < n + 256; x += gridDim.x * kHugeWG) {
        const uint32_t a = Jp[x];
        const uint32_t b = a && x + a < n ? Jp[x + a] : 0u;
        Jk[x] = (uint16_t)(b ? a + b : 0u);
    }
}

// 4. the chain (one lane).  K1's checks where there is no shortcut.
__global__ void __launch_bounds__(64) k_h_walk(const uint8_t *src, uint32_t n, uint32_t hdr, uint32_t m,
                                               const uint32_t *code, const uint8_t *delta, const uint16_t *J,
                                               uint32_t nmax, HugeSeg *seg, HugeCtl *ctl) {
    if (threadIdx.x != 0 || ctl->st != QLZX_OK) return;  // a record CRC mismatch stops here
    const uint32_t gmax = (uint32_t)huge_gmax(m);
    uint32_t x = hdr, g = 0, ns = 0, klast = 31;
    int st = QLZX_OK;
    for (;;) {
        if (x + 4 > n) break;  // the stream ends at a control word
        int k = (int)kHugeLevels;
        uint32_t j = 0;
        for (; k >= 1; k--) {
            j = J[(size_t)(k - 1) * (nmax + 256) + x];
            if (j && g + (1u << k) <= gmax) break;
        }
        if (k >= 1) {
            seg[ns++] = HugeSeg{x, g, 1u << k, 0};
            g += 1u << k;
            x += j;
            continue;
        }
        if (g >= gmax) { st = QLZX_E_CORRUPT; break; }
        const uint32_t d = delta[x];
        seg[ns++] = HugeSeg{x, g, 1, 0};
        g++;
        if (d) { x += d; continue; }
        const uint32_t cw = hg_ld32(src + x);
        if (!(cw >> 31)) { st = QLZX_E_CORRUPT; break; }  // C1
        uint32_t p = x + 4, kk = 0;
        for (; kk < 31 && p < n; kk++) {
            const uint32_t c = ((cw >> kk) & 1u) ? hg_code(code, p) : 0u;
            if (p + c + 1 > n) { st = QLZX_E_CORRUPT; break; }  // C2
            p += c + 1;
        }
        if (st != QLZX_OK) break;
        if (kk < 31) { klast = kk; break; }  // the stream ends inside this group
        x = p;
    }
    if (st == QLZX_OK && g == 0) st = QLZX_E_CORRUPT;
    ctl->ngroups = g;
    ctl->nseg = ns;
    ctl->klast = klast;
    ctl->st = (uint32_t)st;
    ctl->bad = 0;
    ctl->done = 0;
    ctl->tail_idx = 0xffffffffu;
    ctl->max_match = 0;
}

__global__ void __launch_bounds__(kHugeWG) k_h_expand(const uint8_t *delta, const HugeSeg *seg, const HugeCtl *ctl,
                                                   uint32_t *glist) {
    const uint32_t ns = ctl->st == QLZX_OK ? ctl->nseg : 0u;
    for (uint32_t s = blockIdx.x * kHugeWG + threadIdx.x; s < ns; s += gridDim.x * kHugeWG) {
        const HugeSeg e = seg[s];
        uint32_t x = e.x;
        for (uint32_t c = 0; c < e.cnt; c++) {
            glist[e.g + c] = x;
            x += delta[x];
        }
    }
}

// Items of group g: calls f(item index k, is match, token, stream position, token bytes, output length).
template <typename F>
__device__ __forceinline__ void hg_items(const uint8_t *src, uint32_t n, const uint32_t *code, uint32_t x, uint32_t nk,
                                         F &&f) {
    const uint32_t cw = hg_ld32(src + x);
    uint32_t p = x + 4;
    for (uint32_t k = 0; k < nk; k++) {
        const bool ism = (cw >> k) & 1u;
        const uint32_t t = p + 4 <= n ? hg_ld32(src + p) : (hg_ld32(src + n - 4) >> (8 * (p + 4 - n)));
        uint32_t off = 0, len = 1, tl = 1;
        if (ism) decode_tok_bf(t, off, len, tl);
        f(k, ism, t, p, tl, off, len);
        p += tl;
    }
}

__global__ void __launch_bounds__(kHugeWG) k_h_glen(const uint8_t *src, uint32_t n, const uint32_t *code,
                                                 const uint32_t *glist, const HugeCtl *ctl, uint32_t *glen) {
    if (ctl->st != QLZX_OK) return;
    const uint32_t ng = ctl->ngroups, klast = ctl->klast;
    for (uint32_t g = blockIdx.x * kHugeWG + threadIdx.x; g < ng; g += gridDim.x * kHugeWG) {
        uint32_t sum = 0;
        hg_items(src, n, code, glist[g], g + 1 == ng ? klast : 31u,
                 [&](uint32_t, bool, uint32_t, uint32_t, uint32_t, uint32_t, uint32_t len) { sum += len; });
        glen[g] = sum;
    }
}

// exclusive scan of glen (in place) by one workgroup of 1024 threads
__global__ void __launch_bounds__(1024) k_h_scan(uint32_t *glen, const HugeCtl *ctl) {
    __shared__ uint32_t wsum[16];
    __shared__ uint32_t carry;
    if (ctl->st != QLZX_OK) return;
    const uint32_t ng = ctl->ngroups, tid = threadIdx.x;
    if (tid == 0) carry = 0;
    __syncthreads();
    for (uint32_t base = 0; base < ng; base += 1024 * 8) {
        uint32_t v[8], s = 0;
#pragma unroll
        for (uint32_t j = 0; j < 8; j++) {
            const uint32_t g = base + tid * 8 + j;
            v[j] = g < ng ? glen[g] : 0u;
            s += v[j];
        }
        uint32_t total;
        const uint32_t ex = block_excl<false>(s, wsum, total) + carry;
        uint32_t acc = ex;
#pragma unroll
        for (uint32_t j = 0; j < 8; j++) {
            const uint32_t g = base + tid * 8 + j;
            if (g < ng) glen[g] = acc;
            acc += v[j];
        }
        __syncthreads();
        if (tid == 0) carry += total;
        __syncthreads();
    }
}

__global__ void __launch_bounds__(kHugeWG) k_h_items(const uint8_t *src, uint32_t n, uint32_t hdr, uint32_t m,
                                                  const uint32_t *code, const uint32_t *glist, const uint32_t *gd,
                                                  HugeCtl *ctl, uint32_t *sp, uint8_t *lit) {
    if (ctl->st != QLZX_OK) return;
    const uint32_t ng = ctl->ngroups, klast = ctl->klast;
    const uint32_t tail_from = m > QLZX_TAIL ? m - 1 - QLZX_TAIL : 0;  // quicklz.c:503
    uint32_t bad = 0, done = 0, tail_idx = 0xffffffffu, max_match = 0;
    for (uint32_t g = blockIdx.x * kHugeWG + threadIdx.x; g < ng; g += gridDim.x * kHugeWG) {
        uint32_t d = gd[g];
        hg_items(src, n, code, glist[g], g + 1 == ng ? klast : 31u,
                 [&](uint32_t k, bool ism, uint32_t t, uint32_t pos, uint32_t tl, uint32_t off, uint32_t len) {
                     const uint32_t I = g * 31 + k;
                     if (d < m) {
                         if (ism) {
                             max_match = max(max_match, I);
                             if (off < 3 || off > d || (uint64_t)d + len + 4 > m) {
                                 bad = 1;  // C3 (and no match within the last 4 bytes)
                             } else {
                                 for (uint32_t j = 0; j < len; j++) sp[d + j] = d + j - off;
                             }
                         } else {
                             sp[d] = d;
                             lit[d] = (uint8_t)t;
                             if (d >= tail_from) tail_idx = min(tail_idx, I);
                         }
                         if ((uint64_t)d + len == m) {  // C5: the item completing dsize ends the stream
                             done = 1;
                             const uint32_t ip_end = pos + tl;
                             if (!(ip_end == n || (ip_end < hdr + 9 && n == hdr + 9))) bad = 1;
                         }
                     }
                     d += len;
                 });
    }
    if (bad) atomicOr(&ctl->bad, 1u);
    if (done) atomicOr(&ctl->done, 1u);
    if (tail_idx != 0xffffffffu) atomicMin(&ctl->tail_idx, tail_idx);
    if (max_match) atomicMax(&ctl->max_match, max_match);
}

// s[p] <- s[s[p]]; a stale read is an earlier link of the same chain, so it costs only a round
__global__ void __launch_bounds__(kHugeWG) k_h_jumpround(uint32_t *sp, uint32_t m, uint32_t *changed) {
    uint32_t ch = 0;
    for (uint32_t p = blockIdx.x * kHugeWG + threadIdx.x; p < m; p += gridDim.x * kHugeWG) {
        const uint32_t s = sp[p];
        const uint32_t t = sp[s];
        if (t != s) {
            sp[p] = t;
            ch = 1;
        }
    }
    if (__ballot(ch) && (threadIdx.x & 63) == 0) atomicOr(changed, 1u);
}

__global__ void __launch_bounds__(kHugeWG) k_h_gather(const uint32_t *sp, const uint8_t *lit, uint32_t m, uint8_t *dst) {
    for (uint32_t q = blockIdx.x * kHugeWG + threadIdx.x; q < (m + 3) / 4; q += gridDim.x * kHugeWG) {
        const uint32_t p = 4 * q;
        if (p + 4 <= m) {
            const uint4 s = *(const uint4 *)(sp + p);
            const uint32_t w = lit[s.x] | (lit[s.y] << 8) | (lit[s.z] << 16) | ((uint32_t)lit[s.w] << 24);
            if ((((uintptr_t)dst) & 3u) == 0) *(uint32_t *)(dst + p) = w;
            else for (uint32_t j = 0; j < 4; j++) dst[p + j] = (uint8_t)(w >> (8 * j));
        } else {
            for (uint32_t j = 0; p + j < m; j++) dst[p + j] = lit[sp[p + j]];
        }
    }
}

// record CRC: raw CRC (from 0) of every kHugeSeg segment, one wave each; then the combine
__global__ void __launch_bounds__(256) k_h_crcseg(const uint8_t *p, uint64_t len, uint32_t *scrc) {
    __shared__ uint32_t tab[kCrcLdsWords];
    load_crc_lds(tab);
    __syncthreads();
    const uint32_t nseg = (uint32_t)((len + kHugeSeg - 1) / kHugeSeg);
    for (uint32_t s = blockIdx.x * 4 + threadIdx.x / 64; s < nseg; s += gridDim.x * 4) {
        const uint64_t o = (uint64_t)s * kHugeSeg;
        const uint32_t l = (uint32_t)min((uint64_t)kHugeSeg, len - o);
        const uint32_t c = wave_crc(tab, p + o, l, 0u, threadIdx.x & 63);
        if ((threadIdx.x & 63) == 0) scrc[s] = c;
    }
}
__global__ void k_h_crccomb_ctl(const uint32_t *scrc, uint64_t len, HugeCtl *ctl) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    const uint32_t nseg = (uint32_t)((len + kHugeSeg - 1) / kHugeSeg);
    uint32_t acc = ctl->crc;  // the initial state (k_h_crcinit)
    for (uint32_t s = 0; s < nseg; s++) {
        const uint64_t l = min((uint64_t)kHugeSeg, len - (uint64_t)s * kHugeSeg);
        acc = crc_shift(acc, l) ^ scrc[s];
    }
    ctl->crc = acc;
}
// stored values and early verdicts: only while no CRC mismatch was found
__global__ void __launch_bounds__(kHugeWG) k_h_copy_if(const HugeCtl *ctl, const uint8_t *s, uint8_t *d, uint64_t len) {
    if (ctl->st != QLZX_OK) return;
    for (uint64_t p = (uint64_t)(blockIdx.x * kHugeWG + threadIdx.x); p < len; p += (uint64_t)gridDim.x * kHugeWG) d[p] = s[p];
}
__global__ void k_h_setstatus_ok_if(const HugeCtl *ctl, int32_t *status, uint32_t *dsize_out, int32_t st, uint32_t ds) {
    if (threadIdx.x != 0 || blockIdx.x != 0 || ctl->st != QLZX_OK) return;
    *status = st;
    if (dsize_out) *dsize_out = ds;
}

// Pending large blocks of a batch (status kPending after K1): {block, csize, dsize, compressed}
struct HugeItem {
    uint32_t i, csize, dsize, comp;
};
__global__ void __launch_bounds__(256) k_h_pending(qlzx_blocks b, const int32_t *status, uint32_t *count,
                                                   HugeItem *items) {
    for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < b.n; i += gridDim.x * 256) {
        if (status[i] != kPending) continue;
        const Header h = parse_header(b.src + b.src_off[i]);
        const uint32_t j = atomicAdd(count, 1u);
        items[j] = HugeItem{i, h.csize, h.dsize, h.compressed ? 1u : 0u};
    }
}

}  // namespace qlzx
