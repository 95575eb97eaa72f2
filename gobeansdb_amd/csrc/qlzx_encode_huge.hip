// qlzx_encode_huge.hip -- level-3 compress of ONE large value (n > 64 KiB, up to BodyMax = 50 MiB,
// config/mc_config.go:7; TryCompress compresses whole bodies, store/item.go:149-151) by the whole GPU.
//
// qlz_compress_core (quicklz.c:197-494) is a serial loop, but at level 3 every position of the main
// loop is inserted into the hash table, in order (the item start at quicklz.c:356, the bytes of
// a match at 366-372).  So the table a position i sees is a pure function of the positions before
// it: bucket h = hash(fetch(i)) holds, in slot k, the latest earlier position of h whose insertion
// rank r' has r' mod 16 == k, and the slots read are k < min(r mod 256, 16) with r = the number of
// earlier positions of h (hash_counter is a byte: quicklz.c:316,331,357).  Position-parallel:
//   1. hash of every main-loop position; stable radix sort by hash (rocPRIM) -> per bucket the
//      positions in order, so position i's candidates are the <= 16 entries before it;
//   2. per position: the best match (longest, ties to the latest candidate, quicklz.c:319-354)
//      and whether the loop takes it (length > 2, offset < 131071, quicklz.c:361);
//   3. the greedy parse (next = i + length, or i + 1 for a literal) by pointer doubling:
//      J_k = the item start 2^k items on (P = leaving the main loop), one lane walks the largest
//      valid jumps from position 0 and threads expand the jumps level by level into the item list;
//   4. token sizes (quicklz.c:377-406), an exclusive scan for the output offsets, the bail-out test
//      at every control word (quicklz.c:218), then every control word and item written in parallel.
// Output equals the lane encoder's and the reference's byte for byte (tests/test_gpu_large.py).
#include <rocprim/rocprim.hpp>

namespace qlzx {

constexpr uint32_t kHeWG = 256, kHeGrid = 2048;
constexpr uint32_t kHeLevelsMax = 12;  // J_0 .. J_11: 2048 items per top jump

struct HeCtl {
    uint32_t m;       // items of the main loop
    uint32_t tail0;   // first position after the main loop's last item
    uint32_t bail;    // 1: the value stays stored (quicklz.c:218)
    uint32_t pad;
    uint32_t U[kHeLevelsMax + 1];  // U[k]: items covered by jumps of level >= k (a prefix)
};

__device__ __forceinline__ uint32_t he_ld32(const uint8_t *p) {  // unaligned, always a vector load
    uint64_t a = (uint64_t)(uintptr_t)p;
    asm volatile("" : "+v"(a));
    return *(const uint32_t *)(uintptr_t)a;
}
__device__ __forceinline__ uint32_t he_ld24(const uint8_t *p) { return he_ld32(p) & 0xffffffu; }

// main-loop positions: ip <= n - 1 - QLZX_TAIL (quicklz.c:204,213)
__host__ __device__ inline uint32_t he_positions(uint32_t n) { return n > QLZX_TAIL ? n - QLZX_TAIL : 0u; }
__host__ inline uint32_t he_levels(uint32_t P) {
    uint32_t L = 1;
    while (L < kHeLevelsMax && (1ull << L) * 64 <= P) L++;
    return L;
}

__global__ void __launch_bounds__(kHeWG) k_he_keys(const uint8_t *src, uint32_t P, uint16_t *key, uint32_t *pos) {
    for (uint32_t i = blockIdx.x * kHeWG + threadIdx.x; i < P; i += gridDim.x * kHeWG) {
        const uint32_t f = (uint32_t)src[i] | ((uint32_t)src[i + 1] << 8) | ((uint32_t)src[i + 2] << 16);
        key[i] = (uint16_t)(((f >> 12) ^ f) & (QLZX_BUCKETS - 1));  // hash_func, quicklz.c:70
        pos[i] = i;
    }
}

// first sorted index of every bucket present
__global__ void __launch_bounds__(kHeWG) k_he_base(const uint16_t *key_s, uint32_t P, uint32_t *base) {
    for (uint32_t t = blockIdx.x * kHeWG + threadIdx.x; t < P; t += gridDim.x * kHeWG)
        if (t == 0 || key_s[t] != key_s[t - 1]) base[key_s[t]] = t;
}

// Best match of every main-loop position, in sorted order (thread t: the t-th position of the
// sort).  MO[i] = length | offset << 8 when the loop takes it, else 0.
__global__ void __launch_bounds__(kHeWG) k_he_match(const uint8_t *src, uint32_t n, uint32_t P, const uint16_t *key_s,
                                                    const uint32_t *pos_s, const uint32_t *base, uint32_t *MO) {
    for (uint32_t t = blockIdx.x * kHeWG + threadIdx.x; t < P; t += gridDim.x * kHeWG) {
        const uint32_t h = key_s[t], i = pos_s[t], r = t - base[h];
        const uint32_t c = r & 255u, slots = c < QLZX_SLOTS ? c : QLZX_SLOTS;  // quicklz.c:316,331
        const uint32_t f = he_ld24(src + i);
        const uint32_t limit = min(255u, n - 4 - i);  // `remaining`, quicklz.c:310
        uint32_t best_m = 0, best_o = 0;
        const uint32_t nd = min(r, (uint32_t)QLZX_SLOTS);
        for (uint32_t d = 1; d <= nd; d++) {  // latest first: a tie keeps the later candidate
            if (((r - d) & (QLZX_SLOTS - 1)) >= slots) continue;
            const uint32_t o = pos_s[t - d];
            if (o + 2 >= i || he_ld24(src + o) != f) continue;  // o < src - MINOFFSET, fetch equal
            uint32_t m = 3;
            while (m + 4 <= limit) {
                const uint32_t x = he_ld32(src + o + m) ^ he_ld32(src + i + m);
                if (x) {
                    m += (uint32_t)__builtin_ctz(x) >> 3;
                    goto done;
                }
                m += 4;
            }
            while (m < limit && src[o + m] == src[i + m]) m++;
        done:
            if (m > best_m) best_m = m, best_o = o;
        }
        MO[i] = (best_m > 2 && i - best_o < QLZX_MAX_OFFSET) ? (best_m | ((i - best_o) << 8)) : 0u;
    }
}

// J_0[i] = the next item start (P once it leaves the main loop); J_0[P] = P
__global__ void __launch_bounds__(kHeWG) k_he_jump0(const uint32_t *MO, uint32_t P, uint32_t *J0) {
    for (uint32_t i = blockIdx.x * kHeWG + threadIdx.x; i <= P; i += gridDim.x * kHeWG) {
        if (i == P) { J0[i] = P; continue; }
        const uint32_t ml = MO[i] & 255u, nx = i + (ml ? ml : 1u);
        J0[i] = nx < P ? nx : P;
    }
}
__global__ void __launch_bounds__(kHeWG) k_he_jumpk(const uint32_t *Jp, uint32_t P, uint32_t *Jk) {
    for (uint32_t i = blockIdx.x * kHeWG + threadIdx.x; i <= P; i += gridDim.x * kHeWG) Jk[i] = Jp[Jp[i]];
}

// One lane: from position 0, the largest jump that stays in the main loop (levels only fall);
// the start of every jump goes to ITEM[its first item].
__global__ void k_he_walk(const uint32_t *J, uint32_t P, uint32_t L, const uint32_t *MO, uint32_t *ITEM, HeCtl *ctl) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    uint32_t x = 0, t = 0, k = L - 1, last = 0;
    for (uint32_t q = 0; q <= kHeLevelsMax; q++) ctl->U[q] = 0;
    if (P == 0) {
        ctl->m = 0;
        ctl->tail0 = 0;
        return;
    }
    while (x != P) {
        while (k > 0 && J[(size_t)k * (P + 1) + x] == P) {
            ctl->U[k] = t;  // items [0, t) are covered by jumps of level >= k
            k--;
        }
        ITEM[t] = x;
        last = x;
        t += 1u << k;
        x = J[(size_t)k * (P + 1) + x];
    }
    ctl->U[0] = t;
    ctl->m = t;
    const uint32_t ml = MO[last] & 255u;  // the last item is a single step (level 0)
    ctl->tail0 = last + (ml ? ml : 1u);
}

// level k -> k - 1: the second half of every level-k jump inside [0, U[k])
__global__ void __launch_bounds__(kHeWG) k_he_expand(const uint32_t *Jk1, const HeCtl *ctl, uint32_t k, uint32_t *ITEM) {
    const uint32_t nj = ctl->U[k] >> k;
    for (uint32_t j = blockIdx.x * kHeWG + threadIdx.x; j < nj; j += gridDim.x * kHeWG) {
        const uint32_t u = j << k;
        ITEM[u + (1u << (k - 1))] = Jk1[ITEM[u]];
    }
}

__device__ __forceinline__ uint32_t he_tok_bytes(uint32_t ml, uint32_t off) {  // quicklz.c:377-406
    if (ml == 3 && off <= 63) return 1;
    if (ml == 3 && off <= 16383) return 2;
    if (ml <= 18 && off <= 1023) return 2;
    if (ml <= 33) return 3;
    return 4;
}
__device__ __forceinline__ uint32_t he_tok(uint32_t ml, uint32_t off) {
    if (ml == 3 && off <= 63) return off << 2;
    if (ml == 3 && off <= 16383) return (off << 2) | 1u;
    if (ml <= 18 && off <= 1023) return ((ml - 3) << 2) | (off << 6) | 2u;
    if (ml <= 33) return ((ml - 2) << 2) | (off << 7) | 3u;
    return ((ml - 3) << 7) | (off << 15) | 3u;
}

// output bytes of every item (main-loop items, then the literal tail); sizes[ntot] = 0
__global__ void __launch_bounds__(kHeWG) k_he_sizes(const uint32_t *ITEM, const uint32_t *MO, const HeCtl *ctl,
                                                    uint32_t ntot, uint32_t *sizes) {
    const uint32_t m = ctl->m;
    for (uint32_t t = blockIdx.x * kHeWG + threadIdx.x; t <= ntot; t += gridDim.x * kHeWG) {
        uint32_t sz = t < ntot ? 1u : 0u;
        if (t < m) {
            const uint32_t mo = MO[ITEM[t]], ml = mo & 255u;
            if (ml) sz = he_tok_bytes(ml, mo >> 8);
        }
        sizes[t] = sz;
    }
}

// the bail-out test at every control word the main loop starts (quicklz.c:215-219): at item 31 g
// (g >= 1), ip = its position, op = where its control word goes
__global__ void __launch_bounds__(kHeWG) k_he_bail(const uint32_t *ITEM, const uint32_t *S, uint32_t n, uint32_t bias,
                                                   HeCtl *ctl) {
    const uint32_t m = ctl->m;
    for (uint32_t g = 1 + blockIdx.x * kHeWG + threadIdx.x; 31u * g < m; g += gridDim.x * kHeWG) {
        const uint64_t ip = ITEM[31u * g], op = 4ull * g + S[31u * g];
        if (ip > 3ull * (n >> 2) && op + bias > ip - (ip >> 5)) atomicOr(&ctl->bail, 1u);
    }
}

// control words (one thread per group) and items (one thread per item) into dst + hdr
__global__ void __launch_bounds__(kHeWG) k_he_write(const uint8_t *src, const uint32_t *ITEM, const uint32_t *MO,
                                                    const uint32_t *S, const HeCtl *ctl, uint32_t ntot, uint8_t *out) {
    const uint32_t m = ctl->m, tail0 = ctl->tail0, ng = (ntot + 30) / 31;
    for (uint32_t t = blockIdx.x * kHeWG + threadIdx.x; t < ntot; t += gridDim.x * kHeWG) {
        const uint32_t g = t / 31, o = 4 * (g + 1) + S[t];
        const uint32_t p = t < m ? ITEM[t] : tail0 + (t - m);
        const uint32_t mo = t < m ? MO[p] : 0u, ml = mo & 255u;
        if (ml) {
            const uint32_t v = he_tok(ml, mo >> 8), nb = he_tok_bytes(ml, mo >> 8);
            for (uint32_t b = 0; b < nb; b++) out[o + b] = (uint8_t)(v >> (8 * b));
        } else {
            out[o] = src[p];
        }
        if (t % 31 == 0 && g < ng) {  // the group's control word: bit j = item 31 g + j is a match
            uint32_t cw = 0x80000000u;
            for (uint32_t j = 0; j < 31 && t + j < m; j++) cw |= ((MO[ITEM[t + j]] & 255u) ? 1u : 0u) << j;
            const uint32_t co = 4 * g + S[t];
            for (uint32_t b = 0; b < 4; b++) out[co + b] = (uint8_t)(cw >> (8 * b));
        }
    }
}

__global__ void __launch_bounds__(kHeWG) k_he_copy(const uint8_t *s, uint8_t *d, uint64_t len) {
    for (uint64_t p = (uint64_t)(blockIdx.x * kHeWG + threadIdx.x); p < len; p += (uint64_t)gridDim.x * kHeWG) d[p] = s[p];
}
__global__ void k_he_header(uint8_t *dst, bool compressed, uint32_t csize, uint32_t n, uint32_t *csize_out,
                            int32_t *status) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    const uint32_t f = 2u | (compressed ? 1u : 0u) | 0x4Cu;  // long header, level 3 (quicklz.c:757-772)
    dst[0] = (uint8_t)f;
    for (uint32_t b = 0; b < 4; b++) dst[1 + b] = (uint8_t)(csize >> (8 * b)), dst[5 + b] = (uint8_t)(n >> (8 * b));
    *csize_out = csize;
    if (status) *status = QLZX_OK;
}

// Large blocks of a compress batch: {block, length}
struct HeItem {
    uint32_t i, n;
};
__global__ void __launch_bounds__(256) k_he_pending(qlzx_blocks b, uint32_t min_len, uint32_t *count, HeItem *items) {
    for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < b.n; i += gridDim.x * 256) {
        const uint32_t n = b.src_len[i];
        if (n < min_len) continue;
        const uint32_t j = atomicAdd(count, 1u);
        items[j] = HeItem{i, n};
    }
}

// Workspace of one value of up to `nmax` bytes (carved in this order).
struct HeWs {
    uint16_t *key, *key_s;
    uint32_t *pos, *pos_s, *base, *MO, *J, *ITEM, *sizes, *S, *scrc;
    HeCtl *ctl;
    void *tmp;
    size_t tmp_bytes;
};
inline size_t he_ws_layout(uint32_t nmax, uint8_t *ws, HeWs *w) {
    const uint32_t P = he_positions(nmax), L = he_levels(P);
    size_t sort_tmp = 0, scan_tmp = 0;
    (void)rocprim::radix_sort_pairs(nullptr, sort_tmp, (const uint16_t *)nullptr, (uint16_t *)nullptr,
                              (const uint32_t *)nullptr, (uint32_t *)nullptr, (size_t)P, 0, 12);
    (void)rocprim::exclusive_scan(nullptr, scan_tmp, (const uint32_t *)nullptr, (uint32_t *)nullptr, 0u, (size_t)nmax + 1,
                            rocprim::plus<uint32_t>());
    size_t o = 0;
    auto take = [&](size_t bytes) {
        const size_t at = o;
        o += (bytes + 255) & ~(size_t)255;
        return ws ? ws + at : nullptr;
    };
    uint8_t *p;
    p = take(sizeof(HeCtl));
    if (w) w->ctl = (HeCtl *)p;
    p = take((size_t)P * 2);
    if (w) w->key = (uint16_t *)p;
    p = take((size_t)P * 2);
    if (w) w->key_s = (uint16_t *)p;
    p = take((size_t)P * 4);
    if (w) w->pos = (uint32_t *)p;
    p = take((size_t)P * 4);
    if (w) w->pos_s = (uint32_t *)p;
    p = take((size_t)QLZX_BUCKETS * 4);
    if (w) w->base = (uint32_t *)p;
    p = take((size_t)P * 4 + 4);
    if (w) w->MO = (uint32_t *)p;
    p = take((size_t)L * (P + 1) * 4);
    if (w) w->J = (uint32_t *)p;
    p = take((size_t)P * 4 + 4);
    if (w) w->ITEM = (uint32_t *)p;
    p = take(((size_t)nmax + 1) * 4);
    if (w) w->sizes = (uint32_t *)p;
    p = take(((size_t)nmax + 1) * 4);
    if (w) w->S = (uint32_t *)p;
    p = take(((size_t)nmax + 400) / kHugeSeg * 4 + 64);
    if (w) w->scrc = (uint32_t *)p;
    const size_t tb = std::max(sort_tmp, scan_tmp);
    p = take(tb);
    if (w) w->tmp = p, w->tmp_bytes = tb;
    return o;
}

}  // namespace qlzx
