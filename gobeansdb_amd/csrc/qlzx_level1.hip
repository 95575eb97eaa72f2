// qlzx_level1.hip -- the level-1 branch of gobeansdb's Go QuickLZ (quicklz/quicklz.go, a
// translation of QuickLZ.java 1.5.0): Compress(src, 1) (quicklz.go:80-191, 262-289) and
// Decompress of level-1 and stored streams (quicklz.go:291-431).  Production gobeansdb
// writes level 3 through cgo (cquicklz.go), so this path only serves the Go API surface
//  and is built for exactness, not speed: one LANE per block, the
// reference loop restated with index arithmetic, hash tables in a per-block HBM workspace.
//
// Level 1 cannot be decoded item-parallel the way K1/K2 decode level 3: a match token
// names a hash bucket, and the bucket's content is the position the DECODER last hashed
// there, i.e. it depends on every byte decoded before it.  Blocks are independent, so a
// batch still fills the chip one lane per block.
//
// Go bounds-checks every slice index and panics on a violation.  The decoder returns
// QLZX_E_CORRUPT exactly where Go Decompress would panic, and it zero-fills the
// destination first, because Go's make([]byte, size) does and a corrupt stream may read
// destination bytes that were never written.  Parity: oracle/qlz_oracle_l1.c, itself
// cross-checked against the reference quicklz.c compiled at level 1 (oracle/Makefile).
#include "qlzx_device.h"

namespace qlzx {

constexpr uint32_t kL1Hash = 4096;
// per-block workspace: u32 hashtable[4096] | u32 cachetable[4096] | u8 counter[4096]
constexpr size_t kL1WsBlock = 2 * 4 * kL1Hash + kL1Hash;
// the decoder uses only the hashtable
constexpr size_t kL1DecWsBlock = 4 * kL1Hash;
// launches cover at most this many blocks, reusing one bounded workspace chunk after chunk
constexpr uint32_t kL1Chunk = 65536;

__device__ __forceinline__ uint32_t l1_bucket(uint32_t f) { return ((f >> 12) ^ f) & (kL1Hash - 1); }
__device__ __forceinline__ uint32_t l1_rd3(const uint8_t *s, int64_t i) {
    return s[i] | ((uint32_t)s[i + 1] << 8) | ((uint32_t)s[i + 2] << 16);
}
__device__ __forceinline__ void l1_put(uint8_t *p, uint64_t v, int n) {
    for (int j = 0; j < n; j++) p[j] = (uint8_t)(v >> (8 * j));
}
// quicklz.go:66-78 writeHeader: bytes 1..4 = compressed size, 5..8 = decompressed size
__device__ __forceinline__ void l1_header(uint8_t *d, bool compressible, uint64_t csize, uint64_t dsize) {
    d[0] = (uint8_t)(2 | (compressible ? 1 : 0) | (1 << 2) | (1 << 6));
    l1_put(d + 1, csize, 4);
    l1_put(d + 5, dsize, 4);
}

__device__ void l1_zero(uint8_t *p, uint64_t n) {
    uint64_t i = 0;
    for (; i < n && (((uintptr_t)(p + i)) & 15u); i++) p[i] = 0;
    for (; i + 16 <= n; i += 16) *(uint4 *)(p + i) = make_uint4(0, 0, 0, 0);
    for (; i < n; i++) p[i] = 0;
}

__global__ void __launch_bounds__(64) k_dec_go_l1(qlzx_blocks b, const uint32_t *dst_cap, uint32_t *dsize_out,
                                                  int32_t *status, uint8_t *ws, uint32_t first, uint32_t count) {
    const uint32_t li = blockIdx.x * 64 + threadIdx.x;
    if (li >= count) return;
    const uint32_t i = first + li;
    const uint8_t *s = b.src + b.src_off[i];
    uint8_t *dst = b.dst + b.dst_off[i];
    const int64_t n = b.src_len[i];
    int st = QLZX_E_CORRUPT;
    int64_t size = 0;
    if (n < 1 || n < ((s[0] & 2u) ? 9 : 3)) {
        st = QLZX_E_HEADER;  // SizeDecompressed indexes past the buffer
    } else {
        const bool h9 = (s[0] & 2u) != 0;
        const int64_t hdr = h9 ? 9 : 3;
        size = h9 ? (int64_t)((uint32_t)s[5] | ((uint32_t)s[6] << 8) | ((uint32_t)s[7] << 16) | ((uint32_t)s[8] << 24))
                  : (int64_t)s[2];
        const int level = (s[0] >> 2) & 3;
        if (level != 1 && level != 3) st = QLZX_E_LEVEL;
        else if (dst_cap && (uint64_t)size > dst_cap[i]) st = QLZX_E_DST_CAP;
        else if ((s[0] & 1u) == 0) {  // stored: copy() takes min(size, len - hdr), the rest stays 0
            const int64_t k = n - hdr < size ? n - hdr : size;
            for (int64_t q = 0; q < k; q++) dst[q] = s[hdr + q];
            l1_zero(dst + k, (uint64_t)(size - k));
            st = QLZX_OK;
        } else if (level != 1) {
            st = QLZX_E_LEVEL;  // compressed level 3: qlzx_decompress_batch's
        } else {
            l1_zero(dst, (uint64_t)size);
            uint32_t *ht = (uint32_t *)(ws + (size_t)li * kL1DecWsBlock);
            for (uint32_t q = 0; q < kL1Hash; q += 4) *(uint4 *)(ht + q) = make_uint4(0, 0, 0, 0);
            int64_t src = hdr, d = 0, last_hashed = -1;
            const int64_t last_match_start = size - 11;
            uint64_t cword = 1;
            uint32_t fetch = 0;
#define NEED_SRC(x) if ((x) < 0 || (x) >= n) break
#define NEED_DST(x) if ((x) < 0 || (x) >= size) break
            for (;;) {  // every iteration moves src forward; leaving by `break` = a Go panic
                if (cword == 1) {
                    NEED_SRC(src + 3);
                    cword = (uint64_t)s[src] | ((uint64_t)s[src + 1] << 8) | ((uint64_t)s[src + 2] << 16) |
                            ((uint64_t)s[src + 3] << 24);
                    src += 4;
                    if (d <= last_match_start) {
                        NEED_SRC(src + 2);
                        fetch = l1_rd3(s, src);
                    }
                }
                if (cword & 1u) {
                    cword >>= 1;
                    uint32_t hash = (fetch >> 4) & 0xfffu;
                    const int64_t off2 = ht[hash];
                    int64_t matchlen;
                    if (fetch & 0xfu) {
                        matchlen = (fetch & 0xfu) + 2;
                        src += 2;
                    } else {
                        NEED_SRC(src + 2);
                        matchlen = s[src + 2];
                        src += 3;
                    }
                    // destination[dst+0..2] = destination[offset2+0..2], then i = 3..matchlen-1
                    const int64_t ncopy = matchlen > 3 ? matchlen : 3;
                    if (off2 + ncopy - 1 >= size || d + ncopy - 1 >= size) break;
                    for (int64_t q = 0; q < ncopy; q++) dst[d + q] = dst[off2 + q];
                    d += matchlen;
                    NEED_DST(last_hashed + 3);
                    fetch = l1_rd3(dst, last_hashed + 1);
                    bool oob = false;
                    while (last_hashed < d - matchlen) {
                        last_hashed++;
                        ht[l1_bucket(fetch)] = (uint32_t)last_hashed;
                        if (last_hashed + 3 >= size) { oob = true; break; }
                        fetch = ((fetch >> 8) & 0xffffu) | ((uint32_t)dst[last_hashed + 3] << 16);
                    }
                    if (oob) break;
                    NEED_SRC(src + 2);
                    fetch = l1_rd3(s, src);
                    last_hashed = d - 1;
                } else if (d <= last_match_start) {
                    NEED_SRC(src);
                    NEED_DST(d);
                    dst[d++] = s[src++];
                    cword >>= 1;
                    while (last_hashed < d - 3) {
                        last_hashed++;
                        ht[l1_bucket(l1_rd3(dst, last_hashed))] = (uint32_t)last_hashed;
                    }
                    NEED_SRC(src + 2);
                    fetch = ((fetch >> 8) & 0xffffu) | ((uint32_t)s[src + 2] << 16);
                } else {
                    bool oob = false;
                    while (d <= size - 1) {
                        if (cword == 1) {
                            src += 4;
                            cword = 0x80000000u;
                        }
                        if (src >= n) { oob = true; break; }
                        dst[d++] = s[src++];
                        cword >>= 1;
                    }
                    if (!oob) st = QLZX_OK;
                    break;
                }
            }
#undef NEED_SRC
#undef NEED_DST
        }
    }
    status[i] = st;
    if (dsize_out) dsize_out[i] = st == QLZX_OK ? (uint32_t)size : 0u;
}

// Go Compress(src, 1).  dst capacity >= len + 400 (quicklz.go:84); empty input: QLZX_E_EMPTY
// (Go returns nil).
__global__ void __launch_bounds__(64) k_enc_go_l1(qlzx_blocks b, uint32_t *csize, int32_t *status, uint8_t *ws,
                                                  uint32_t first, uint32_t count) {
    const uint32_t li = blockIdx.x * 64 + threadIdx.x;
    if (li >= count) return;
    const uint32_t i = first + li;
    const uint8_t *s = b.src + b.src_off[i];
    uint8_t *d = b.dst + b.dst_off[i];
    const int64_t len = b.src_len[i];
    if (len == 0) {
        csize[i] = 0;
        if (status) status[i] = QLZX_E_EMPTY;
        return;
    }
    uint32_t *ht = (uint32_t *)(ws + (size_t)li * kL1WsBlock);
    uint32_t *cache_t = ht + kL1Hash;
    uint8_t *counter = (uint8_t *)(cache_t + kL1Hash);
    for (uint32_t q = 0; q < 2 * kL1Hash + kL1Hash / 4; q += 4) *(uint4 *)(ht + q) = make_uint4(0, 0, 0, 0);
    int64_t src = 0, dst = 9 + 4, cword_ptr = 9, lits = 0;
    uint32_t cword = 0x80000000u, fetch = 0;
    const int64_t last_match_start = len - 6 - 4 - 1;  // UNCONDITIONAL_MATCHLEN, UNCOMPRESSED_END
    if (src <= last_match_start) fetch = l1_rd3(s, 0);
    while (src <= last_match_start) {
        if (cword & 1u) {
            if (src > 3 * (len >> 2) && dst > src - (src >> 5)) {  // quicklz.go:127-133: store
                l1_header(d, false, (uint64_t)len + 9, (uint64_t)len);
                for (int64_t q = 0; q < len; q++) d[9 + q] = s[q];
                csize[i] = (uint32_t)(len + 9);
                if (status) status[i] = QLZX_OK;
                return;
            }
            l1_put(d + cword_ptr, (cword >> 1) | 0x80000000u, 4);
            cword_ptr = dst;
            dst += 4;
            cword = 0x80000000u;
        }
        uint32_t hash = l1_bucket(fetch);
        const int64_t o = ht[hash];
        const uint32_t cache = cache_t[hash] ^ fetch;
        cache_t[hash] = fetch;
        ht[hash] = (uint32_t)src;
        const uint8_t c0 = s[src];
        const bool rle = src == o + 1 && lits >= 3 && src > 3 && c0 == s[src - 3] && c0 == s[src - 2] &&
                         c0 == s[src - 1] && c0 == s[src + 1] && c0 == s[src + 2];
        if (cache == 0 && counter[hash] != 0 && (src - o > 2 || rle)) {
            cword = (cword >> 1) | 0x80000000u;
            if (s[o + 3] != s[src + 3]) {
                const uint32_t f = 1u | (hash << 4);
                d[dst] = (uint8_t)f;
                d[dst + 1] = (uint8_t)(f >> 8);
                src += 3;
                dst += 2;
            } else {
                const int64_t old = src;
                const int64_t remaining = len - 4 - src <= 255 ? len - 4 - src : 255;
                src += 4;
                if (s[o + src - old] == s[src]) {
                    src++;
                    if (s[o + src - old] == s[src]) {
                        src++;
                        while (s[o + (src - old)] == s[src] && (src - old) < remaining) src++;
                    }
                }
                const uint32_t matchlen = (uint32_t)(src - old);
                hash <<= 4;
                if (matchlen < 18) {
                    const uint32_t f = hash | (matchlen - 2);
                    d[dst] = (uint8_t)f;
                    d[dst + 1] = (uint8_t)(f >> 8);
                    dst += 2;
                } else {
                    l1_put(d + dst, hash | (matchlen << 16), 3);
                    dst += 3;
                }
            }
            lits = 0;
            fetch = l1_rd3(s, src);
        } else {
            lits++;
            counter[hash] = 1;
            d[dst] = c0;
            cword >>= 1;
            src++;
            dst++;
            fetch = ((fetch >> 8) & 0xffffu) | ((uint32_t)s[src + 2] << 16);
        }
    }
    while (src <= len - 1) {  // quicklz.go:262-273
        if (cword & 1u) {
            l1_put(d + cword_ptr, (cword >> 1) | 0x80000000u, 4);
            cword_ptr = dst;
            dst += 4;
            cword = 0x80000000u;
        }
        d[dst++] = s[src++];
        cword >>= 1;
    }
    while ((cword & 1u) != 1u) cword >>= 1;
    l1_put(d + cword_ptr, (cword >> 1) | 0x80000000u, 4);
    l1_header(d, true, (uint64_t)dst, (uint64_t)len);
    csize[i] = (uint32_t)dst;
    if (status) status[i] = QLZX_OK;
}

}  // namespace qlzx
