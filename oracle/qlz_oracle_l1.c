/*
 * oracle/qlz_oracle_l1.c -- TEST INFRASTRUCTURE ONLY (see qlz_oracle.h).
 *
 * The level-1 branch of gobeansdb's Go QuickLZ (quicklz/quicklz.go, a translation of
 * QuickLZ.java 1.5.0): Compress(src, 1) (quicklz.go:80-191 plus the shared tail
 * 262-289) and Decompress of level-1 and stored streams (quicklz.go:291-431).  Restated
 * from the Go source with index arithmetic; production gobeansdb writes level 3 only
 * (cquicklz.go), so this path serves the Go API surface.
 *
 * Go bounds-checks every slice access and panics on a violation.  The decoder here
 * returns ORC_E_CORRUPT exactly where Go Decompress would panic (index out of range
 * on the source or the destination), and reads of destination bytes not yet written
 * see 0, as Go's make([]byte, size) does.
 */
#include <stdlib.h>
#include <string.h>

#include "qlz_oracle.h"

#define L1_HASH 4096
#define L1_HDR 9
#define L1_CWORD 4

static inline uint32_t bucket1(uint32_t f) { return ((f >> 12) ^ f) & (L1_HASH - 1); }

static void put_le(uint8_t *p, uint64_t v, int n) {
    for (int j = 0; j < n; j++) p[j] = (uint8_t)(v >> (8 * j));
}

/* quicklz.go:66-78 writeHeader(dst, level, compressible, sizeCompressed, sizeDecompressed):
 * bytes 1..4 get the 4th argument's value and 5..8 the 5th's (the call sites pass them
 * so that 1..4 holds the compressed and 5..8 the decompressed size). */
static void go_header(uint8_t *d, int level, int compressible, uint64_t at1, uint64_t at5) {
    d[0] = (uint8_t)(2 | (compressible ? 1 : 0) | (level << 2) | (1 << 6));
    put_le(d + 1, at1, 4);
    put_le(d + 5, at5, 4);
}

static inline uint32_t rd3(const uint8_t *s, size_t i) {
    return s[i] | ((uint32_t)s[i + 1] << 8) | ((uint32_t)s[i + 2] << 16);
}

size_t orc_compress_go_l1(const uint8_t *s, size_t n, uint8_t *d) {
    if (n == 0) return 0; /* quicklz.go:109-111: nil */
    int32_t *hashtable = calloc(L1_HASH, sizeof(int32_t));
    uint32_t *cachetable = calloc(L1_HASH, sizeof(uint32_t));
    uint8_t *counter = calloc(L1_HASH, 1);
    const int64_t len = (int64_t)n;
    int64_t src = 0, dst = L1_HDR + L1_CWORD, cword_ptr = L1_HDR, lits = 0;
    uint32_t cword = 0x80000000u, fetch = 0;
    const int64_t last_match_start = len - 6 - 4 - 1; /* UNCONDITIONAL_MATCHLEN, UNCOMPRESSED_END */
    size_t out = 0;
    memset(d, 0, n + 400);
    if (src <= last_match_start) fetch = rd3(s, 0);
    while (src <= last_match_start) {
        if (cword & 1u) {
            if (src > 3 * (len >> 2) && dst > src - (src >> 5)) { /* quicklz.go:127-133: stored */
                go_header(d, 1, 0, (uint64_t)len + L1_HDR, (uint64_t)len);
                memcpy(d + L1_HDR, s, n);
                out = n + L1_HDR;
                goto done;
            }
            put_le(d + cword_ptr, (cword >> 1) | 0x80000000u, 4);
            cword_ptr = dst;
            dst += L1_CWORD;
            cword = 0x80000000u;
        }
        uint32_t hash = bucket1(fetch);
        const int64_t o = hashtable[hash];
        const uint32_t cache = cachetable[hash] ^ fetch;
        cachetable[hash] = fetch;
        hashtable[hash] = (int32_t)src;
        const int rle = src == o + 1 && lits >= 3 && src > 3 && s[src] == s[src - 3] && s[src] == s[src - 2] &&
                        s[src] == s[src - 1] && s[src] == s[src + 1] && s[src] == s[src + 2];
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
                int64_t remaining = 255;
                if (len - 4 - src <= 255) remaining = len - 4 - src;
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
                    put_le(d + dst, hash | (matchlen << 16), 3);
                    dst += 3;
                }
            }
            lits = 0;
            fetch = rd3(s, (size_t)src);
        } else {
            lits++;
            counter[hash] = 1;
            d[dst] = s[src];
            cword >>= 1;
            src++;
            dst++;
            fetch = ((fetch >> 8) & 0xffffu) | ((uint32_t)s[src + 2] << 16);
        }
    }
    while (src <= len - 1) { /* quicklz.go:262-273 */
        if (cword & 1u) {
            put_le(d + cword_ptr, (cword >> 1) | 0x80000000u, 4);
            cword_ptr = dst;
            dst += L1_CWORD;
            cword = 0x80000000u;
        }
        d[dst++] = s[src++];
        cword >>= 1;
    }
    while ((cword & 1u) != 1u) cword >>= 1;
    put_le(d + cword_ptr, (cword >> 1) | 0x80000000u, 4);
    go_header(d, 1, 1, (uint64_t)dst, (uint64_t)len);
    out = (size_t)dst;
done:
    free(hashtable);
    free(cachetable);
    free(counter);
    return out;
}

/* Go Decompress (quicklz.go:291-431) for stored streams of any level and compressed
 * level-1 streams; compressed level-3 streams are orc_decompress's.  On success *out_len
 * = SizeDecompressed and dst[0, *out_len) is the result. */
int orc_decompress_go_l1(const uint8_t *s, size_t slen, uint8_t *dst, size_t dst_cap, size_t *out_len) {
    *out_len = 0;
    if (slen < 1) return ORC_E_HEADER;
    const size_t hdr = (s[0] & 2) ? 9 : 3;
    if (slen < hdr) return ORC_E_HEADER; /* SizeDecompressed indexes past the buffer */
    const int64_t size = (int64_t)orc_size_decompressed(s);
    const int level = (s[0] >> 2) & 3;
    if (level != 1 && level != 3) return ORC_E_LEVEL;
    if ((uint64_t)size > dst_cap) return ORC_E_DST_CAP;
    memset(dst, 0, (size_t)size);
    if ((s[0] & 1) != 1) { /* quicklz.go:310-314: copy() takes min(size, len - hdr) */
        const size_t k = slen - hdr < (size_t)size ? slen - hdr : (size_t)size;
        memcpy(dst, s + hdr, k);
        *out_len = (size_t)size;
        return ORC_OK;
    }
    if (level != 1) return ORC_E_LEVEL;
    int32_t *ht = calloc(L1_HASH, sizeof(int32_t));
    const int64_t n = (int64_t)slen;
    int64_t src = (int64_t)hdr, d = 0, last_hashed = -1;
    const int64_t last_match_start = size - 11;
    uint64_t cword = 1;
    uint32_t fetch = 0;
    int st = ORC_E_CORRUPT;
#define NEED_SRC(i) do { if ((i) < 0 || (i) >= n) goto out; } while (0)
#define NEED_DST(i) do { if ((i) < 0 || (i) >= size) goto out; } while (0)
    for (;;) {
        if (cword == 1) {
            NEED_SRC(src + 3);
            cword = (uint64_t)s[src] | ((uint64_t)s[src + 1] << 8) | ((uint64_t)s[src + 2] << 16) |
                    ((uint64_t)s[src + 3] << 24);
            src += 4;
            if (d <= last_match_start) {
                NEED_SRC(src + 2);
                fetch = rd3(s, (size_t)src);
            }
        }
        if (cword & 1) {
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
            /* destination[dst+0..2] = destination[offset2+0..2], then i = 3..matchlen-1 */
            const int64_t ncopy = matchlen > 3 ? matchlen : 3;
            for (int64_t i = 0; i < ncopy; i++) {
                NEED_DST(off2 + i);
                NEED_DST(d + i);
                dst[d + i] = dst[off2 + i];
            }
            d += matchlen;
            NEED_DST(last_hashed + 3);
            fetch = rd3(dst, (size_t)(last_hashed + 1));
            while (last_hashed < d - matchlen) {
                last_hashed++;
                hash = bucket1(fetch);
                ht[hash] = (int32_t)last_hashed;
                NEED_DST(last_hashed + 3);
                fetch = ((fetch >> 8) & 0xffffu) | ((uint32_t)dst[last_hashed + 3] << 16);
            }
            NEED_SRC(src + 2);
            fetch = rd3(s, (size_t)src);
            last_hashed = d - 1;
        } else if (d <= last_match_start) {
            NEED_SRC(src);
            NEED_DST(d);
            dst[d++] = s[src++];
            cword >>= 1;
            while (last_hashed < d - 3) {
                last_hashed++;
                const uint32_t f2 = rd3(dst, (size_t)last_hashed);
                ht[bucket1(f2)] = (int32_t)last_hashed;
            }
            NEED_SRC(src + 2);
            fetch = ((fetch >> 8) & 0xffffu) | ((uint32_t)s[src + 2] << 16);
        } else {
            while (d <= size - 1) {
                if (cword == 1) {
                    src += L1_CWORD;
                    cword = 0x80000000u;
                }
                NEED_SRC(src);
                dst[d++] = s[src++];
                cword >>= 1;
            }
            *out_len = (size_t)size;
            st = ORC_OK;
            goto out;
        }
    }
#undef NEED_SRC
#undef NEED_DST
out:
    free(ht);
    return st;
}
