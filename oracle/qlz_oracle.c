/*
 * oracle/qlz_oracle.c -- TEST INFRASTRUCTURE ONLY (see qlz_oracle.h).
 *
 * A plain-C restatement of QuickLZ 1.4.1 level 3 as gobeansdb builds it
 * (quicklz/quicklz.h:25-31: level 3, QLZ_STREAMING_BUFFER 0, not memory
 * safe) plus the record CRC32 of store/crc32.go.  Written from the format
 * description, not copied: byte streams are addressed by indices, the hash
 * table stores indices, and the decoder is bounds-checked.
 */
#include "qlz_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#define HASH_BUCKETS 4096u  /* QLZ_HASH_VALUES, quicklz.h:62 */
#define BUCKET_SLOTS 16u    /* QLZ_POINTERS, quicklz.h:61 */
#define TAIL_LITERALS 10    /* UNCONDITIONAL_MATCHLEN + UNCOMPRESSED_END, quicklz.c:24-25 */
#define MAX_OFFSET 131071u  /* quicklz.c:361 */

static inline uint32_t ld24(const uint8_t *p) { return p[0] | (p[1] << 8) | ((uint32_t)p[2] << 16); }
static inline uint32_t ld32(const uint8_t *p) {
    return p[0] | (p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
static inline void st32(uint8_t *p, uint32_t v) {
    p[0] = (uint8_t)v; p[1] = (uint8_t)(v >> 8); p[2] = (uint8_t)(v >> 16); p[3] = (uint8_t)(v >> 24);
}
/* quicklz.c:65-72 (level 3) */
static inline uint32_t bucket_of(uint32_t f) { return ((f >> 12) ^ f) & (HASH_BUCKETS - 1); }

/* quicklz.c:674-690 / quicklz.go:32-51 */
size_t orc_size_decompressed(const uint8_t *src) {
    return (src[0] & 2) ? ld32(src + 5) : src[2];
}
size_t orc_size_compressed(const uint8_t *src) {
    return (src[0] & 2) ? ld32(src + 1) : src[1];
}

/*
 * Level-3 core encoder: quicklz.c:197-227 (control words + bail-out),
 * :305-414 (candidate search, insertion, token emission), :449-494 (tail).
 * `bail_bias` = 0 gives the C rule of :218; 9 gives Go's rule
 * (quicklz.go:119 compares dst including the 9-byte header).
 * Returns the core length (>= 9) or 0 when the block is left stored.
 */
static size_t encode_core(const uint8_t *in, size_t n, uint8_t *out, uint32_t *slots,
                          uint8_t *count, size_t bail_bias) {
    const long long last_start = (long long)n - 1 - TAIL_LITERALS;
    size_t ip = 0, op = 4, cw_pos = 0;
    uint32_t cw = 0x80000000u;
    memset(count, 0, HASH_BUCKETS);

    while ((long long)ip <= last_start) {
        if (cw & 1u) {
            if (ip > 3 * (n >> 2) && op + bail_bias > ip - (ip >> 5)) return 0;
            st32(out + cw_pos, (cw >> 1) | 0x80000000u);
            cw_pos = op;
            op += 4;
            cw = 0x80000000u;
        }
        const uint32_t f = ld24(in + ip);
        const uint32_t h = bucket_of(f);
        const uint8_t c = count[h];
        size_t limit = n - 4 - ip; /* quicklz.c:310 */
        if (limit > 255) limit = 255;
        uint32_t best_len = 0;
        size_t best_pos = 0;
        for (uint32_t k = 0; k < BUCKET_SLOTS && k < c; k++) {
            const size_t o = slots[h * BUCKET_SLOTS + k];
            if (o + 2 >= ip || ld24(in + o) != f) continue; /* o < src - MINOFFSET */
            uint32_t m = 3;
            while (m < limit && in[o + m] == in[ip + m]) m++;
            if (m > best_len || (m == best_len && o > best_pos)) { best_len = m; best_pos = o; }
        }
        slots[h * BUCKET_SLOTS + (c & (BUCKET_SLOTS - 1))] = (uint32_t)ip;
        count[h] = (uint8_t)(c + 1);

        if (best_len > 2 && ip - best_pos < MAX_OFFSET) {
            /* every position inside the match is inserted (quicklz.c:366-372) */
            for (uint32_t u = 1; u < best_len; u++) {
                const uint32_t h2 = bucket_of(ld24(in + ip + u));
                const uint8_t c2 = count[h2]++;
                slots[h2 * BUCKET_SLOTS + (c2 & (BUCKET_SLOTS - 1))] = (uint32_t)(ip + u);
            }
            const uint32_t off = (uint32_t)(ip - best_pos), ml = best_len;
            cw = (cw >> 1) | 0x80000000u;
            ip += ml;
            /* token table, quicklz.c:377-406 */
            if (ml == 3 && off <= 63) {
                out[op++] = (uint8_t)(off << 2);
            } else if (ml == 3 && off <= 16383) {
                const uint32_t t = (off << 2) | 1u;
                out[op++] = (uint8_t)t; out[op++] = (uint8_t)(t >> 8);
            } else if (ml <= 18 && off <= 1023) {
                const uint32_t t = ((ml - 3) << 2) | (off << 6) | 2u;
                out[op++] = (uint8_t)t; out[op++] = (uint8_t)(t >> 8);
            } else if (ml <= 33) {
                const uint32_t t = ((ml - 2) << 2) | (off << 7) | 3u;
                out[op++] = (uint8_t)t; out[op++] = (uint8_t)(t >> 8); out[op++] = (uint8_t)(t >> 16);
            } else {
                const uint32_t t = ((ml - 3) << 7) | (off << 15) | 3u;
                st32(out + op, t);
                op += 4;
            }
        } else {
            out[op++] = in[ip++];
            cw >>= 1;
        }
    }
    while (ip < n) { /* literal tail, no hashing at level 3 */
        if (cw & 1u) {
            st32(out + cw_pos, (cw >> 1) | 0x80000000u);
            cw_pos = op;
            op += 4;
            cw = 0x80000000u;
        }
        out[op++] = in[ip++];
        cw >>= 1;
    }
    while (!(cw & 1u)) cw >>= 1;
    st32(out + cw_pos, (cw >> 1) | 0x80000000u);
    return op < 9 ? 9 : op; /* quicklz.c:493 */
}

static void put_header(uint8_t *dst, size_t hdr, int compressed, size_t csize, size_t dsize) {
    /* byte 0 = 01SSLLHC, quicklz.c:754-772 */
    if (hdr == 3) {
        dst[0] = (uint8_t)(compressed ? 1 : 0);
        dst[1] = (uint8_t)csize;
        dst[2] = (uint8_t)dsize;
    } else {
        dst[0] = (uint8_t)(2 | (compressed ? 1 : 0));
        st32(dst + 1, (uint32_t)csize);
        st32(dst + 5, (uint32_t)dsize);
    }
    dst[0] |= (uint8_t)((3 << 2) | (1 << 6));
}

static size_t compress_common(const uint8_t *src, size_t n, uint8_t *dst, int go_mode) {
    if (go_mode) {
        if (n == 0) return 0;
    } else if (n == 0 || n > 0xffffffffull - 400) {
        return 0;
    }
    const size_t hdr = (!go_mode && n < 216) ? 3 : 9; /* quicklz.c:708-711 */
    uint32_t *slots = (uint32_t *)malloc(sizeof(uint32_t) * HASH_BUCKETS * BUCKET_SLOTS);
    uint8_t *count = (uint8_t *)malloc(HASH_BUCKETS);
    memset(dst, 0, hdr + 9);
    size_t core = encode_core(src, n, dst + hdr, slots, count, go_mode ? 9 : 0);
    free(slots);
    free(count);
    if (go_mode && core == 9 && n < 5) core = n + 4; /* Go has no 9-byte core minimum */
    if (core == 0) {
        memcpy(dst + hdr, src, n);
        put_header(dst, hdr, 0, n + hdr, n);
        return n + hdr;
    }
    put_header(dst, hdr, 1, core + hdr, n);
    return core + hdr;
}

size_t orc_compress(const uint8_t *src, size_t n, uint8_t *dst) { return compress_common(src, n, dst, 0); }
size_t orc_compress_go(const uint8_t *src, size_t n, uint8_t *dst) { return compress_common(src, n, dst, 1); }

/*
 * Level-3 decoder: quicklz.c:496-672 / quicklz.go:291-431.  On every stream
 * qlz_compress (C or Go mode) can produce, the output equals the reference's.
 * Malformed input -- undefined behaviour in the reference, which is built
 * without QLZ_MEMORY_SAFE (quicklz.h:31) -- is rejected by these checks, which
 * the HIP decoders implement identically:
 *   C1 every control word is fully inside csize and has its sentinel bit 31
 *   C2 every token / literal byte lies inside csize
 *   C3 matches: 3 <= offset <= op and op + len + 4 <= dsize (quicklz.c:613-619)
 *   C4 after the first literal at op >= dsize-11 (the tail loop of
 *      quicklz.c:645-668) every further item is a literal
 *   C5 the stream ends with the item that completes dsize, except for the
 *      zero padding up to the 9-byte core minimum (quicklz.c:493)
 */
int orc_decompress(const uint8_t *src, size_t src_len, uint8_t *dst, size_t dst_cap, size_t *out_len) {
    if (src_len < 3) return ORC_E_HEADER;
    const size_t hdr = (src[0] & 2) ? 9 : 3;
    if (src_len < hdr) return ORC_E_HEADER;
    const size_t csize = orc_size_compressed(src), dsize = orc_size_decompressed(src);
    if (csize != src_len) return ORC_E_SIZE_COMPRESSED;
    if (((src[0] >> 2) & 3) != 3) return ORC_E_LEVEL;
    if (dsize > dst_cap) return ORC_E_DST_CAP;
    if (!(src[0] & 1)) {
        if (csize < hdr + dsize) return ORC_E_CORRUPT;
        memcpy(dst, src + hdr, dsize);
        *out_len = dsize;
        return ORC_OK;
    }
    size_t ip = hdr, op = 0;
    uint32_t cw = 1;
    int tail = 0;
    while (op < dsize) {
        if (cw == 1) {
            if (ip + 4 > csize) return ORC_E_CORRUPT;                       /* C1 */
            cw = ld32(src + ip);
            if (!(cw >> 31)) return ORC_E_CORRUPT;                          /* C1 */
            ip += 4;
        }
        if (ip >= csize) return ORC_E_CORRUPT;                              /* C2 */
        if (cw & 1u) {
            if (tail) return ORC_E_CORRUPT;                                 /* C4 */
            const uint32_t b0 = src[ip];
            const uint32_t tl = (b0 & 3) == 0 ? 1 : (b0 & 3) != 3 ? 2 : (b0 & 127) != 3 ? 3 : 4;
            if (ip + tl > csize) return ORC_E_CORRUPT;                      /* C2 */
            uint32_t t = 0;
            for (uint32_t k = 0; k < tl; k++) t |= (uint32_t)src[ip + k] << (8 * k);
            uint32_t off, ml;
            if ((t & 3) == 0) { off = (t & 0xff) >> 2; ml = 3; }
            else if ((t & 2) == 0) { off = (t & 0xffff) >> 2; ml = 3; }
            else if ((t & 1) == 0) { off = (t & 0xffff) >> 6; ml = ((t >> 2) & 15) + 3; }
            else if ((t & 127) != 3) { off = (t >> 7) & 0x1ffff; ml = ((t >> 2) & 0x1f) + 2; }
            else { off = t >> 15; ml = ((t >> 7) & 255) + 3; }
            ip += tl;
            if (off < 3 || off > op || op + ml + 4 > dsize) return ORC_E_CORRUPT;  /* C3 */
            for (uint32_t i = 0; i < ml; i++) dst[op + i] = dst[op - off + i];   /* forward copy */
            op += ml;
        } else {
            if ((long long)op >= (long long)dsize - 1 - TAIL_LITERALS) tail = 1;
            dst[op++] = src[ip++];
        }
        cw >>= 1;
    }
    if (!(ip == csize || (ip < hdr + 9 && csize == hdr + 9))) return ORC_E_CORRUPT;  /* C5 */
    *out_len = dsize;
    return ORC_OK;
}

/* CRC-32/IEEE reflected table (poly 0xEDB88320), as store/crc32.go:5-59 */
static uint32_t crc_table[256];
static pthread_once_t crc_once = PTHREAD_ONCE_INIT;
static void crc_init(void) {
    for (uint32_t i = 0; i < 256; i++) {
        uint32_t c = i;
        for (int k = 0; k < 8; k++) c = (c & 1) ? (c >> 1) ^ 0xEDB88320u : c >> 1;
        crc_table[i] = c;
    }
}
uint32_t orc_crc32_write(uint32_t crc, const uint8_t *buf, size_t len) {
    pthread_once(&crc_once, crc_init);
    for (size_t i = 0; i < len; i++) crc = crc_table[(crc ^ buf[i]) & 0xff] ^ (crc >> 8);
    return crc;
}

/* ---------------- synthetic workloads ---------------- */
static inline uint64_t sm64(uint64_t *s) {
    uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
uint64_t orc_block_seed(uint64_t seed, uint64_t block_id) {
    uint64_t s = seed ^ (block_id * 0xD1B54A32D192ED03ull);
    return sm64(&s);
}
static uint32_t zipf_pick(const uint32_t *cdf, uint32_t nwords, uint32_t u) {
    uint32_t lo = 0, hi = nwords - 1; /* first k with cdf[k] > u */
    while (lo < hi) {
        uint32_t mid = (lo + hi) >> 1;
        if (cdf[mid] > u) hi = mid; else lo = mid + 1;
    }
    return lo;
}
void orc_gen_text(uint64_t block_seed, const uint8_t *vocab, const uint32_t *vocab_off,
                  const uint32_t *zipf_cdf, uint32_t nwords, uint8_t *out, size_t n) {
    uint64_t s = block_seed;
    size_t p = 0;
    while (p < n) {
        const uint64_t r = sm64(&s);
        const uint32_t w = zipf_pick(zipf_cdf, nwords, (uint32_t)r);
        for (uint32_t i = vocab_off[w]; i < vocab_off[w + 1] && p < n; i++) out[p++] = vocab[i];
        if ((uint32_t)(r >> 32) % 100u < 8u) {
            if (p < n) out[p++] = '.';
        }
        if (p < n) out[p++] = ' ';
    }
}
void orc_gen_image(uint64_t block_seed, const uint8_t *vocab, const uint32_t *vocab_off,
                   const uint32_t *zipf_cdf, uint32_t nwords, uint8_t *out, size_t n) {
    uint64_t s = block_seed;
    const uint64_t kind = sm64(&s);
    if ((kind & 3) != 0) { /* 75 %: uniform random bytes */
        for (size_t p = 0; p < n; p += 8) {
            uint64_t r = sm64(&s);
            for (int b = 0; b < 8 && p + b < n; b++) out[p + b] = (uint8_t)(r >> (8 * b));
        }
        return;
    }
    /* 25 %: noisy text, 40 + (kind>>8)%6 percent of bytes replaced */
    orc_gen_text(sm64(&s), vocab, vocab_off, zipf_cdf, nwords, out, n);
    const uint32_t pct = 40u + (uint32_t)((kind >> 8) % 6u);
    for (size_t p = 0; p < n; p++) {
        const uint64_t r = sm64(&s);
        if ((uint32_t)r % 100u < pct) out[p] = (uint8_t)(r >> 32);
    }
}

/* ---------------- CPU baseline harness ---------------- */
typedef struct {
    const uint8_t *src; const uint64_t *src_off; const uint32_t *src_len;
    uint8_t *dst; const uint64_t *dst_off;
    uint32_t lo, hi; int cgo; int mode;
} job_t;

static void *run_job(void *arg) {
    job_t *j = (job_t *)arg;
    for (uint32_t i = j->lo; i < j->hi; i++) {
        const uint8_t *s = j->src + j->src_off[i];
        uint8_t *d = j->dst + j->dst_off[i];
        if (j->mode == 0) {
            size_t out = 0;
            uint8_t *tmp = d;
            if (j->cgo) tmp = (uint8_t *)malloc(orc_size_decompressed(s) + 1); /* cquicklz.go:45 */
            orc_decompress(s, j->src_len[i], tmp, orc_size_decompressed(s), &out);
            if (j->cgo) { d[0] = tmp[0]; free(tmp); }
        } else {
            if (j->cgo) { /* cquicklz.go:24-34: output + 528,400 B scratch per call */
                uint8_t *scratch = (uint8_t *)malloc(528400);
                uint8_t *tmp = (uint8_t *)malloc(j->src_len[i] + 400);
                scratch[0] = 0;
                orc_compress(s, j->src_len[i], tmp);
                d[0] = tmp[0];
                free(tmp);
                free(scratch);
            } else {
                orc_compress(s, j->src_len[i], d);
            }
        }
    }
    return NULL;
}

static double run_threads(const uint8_t *src, const uint64_t *src_off, const uint32_t *src_len,
                          uint8_t *dst, const uint64_t *dst_off, uint32_t n, int threads, int cgo,
                          int mode) {
    if (threads < 1) threads = 1;
    pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * threads);
    job_t *jobs = (job_t *)malloc(sizeof(job_t) * threads);
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (int t = 0; t < threads; t++) {
        jobs[t] = (job_t){src, src_off, src_len, dst, dst_off,
                          (uint32_t)((uint64_t)n * t / threads),
                          (uint32_t)((uint64_t)n * (t + 1) / threads), cgo, mode};
        pthread_create(&th[t], NULL, run_job, &jobs[t]);
    }
    for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    free(th);
    free(jobs);
    return (t1.tv_sec - t0.tv_sec) * 1e9 + (t1.tv_nsec - t0.tv_nsec);
}
double orc_bench_decompress(const uint8_t *src, const uint64_t *src_off, const uint32_t *src_len,
                            uint8_t *dst, const uint64_t *dst_off, uint32_t n, int threads,
                            int cgo_faithful) {
    return run_threads(src, src_off, src_len, dst, dst_off, n, threads, cgo_faithful, 0);
}
double orc_bench_compress(const uint8_t *src, const uint64_t *src_off, const uint32_t *src_len,
                          uint8_t *dst, const uint64_t *dst_off, uint32_t n, int threads,
                          int cgo_faithful) {
    return run_threads(src, src_off, src_len, dst, dst_off, n, threads, cgo_faithful, 1);
}

/* ---------------- reference timing harness ----------------
 * Times the REFERENCE codec (oracle/_ref/libqlzref.so, quicklz.c compiled from
 * /root/reference by oracle/Makefile) through the function pointers bench.py
 * passes in: qlz_decompress(src, dst, scratch) / qlz_compress(src, dst, size,
 * scratch), the calls quicklz/cquicklz.go:23-101 make.  Each thread owns the
 * reference's scratch (16 B decompress, 528,400 B compress: quicklz.h:
 * QLZ_SCRATCH_*), allocated once, as a long-lived cgo caller would. */
typedef size_t (*ref_dec_fn)(const char *, void *, char *);
typedef size_t (*ref_comp_fn)(const void *, char *, size_t, char *);
typedef struct {
    const uint8_t *src; const uint64_t *src_off; const uint32_t *src_len;
    uint8_t *dst; const uint64_t *dst_off;
    uint32_t lo, hi; void *fn; int mode;
} rjob_t;

/* mode bit 0: 0 decompress, 1 compress.  Bit 1 (cgo-faithful): every call allocates what
 * the Go wrappers allocate -- CCompress a len+400 output CArray and a 528,400-B scratch
 * (quicklz/cquicklz.go:24-34), CDecompress a dsize output CArray and a 16-B buffer
 * (cquicklz.go:45-49) -- and frees them after copying one byte out (so the call cannot be
 * elided); otherwise each thread owns one scratch and writes into dst. */
static void *run_rjob(void *arg) {
    rjob_t *j = (rjob_t *)arg;
    const int comp = j->mode & 1, cgo = (j->mode >> 1) & 1;
    char *scratch = cgo ? NULL : (char *)malloc(comp ? 528400 : 16);
    if (scratch && comp) memset(scratch, 0, 528400);
    for (uint32_t i = j->lo; i < j->hi; i++) {
        const uint8_t *s = j->src + j->src_off[i];
        uint8_t *d = j->dst + j->dst_off[i];
        if (cgo) {
            const size_t outn = comp ? (size_t)j->src_len[i] + 400 : orc_size_decompressed(s);
            uint8_t *out = (uint8_t *)malloc(outn ? outn : 1);
            char *sc = (char *)malloc(comp ? 528400 : 16);
            if (comp) ((ref_comp_fn)j->fn)(s, (char *)out, j->src_len[i], sc);
            else ((ref_dec_fn)j->fn)((const char *)s, out, sc);
            d[0] = out[0];
            free(sc);
            free(out);
        } else if (!comp) {
            ((ref_dec_fn)j->fn)((const char *)s, d, scratch);
        } else {
            ((ref_comp_fn)j->fn)(s, (char *)d, j->src_len[i], scratch);
        }
    }
    free(scratch);
    return NULL;
}

double orc_bench_ref(void *fn, const uint8_t *src, const uint64_t *src_off, const uint32_t *src_len,
                     uint8_t *dst, const uint64_t *dst_off, uint32_t n, int threads, int mode) {
    if (threads < 1) threads = 1;
    pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * threads);
    rjob_t *jobs = (rjob_t *)malloc(sizeof(rjob_t) * threads);
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (int t = 0; t < threads; t++) {
        jobs[t] = (rjob_t){src, src_off, src_len, dst, dst_off,
                           (uint32_t)((uint64_t)n * t / threads),
                           (uint32_t)((uint64_t)n * (t + 1) / threads), fn, mode};
        pthread_create(&th[t], NULL, run_rjob, &jobs[t]);
    }
    for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    free(th);
    free(jobs);
    return (t1.tv_sec - t0.tv_sec) * 1e9 + (t1.tv_nsec - t0.tv_nsec);
}

/* ---- c4 CPU baseline: the reference record loop (test infrastructure / baseline only) ----
 * One thread per range of records, each walking its range the way
 * store/bucket.go:89-117 (buildHintFromData) drives DataStreamReader.Next
 * (store/datafile.go:228-277): decode the 24-B header, CRC-verify
 * header[4:24] | key | value with the reference crc32_write (store/datafile.go:66-76,
 * 161-168), Payload.Decompress through the reference qlz_decompress when FLAG_COMPRESS
 * is set (store/item.go:163-176; cgo = 1 allocates the output as CDecompress does),
 * then Getvhash (store/item.go:89-100, utils/hash.go:8-16).  Returns the wall time in ns;
 * *bad counts records whose CRC or decompress failed (0 on a valid chunk). */
typedef uint32_t (*ref_crc_fn)(uint32_t, unsigned char *, int);
typedef struct {
    const uint8_t *data; uint64_t lo, hi; void *dec; void *crc; int cgo;
    uint64_t bad; uint32_t hsum;
} pjob_t;

static uint32_t fnv1a_sx(const uint8_t *p, size_t n) {  /* utils/hash.go:8-16 */
    uint32_t h = 0x811C9DC5u;
    for (size_t i = 0; i < n; i++) {
        h ^= (uint32_t)(int32_t)(int8_t)p[i];
        h *= 0x01000193u;
    }
    return h;
}
static uint16_t getvhash(const uint8_t *v, size_t n) {  /* store/item.go:89-100 */
    uint32_t h = (uint32_t)n * 97u;
    if (n <= 1024) h += fnv1a_sx(v, n);
    else {
        h += fnv1a_sx(v, 512);
        h *= 97u;
        h += fnv1a_sx(v + n - 512, 512);
    }
    return (uint16_t)h;
}

static void *run_pjob(void *arg) {
    pjob_t *j = (pjob_t *)arg;
    ref_crc_fn crc = (ref_crc_fn)j->crc;
    ref_dec_fn dec = (ref_dec_fn)j->dec;
    char scratch[16];
    uint8_t *reuse = (uint8_t *)malloc(64u << 20);
    uint64_t pos = j->lo;
    while (pos + 24 <= j->hi) {
        const uint8_t *h = j->data + pos;
        const uint32_t stored = ld32(h), flag = ld32(h + 8), ksz = ld32(h + 16), vsz = ld32(h + 20);
        const uint8_t *key = h + 24, *val = key + ksz;
        uint32_t c = crc(0xFFFFFFFFu, (unsigned char *)h + 4, 20);
        if (ksz) c = crc(c, (unsigned char *)key, (int)ksz);
        if (vsz) c = crc(c, (unsigned char *)val, (int)vsz);
        if (~c != stored) j->bad++;
        const uint8_t *body = val;
        size_t blen = vsz;
        uint8_t *tmp = NULL;
        if (flag & 0x10000u) {
            const size_t dsz = orc_size_decompressed(val);
            uint8_t *out = j->cgo ? (tmp = (uint8_t *)malloc(dsz ? dsz : 1)) : reuse;
            if (dec((const char *)val, out, scratch) != dsz) j->bad++;
            body = out;
            blen = dsz;
        }
        j->hsum += getvhash(body, blen);
        free(tmp);
        pos += (24 + (uint64_t)ksz + vsz + 255) & ~(uint64_t)255;
    }
    free(reuse);
    return NULL;
}

double orc_bench_replay(void *dec, void *crc, const uint8_t *data, const uint64_t *cuts, int threads, int cgo,
                        uint64_t *bad) {
    if (threads < 1) threads = 1;
    pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * threads);
    pjob_t *jobs = (pjob_t *)malloc(sizeof(pjob_t) * threads);
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (int t = 0; t < threads; t++) {
        jobs[t] = (pjob_t){data, cuts[t], cuts[t + 1], dec, crc, cgo, 0, 0};
        pthread_create(&th[t], NULL, run_pjob, &jobs[t]);
    }
    uint64_t b = 0;
    for (int t = 0; t < threads; t++) {
        pthread_join(th[t], NULL);
        b += jobs[t].bad;
    }
    clock_gettime(CLOCK_MONOTONIC, &t1);
    if (bad) *bad = b;
    free(th);
    free(jobs);
    return (t1.tv_sec - t0.tv_sec) * 1e9 + (t1.tv_nsec - t0.tv_nsec);
}
