/*
 * oracle/qlz_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the gobeansdb QuickLZ (1.4.1, level 3, streaming off)
 * codec and record CRC32.  It is the parity checker for the HIP product
 * path and the CPU baseline timed by bench.py's cpu_baseline leg.  Only
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline may load it;
 * the product library (gobeansdb_amd/) never links or calls it.
 *
 * Pinned against: the reference quicklz.c compiled from /root/reference
 * (oracle/_ref, see oracle/Makefile) through the golden vectors under
 * tests/golden/, the Go KAT in quicklz/quicklz_test.go:9-14, and
 * zlib.crc32 == store/crc32.go:61-68 (+ the ~0 init / final xor of
 * store/crc32.go:77-88).
 */
#ifndef QLZ_ORACLE_H
#define QLZ_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* status codes shared with the HIP path (include/qlzx.h) */
#define ORC_OK 0
#define ORC_E_SIZE_COMPRESSED 1 /* header csize != buffer length (cquicklz.go:90-94) */
#define ORC_E_CORRUPT 2         /* stream fails QLZ_MEMORY_SAFE checks (quicklz.c:519-657) */
#define ORC_E_LEVEL 3           /* header level is not 3 */
#define ORC_E_DST_CAP 4         /* dsize exceeds destination capacity */
#define ORC_E_HEADER 6          /* buffer shorter than the header it announces */

size_t orc_size_decompressed(const uint8_t *src);
size_t orc_size_compressed(const uint8_t *src);

/* C-library semantics (quicklz.c:692-775).  dst must hold n + 400 bytes and
 * is zero-filled up to the 9-byte core minimum, so outputs of < 5-byte
 * inputs are deterministic.  Returns the compressed size, 0 on error. */
size_t orc_compress(const uint8_t *src, size_t n, uint8_t *dst);

/* Go quicklz.Compress(src, 3) semantics (quicklz.go:80-289): always a
 * 9-byte header, bail-out compares dst *including* the header, and empty
 * input returns 0 (nil).  dst must hold n + 400 bytes. */
size_t orc_compress_go(const uint8_t *src, size_t n, uint8_t *dst);

/* Go quicklz.Compress(src, 1) (quicklz.go:80-191,262-289; qlz_oracle_l1.c).  dst must hold
 * n + 400 bytes.  Returns the compressed size, 0 (nil) for empty input. */
size_t orc_compress_go_l1(const uint8_t *src, size_t n, uint8_t *dst);

/* Go quicklz.Decompress (quicklz.go:291-431) of a stored stream (any level) or a compressed
 * level-1 stream; ORC_E_CORRUPT where Go panics on an index, ORC_E_LEVEL for compressed
 * level 3 (orc_decompress) and levels other than 1/3. */
int orc_decompress_go_l1(const uint8_t *src, size_t src_len, uint8_t *dst, size_t dst_cap, size_t *out_len);

/* Memory-safe level-3 decoder.  On valid streams the output equals
 * qlz_decompress (quicklz.c:777-836) and Go Decompress (quicklz.go:291-431).
 * Returns a status code; *out_len receives dsize on success. */
int orc_decompress(const uint8_t *src, size_t src_len, uint8_t *dst,
                   size_t dst_cap, size_t *out_len);

/* store/crc32.go:61-68: raw table update, no pre/post inversion. */
uint32_t orc_crc32_write(uint32_t crc, const uint8_t *buf, size_t len);

/* --- synthetic workloads (spec in DESIGN.md §5) --- */
uint64_t orc_block_seed(uint64_t seed, uint64_t block_id);
void orc_gen_text(uint64_t block_seed, const uint8_t *vocab, const uint32_t *vocab_off,
                  const uint32_t *zipf_cdf, uint32_t nwords, uint8_t *out, size_t n);
void orc_gen_image(uint64_t block_seed, const uint8_t *vocab, const uint32_t *vocab_off,
                   const uint32_t *zipf_cdf, uint32_t nwords, uint8_t *out, size_t n);

/* cpu baseline: compress/decompress a batch with T threads; returns ns */
double orc_bench_decompress(const uint8_t *src, const uint64_t *src_off,
                            const uint32_t *src_len, uint8_t *dst,
                            const uint64_t *dst_off, uint32_t n, int threads,
                            int cgo_faithful);
double orc_bench_compress(const uint8_t *src, const uint64_t *src_off,
                          const uint32_t *src_len, uint8_t *dst,
                          const uint64_t *dst_off, uint32_t n, int threads,
                          int cgo_faithful);
/* times the reference codec through fn (qlz_decompress when mode 0, qlz_compress when 1) */
double orc_bench_ref(void *fn, const uint8_t *src, const uint64_t *src_off, const uint32_t *src_len,
                     uint8_t *dst, const uint64_t *dst_off, uint32_t n, int threads, int mode);

#ifdef __cplusplus
}
#endif
#endif
