/*
 * include/qlzx.h -- C ABI of libqlzx.so, the MI355X (gfx950) QuickLZ level-3
 * codec + record CRC32 for gobeansdb.
 *
 * Two layers:
 *
 * 1. Drop-in symbols.  cgo compiles every .c of quicklz/ and includes
 *    quicklz.h (quicklz/cquicklz.go:3-8), so a drop-in replacement exports
 *    exactly the quicklz.h surface with identical semantics.  Each entry
 *    below names the reference function it replaces.  These run on the GPU
 *    (a batch of one, staged through pinned memory by the host runtime);
 *    there is no CPU codec in this library.
 *
 * 2. Batch device API (qlzx_*).  Thousands of independent value blocks per
 *    launch, device-resident inputs/outputs, per-block status.  All pointers
 *    are device pointers; `stream` is a hipStream_t (NULL = default stream).
 *    Nothing here allocates: callers pass a workspace sized by the matching
 *    *_workspace_size() call, so launches are graph-capturable.
 *
 * Status codes reproduce the reference wrapper errors and add the
 * memory-safety checks the reference leaves out (quicklz.h:31 builds without
 * QLZ_MEMORY_SAFE).
 */
#ifndef QLZX_H
#define QLZX_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---------------- layer 1: quicklz.h drop-in ---------------- */

/* quicklz/quicklz.c:674-681 -- dsize from the 3/9-byte header. */
size_t qlz_size_decompressed(const char *source);
/* quicklz/quicklz.c:683-690 -- csize (header included). */
size_t qlz_size_compressed(const char *source);
/* quicklz/quicklz.c:777-836 -- decompress one block; returns dsize.
 * `scratch_decompress` (>= 16 B, QLZ_SCRATCH_DECOMPRESS) is accepted and unused.
 * A corrupt stream returns 0 instead of the reference's undefined behaviour
 * (qlzx_last_status() says why).
 * Fail-stop: the three GPU-backed drop-ins (qlz_decompress, qlz_compress,
 * crc32_write) have no error channel in their callers (quicklz/cquicklz.go:38-40,
 * store/crc32.go:81-84), so a runtime failure (no device, a HIP error) prints
 * qlzx_last_error() to stderr and abort()s instead of returning a wrong value. */
size_t qlz_decompress(const char *source, void *destination, char *scratch_decompress);
/* quicklz/quicklz.c:692-775 -- compress one block (level 3); returns csize,
 * 0 if size == 0 or size > 0xffffffff-400.  destination >= size + 400 bytes.
 * `scratch_compress` (>= 528400 B, QLZ_SCRATCH_COMPRESS) is accepted and unused. */
size_t qlz_compress(const void *source, char *destination, size_t size, char *scratch_compress);
/* quicklz/quicklz.c:31-58 -- 0:3 1:528400 2:16 3:0 6:0 7:1 8:4 9:1, else -1. */
int qlz_get_setting(int setting);
/* store/crc32.go:61-68 -- raw reflected CRC-32/IEEE table update (no
 * pre/post inversion; the Go wrapper applies ~ at store/crc32.go:78,87). */
uint32_t crc32_write(uint32_t crc, unsigned char *buf, int len);

/* ---------------- layer 2: batch device API ---------------- */

enum qlzx_status {
    QLZX_OK = 0,
    QLZX_E_SIZE_COMPRESSED = 1, /* header csize != src_len   (quicklz/cquicklz.go:90-94) */
    QLZX_E_CORRUPT = 2,         /* stream fails the QLZ_MEMORY_SAFE checks (quicklz.c:519-657) */
    QLZX_E_LEVEL = 3,           /* header level != 3 (quicklz.go:304-308 panics) */
    QLZX_E_DST_CAP = 4,         /* dsize > dst capacity (cquicklz.go:45 allocates exactly dsize) */
    QLZX_E_CRC = 5,             /* record CRC mismatch (store/datafile.go:161-168) */
    QLZX_E_HEADER = 6,          /* src_len shorter than the header */
    QLZX_E_EMPTY = 7,           /* compress of an empty value (cquicklz.go:36 panics) */
    QLZX_E_TOO_LARGE = 8,       /* compress size > 0xffffffff-400 (quicklz.c:705) */
    QLZX_E_MAX_DSIZE = 9,       /* dsize > the batch's max_dsize argument (caller contract) */
    QLZX_E_RUNTIME = 10         /* single call: no result, the GPU runtime failed (qlzx_last_error) */
};

enum qlzx_return {
    QLZX_R_OK = 0,
    QLZX_R_BAD_ARG = -1,
    QLZX_R_WORKSPACE = -2,      /* workspace too small */
    QLZX_R_HIP = -3,            /* a HIP runtime call failed */
    QLZX_R_NO_DEVICE = -4
};

/*
 * Blocks are addressed by byte offsets into one base buffer each side:
 * block i = src[src_off[i] .. src_off[i]+src_len[i]).
 */
typedef struct qlzx_blocks {
    const uint8_t *src;
    const uint64_t *src_off;
    const uint32_t *src_len;
    uint8_t *dst;
    const uint64_t *dst_off;
    uint32_t n;
} qlzx_blocks;

/* Decompress: replaces CDecompressSafe (quicklz/cquicklz.go:84-101) per block.
 *   dst_cap[i]   capacity of block i's destination (nullable: unbounded)
 *   dsize[i]     out: decompressed size (0 on error)             (nullable)
 *   status[i]    out: enum qlzx_status                           (required)
 *   crc_state[i] in: raw CRC state after header[4:24] ‖ key (store/datafile.go:66-72);
 *                nullable = no CRC
 *   crc_expect[i] in: stored record CRC (header[0:4]); nullable = no check
 *   crc_out[i]   out: ~crc_write(crc_state, compressed value)    (nullable)
 *   max_dsize    upper bound on dsize over the batch (selects kernels; blocks
 *                above the fast-path limit take the general kernel).  A block whose
 *                header dsize exceeds it is not decoded: status QLZX_E_MAX_DSIZE.
 * The record CRC is computed over the compressed bytes in the same pass that
 * decodes them (fused).
 * Values over 64 KiB (max_dsize > 65536): the batch decoder decodes every block up to 64 KiB
 * asynchronously, then each larger block in its own whole-GPU pass, one block at a time; that
 * phase reads counts back and synchronises `stream` several times per large block, so the call
 * returns only after it (blocks up to 64 KiB never do).  The workspace then also holds the
 * whole-GPU decoder's scratch: about 31.7 x max_dsize bytes (8 u16 jump levels over 1.5 x
 * max_dsize plus a u32 source index per output byte), e.g. 1.66 GB at the 50 MiB body limit.
 * qlzx_decompress_workspace_size includes it; size max_dsize from the largest header dsize
 * actually pending (as replay does), not from a configured bound.
 * Workspace of the batch decoder itself: one region per chunk in flight -- 1 for a call of one
 * chunk, 2 when K1 of the next chunk overlaps K2 of this one, 3 for calls of values over 16 KiB
 * in three chunks or more (the last chunk's K1 starts first).  A smaller workspace (at least one
 * region) still decodes, with less overlap. */
size_t qlzx_decompress_workspace_size(uint32_t n, uint32_t max_dsize);
int qlzx_decompress_batch(const qlzx_blocks *b, const uint32_t *dst_cap, uint32_t *dsize,
                          int32_t *status, const uint32_t *crc_state, const uint32_t *crc_expect,
                          uint32_t *crc_out, uint32_t max_dsize, void *workspace,
                          size_t workspace_bytes, void *stream);

/* Compress: replaces CCompress (quicklz/cquicklz.go:23-42) per block.
 *   dst capacity per block must be >= src_len[i] + 400 (cquicklz.go:24).  The encoder may
 *                write anywhere in [0, src_len[i] + 400) of a destination (a speculative
 *                stored copy lands there before the parse decides); only [0, csize[i]) is
 *                the result, the bytes past it are unspecified.
 *   csize[i]     out: compressed size (0 + status on error)      (required)
 *   status[i]    out: enum qlzx_status                           (nullable)
 *   crc_state / crc_out: as above, over the *compressed* output (the value
 *   bytes of the record written by store/datafile.go:307-330).  Fused.
 *   max_len      upper bound on src_len over the batch
 * Values over 64 KiB (max_len > 65536) are encoded by a whole-GPU pass each, one at a time,
 * after the batch's smaller blocks; like the decoder, that phase synchronises `stream` several
 * times per large block, and the workspace grows by about 76 x max_len bytes (jump levels, sort
 * keys and scans; 3.99 GB at 50 MiB), included in qlzx_compress_workspace_size. */
#define QLZX_F_GO_COMPAT 1u /* Go quicklz.Compress(src, 3) output (quicklz.go:80-289): always a
                              9-byte header, bail-out counts the header, no 9-byte core minimum */
size_t qlzx_compress_workspace_size(uint32_t n, uint32_t max_len);
int qlzx_compress_batch(const qlzx_blocks *b, uint32_t *csize, int32_t *status,
                        const uint32_t *crc_state, uint32_t *crc_out, uint32_t max_len,
                        uint32_t flags, void *workspace, size_t workspace_bytes, void *stream);

#define QLZX_F_LEVEL1 2u    /* Go quicklz.Compress(src, 1) (quicklz.go:80-191): qlzx_compress1 only */

/* Single-block helper on the GPU with `flags` (used by the quicklz.Compress mirror);
 * same contract as qlz_compress. */
size_t qlzx_compress1(const void *source, char *destination, size_t size, uint32_t flags);

/* ---- Go quicklz level 1 (quicklz.go:80-191 and 291-431) ----
 * One lane per block with its hash tables in `workspace` (16-B aligned,
 * qlzx_go_l1_workspace_size(n) bytes for compress, qlzx_go_decompress_workspace_size(n)
 * for decompress; both bounded: launches of at most 65536 blocks reuse them).  Production gobeansdb writes level 3 through
 * cgo; these serve the Go Compress(src, 1) / Decompress surface.
 * compress:   dst capacity >= src_len + 400 per block; empty block -> QLZX_E_EMPTY
 *             (Go returns nil); output bytes = Go Compress(src, 1).
 * decompress: Go Decompress of stored streams (any level) and compressed level-1
 *             streams; QLZX_E_CORRUPT where Go would panic on an index, QLZX_E_LEVEL
 *             for compressed level 3 (use qlzx_decompress_batch) and levels 0/2. */
size_t qlzx_go_l1_workspace_size(uint32_t n);
int qlzx_go_l1_compress_batch(const qlzx_blocks *b, uint32_t *csize, int32_t *status, void *workspace,
                              size_t workspace_bytes, void *stream);
int qlzx_go_decompress_batch(const qlzx_blocks *b, const uint32_t *dst_cap, uint32_t *dsize, int32_t *status,
                             void *workspace, size_t workspace_bytes, void *stream);
/* Workspace of qlzx_go_decompress_batch (the decoder needs only the 16 KiB hashtable per
 * block; launches cover at most 65536 blocks and reuse it). */
size_t qlzx_go_decompress_workspace_size(uint32_t n);
/* Single-block Go Decompress of a stored or level-1 stream of source_len bytes into
 * destination (capacity dst_cap): returns the decompressed size (0 is a valid empty
 * result), QLZX_GO_ERROR on error; qlzx_last_status() then holds the block's
 * enum qlzx_status (QLZX_E_CORRUPT where Go panics) and qlzx_last_error() the reason. */
#define QLZX_GO_ERROR ((size_t)-1)
size_t qlzx_go_decompress1(const char *source, size_t source_len, void *destination, size_t dst_cap);

/* CRC32 of many buffers: out[i] = crc32_write(init ? init[i] : 0xffffffff, src_i) ^ (final_xor).
 * final_xor = 0 returns the raw state; 0xffffffff the store/crc32.go get() value. */
int qlzx_crc32_batch(const uint8_t *src, const uint64_t *src_off, const uint32_t *src_len,
                     uint32_t n, const uint32_t *init, uint32_t final_xor, uint32_t *out,
                     void *stream);

/* Synthetic workloads: block i = gen(seed, first_id + i) of src_len[i] bytes
 * written at dst + dst_off[i].  kind 0 = text-like, 1 = image-like.  Tables come from
 * gobeansdb_amd/synth.py (vocab bytes, vocab offsets[nwords+1], zipf cdf[nwords]). */
int qlzx_synth_batch(int kind, uint64_t seed, uint64_t first_id, uint8_t *dst,
                     const uint64_t *dst_off, const uint32_t *len, uint32_t n,
                     const uint8_t *vocab, const uint32_t *vocab_off, const uint32_t *zipf_cdf,
                     uint32_t nwords, void *stream);

/* ---- write-side record encode ----
 * Record CRC = ~crc_write(~0, header[4:24] ‖ key ‖ value) (store/datafile.go:66-88).
 * qlzx_compress_batch fuses the value's raw CRC (crc_state = 0, crc_out = ~raw);
 * this folds the header+key prefix in afterwards:
 *   out[i] = (raw_a[i] * x^(8 len_b[i]) ^ raw_b[i]) ^ final_xor
 * i.e. the raw state of A ‖ B from the raw state of A and the raw CRC (from 0) of B. */
int qlzx_crc32_combine(const uint32_t *raw_a, const uint32_t *raw_b, const uint32_t *len_b, uint32_t n,
                       uint32_t final_xor, uint32_t *out, void *stream);
/* dst[dst_off[i] ..+ len[i]) = src[src_off[i] ..+ len[i]) (record assembly, WriteRecord.append). */
int qlzx_copy_batch(const uint8_t *src, const uint64_t *src_off, const uint32_t *len, uint8_t *dst,
                    const uint64_t *dst_off, uint32_t n, void *stream);

/* ---- .data chunk replay ----
 * Replaces the DataStreamReader.Next loop of buildHintFromData
 * (store/datafile.go:202-277, store/bucket.go:89-117) over one chunk file that
 * is resident in device memory: the records the sequential reader would
 * return from `start` (a multiple of 256), in order, each with its offset and
 * sizeBroken (bytes skipped by the nextValid resync).  CRCs are verified
 * (store/datafile.go:161-168) as part of record discovery.
 *   max_key  MaxKeyLen (config/mc_config.go:6, 250); body_max BodyMax (50 MiB)
 *   rec_off / rec_broken: capacity size/256 + 1 entries
 *   result[0] = records found; result[1] = 1 if the reader stops on an error
 *   (unexpected EOF: partial header or truncated record) after them;
 *   result[2] = header-plausible slots, result[3] = CRC-valid slots. */
size_t qlzx_replay_workspace_size(uint64_t size);
int qlzx_replay_index(const uint8_t *data, uint64_t size, uint64_t start, uint32_t max_key, uint64_t body_max,
                      uint64_t *rec_off, uint32_t *rec_broken, uint32_t *result, void *workspace,
                      size_t workspace_bytes, void *stream);

/* Around the batch decoder (Payload.Decompress of the FLAG_COMPRESS records, store/item.go:163-176),
 * without host parsing.  `result` is qlzx_replay_index's (result[0] = n records); `cap` the
 * capacity of rec_off and of every per-record array below.
 * qlzx_replay_plan: hdr[6 j..] = the 24-B header of record j (crc, ts, flag, ver, ksz, vsz); the
 *   compressed records in record order: comp_idx (record), comp_off/comp_len (body in `data`),
 *   comp_dsize (QuickLZ header dsize, quicklz.go:32-44; 0 if the body is shorter than a header),
 *   comp_dst_off (256-B-aligned offsets in one packed output buffer);
 *   totals[5] = {n, ncomp, max dsize, output bytes (lo, hi)} -- the only values a caller needs on
 *   the host (to size the output buffer and the decoder launch).
 * qlzx_replay_finish: after qlzx_decompress_batch over the ncomp compressed records (comp_status,
 *   comp_dsize = its dsize output): per record the flag (FLAG_COMPRESS cleared when the value
 *   decoded), value_len, where the value lives (in_out 1: outbuf + val_off, 0: data + val_off; a
 *   failed decode keeps the raw body, as the reference swallows the error) and Getvhash. */
size_t qlzx_replay_plan_workspace_size(uint32_t cap);
int qlzx_replay_plan(const uint8_t *data, const uint64_t *rec_off, const uint32_t *result, uint32_t cap,
                     int32_t *hdr, uint32_t *comp_idx, uint64_t *comp_off, uint32_t *comp_len, uint32_t *comp_dsize,
                     uint64_t *comp_dst_off, uint32_t *totals, void *workspace, size_t workspace_bytes, void *stream);
int qlzx_replay_finish(const uint8_t *data, const uint64_t *rec_off, const uint32_t *result, const uint32_t *totals,
                       const uint32_t *comp_idx, const int32_t *comp_status, const uint32_t *comp_dsize,
                       const uint64_t *comp_dst_off, const uint8_t *outbuf, uint32_t cap, int32_t *flag,
                       int32_t *value_len, uint8_t *in_out, uint64_t *val_off, uint16_t *vhash, void *stream);

/* Getvhash (store/item.go:89-100, Fnv1a of utils/hash.go:8-16) of n values. */
int qlzx_vhash_batch(const uint8_t *src, const uint64_t *off, const uint32_t *len, uint32_t n, uint16_t *out,
                     void *stream);

/* enum qlzx_status of the calling thread's last single-block call (qlz_decompress,
 * qlzx_compress1, qlzx_go_decompress1). */
int qlzx_last_status(void);

/* Last error message of the calling thread (empty if none). */
const char *qlzx_last_error(void);

/* One record read in ONE request, as readRecordAt + Payload.Decompress use it
 * (store/datafile.go:161-168, store/item.go:163-176): the record CRC continued from `crc_state`
 * (crc32_write from ~0 over header[4:24] then the key) over the `vlen` value bytes is checked
 * against the stored `crc_expect` (~state == crc_expect), and only then, when `compressed`
 * (FLAG_COMPRESS), the value is decompressed into dst (dst_cap >= its dsize).  Replaces the
 * value's crc32_write and the qlz_decompress of the same GET (two GPU round trips) with one.
 * *status: QLZX_OK, QLZX_E_CRC (nothing decoded), or the decode status; *out_len: the value's
 * length after the step (vlen when not compressed, which is not copied).  Returns a qlzx_return
 * code (runtime failure). */
int qlzx_read_record1(const void *value, size_t vlen, uint32_t crc_state, uint32_t crc_expect, int compressed,
                      void *dst, size_t dst_cap, size_t *out_len, int32_t *status);

/* Library/version info: fills `buf` with a short description (arch, kernels, source hash). */
int qlzx_info(char *buf, size_t len);

/* INTERNAL test hook, inert unless the process was started with QLZX_TEST_HOOKS=1 (read once;
 * otherwise it returns QLZX_R_BAD_ARG and changes nothing).
 * For the request path behind the drop-ins (values <= 64 KiB): the next batch the
 * current device's service launches fails -- mode 1: its kernel runs but publishes no
 * completion (caught through the batch event), mode 2: the launch itself fails.  Every request
 * of that batch then fails with QLZX_R_HIP (qlzx_compress1 returns 0, the quicklz.h drop-ins
 * stop the process).  For qlzx_decompress_batch: mode 3 / 4 makes its next K1 / K2 launch fail,
 * and the call returns QLZX_R_HIP.  Returns a qlzx_return code. */
int qlzx_service_test_fault(int mode);

#ifdef __cplusplus
}
#endif
#endif
