// qlzx_decode_lane8.hip -- general-size level-3 decoder, one LANE per block,
// output written straight to the block's destination with 8-byte wild copies.
//
// This is the catch-all path: any dsize, including BodyMax = 50 MiB values
// (config/mc_config.go:7); the batch fast path (qlzx_decode_wave.hip) owns
// blocks up to QLZX_FAST_MAX_DSIZE.  Each lane walks its block's control-word /
// token chain (quicklz.c:513-671) and executes it directly: the history is the
// destination buffer itself, so a match source is an earlier part of the
// lane's own output (single-lane program order makes its earlier stores
// visible to its later loads).  One "step" = the literal run before the next
// match (<= 4 bytes, one 8-byte wild store) + that match (8-byte wild
// load/store chunks).  Bytes a wild store writes past the item's end are
// rewritten by later items, in order; no store ever leaves [0, dsize).  Rare
// cases (long literal runs, short-period overlapping matches, the last bytes of
// the block or of the stream) take the byte-serial item path, which is the
// oracle's decode loop verbatim (oracle/qlz_oracle.c:orc_decompress, checks
// C1-C5).  Header/size checks as CDecompressSafe
// (cquicklz.go:84-101); the record CRC (store/datafile.go:66-76) is continued
// over the compressed bytes before the decode, as readRecordAt verifies it
// before Payload.Decompress.
//
// As the batch path for 16 KiB blocks it is 3.4x slower than K1/K2 (every
// lane's recent output competes for L2), so it serves the large
// values only, and every block of a batch given no workspace.
#include "qlzx_device.h"

namespace qlzx {

__device__ __forceinline__ uint64_t ldu64(const uint8_t *p) { return *(const uint64_t *)p; }  // unaligned mode
__device__ __forceinline__ void stu64(uint8_t *p, uint64_t v) { *(uint64_t *)p = v; }
__device__ __forceinline__ uint32_t ldu32(const uint8_t *p) { return *(const uint32_t *)p; }

__device__ int decode_lane8(const uint8_t *src, uint32_t len, uint8_t *dst, uint64_t cap, uint32_t max_dsize,
                            uint32_t &dsize_out) {
    dsize_out = 0;
    if (len < 3) return QLZX_E_HEADER;
    const uint32_t hdr = (src[0] & 2u) ? 9u : 3u;
    if (len < hdr) return QLZX_E_HEADER;
    const Header h = parse_header(src);
    if (h.csize != len) return QLZX_E_SIZE_COMPRESSED;
    if (h.level != 3) return QLZX_E_LEVEL;
    if ((uint64_t)h.dsize > cap) return QLZX_E_DST_CAP;
    if (h.dsize > max_dsize) return QLZX_E_MAX_DSIZE;  // K1's order of checks
    const uint32_t csize = h.csize, dsize = h.dsize;
    if (!h.compressed) {  // stored block (quicklz.c:808-811)
        if ((uint64_t)csize < (uint64_t)hdr + dsize) return QLZX_E_CORRUPT;
        const uint8_t *s = src + hdr;
        uint32_t p = 0;
        for (; p + 8 <= dsize; p += 8) stu64(dst + p, ldu64(s + p));
        for (; p < dsize; p++) dst[p] = s[p];
        dsize_out = dsize;
        return QLZX_OK;
    }
    uint32_t ip = hdr, op = 0, cw = 1;
    bool tail = false;
    const int64_t tail_from = (int64_t)dsize - 1 - QLZX_TAIL;
    while (op < dsize) {
        if (cw == 1) {
            if (ip + 4 > csize) return QLZX_E_CORRUPT;  // C1
            cw = ldu32(src + ip);
            if (!(cw >> 31)) return QLZX_E_CORRUPT;      // C1: sentinel bit (quicklz.c:221)
            ip += 4;
        }
        const uint32_t r = __builtin_ctz(cw);  // literals before the next match (or the sentinel)
        if (ip + 8 <= csize && op + 24 <= dsize && r <= 4) {
            // ---- fast step: r literals (+ the match after them); C2-C4 hold by construction ----
            const uint64_t w = ldu64(src + ip);
            if (r) stu64(dst + op, w);  // wild: bytes past r are rewritten later
            op += r;
            ip += r;
            cw >>= r;
            if (cw == 1) continue;  // the run ended the group
            const uint32_t t = (uint32_t)(w >> (8 * r));
            uint32_t off, ml;
            const uint32_t tl = decode_token(t, off, ml);  // ip + tl <= ip0 + 8 <= csize (C2)
            ip += tl;
            cw >>= 1;
            if (off < 3 || off > op || op + ml + 4 > dsize) return QLZX_E_CORRUPT;  // C3
            uint8_t *d = dst + op;
            const uint8_t *s = d - off;
            if ((off >= 8 || ml <= off) && op + ((ml + 7) & ~7u) <= dsize) {
                for (uint32_t c = 0; c < ml; c += 8) stu64(d + c, ldu64(s + c));
            } else {
                for (uint32_t c = 0; c < ml; c++) d[c] = s[c];  // forward (overlapping) copy
            }
            op += ml;
            continue;
        }
        // ---- one item, byte-serial (oracle/qlz_oracle.c:orc_decompress) ----
        if (ip >= csize) return QLZX_E_CORRUPT;  // C2
        if (cw & 1u) {
            if (tail) return QLZX_E_CORRUPT;  // C4
            const uint32_t tl = token_bytes(src[ip]);
            if (ip + tl > csize) return QLZX_E_CORRUPT;  // C2
            uint32_t t = 0;
            for (uint32_t k = 0; k < tl; k++) t |= (uint32_t)src[ip + k] << (8 * k);
            uint32_t off, ml;
            ip += decode_token(t, off, ml);
            if (off < 3 || off > op || op + ml + 4 > dsize) return QLZX_E_CORRUPT;  // C3
            for (uint32_t c = 0; c < ml; c++) dst[op + c] = dst[op - off + c];
            op += ml;
        } else {
            if ((int64_t)op >= tail_from) tail = true;  // tail loop (quicklz.c:645-668)
            dst[op++] = src[ip++];
        }
        cw >>= 1;
    }
    if (!(ip == csize || (ip < hdr + 9 && csize == hdr + 9))) return QLZX_E_CORRUPT;  // C5
    dsize_out = dsize;
    return QLZX_OK;
}

// Handles blocks with min_dsize <= dsize (smaller ones belong to the fast path when it
// runs; min_dsize = 0 -> all).  A block whose header dsize exceeds the caller's max_dsize is
// not decoded: QLZX_E_MAX_DSIZE (include/qlzx.h, the batch contract), so a caller that sizes
// its destinations by max_dsize is never written past them.
__global__ void __launch_bounds__(256) k_dec_lane8(qlzx_blocks b, const uint32_t *dst_cap, uint32_t *dsize,
                                                   int32_t *status, const uint32_t *crc_state,
                                                   const uint32_t *crc_expect, uint32_t *crc_out,
                                                   uint32_t min_dsize, uint32_t max_dsize) {
    __shared__ uint32_t tab[256];
    load_crc_table(tab);
    __syncthreads();
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= b.n) return;
    const uint8_t *src = b.src + b.src_off[i];
    const uint32_t len = b.src_len[i];
    if (min_dsize) {  // header errors of fast-path batches are reported by K1
        if (len < 3) return;
        const uint32_t hb = (src[0] & 2u) ? 9u : 3u;
        if (len < hb || parse_header(src).dsize < min_dsize) return;  // owned by the fast path
    }
    int st = QLZX_OK;
    if (crc_state || crc_expect || crc_out) {  // record CRC over the stored (compressed) value bytes
        uint32_t c = crc_state ? crc_state[i] : 0xffffffffu;
        uint32_t k = 0;
        for (; k + 4 <= len; k += 4) c = crc_word(tab, c, ldu32(src + k));
        for (; k < len; k++) c = crc_byte(tab, c, src[k]);
        c = ~c;
        if (crc_out) crc_out[i] = c;
        if (crc_expect && c != crc_expect[i]) st = QLZX_E_CRC;  // store/datafile.go:161-168: before decode
    }
    uint32_t ds = 0;
    if (st == QLZX_OK) st = decode_lane8(src, len, b.dst + b.dst_off[i], dst_cap ? dst_cap[i] : ~0ull, max_dsize, ds);
    if (dsize) dsize[i] = ds;
    status[i] = st;
}

}  // namespace qlzx
