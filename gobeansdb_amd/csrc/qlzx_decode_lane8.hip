// qlzx_decode_lane8.hip -- batched level-3 decoder, one LANE per block, output
// written straight to the block's destination in HBM with 8-byte wild copies.
//
// Each lane walks its block's control-word/token chain (quicklz.c:513-671) and
// executes it directly: the history is the destination buffer itself, so a
// match source is an earlier part of the lane's own output (single-lane
// program order makes its earlier stores visible to its later loads).  One
// "step" = the literal run before the next match (<= 4 bytes, one 8-byte
// wild store) + that match (8-byte wild load/store chunks).  Bytes a wild
// store writes past the item's end are rewritten by later items, in order;
// no store ever leaves [0, dsize).  Rare cases (long literal runs, short-period
// overlapping matches, the last bytes of the block or of the stream) take the
// byte-serial item path, which is the oracle's decode loop verbatim
// (oracle/qlz_oracle.c:orc_decompress, checks C1-C5).
#include "qlzx_device.h"

namespace qlzx {

__device__ __forceinline__ uint64_t ldu64(const uint8_t *p) { return *(const uint64_t *)p; }  // unaligned mode
__device__ __forceinline__ void stu64(uint8_t *p, uint64_t v) { *(uint64_t *)p = v; }
__device__ __forceinline__ uint32_t ldu32(const uint8_t *p) { return *(const uint32_t *)p; }

__global__ void __launch_bounds__(256) k_dec_lane8(qlzx_blocks b, const uint32_t *dst_cap, uint32_t *dsize_out,
                                                   int32_t *status, uint32_t max_fast) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= b.n) return;
    const uint8_t *src = b.src + b.src_off[i];
    uint8_t *dst = b.dst + b.dst_off[i];
    const uint32_t len = b.src_len[i];
    int st = QLZX_OK;
    uint32_t csize = 0, dsize = 0, hdr = 0;
    bool compressed = false;
    if (len < 3) st = QLZX_E_HEADER;
    else {
        hdr = (src[0] & 2u) ? 9u : 3u;
        if (len < hdr) st = QLZX_E_HEADER;
        else {
            const Header h = parse_header(src);
            csize = h.csize;
            dsize = h.dsize;
            compressed = h.compressed;
            if (h.csize != len) st = QLZX_E_SIZE_COMPRESSED;
            else if (h.level != 3) st = QLZX_E_LEVEL;
            else if (dst_cap && h.dsize > dst_cap[i]) st = QLZX_E_DST_CAP;
            else if (max_fast && h.dsize > max_fast) return;  // another kernel owns it
            else if (!h.compressed && csize < hdr + dsize) st = QLZX_E_CORRUPT;
        }
    }
    if (st == QLZX_OK && !compressed) {  // stored block (quicklz.c:808-811)
        const uint8_t *s = src + hdr;
        uint32_t p = 0;
        for (; p + 8 <= dsize; p += 8) stu64(dst + p, ldu64(s + p));
        for (; p < dsize; p++) dst[p] = s[p];
    } else if (st == QLZX_OK) {
        uint32_t ip = hdr, op = 0, cw = 1;
        bool tail = false;
        const int64_t tail_from = (int64_t)dsize - 1 - QLZX_TAIL;
        while (op < dsize) {
            if (cw == 1) {
                if (ip + 4 > csize) { st = QLZX_E_CORRUPT; break; }  // C1
                cw = ldu32(src + ip);
                if (!(cw >> 31)) { st = QLZX_E_CORRUPT; break; }      // C1
                ip += 4;
            }
            const uint32_t r = __builtin_ctz(cw);  // literals before the next match (or the sentinel)
            if (ip + 8 <= csize && op + 24 <= dsize && r <= 4) {
                // ---- fast step: r literals (+ the match after them) ----
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
                if (off < 3 || off > op || op + ml + 4 > dsize) { st = QLZX_E_CORRUPT; break; }  // C3
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
            if (ip >= csize) { st = QLZX_E_CORRUPT; break; }  // C2
            if (cw & 1u) {
                if (tail) { st = QLZX_E_CORRUPT; break; }  // C4
                const uint32_t tl = token_bytes(src[ip]);
                if (ip + tl > csize) { st = QLZX_E_CORRUPT; break; }  // C2
                uint32_t t = 0;
                for (uint32_t k = 0; k < tl; k++) t |= (uint32_t)src[ip + k] << (8 * k);
                uint32_t off, ml;
                ip += decode_token(t, off, ml);
                if (off < 3 || off > op || op + ml + 4 > dsize) { st = QLZX_E_CORRUPT; break; }  // C3
                for (uint32_t c = 0; c < ml; c++) dst[op + c] = dst[op - off + c];
                op += ml;
            } else {
                if ((int64_t)op >= tail_from) tail = true;  // tail loop (quicklz.c:645-668)
                dst[op++] = src[ip++];
            }
            cw >>= 1;
        }
        if (st == QLZX_OK && !(ip == csize || (ip < hdr + 9 && csize == hdr + 9))) st = QLZX_E_CORRUPT;  // C5
    }
    status[i] = st;
    if (dsize_out) dsize_out[i] = st == QLZX_OK ? dsize : 0;
}

}  // namespace qlzx
