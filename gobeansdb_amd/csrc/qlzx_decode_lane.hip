// qlzx_decode_lane.hip -- general-size level-3 decoder, one lane per block.
//
// This is the catch-all path: any dsize (the batch fast path handles blocks
// up to QLZX_FAST_MAX_DSIZE with the whole history in LDS; see
// qlzx_decode_wave.hip).  History lives in the destination buffer itself
// (global memory), so it serves blocks of any size, including BodyMax = 50 MiB
// values (config/mc_config.go:7).
//
// Semantics: quicklz.c:496-672 (qlz_decompress_core) on every stream the
// encoder can produce; malformed streams are rejected by checks C1-C5 of
// oracle/qlz_oracle.c:orc_decompress; header/size checks of
// CDecompressSafe (cquicklz.go:84-101).
// The record CRC (store/datafile.go:66-76) is continued over the compressed
// bytes in the same kernel.
#include "qlzx_device.h"

namespace qlzx {

__device__ int decode_block_lane(const uint8_t *src, uint32_t src_len, uint8_t *dst, uint64_t cap,
                                 uint32_t &dsize_out) {
    dsize_out = 0;
    if (src_len < 3) return QLZX_E_HEADER;
    const uint32_t hb = (src[0] & 2u) ? 9u : 3u;
    if (src_len < hb) return QLZX_E_HEADER;
    const Header h = parse_header(src);
    if (h.csize != src_len) return QLZX_E_SIZE_COMPRESSED;
    if (h.level != 3) return QLZX_E_LEVEL;
    if ((uint64_t)h.dsize > cap) return QLZX_E_DST_CAP;
    const uint32_t csize = h.csize, dsize = h.dsize;
    if (!h.compressed) {  // stored block (quicklz.c:808-811)
        if ((uint64_t)csize < (uint64_t)h.hdr + dsize) return QLZX_E_CORRUPT;
        for (uint32_t i = 0; i < dsize; i++) dst[i] = src[h.hdr + i];
        dsize_out = dsize;
        return QLZX_OK;
    }
    // checks C1-C5 of oracle/qlz_oracle.c:orc_decompress
    uint32_t ip = h.hdr, op = 0, cw = 1;
    bool tail = false;
    const int64_t tail_from = (int64_t)dsize - 1 - QLZX_TAIL;
    while (op < dsize) {
        if (cw == 1) {
            if (ip + 4 > csize) return QLZX_E_CORRUPT;
            cw = ld_u32_bytes(src + ip);
            if (!(cw >> 31)) return QLZX_E_CORRUPT;  // sentinel bit (quicklz.c:221)
            ip += 4;
        }
        if (ip >= csize) return QLZX_E_CORRUPT;
        if (cw & 1u) {
            if (tail) return QLZX_E_CORRUPT;
            const uint32_t tl = token_bytes(src[ip]);
            if (ip + tl > csize) return QLZX_E_CORRUPT;
            uint32_t t = 0;
            for (uint32_t k = 0; k < tl; k++) t |= (uint32_t)src[ip + k] << (8 * k);
            uint32_t off, len;
            ip += decode_token(t, off, len);
            if (off < 3 || off > op || (uint64_t)op + len + 4 > dsize) return QLZX_E_CORRUPT;
            uint8_t *d = dst + op;
            const uint8_t *s = d - off;
            for (uint32_t i = 0; i < len; i++) d[i] = s[i];  // forward (overlapping) copy
            op += len;
        } else {
            if ((int64_t)op >= tail_from) tail = true;  // tail loop (quicklz.c:645-668)
            dst[op++] = src[ip++];
        }
        cw >>= 1;
    }
    if (!(ip == csize || (ip < h.hdr + 9 && csize == h.hdr + 9))) return QLZX_E_CORRUPT;
    dsize_out = dsize;
    return QLZX_OK;
}

// Handles blocks with dsize >= min_dsize (smaller ones belong to the fast path
// when it runs; min_dsize = 0 -> all).
__global__ void __launch_bounds__(256) k_decode_lane(qlzx_blocks b, const uint32_t *dst_cap,
                                                     uint32_t *dsize, int32_t *status,
                                                     const uint32_t *crc_state,
                                                     const uint32_t *crc_expect, uint32_t *crc_out,
                                                     uint32_t min_dsize) {
    __shared__ uint32_t tab[256];
    load_crc_table(tab);
    __syncthreads();
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= b.n) return;
    const uint8_t *src = b.src + b.src_off[i];
    const uint32_t len = b.src_len[i];
    if (min_dsize && len >= 3) {
        const uint32_t hb = (src[0] & 2u) ? 9u : 3u;
        if (len >= hb && parse_header(src).dsize < min_dsize) return;  // owned by the fast path
    }
    int st = QLZX_OK;
    if (crc_state || crc_expect || crc_out) {  // record CRC over the stored (compressed) value bytes
        uint32_t c = crc_state ? crc_state[i] : 0xffffffffu;
        for (uint32_t k = 0; k < len; k++) c = crc_byte(tab, c, src[k]);
        c = ~c;
        if (crc_out) crc_out[i] = c;
        if (crc_expect && c != crc_expect[i]) st = QLZX_E_CRC;
    }
    uint32_t ds = 0;
    if (st == QLZX_OK)
        st = decode_block_lane(src, len, b.dst + b.dst_off[i], dst_cap ? dst_cap[i] : ~0ull, ds);
    if (dsize) dsize[i] = ds;
    status[i] = st;
}

}  // namespace qlzx
