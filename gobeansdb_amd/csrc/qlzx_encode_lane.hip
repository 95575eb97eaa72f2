// qlzx_encode_lane.hip -- general-size level-3 encoder, one lane per block.
//
// Catch-all compress path for values of any size (the fast batch path is
// qlzx_encode_wg.hip).  Each lane owns a hash-table slab in the workspace:
// 4096 buckets x 16 u32 positions + 4096 u8 counters, exactly the state of
// quicklz.c:197-494 (qlz_compress_core, level 3) with positions instead of
// pointers.  Output is bit-identical to qlz_compress (quicklz.c:692-775) with
// the destination zero-filled up to the 9-byte core minimum.
#include "qlzx_device.h"

namespace qlzx {

constexpr size_t kLaneSlab = (size_t)QLZX_BUCKETS * QLZX_SLOTS * 4 + QLZX_BUCKETS;

__device__ __forceinline__ uint32_t ld24(const uint8_t *p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16);
}
__device__ __forceinline__ uint32_t bucket_of(uint32_t f) { return ((f >> 12) ^ f) & (QLZX_BUCKETS - 1); }
__device__ __forceinline__ void st32(uint8_t *p, uint32_t v) {
    p[0] = (uint8_t)v; p[1] = (uint8_t)(v >> 8); p[2] = (uint8_t)(v >> 16); p[3] = (uint8_t)(v >> 24);
}

// quicklz.c:197-494. Returns the raw core size (callers apply the 9-byte
// minimum of quicklz.c:493) or 0 when the block stays stored.  bail_bias = 9
// gives Go's bail-out rule (quicklz.go:119 counts the header).
__device__ uint32_t encode_core_lane(const uint8_t *in, uint32_t n, uint8_t *out, uint32_t *slots,
                                     uint8_t *count, uint32_t bail_bias) {
    for (uint32_t k = 0; k < QLZX_BUCKETS; k++) count[k] = 0;
    const int64_t last_start = (int64_t)n - 1 - QLZX_TAIL;
    uint32_t ip = 0, op = 4, cw_pos = 0, cw = 0x80000000u;
    while ((int64_t)ip <= last_start) {
        if (cw & 1u) {
            if (ip > 3u * (n >> 2) && op + bail_bias > ip - (ip >> 5)) return 0;  // quicklz.c:218
            st32(out + cw_pos, (cw >> 1) | 0x80000000u);
            cw_pos = op;
            op += 4;
            cw = 0x80000000u;
        }
        const uint32_t f = ld24(in + ip), h = bucket_of(f);
        const uint32_t c = count[h];
        uint32_t limit = n - 4 - ip;
        if (limit > 255) limit = 255;
        uint32_t best_len = 0, best_pos = 0;
        const uint32_t ncand = c < QLZX_SLOTS ? c : QLZX_SLOTS;
        for (uint32_t k = 0; k < ncand; k++) {
            const uint32_t o = slots[h * QLZX_SLOTS + k];
            if (o + 2 >= ip || ld24(in + o) != f) continue;
            uint32_t m = 3;
            while (m < limit && in[o + m] == in[ip + m]) m++;
            if (m > best_len || (m == best_len && o > best_pos)) { best_len = m; best_pos = o; }
        }
        slots[h * QLZX_SLOTS + (c & (QLZX_SLOTS - 1))] = ip;
        count[h] = (uint8_t)(c + 1);
        if (best_len > 2 && ip - best_pos < QLZX_MAX_OFFSET) {
            for (uint32_t u = 1; u < best_len; u++) {
                const uint32_t h2 = bucket_of(ld24(in + ip + u));
                const uint32_t c2 = count[h2];
                count[h2] = (uint8_t)(c2 + 1);
                slots[h2 * QLZX_SLOTS + (c2 & (QLZX_SLOTS - 1))] = ip + u;
            }
            const uint32_t off = ip - best_pos, ml = best_len;
            cw = (cw >> 1) | 0x80000000u;
            ip += ml;
            if (ml == 3 && off <= 63) {
                out[op++] = (uint8_t)(off << 2);
            } else if (ml == 3 && off <= 16383) {
                const uint32_t t = (off << 2) | 1u;
                out[op] = (uint8_t)t; out[op + 1] = (uint8_t)(t >> 8); op += 2;
            } else if (ml <= 18 && off <= 1023) {
                const uint32_t t = ((ml - 3) << 2) | (off << 6) | 2u;
                out[op] = (uint8_t)t; out[op + 1] = (uint8_t)(t >> 8); op += 2;
            } else if (ml <= 33) {
                const uint32_t t = ((ml - 2) << 2) | (off << 7) | 3u;
                out[op] = (uint8_t)t; out[op + 1] = (uint8_t)(t >> 8); out[op + 2] = (uint8_t)(t >> 16);
                op += 3;
            } else {
                st32(out + op, ((ml - 3) << 7) | (off << 15) | 3u);
                op += 4;
            }
        } else {
            out[op++] = in[ip++];
            cw >>= 1;
        }
    }
    while (ip < n) {
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
    return op;
}

__device__ void write_header(uint8_t *dst, uint32_t hdr, bool compressed, uint32_t csize,
                             uint32_t dsize) {
    if (hdr == 3) {
        dst[0] = (uint8_t)((compressed ? 1 : 0) | 0x4C);
        dst[1] = (uint8_t)csize;
        dst[2] = (uint8_t)dsize;
    } else {
        dst[0] = (uint8_t)(2 | (compressed ? 1 : 0) | 0x4C);
        st32(dst + 1, csize);
        st32(dst + 5, dsize);
    }
}

// quicklz.c:692-775 for one block (Go quicklz.go:80-289 with QLZX_F_GO_COMPAT).
// Returns csize (0 on error).
__device__ uint32_t compress_block_lane(const uint8_t *src, uint32_t n, uint8_t *dst, uint32_t *slots,
                                        uint8_t *count, uint32_t flags, int &st) {
    const bool go = (flags & QLZX_F_GO_COMPAT) != 0;
    if (n == 0) { st = QLZX_E_EMPTY; return 0; }
    if ((uint64_t)n > 0xffffffffull - 400) { st = QLZX_E_TOO_LARGE; return 0; }
    const uint32_t hdr = (n < 216 && !go) ? 3u : 9u;
    for (uint32_t k = 0; k < hdr + 9; k++) dst[k] = 0;
    uint32_t core = encode_core_lane(src, n, dst + hdr, slots, count, go ? 9u : 0u);
    if (core && core < 9 && !go) core = 9;  // quicklz.c:493
    st = QLZX_OK;
    if (core == 0) {
        for (uint32_t k = 0; k < n; k++) dst[hdr + k] = src[k];
        write_header(dst, hdr, false, n + hdr, n);
        return n + hdr;
    }
    write_header(dst, hdr, true, core + hdr, n);
    return core + hdr;
}

// Grid-stride over blocks; lane t owns slab t of the workspace.  Blocks with
// src_len < min_len (the fast path) or > max_len (the whole-GPU path) are skipped (0: no bound).
__global__ void __launch_bounds__(64) k_encode_lane(qlzx_blocks b, uint32_t *csize, int32_t *status,
                                                    const uint32_t *crc_state, uint32_t *crc_out,
                                                    uint8_t *ws, uint32_t nlanes, uint32_t min_len,
                                                    uint32_t max_len, uint32_t flags) {
    __shared__ uint32_t tab[256];
    load_crc_table(tab);
    __syncthreads();
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= nlanes) return;
    uint8_t *slab = ws + (size_t)t * kLaneSlab;
    uint32_t *slots = (uint32_t *)slab;
    uint8_t *count = slab + (size_t)QLZX_BUCKETS * QLZX_SLOTS * 4;
    for (uint32_t i = t; i < b.n; i += nlanes) {
        const uint32_t n = b.src_len[i];
        if (min_len && n < min_len) continue;  // the workgroup kernel owns it (including n == 0)
        if (max_len && n > max_len) continue;  // the whole-GPU encoder owns it (qlzx_encode_huge.hip)
        int st = QLZX_OK;
        uint8_t *dst = b.dst + b.dst_off[i];
        const uint32_t r = compress_block_lane(b.src + b.src_off[i], n, dst, slots, count, flags, st);
        csize[i] = r;
        if (status) status[i] = st;
        if (crc_state && crc_out) {
            uint32_t c = crc_state[i];
            for (uint32_t k = 0; k < r; k++) c = crc_byte(tab, c, dst[k]);
            crc_out[i] = ~c;
        }
    }
}

}  // namespace qlzx
