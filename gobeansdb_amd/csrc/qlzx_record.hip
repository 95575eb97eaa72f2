// qlzx_record.hip -- write-side record encode helpers:
// CRC combine for the fused record CRC and a batched block copy for assembling
// 256-B-padded .data records (store/datafile.go:78-88, 307-330).
//
// The record CRC covers header[4:24] ‖ key ‖ value (store/datafile.go:66-76),
// and header[20:24] is the *compressed* size, known only after compress.  The
// compressor therefore fuses the CRC of the value alone (raw state 0) and the
// prefix is folded in afterwards with the linearity of the raw CRC state:
//   crc_write(s, V) = s * x^(8|V|) ^ crc_write(0, V).
#include "qlzx_device.h"

namespace qlzx {

// out[i] = (raw_a[i] * x^(8 len_b[i]) ^ raw_b[i]) ^ final_xor
__global__ void __launch_bounds__(256) k_crc_combine(const uint32_t *raw_a, const uint32_t *raw_b,
                                                     const uint32_t *len_b, uint32_t n, uint32_t final_xor,
                                                     uint32_t *out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    out[i] = (crc_shift(raw_a[i], len_b[i]) ^ raw_b[i]) ^ final_xor;
}

// dst[dst_off[i] .. + len[i]) = src[src_off[i] .. + len[i]); one wave per block,
// 16 B per lane when both sides are 16-B aligned, bytes otherwise.
__global__ void __launch_bounds__(256) k_copy_blocks(const uint8_t *src, const uint64_t *src_off,
                                                     const uint32_t *len, uint8_t *dst, const uint64_t *dst_off,
                                                     uint32_t n) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t i = blockIdx.x * 4 + threadIdx.x / 64;
    if (i >= n) return;
    const uint8_t *s = src + src_off[i];
    uint8_t *d = dst + dst_off[i];
    const uint32_t l = len[i];
    if ((((uintptr_t)s | (uintptr_t)d) & 15u) == 0) {
        const uint32_t n16 = l / 16;
        for (uint32_t k = lane; k < n16; k += 64) ((uint4 *)d)[k] = ((const uint4 *)s)[k];
        for (uint32_t k = n16 * 16 + lane; k < l; k += 64) d[k] = s[k];
    } else {
        for (uint32_t k = lane; k < l; k += 64) d[k] = s[k];
    }
}

}  // namespace qlzx
