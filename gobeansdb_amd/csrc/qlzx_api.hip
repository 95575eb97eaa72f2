// qlzx_api.hip -- host runtime + C ABI of libqlzx.so (declared in include/qlzx.h).
//
// Unity build: the kernel sources are included here so the device tables
// (qlzx_tables.hip) link without relocatable device code.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>

#include "qlzx_tables.hip"
#include "qlzx_crc.hip"
#include "qlzx_decode_wave.hip"
#include "qlzx_decode_lane8.hip"
#include "qlzx_decode_huge.hip"
#include "qlzx_encode_lane.hip"
#include "qlzx_encode_wg.hip"
#include "qlzx_encode_huge.hip"
#include "qlzx_replay.hip"
#include "qlzx_record.hip"
#include "qlzx_level1.hip"

namespace {

thread_local std::string t_last_error;

int fail(int code, const char *what, hipError_t e = hipSuccess) {
    t_last_error = what;
    if (e != hipSuccess) {
        t_last_error += ": ";
        t_last_error += hipGetErrorString(e);
    }
    return code;
}

#define HIP_OK(expr)                                                     \
    do {                                                                 \
        hipError_t _e = (expr);                                          \
        if (_e != hipSuccess) return fail(QLZX_R_HIP, #expr, _e);       \
    } while (0)

inline uint32_t ld32h(const unsigned char *p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

constexpr uint32_t kMaxLaneSlabs = 4096;  // concurrent lane encoders for the general path

}  // namespace

#include "qlzx_service.hip"

#ifdef QLZX_PROFILE
namespace qlzx {
__device__ unsigned long long *g_prof = nullptr;
}
extern "C" int qlzx_profile_set(void *dev_buf) {
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(qlzx::g_prof), &dev_buf, sizeof(void *));
}
#endif

extern "C" {

const char *qlzx_last_error(void) { return t_last_error.c_str(); }

#ifndef QLZX_SRC_HASH
#define QLZX_SRC_HASH "unknown"
#endif
// the source hash of the build (gobeansdb_amd/build.py source_hash); also greppable in the binary
extern __attribute__((used)) const char qlzx_src_hash_tag[] = "qlzx-src-hash:" QLZX_SRC_HASH;

int qlzx_info(char *buf, size_t len) {
    const char *s =
        "libqlzx: QuickLZ 1.4.1 level 3 + record CRC32 for gobeansdb; target gfx950 (MI355X); "
        "decode: wave-per-block LDS history (dsize<=" QLZX_STR(QLZX_FAST_MAX_DSIZE)
        ") + lane-per-block general; encode: workgroup-per-block position-parallel "
        "(len<=" QLZX_STR(QLZX_WG_MAX_LEN) ") + lane-per-block general; src " QLZX_SRC_HASH;
    if (!buf || !len) return (int)strlen(s);
    snprintf(buf, len, "%s", s);
    return 0;
}

/* ---------------- quicklz.h drop-in: header helpers (quicklz.c:674-690) ---------------- */
size_t qlz_size_decompressed(const char *source) {
    const unsigned char *s = (const unsigned char *)source;
    return (s[0] & 2) ? ld32h(s + 5) : s[2];
}
size_t qlz_size_compressed(const char *source) {
    const unsigned char *s = (const unsigned char *)source;
    return (s[0] & 2) ? ld32h(s + 1) : s[1];
}
int qlz_get_setting(int setting) {  // quicklz.c:31-58 as built by quicklz.h:25-31
    switch (setting) {
        case 0: return 3;       // QLZ_COMPRESSION_LEVEL
        case 1: return 528400;  // QLZ_SCRATCH_COMPRESS
        case 2: return 16;      // QLZ_SCRATCH_DECOMPRESS
        case 3: return 0;       // QLZ_STREAMING_BUFFER
        case 6: return 0;       // QLZ_MEMORY_SAFE (the reference build); this library always checks
        case 7: return 1;
        case 8: return 4;
        case 9: return 1;
    }
    return -1;
}

/* ---------------- batch device API ---------------- */

size_t qlzx_decompress_workspace_size(uint32_t n, uint32_t max_dsize) {
    // two halves for batches of more than one chunk: K1/K2 of consecutive chunks overlap (three
    // for mixed sizes over three chunks or more: the last chunk's K1 starts first)
    const size_t one = qlzx::decode_wave_ws_bytes(n, max_dsize);
    size_t ws = qlzx::decode_wave_halves(n, max_dsize) * one;
    if (max_dsize > QLZX_FAST_MAX_DSIZE)  // large values: the pending list and the whole-GPU decoder
        ws += align_up((size_t)n * sizeof(qlzx::HugeItem) + 256, 256) + qlzx::huge_ws_layout(max_dsize, nullptr, nullptr);
    return ws;
}

}  // extern "C"

namespace {

__global__ void k_h_setstatus(int32_t *status, uint32_t *dsize_out, int32_t st, uint32_t ds) {
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        *status = st;
        if (dsize_out) *dsize_out = ds;
    }
}
// record CRC verdict of one large block: crc_out, and QLZX_E_CRC (nothing decoded) on a mismatch
__global__ void k_h_crcverdict(qlzx::HugeCtl *ctl, const uint32_t *crc_expect, uint32_t *crc_out, int32_t *status,
                               uint32_t *dsize_out) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    const uint32_t c = ~ctl->crc;
    if (crc_out) *crc_out = c;
    if (crc_expect && c != *crc_expect) {
        ctl->st = QLZX_E_CRC;
        *status = QLZX_E_CRC;
        if (dsize_out) *dsize_out = 0;
    }
}
__global__ void k_h_crcinit(qlzx::HugeCtl *ctl, const uint32_t *crc_state) {
    if (threadIdx.x == 0 && blockIdx.x == 0) ctl->crc = crc_state ? *crc_state : 0xffffffffu;
}

// One large block (dsize > QLZX_FAST_MAX_DSIZE) by the whole GPU (qlzx_decode_huge.hip).  The host
// knows the sizes from the pending list; it synchronises to read the verdict of the parse and
// the pointer-jumping flags.
int huge_one(const uint8_t *src, uint32_t csize, uint8_t *dst, uint32_t dsize, bool comp, uint32_t max_dsize,
             const uint32_t *crc_state, const uint32_t *crc_expect, uint32_t *crc_out, int32_t *status,
             uint32_t *dsize_out, uint8_t *ws, hipStream_t s) {
    using namespace qlzx;
    HugeWs w;
    huge_ws_layout(max_dsize, ws, &w);
    const uint32_t nmax = (uint32_t)huge_nmax(max_dsize);
    const dim3 G(kHugeGrid), B(kHugeWG);
    HIP_OK(hipMemsetAsync(w.ctl, 0, sizeof(HugeCtl), s));
    const bool crc = crc_state || crc_expect || crc_out;
    if (crc) {
        hipLaunchKernelGGL(k_h_crcseg, dim3(std::min<uint32_t>((csize + kHugeSeg * 4 - 1) / (kHugeSeg * 4), 1024)),
                           dim3(256), 0, s, src, (uint64_t)csize, w.scrc);
        hipLaunchKernelGGL(k_h_crcinit, dim3(1), dim3(64), 0, s, w.ctl, crc_state);
        // the combine reads the initial state from ctl->crc
        hipLaunchKernelGGL(k_h_crccomb_ctl, dim3(1), dim3(64), 0, s, w.scrc, (uint64_t)csize, w.ctl);
        hipLaunchKernelGGL(k_h_crcverdict, dim3(1), dim3(64), 0, s, w.ctl, crc_expect, crc_out, status, dsize_out);
    }
    const uint32_t hdr = 9;  // header of a value over 64 KiB: always 9 bytes (quicklz.c:771-772)
    if (!comp) {  // stored (quicklz.c:808-811)
        if ((uint64_t)csize < (uint64_t)hdr + dsize) {
            hipLaunchKernelGGL(k_h_setstatus_ok_if, dim3(1), dim3(64), 0, s, w.ctl, status, dsize_out, QLZX_E_CORRUPT, 0u);
        } else {
            hipLaunchKernelGGL(k_h_copy_if, G, B, 0, s, w.ctl, src + hdr, dst, (uint64_t)dsize);
            hipLaunchKernelGGL(k_h_setstatus_ok_if, dim3(1), dim3(64), 0, s, w.ctl, status, dsize_out, QLZX_OK, dsize);
        }
        HIP_OK(hipGetLastError());
        return QLZX_R_OK;
    }
    if (csize > nmax) {  // longer than any stream of dsize bytes can be: trailing garbage (C5)
        hipLaunchKernelGGL(k_h_setstatus_ok_if, dim3(1), dim3(64), 0, s, w.ctl, status, dsize_out, QLZX_E_CORRUPT, 0u);
        HIP_OK(hipGetLastError());
        return QLZX_R_OK;
    }
    hipLaunchKernelGGL(k_h_codes, G, B, 0, s, src, csize, w.code);
    hipLaunchKernelGGL(k_h_delta, G, B, 0, s, src, csize, hdr, (const uint32_t *)w.code, w.delta);
    hipLaunchKernelGGL(k_h_jump1, G, B, 0, s, (const uint8_t *)w.delta, csize, w.J);
    for (uint32_t k = 2; k <= kHugeLevels; k++)
        hipLaunchKernelGGL(k_h_jumpk, G, B, 0, s, (const uint16_t *)(w.J + (size_t)(k - 2) * (nmax + 256)), csize,
                           w.J + (size_t)(k - 1) * (nmax + 256));
    hipLaunchKernelGGL(k_h_walk, dim3(1), dim3(64), 0, s, src, csize, hdr, dsize, (const uint32_t *)w.code,
                       (const uint8_t *)w.delta, (const uint16_t *)w.J, nmax, w.seg, w.ctl);
    hipLaunchKernelGGL(k_h_expand, G, B, 0, s, (const uint8_t *)w.delta, (const HugeSeg *)w.seg,
                       (const HugeCtl *)w.ctl, w.glist);
    hipLaunchKernelGGL(k_h_glen, G, B, 0, s, src, csize, (const uint32_t *)w.code, (const uint32_t *)w.glist,
                       (const HugeCtl *)w.ctl, w.glen);
    hipLaunchKernelGGL(k_h_scan, dim3(1), dim3(1024), 0, s, w.glen, (const HugeCtl *)w.ctl);
    hipLaunchKernelGGL(k_h_items, G, B, 0, s, src, csize, hdr, dsize, (const uint32_t *)w.code,
                       (const uint32_t *)w.glist, (const uint32_t *)w.glen, w.ctl, w.src, w.lit);
    HIP_OK(hipGetLastError());
    HugeCtl h;
    HIP_OK(hipMemcpyAsync(&h, w.ctl, sizeof(HugeCtl), hipMemcpyDeviceToHost, s));
    HIP_OK(hipStreamSynchronize(s));
    if (h.st == QLZX_E_CRC) return QLZX_R_OK;  // already reported
    const bool corrupt = h.st != QLZX_OK || h.bad || !h.done || (h.tail_idx != 0xffffffffu && h.max_match > h.tail_idx);
    if (corrupt) {
        hipLaunchKernelGGL(k_h_setstatus, dim3(1), dim3(64), 0, s, status, dsize_out, (int32_t)QLZX_E_CORRUPT, 0u);
        HIP_OK(hipGetLastError());
        return QLZX_R_OK;
    }
    // pointer jumping, four rounds per check of the last round's flag
    for (uint32_t r = 0;; r += 4) {
        if (r + 4 > 64) return fail(QLZX_R_HIP, "huge decode: pointer jumping did not converge");
        for (uint32_t j = 0; j < 4; j++)
            hipLaunchKernelGGL(k_h_jumpround, G, B, 0, s, w.src, dsize, w.ctl->changed + r + j);
        uint32_t ch = 0;
        HIP_OK(hipMemcpyAsync(&ch, w.ctl->changed + r + 3, 4, hipMemcpyDeviceToHost, s));
        HIP_OK(hipStreamSynchronize(s));
        if (!ch) break;
    }
    hipLaunchKernelGGL(k_h_gather, G, B, 0, s, (const uint32_t *)w.src, (const uint8_t *)w.lit, dsize, dst);
    hipLaunchKernelGGL(k_h_setstatus, dim3(1), dim3(64), 0, s, status, dsize_out, (int32_t)QLZX_OK, dsize);
    HIP_OK(hipGetLastError());
    return QLZX_R_OK;
}

// The pending large blocks of a batch (K1 left them kPending): listed on the device, read back
// once, then decoded one at a time by huge_one.
int huge_pass(const qlzx_blocks &b, const uint32_t *crc_state, const uint32_t *crc_expect, uint32_t *crc_out,
              int32_t *status, uint32_t *dsize_out, uint32_t max_dsize, uint8_t *ws, hipStream_t s) {
    using namespace qlzx;
    uint32_t *count = (uint32_t *)ws;
    HugeItem *items = (HugeItem *)(ws + 256);
    uint8_t *hws = ws + align_up((size_t)b.n * sizeof(HugeItem) + 256, 256);
    HIP_OK(hipMemsetAsync(count, 0, 4, s));
    hipLaunchKernelGGL(k_h_pending, dim3(std::min<uint32_t>((b.n + 255) / 256, 4096)), dim3(256), 0, s, b,
                       (const int32_t *)status, count, items);
    HIP_OK(hipGetLastError());
    uint32_t np = 0;
    HIP_OK(hipMemcpyAsync(&np, count, 4, hipMemcpyDeviceToHost, s));
    HIP_OK(hipStreamSynchronize(s));
    if (np == 0) return QLZX_R_OK;
    std::vector<HugeItem> hl(np);
    HIP_OK(hipMemcpyAsync(hl.data(), items, np * sizeof(HugeItem), hipMemcpyDeviceToHost, s));
    std::vector<uint64_t> so(np), dof(np);
    HIP_OK(hipStreamSynchronize(s));
    for (uint32_t j = 0; j < np; j++) {
        HIP_OK(hipMemcpyAsync(&so[j], b.src_off + hl[j].i, 8, hipMemcpyDeviceToHost, s));
        HIP_OK(hipMemcpyAsync(&dof[j], b.dst_off + hl[j].i, 8, hipMemcpyDeviceToHost, s));
    }
    HIP_OK(hipStreamSynchronize(s));
    for (uint32_t j = 0; j < np; j++) {
        const uint32_t i = hl[j].i;
        if (int r = huge_one(b.src + so[j], hl[j].csize, b.dst + dof[j], hl[j].dsize, hl[j].comp != 0, max_dsize,
                             crc_state ? crc_state + i : nullptr, crc_expect ? crc_expect + i : nullptr,
                             crc_out ? crc_out + i : nullptr, status + i, dsize_out ? dsize_out + i : nullptr, hws, s))
            return r;
    }
    return QLZX_R_OK;
}

__global__ void k_he_fail(int32_t *status, uint32_t *csize, int32_t st) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    if (status) *status = st;
    *csize = 0;
}
__global__ void k_he_crcfin(const uint32_t *scrc, uint64_t len, const uint32_t *crc_state, uint32_t *crc_out) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    const uint32_t nseg = (uint32_t)((len + qlzx::kHugeSeg - 1) / qlzx::kHugeSeg);
    uint32_t acc = *crc_state;
    for (uint32_t k = 0; k < nseg; k++)
        acc = qlzx::crc_shift(acc, min((uint64_t)qlzx::kHugeSeg, len - (uint64_t)k * qlzx::kHugeSeg)) ^ scrc[k];
    *crc_out = ~acc;  // as the lane encoder: ~crc over the output from crc_state
}

// One value of n > 64 KiB bytes by the whole GPU (qlzx_encode_huge.hip).  The host synchronises
// twice: for the parse's item count, and for the bail-out verdict and the output size.
int huge_encode_one(const uint8_t *src, uint32_t n, uint8_t *dst, uint32_t flags, const uint32_t *crc_state,
                    uint32_t *crc_out, uint32_t *csize_out, int32_t *status, uint32_t nmax, uint8_t *ws,
                    hipStream_t s) {
    using namespace qlzx;
    HeWs w;
    he_ws_layout(nmax, ws, &w);
    const uint32_t P = he_positions(n), L = he_levels(P);
    const dim3 G(kHeGrid), B(kHeWG);
    HIP_OK(hipMemsetAsync(w.ctl, 0, sizeof(HeCtl), s));
    hipLaunchKernelGGL(k_he_keys, G, B, 0, s, src, P, w.key, w.pos);
    size_t tb = w.tmp_bytes;
    if (rocprim::radix_sort_pairs(w.tmp, tb, (const uint16_t *)w.key, w.key_s, (const uint32_t *)w.pos, w.pos_s,
                                  (size_t)P, 0, 12, s) != hipSuccess)
        return fail(QLZX_R_HIP, "huge encode: radix sort");
    hipLaunchKernelGGL(k_he_base, G, B, 0, s, (const uint16_t *)w.key_s, P, w.base);
    hipLaunchKernelGGL(k_he_match, G, B, 0, s, src, n, P, (const uint16_t *)w.key_s, (const uint32_t *)w.pos_s,
                       (const uint32_t *)w.base, w.MO);
    hipLaunchKernelGGL(k_he_jump0, G, B, 0, s, (const uint32_t *)w.MO, P, w.J);
    for (uint32_t k = 1; k < L; k++)
        hipLaunchKernelGGL(k_he_jumpk, G, B, 0, s, (const uint32_t *)(w.J + (size_t)(k - 1) * (P + 1)), P,
                           w.J + (size_t)k * (P + 1));
    hipLaunchKernelGGL(k_he_walk, dim3(1), dim3(64), 0, s, (const uint32_t *)w.J, P, L, (const uint32_t *)w.MO,
                       w.ITEM, w.ctl);
    for (uint32_t k = L - 1; k >= 1; k--)
        hipLaunchKernelGGL(k_he_expand, G, B, 0, s, (const uint32_t *)(w.J + (size_t)(k - 1) * (P + 1)),
                           (const HeCtl *)w.ctl, k, w.ITEM);
    HIP_OK(hipGetLastError());
    HeCtl h;
    HIP_OK(hipMemcpyAsync(&h, w.ctl, sizeof(HeCtl), hipMemcpyDeviceToHost, s));
    HIP_OK(hipStreamSynchronize(s));
    if (h.tail0 > n || h.m > P) return fail(QLZX_R_HIP, "huge encode: parse out of range");
    const uint32_t ntot = h.m + (n - h.tail0);
    hipLaunchKernelGGL(k_he_sizes, G, B, 0, s, (const uint32_t *)w.ITEM, (const uint32_t *)w.MO,
                       (const HeCtl *)w.ctl, ntot, w.sizes);
    tb = w.tmp_bytes;
    if (rocprim::exclusive_scan(w.tmp, tb, (const uint32_t *)w.sizes, w.S, 0u, (size_t)ntot + 1,
                                rocprim::plus<uint32_t>(), s) != hipSuccess)
        return fail(QLZX_R_HIP, "huge encode: scan");
    const uint32_t bias = (flags & QLZX_F_GO_COMPAT) ? 9u : 0u;  // Go counts the header (quicklz.go:119)
    hipLaunchKernelGGL(k_he_bail, G, B, 0, s, (const uint32_t *)w.ITEM, (const uint32_t *)w.S, n, bias, w.ctl);
    uint32_t tot = 0;
    HIP_OK(hipMemcpyAsync(&tot, w.S + ntot, 4, hipMemcpyDeviceToHost, s));
    HIP_OK(hipMemcpyAsync(&h, w.ctl, sizeof(HeCtl), hipMemcpyDeviceToHost, s));
    HIP_OK(hipStreamSynchronize(s));
    const uint32_t hdr = 9;  // n > 64 KiB >= 216 (quicklz.c:708-711)
    uint32_t cs;
    if (!h.bail) {
        const uint32_t core = 4 * ((ntot + 30) / 31) + tot;
        cs = hdr + core;
        hipLaunchKernelGGL(k_he_write, G, B, 0, s, src, (const uint32_t *)w.ITEM, (const uint32_t *)w.MO,
                           (const uint32_t *)w.S, (const HeCtl *)w.ctl, ntot, dst + hdr);
    } else {  // stored (quicklz.c:722-727)
        cs = n + hdr;
        hipLaunchKernelGGL(k_he_copy, G, B, 0, s, src, dst + hdr, (uint64_t)n);
    }
    hipLaunchKernelGGL(k_he_header, dim3(1), dim3(64), 0, s, dst, !h.bail, cs, n, csize_out, status);
    if (crc_state && crc_out) {
        hipLaunchKernelGGL(k_h_crcseg, dim3(std::min<uint32_t>((cs + kHugeSeg * 4 - 1) / (kHugeSeg * 4), 1024)),
                           dim3(256), 0, s, (const uint8_t *)dst, (uint64_t)cs, w.scrc);
        hipLaunchKernelGGL(k_he_crcfin, dim3(1), dim3(64), 0, s, (const uint32_t *)w.scrc, (uint64_t)cs, crc_state,
                           crc_out);
    }
    HIP_OK(hipGetLastError());
    return QLZX_R_OK;
}

// The values over 64 KiB of a compress batch: listed on the device, read back once, then
// compressed one at a time by huge_encode_one.
int huge_encode_pass(const qlzx_blocks &b, uint32_t *csize, int32_t *status, const uint32_t *crc_state,
                     uint32_t *crc_out, uint32_t flags, uint32_t max_len, uint8_t *ws, hipStream_t s) {
    using namespace qlzx;
    uint32_t *count = (uint32_t *)ws;
    HeItem *items = (HeItem *)(ws + 256);
    uint8_t *hws = ws + align_up((size_t)std::max<uint32_t>(b.n, 1) * sizeof(HeItem) + 256, 256);
    HIP_OK(hipMemsetAsync(count, 0, 4, s));
    hipLaunchKernelGGL(k_he_pending, dim3(std::min<uint32_t>((b.n + 255) / 256, 4096)), dim3(256), 0, s, b,
                       (uint32_t)QLZX_WG_MAX_LEN + 1, count, items);
    HIP_OK(hipGetLastError());
    uint32_t np = 0;
    HIP_OK(hipMemcpyAsync(&np, count, 4, hipMemcpyDeviceToHost, s));
    HIP_OK(hipStreamSynchronize(s));
    if (np == 0) return QLZX_R_OK;
    std::vector<HeItem> hl(np);
    HIP_OK(hipMemcpyAsync(hl.data(), items, np * sizeof(HeItem), hipMemcpyDeviceToHost, s));
    std::vector<uint64_t> so(np), dof(np);
    HIP_OK(hipStreamSynchronize(s));
    for (uint32_t j = 0; j < np; j++) {
        HIP_OK(hipMemcpyAsync(&so[j], b.src_off + hl[j].i, 8, hipMemcpyDeviceToHost, s));
        HIP_OK(hipMemcpyAsync(&dof[j], b.dst_off + hl[j].i, 8, hipMemcpyDeviceToHost, s));
    }
    HIP_OK(hipStreamSynchronize(s));
    for (uint32_t j = 0; j < np; j++) {
        const uint32_t i = hl[j].i;
        if (hl[j].n > max_len || (uint64_t)hl[j].n > 0xffffffffull - 400) {  // as the lane encoder reports it
            hipLaunchKernelGGL(k_he_fail, dim3(1), dim3(64), 0, s, status ? status + i : nullptr, csize + i,
                               (int32_t)QLZX_E_TOO_LARGE);
            continue;
        }
        if (int r = huge_encode_one(b.src + so[j], hl[j].n, b.dst + dof[j], flags, crc_state ? crc_state + i : nullptr,
                                    crc_out ? crc_out + i : nullptr, csize + i, status ? status + i : nullptr, max_len,
                                    hws, s))
            return r;
    }
    return QLZX_R_OK;
}

}  // namespace

extern "C" {

int qlzx_decompress_batch(const qlzx_blocks *b, const uint32_t *dst_cap, uint32_t *dsize,
                          int32_t *status, const uint32_t *crc_state, const uint32_t *crc_expect,
                          uint32_t *crc_out, uint32_t max_dsize, void *workspace,
                          size_t workspace_bytes, void *stream) {
    if (!b || !status) return fail(QLZX_R_BAD_ARG, "qlzx_decompress_batch: null blocks/status");
    if (b->n == 0) return QLZX_R_OK;
    if (!b->src || !b->src_off || !b->src_len || !b->dst || !b->dst_off)
        return fail(QLZX_R_BAD_ARG, "qlzx_decompress_batch: null block array");
    hipStream_t s = (hipStream_t)stream;
    // no workspace: the general lane-per-block kernel for every block
    const bool fast = workspace && workspace_bytes >= qlzx::decode_wave_ws_bytes(b->n, max_dsize);
    if (fast) {
        int r = qlzx::launch_decode_wave(*b, dst_cap, dsize, status, crc_state, crc_expect, crc_out,
                                         max_dsize, workspace, workspace_bytes, s);
        if (r) return fail(QLZX_R_HIP, "decode_wave launch", (hipError_t)r);
    }
    if (fast && max_dsize > QLZX_FAST_MAX_DSIZE &&
        workspace_bytes >= qlzx_decompress_workspace_size(b->n, max_dsize)) {
        // large values: the whole-GPU decoder, one value at a time (synchronises the stream)
        const size_t wave = qlzx_decompress_workspace_size(b->n, QLZX_FAST_MAX_DSIZE);
        return huge_pass(*b, crc_state, crc_expect, crc_out, status, dsize, max_dsize, (uint8_t *)workspace + wave, s);
    }
    if (!fast || max_dsize > QLZX_FAST_MAX_DSIZE) {
        const uint32_t min_dsize = fast ? QLZX_FAST_MAX_DSIZE + 1 : 0;
        hipLaunchKernelGGL(qlzx::k_dec_lane8, dim3((b->n + 255) / 256), dim3(256), 0, s, *b, dst_cap,
                           dsize, status, crc_state, crc_expect, crc_out, min_dsize, max_dsize);
        HIP_OK(hipGetLastError());
    }
    return QLZX_R_OK;
}

size_t qlzx_compress_workspace_size(uint32_t n, uint32_t max_len) {
    // at least one lane slab: QLZX_F_GO_COMPAT batches (flags are not known here) take the lane path
    size_t ws = qlzx::kLaneSlab;
    if (!qlzx::encode_wg_enabled())
        ws = (size_t)std::min<uint32_t>(std::max<uint32_t>(n, 1), kMaxLaneSlabs) * qlzx::kLaneSlab;
    ws = std::max(ws, qlzx::encode_wg_ws_bytes(n, max_len));
    if (max_len > QLZX_WG_MAX_LEN)  // values over 64 KiB: the pending list and the whole-GPU encoder
        ws += align_up((size_t)std::max<uint32_t>(n, 1) * sizeof(qlzx::HeItem) + 256, 256) +
              qlzx::he_ws_layout(max_len, nullptr, nullptr);
    return ws;
}

int qlzx_compress_batch(const qlzx_blocks *b, uint32_t *csize, int32_t *status,
                        const uint32_t *crc_state, uint32_t *crc_out, uint32_t max_len,
                        uint32_t flags, void *workspace, size_t workspace_bytes, void *stream) {
    if (!b || !csize) return fail(QLZX_R_BAD_ARG, "qlzx_compress_batch: null blocks/csize");
    if (b->n == 0) return QLZX_R_OK;
    if (!b->src || !b->src_off || !b->src_len || !b->dst || !b->dst_off)
        return fail(QLZX_R_BAD_ARG, "qlzx_compress_batch: null block array");
    if (workspace_bytes < qlzx_compress_workspace_size(b->n, max_len) || !workspace)
        return fail(QLZX_R_WORKSPACE, "qlzx_compress_batch: workspace too small");
    hipStream_t s = (hipStream_t)stream;
    const bool wg = qlzx::encode_wg_enabled() && !(flags & QLZX_F_GO_COMPAT);
    const bool huge = max_len > QLZX_WG_MAX_LEN;  // values over 64 KiB: qlzx_encode_huge.hip
    if (wg) {
        int r = qlzx::launch_encode_wg(*b, csize, status, crc_state, crc_out, max_len, flags, workspace, s);
        if (r) return fail(QLZX_R_HIP, "encode_wg launch", (hipError_t)r);
    }
    if (!wg) {  // the lane encoder: Go-compat batches (and a disabled workgroup encoder) up to 64 KiB
        const uint32_t nl = (uint32_t)std::min<size_t>(
            std::min<uint32_t>(b->n, kMaxLaneSlabs), workspace_bytes / qlzx::kLaneSlab);
        if (nl == 0) return fail(QLZX_R_WORKSPACE, "qlzx_compress_batch: no lane slab");
        hipLaunchKernelGGL(qlzx::k_encode_lane, dim3((nl + 63) / 64), dim3(64), 0, s, *b, csize, status,
                           crc_state, crc_out, (uint8_t *)workspace, nl, 0u, huge ? (uint32_t)QLZX_WG_MAX_LEN : 0u,
                           flags);
        HIP_OK(hipGetLastError());
    }
    if (huge)  // after the kernels above in stream order: the whole workspace is free again
        return huge_encode_pass(*b, csize, status, crc_state, crc_out, flags, max_len, (uint8_t *)workspace, s);
    return QLZX_R_OK;
}

size_t qlzx_go_l1_workspace_size(uint32_t n) {
    return (size_t)std::min<uint32_t>(std::max<uint32_t>(n, 1), qlzx::kL1Chunk) * qlzx::kL1WsBlock;
}
size_t qlzx_go_decompress_workspace_size(uint32_t n) {
    return (size_t)std::min<uint32_t>(std::max<uint32_t>(n, 1), qlzx::kL1Chunk) * qlzx::kL1DecWsBlock;
}

static int check_l1_args(const qlzx_blocks *b, const void *out, void *workspace, size_t workspace_bytes,
                         size_t need, const char *who) {
    if (!b || !out) return fail(QLZX_R_BAD_ARG, who);
    if (b->n == 0) return QLZX_R_OK;
    if (!b->src || !b->src_off || !b->src_len || !b->dst || !b->dst_off) return fail(QLZX_R_BAD_ARG, who);
    if (!workspace || (((uintptr_t)workspace) & 15u) || workspace_bytes < need) return fail(QLZX_R_WORKSPACE, who);
    return QLZX_R_OK;
}

int qlzx_go_l1_compress_batch(const qlzx_blocks *b, uint32_t *csize, int32_t *status, void *workspace,
                              size_t workspace_bytes, void *stream) {
    if (int r = check_l1_args(b, csize, workspace, workspace_bytes, qlzx_go_l1_workspace_size(b ? b->n : 0),
                              "qlzx_go_l1_compress_batch"))
        return r;
    // chunks of kL1Chunk blocks reuse the workspace (same stream: in order)
    for (uint32_t first = 0; first < b->n; first += qlzx::kL1Chunk) {
        const uint32_t cnt = std::min<uint32_t>(b->n - first, qlzx::kL1Chunk);
        hipLaunchKernelGGL(qlzx::k_enc_go_l1, dim3((cnt + 63) / 64), dim3(64), 0, (hipStream_t)stream, *b, csize,
                           status, (uint8_t *)workspace, first, cnt);
        HIP_OK(hipGetLastError());
    }
    return QLZX_R_OK;
}

int qlzx_go_decompress_batch(const qlzx_blocks *b, const uint32_t *dst_cap, uint32_t *dsize, int32_t *status,
                             void *workspace, size_t workspace_bytes, void *stream) {
    if (int r = check_l1_args(b, status, workspace, workspace_bytes, qlzx_go_decompress_workspace_size(b ? b->n : 0),
                              "qlzx_go_decompress_batch"))
        return r;
    for (uint32_t first = 0; first < b->n; first += qlzx::kL1Chunk) {
        const uint32_t cnt = std::min<uint32_t>(b->n - first, qlzx::kL1Chunk);
        hipLaunchKernelGGL(qlzx::k_dec_go_l1, dim3((cnt + 63) / 64), dim3(64), 0, (hipStream_t)stream, *b, dst_cap,
                           dsize, status, (uint8_t *)workspace, first, cnt);
        HIP_OK(hipGetLastError());
    }
    return QLZX_R_OK;
}

int qlzx_crc32_batch(const uint8_t *src, const uint64_t *src_off, const uint32_t *src_len, uint32_t n,
                     const uint32_t *init, uint32_t final_xor, uint32_t *out, void *stream) {
    if (n == 0) return QLZX_R_OK;
    if (!src || !src_off || !src_len || !out) return fail(QLZX_R_BAD_ARG, "qlzx_crc32_batch: null arg");
    hipLaunchKernelGGL(qlzx::k_crc32, dim3((n + 3) / 4), dim3(256), 0, (hipStream_t)stream, src, src_off,
                       src_len, n, init, final_xor, out);
    HIP_OK(hipGetLastError());
    return QLZX_R_OK;
}

int qlzx_synth_batch(int kind, uint64_t seed, uint64_t first_id, uint8_t *dst, const uint64_t *dst_off,
                     const uint32_t *len, uint32_t n, const uint8_t *vocab, const uint32_t *vocab_off,
                     const uint32_t *zipf_cdf, uint32_t nwords, void *stream) {
    if (n == 0) return QLZX_R_OK;
    if (!dst || !dst_off || !len || !vocab || !vocab_off || !zipf_cdf || nwords == 0)
        return fail(QLZX_R_BAD_ARG, "qlzx_synth_batch: null arg");
    hipLaunchKernelGGL(qlzx::k_synth, dim3((n + 63) / 64), dim3(64), 0, (hipStream_t)stream, kind, seed,
                       first_id, dst, dst_off, len, n, vocab, vocab_off, zipf_cdf, nwords);
    HIP_OK(hipGetLastError());
    return QLZX_R_OK;
}

int qlzx_crc32_combine(const uint32_t *raw_a, const uint32_t *raw_b, const uint32_t *len_b, uint32_t n,
                       uint32_t final_xor, uint32_t *out, void *stream) {
    if (n == 0) return QLZX_R_OK;
    if (!raw_a || !raw_b || !len_b || !out) return fail(QLZX_R_BAD_ARG, "qlzx_crc32_combine: null arg");
    hipLaunchKernelGGL(qlzx::k_crc_combine, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, raw_a, raw_b,
                       len_b, n, final_xor, out);
    HIP_OK(hipGetLastError());
    return QLZX_R_OK;
}

int qlzx_copy_batch(const uint8_t *src, const uint64_t *src_off, const uint32_t *len, uint8_t *dst,
                    const uint64_t *dst_off, uint32_t n, void *stream) {
    if (n == 0) return QLZX_R_OK;
    if (!src || !src_off || !len || !dst || !dst_off) return fail(QLZX_R_BAD_ARG, "qlzx_copy_batch: null arg");
    hipLaunchKernelGGL(qlzx::k_copy_blocks, dim3((n + 3) / 4), dim3(256), 0, (hipStream_t)stream, src, src_off, len,
                       dst, dst_off, n);
    HIP_OK(hipGetLastError());
    return QLZX_R_OK;
}

size_t qlzx_replay_workspace_size(uint64_t size) { return qlzx::replay_ws_layout(size, nullptr, nullptr); }

int qlzx_replay_index(const uint8_t *data, uint64_t size, uint64_t start, uint32_t max_key, uint64_t body_max,
                      uint64_t *rec_off, uint32_t *rec_broken, uint32_t *result, void *workspace,
                      size_t workspace_bytes, void *stream) {
    if ((!data && size) || !rec_off || !rec_broken || !result)
        return fail(QLZX_R_BAD_ARG, "qlzx_replay_index: null arg");
    if (start % 256 != 0 || start > size) return fail(QLZX_R_BAD_ARG, "qlzx_replay_index: start not a slot");
    if (size / 256 >= 0xfffffff0ull) return fail(QLZX_R_BAD_ARG, "qlzx_replay_index: file too large");
    if (!workspace || workspace_bytes < qlzx_replay_workspace_size(size))
        return fail(QLZX_R_WORKSPACE, "qlzx_replay_index: workspace too small");
    const int e = qlzx::launch_replay_index(data, size, start, max_key, body_max, rec_off, rec_broken, result,
                                            workspace, (hipStream_t)stream);
    if (e) return fail(QLZX_R_HIP, "qlzx_replay_index", (hipError_t)e);
    return QLZX_R_OK;
}

size_t qlzx_replay_plan_workspace_size(uint32_t cap) { return qlzx::replay_plan_ws_bytes(cap); }

int qlzx_replay_plan(const uint8_t *data, const uint64_t *rec_off, const uint32_t *result, uint32_t cap,
                     int32_t *hdr, uint32_t *comp_idx, uint64_t *comp_off, uint32_t *comp_len, uint32_t *comp_dsize,
                     uint64_t *comp_dst_off, uint32_t *totals, void *workspace, size_t workspace_bytes, void *stream) {
    if (!rec_off || !result || !hdr || !comp_idx || !comp_off || !comp_len || !comp_dsize || !comp_dst_off || !totals)
        return fail(QLZX_R_BAD_ARG, "qlzx_replay_plan: null arg");
    // data may be null for an empty chunk: nothing is read beyond result[0] = 0 records
    if (!workspace || workspace_bytes < qlzx::replay_plan_ws_bytes(cap))
        return fail(QLZX_R_WORKSPACE, "qlzx_replay_plan: workspace too small");
    const int e = qlzx::launch_replay_plan(data, rec_off, result, cap, hdr, comp_idx, comp_off, comp_len, comp_dsize,
                                           comp_dst_off, totals, workspace, (hipStream_t)stream);
    if (e) return fail(QLZX_R_HIP, "qlzx_replay_plan", (hipError_t)e);
    return QLZX_R_OK;
}

int qlzx_replay_finish(const uint8_t *data, const uint64_t *rec_off, const uint32_t *result, const uint32_t *totals,
                       const uint32_t *comp_idx, const int32_t *comp_status, const uint32_t *comp_dsize,
                       const uint64_t *comp_dst_off, const uint8_t *outbuf, uint32_t cap, int32_t *flag,
                       int32_t *value_len, uint8_t *in_out, uint64_t *val_off, uint16_t *vhash, void *stream) {
    if (!rec_off || !result || !totals || !comp_idx || !comp_status || !comp_dsize || !comp_dst_off || !flag ||
        !value_len || !in_out || !val_off || !vhash)
        return fail(QLZX_R_BAD_ARG, "qlzx_replay_finish: null arg");
    const int e = qlzx::launch_replay_finish(data, rec_off, result, totals, comp_idx, comp_status, comp_dsize,
                                             comp_dst_off, outbuf, cap, flag, value_len, in_out, val_off, vhash,
                                             (hipStream_t)stream);
    if (e) return fail(QLZX_R_HIP, "qlzx_replay_finish", (hipError_t)e);
    return QLZX_R_OK;
}

int qlzx_vhash_batch(const uint8_t *src, const uint64_t *off, const uint32_t *len, uint32_t n, uint16_t *out,
                     void *stream) {
    if (n == 0) return QLZX_R_OK;
    if (!src || !off || !len || !out) return fail(QLZX_R_BAD_ARG, "qlzx_vhash_batch: null arg");
    hipLaunchKernelGGL(qlzx::k_vhash, dim3((n + 63) / 64), dim3(64), 0, (hipStream_t)stream, src, off, len, n,
                       out);
    HIP_OK(hipGetLastError());
    return QLZX_R_OK;
}

}  // extern "C"

/* ---------------- single-call runtime (quicklz.h drop-in on the GPU) ----------------
 * Each calling thread owns a stream, a device buffer and a pinned host buffer, so the
 * symbols are re-entrant like the reference (quicklz.h: one scratch per call).  A call
 * copies the caller's bytes into the pinned buffer, does one H2D, the kernel, one D2H of
 * the result and its descriptor, and one stream synchronisation; the caller's pageable
 * buffers are touched only by host memcpy. */
namespace {

using qlzx::g_hip_down;

struct Meta {  // one-block batch descriptors, device side
    uint64_t src_off, dst_off;
    uint32_t src_len, dst_cap, out_size, crc_in, crc_out;
    int32_t status;
};

struct Ctx {
    hipStream_t s = nullptr;
    uint8_t *d_buf = nullptr;  // [meta 256 | src | dst | ws]
    size_t d_cap = 0;
    uint8_t *h_buf = nullptr;  // pinned: [meta 256 | staging]
    size_t h_cap = 0;
    bool ok = false;
    ~Ctx() {
        if (g_hip_down.load()) return;
        if (d_buf) (void)hipFree(d_buf);
        if (h_buf) (void)hipHostFree(h_buf);
        if (s) (void)hipStreamDestroy(s);
    }
    int init() {
        if (ok) return 0;
        int ndev = 0;
        if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(QLZX_R_NO_DEVICE, "no HIP device");
        qlzx::note_hip_up();
        HIP_OK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
        ok = true;
        return 0;
    }
    // Buffers of a call above kCtxKeep are released after it: a thread keeps at most kCtxKeep
    // of each (the single-call sizes the service does not take are the rare large values).
    static constexpr size_t kCtxKeep = 8u << 20;
    void trim() {
        if (g_hip_down.load()) return;
        if (d_cap > kCtxKeep) (void)hipFree(d_buf), d_buf = nullptr, d_cap = 0;
        if (h_cap > kCtxKeep) (void)hipHostFree(h_buf), h_buf = nullptr, h_cap = 0;
    }
    int reserve(size_t dev_bytes, size_t host_bytes) {
        if (dev_bytes > d_cap) {
            if (d_buf) (void)hipFree(d_buf);
            d_buf = nullptr;
            d_cap = 0;
            const size_t want = align_up(dev_bytes + dev_bytes / 4, 1 << 20);
            HIP_OK(hipMalloc((void **)&d_buf, want));
            d_cap = want;
        }
        if (host_bytes > h_cap) {
            if (h_buf) (void)hipHostFree(h_buf);
            h_buf = nullptr;
            h_cap = 0;
            const size_t want = align_up(host_bytes + host_bytes / 4, 1 << 20);
            HIP_OK(hipHostMalloc((void **)&h_buf, want, hipHostMallocDefault));
            h_cap = want;
        }
        return 0;
    }
};
thread_local Ctx t_ctx;


// The quicklz.h drop-ins have no error channel: cgo's CCompress ignores a 0 return and keeps an
// empty Body (quicklz/cquicklz.go:38-40, then store/item.go:145-159 stores it as "compressed"),
// and crc32_write's result becomes the record CRC (store/crc32.go:81-84).  The reference CPU
// code cannot fail, so a runtime failure here (no device, a HIP error) stops the process with
// the reason instead of returning a plausible wrong value.
// Host CRC-32/IEEE (store/crc32.go:5-59's table, slicing-by-8) for the short slices crc32_write
// receives; the tables are built once from the polynomial.
#ifndef QLZX_CRC_HOST_MAX  // longest crc32_write slice folded on the host (DESIGN.md §3 "Single calls")
#define QLZX_CRC_HOST_MAX 256
#endif
constexpr size_t kCrcHostMax = QLZX_CRC_HOST_MAX;
struct HostCrcTables {
    uint32_t t[8][256];
    HostCrcTables() {
        for (uint32_t b = 0; b < 256; b++) {
            uint32_t c = b;
            for (int k = 0; k < 8; k++) c = (c & 1u) ? (c >> 1) ^ 0xEDB88320u : c >> 1;
            t[0][b] = c;
        }
        for (uint32_t b = 0; b < 256; b++)
            for (int j = 1; j < 8; j++) t[j][b] = (t[j - 1][b] >> 8) ^ t[0][t[j - 1][b] & 0xffu];
    }
};
uint32_t host_crc32(uint32_t crc, const unsigned char *p, size_t n) {
    static const HostCrcTables T;
    uint32_t c = crc;  // crc32_write is the raw table update (store/crc32.go:61-68): no inversions
    for (; n >= 8; n -= 8, p += 8) {
        uint32_t lo, hi;
        memcpy(&lo, p, 4);
        memcpy(&hi, p + 4, 4);
        lo ^= c;
        c = T.t[7][lo & 0xff] ^ T.t[6][(lo >> 8) & 0xff] ^ T.t[5][(lo >> 16) & 0xff] ^ T.t[4][lo >> 24] ^
            T.t[3][hi & 0xff] ^ T.t[2][(hi >> 8) & 0xff] ^ T.t[1][(hi >> 16) & 0xff] ^ T.t[0][hi >> 24];
    }
    for (; n; n--, p++) c = T.t[0][(c ^ *p) & 0xffu] ^ (c >> 8);
    return c;
}

[[noreturn]] void die(const char *who) {
    fprintf(stderr, "libqlzx: %s: %s (GPU runtime failure; the drop-in has no error channel)\n", who,
            t_last_error.empty() ? "unknown error" : t_last_error.c_str());
    fflush(stderr);
    abort();
}

thread_local int t_last_status = QLZX_OK;

#ifndef QLZX_SOLO_ENC_CAP
#define QLZX_SOLO_ENC_CAP 65536u
#endif

// One block through the batch encoder.  Returns a qlzx_return code (runtime failure) and sets
// *csize (0 with t_last_status != OK when the kernel rejects the block).
int compress1(const void *source, char *destination, size_t size, uint32_t flags, size_t *csize) {
    *csize = 0;
    t_last_status = QLZX_E_RUNTIME;  // replaced below; never left over from an earlier call
    if (flags == 0 && size <= qlzx::kSvcMaxLen) {  // the request path (qlzx_service.hip)
        Service *S = service();
        if (!S) return QLZX_R_NO_DEVICE;
        const uint32_t b = S->take_slot();
        memcpy(S->in(b), source, size);
        qlzx::SvcReq r{};
        r.slot = b, r.len = (uint32_t)size, r.cap = (uint32_t)size + 400;
        const int rc = S->run(qlzx::kSvcCompress, r);
        const qlzx::SvcDone d = *(const qlzx::SvcDone *)(S->h_done + b);
        if (rc == QLZX_R_OK) {
            t_last_status = d.status;
            if (d.status == QLZX_OK && (d.out == 0 || d.out > size + 400)) {
                S->give_slot(b);
                return fail(QLZX_R_HIP, "compress1: bad result size");
            }
            if (d.status == QLZX_OK) memcpy(destination, S->out(b), d.out), *csize = d.out;
        }
        S->give_slot(b);
        return rc;
    }
    Ctx &c = t_ctx;
    if (int r = c.init()) return r;
    const bool l1 = (flags & QLZX_F_LEVEL1) != 0;
    // a lone block gets the widest encoder workgroup whatever its size (max_len only picks the
    // kernel: a 4 KiB block on the 64-thread k_encode_wg<4096> is one wave walking every phase)
    const uint32_t max_len = size <= QLZX_SOLO_ENC_CAP ? QLZX_SOLO_ENC_CAP : (uint32_t)size;
    const size_t src_b = align_up(size, 256), dst_b = align_up(size + 400, 256);
    const size_t ws_b = l1 ? qlzx_go_l1_workspace_size(1) : qlzx_compress_workspace_size(1, max_len);
    // pinned: [meta | src staging, reused for the result]
    if (int r = c.reserve(256 + src_b + dst_b + ws_b, 256 + std::max(src_b, dst_b))) return r;
    uint8_t *d_meta = c.d_buf, *d_src = d_meta + 256, *d_dst = d_src + src_b, *d_ws = d_dst + dst_b;
    Meta *m = (Meta *)c.h_buf;
    uint8_t *h_data = c.h_buf + 256;
    memset(m, 0, sizeof(Meta));
    m->src_len = (uint32_t)size;
    memcpy(h_data, source, size);
    // one H2D of descriptor + source (contiguous on both sides)
    HIP_OK(hipMemcpyAsync(d_meta, c.h_buf, 256 + size, hipMemcpyHostToDevice, c.s));
    Meta *dm = (Meta *)d_meta;
    qlzx_blocks b{d_src, &dm->src_off, &dm->src_len, d_dst, &dm->dst_off, 1};
    if (int r = l1 ? qlzx_go_l1_compress_batch(&b, &dm->out_size, &dm->status, d_ws, ws_b, c.s)
                   : qlzx_compress_batch(&b, &dm->out_size, &dm->status, nullptr, nullptr, max_len, flags, d_ws,
                                         ws_b, c.s))
        return r;
    // one D2H of descriptor + the largest possible result, then the only synchronisation
    HIP_OK(hipMemcpyAsync(c.h_buf, d_meta, sizeof(Meta), hipMemcpyDeviceToHost, c.s));
    HIP_OK(hipMemcpyAsync(h_data, d_dst, size + 400, hipMemcpyDeviceToHost, c.s));
    HIP_OK(hipStreamSynchronize(c.s));
    t_last_status = m->status;
    if (m->status != QLZX_OK) return QLZX_R_OK;
    if (m->out_size == 0 || m->out_size > size + 400) return fail(QLZX_R_HIP, "compress1: bad result size");
    memcpy(destination, h_data, m->out_size);
    *csize = m->out_size;
    c.trim();
    return QLZX_R_OK;
}

// One level-3 block through the batch decoder; *dsize = 0 with t_last_status != OK on a
// corrupt stream.
int decompress1(const char *source, void *destination, size_t *dsize_out) {
    *dsize_out = 0;
    const size_t csize = qlz_size_compressed(source), dsize = qlz_size_decompressed(source);
    t_last_status = QLZX_E_RUNTIME;  // replaced below; never left over from an earlier call
    if (csize < 3) {
        t_last_status = QLZX_E_HEADER;
        return QLZX_R_OK;
    }
    if (dsize <= qlzx::kSvcMaxLen && csize <= qlzx::kSoloMaxCsize) {  // the request path
        Service *S = service();
        if (!S) return QLZX_R_NO_DEVICE;
        const uint32_t b = S->take_slot();
        memcpy(S->in(b), source, csize);
        qlzx::SvcReq r{};
        r.slot = b, r.len = (uint32_t)csize, r.cap = (uint32_t)dsize;
        const int rc = S->run(qlzx::kSvcDecode, r);
        const qlzx::SvcDone d = *(const qlzx::SvcDone *)(S->h_done + b);
        if (rc == QLZX_R_OK) {
            t_last_status = d.status;
            if (d.status == QLZX_OK) memcpy(destination, S->out(b), d.out), *dsize_out = d.out;
        }
        S->give_slot(b);
        return rc;
    }
    Ctx &c = t_ctx;
    if (int r = c.init()) return r;
    const size_t src_b = align_up(csize, 256), dst_b = align_up(dsize + 1, 256);
    const size_t ws_b = align_up(qlzx_decompress_workspace_size(1, (uint32_t)dsize), 256);
    if (int r = c.reserve(256 + src_b + dst_b + ws_b, 256 + std::max(src_b, dst_b))) return r;
    uint8_t *d_meta = c.d_buf, *d_src = d_meta + 256, *d_dst = d_src + src_b, *d_ws = d_dst + dst_b;
    Meta *m = (Meta *)c.h_buf;
    uint8_t *h_data = c.h_buf + 256;
    memset(m, 0, sizeof(Meta));
    m->src_len = (uint32_t)csize;
    m->dst_cap = (uint32_t)dsize;
    memcpy(h_data, source, csize);
    HIP_OK(hipMemcpyAsync(d_meta, c.h_buf, 256 + csize, hipMemcpyHostToDevice, c.s));
    Meta *dm = (Meta *)d_meta;
    if (dsize <= QLZX_FAST_MAX_DSIZE && csize <= qlzx::kSoloMaxCsize) {
        // the latency path: one workgroup parses and decodes the block (qlzx_decode_solo.hip)
        static_assert(qlzx::kSoloGmax * sizeof(qlzx::GroupRec) <= (1u << 20), "solo records");
        if (int r = qlzx::launch_decode_solo(
                d_src, (uint32_t)csize, d_dst, (uint32_t)dsize, (uint32_t)dsize, (qlzx::GroupRec *)d_ws, &dm->status,
                &dm->out_size, c.s))
            return fail(QLZX_R_HIP, "decode_solo launch", (hipError_t)r);
    } else {
        qlzx_blocks b{d_src, &dm->src_off, &dm->src_len, d_dst, &dm->dst_off, 1};
        if (int r = qlzx_decompress_batch(&b, &dm->dst_cap, &dm->out_size, &dm->status, nullptr, nullptr, nullptr,
                                          (uint32_t)dsize, d_ws, ws_b, c.s))
            return r;
    }
    HIP_OK(hipMemcpyAsync(c.h_buf, d_meta, sizeof(Meta), hipMemcpyDeviceToHost, c.s));
    if (dsize) HIP_OK(hipMemcpyAsync(h_data, d_dst, dsize, hipMemcpyDeviceToHost, c.s));
    HIP_OK(hipStreamSynchronize(c.s));
    t_last_status = m->status;
    if (m->status == QLZX_OK) {
        memcpy(destination, h_data, dsize);
        *dsize_out = m->out_size;
    }
    c.trim();
    return QLZX_R_OK;
}

}  // namespace

extern "C" {

int qlzx_read_record1(const void *value, size_t vlen, uint32_t crc_state, uint32_t crc_expect, int compressed,
                      void *dst, size_t dst_cap, size_t *out_len, int32_t *status) {
    if (!value && vlen) return fail(QLZX_R_BAD_ARG, "qlzx_read_record1: null value");
    if (!out_len || !status) return fail(QLZX_R_BAD_ARG, "qlzx_read_record1: null out_len / status");
    *out_len = 0;
    *status = QLZX_E_RUNTIME;
    const uint8_t *v = (const uint8_t *)value;
    size_t dsize = 0;
    if (compressed) {
        if (vlen < 3 || vlen < (size_t)((v[0] & 2) ? 9 : 3)) {  // Payload.Decompress: CDecompressSafe's panic
            // the CRC is still checked first, as readRecordAt does before the payload is used
            const uint32_t c = vlen ? crc32_write(crc_state, (unsigned char *)value, (int)vlen) : crc_state;
            *status = (~c != crc_expect) ? QLZX_E_CRC : QLZX_E_HEADER;
            return QLZX_R_OK;
        }
        dsize = qlz_size_decompressed((const char *)value);
        if (!dst || dst_cap < dsize) return fail(QLZX_R_BAD_ARG, "qlzx_read_record1: dst_cap below the value's dsize");
    }
    const bool served = vlen <= qlzx::kSvcIn - 64 &&
                        (!compressed || (dsize <= qlzx::kSvcMaxLen && vlen <= qlzx::kSoloMaxCsize));
    if (served) {  // one request: CRC check, then the decode, in one kernel (qlzx_service.hip)
        Service *S = service();
        if (!S) return QLZX_R_NO_DEVICE;
        const uint32_t b = S->take_slot();
        memcpy(S->in(b), value, vlen);
        qlzx::SvcReq r{};
        r.slot = b, r.len = (uint32_t)vlen, r.cap = (uint32_t)dsize;
        r.arg = crc_state, r.expect = crc_expect;
        r.mode = qlzx::kSvcVerify | (compressed ? 0u : qlzx::kSvcNoDecode);
        const int rc = S->run(qlzx::kSvcDecode, r);
        const qlzx::SvcDone d = *(const qlzx::SvcDone *)(S->h_done + b);
        if (rc == QLZX_R_OK) {
            *status = d.status;
            if (d.status == QLZX_OK) {
                if (compressed) memcpy(dst, S->out(b), d.out), *out_len = d.out;
                else *out_len = vlen;
            }
        }
        S->give_slot(b);
        t_last_status = *status;
        return rc;
    }
    // longer values: the general per-call paths (GPU), CRC first
    const uint32_t c = crc32_write(crc_state, (unsigned char *)value, (int)vlen);
    if (~c != crc_expect) {
        *status = t_last_status = QLZX_E_CRC;
        return QLZX_R_OK;
    }
    if (!compressed) {
        *status = t_last_status = QLZX_OK;
        *out_len = vlen;
        return QLZX_R_OK;
    }
    size_t n = 0;
    const int rc = decompress1((const char *)value, dst, &n);
    *status = t_last_status;
    *out_len = n;
    return rc;
}

int qlzx_last_status(void) { return t_last_status; }

int qlzx_service_test_fault(int mode) {
    // a test hook: armed only in a process started with QLZX_TEST_HOOKS=1 (read once), so no
    // caller of the release library can make another thread's drop-in call fail
    static const bool armed = [] {
        const char *e = std::getenv("QLZX_TEST_HOOKS");
        return e && e[0] == '1';
    }();
    if (!armed) return fail(QLZX_R_BAD_ARG, "qlzx_service_test_fault: test hooks are off (QLZX_TEST_HOOKS=1)");
    if (mode < 1 || mode > 4) return fail(QLZX_R_BAD_ARG, "qlzx_service_test_fault: mode is 1 to 4");
    if (mode >= 3) {  // the batch decoder's next K1 (3) or K2 (4) launch
        qlzx::g_batch_fault.store(mode, std::memory_order_release);
        return QLZX_R_OK;
    }
    Service *S = service();
    if (!S) return QLZX_R_NO_DEVICE;
    S->fault.store(mode, std::memory_order_release);
    return QLZX_R_OK;
}

size_t qlz_compress(const void *source, char *destination, size_t size, char *scratch_compress) {
    (void)scratch_compress;
    if (size == 0 || size > 0xffffffffull - 400) return 0;  // quicklz.c:705-706
    size_t n = 0;
    if (compress1(source, destination, size, 0, &n) || n == 0) die("qlz_compress");
    return n;
}

size_t qlzx_compress1(const void *source, char *destination, size_t size, uint32_t flags) {
    t_last_status = QLZX_E_RUNTIME;
    if (size == 0 || size > 0xffffffffull - 400) {  // quicklz.c:705-706
        t_last_status = size ? QLZX_E_TOO_LARGE : QLZX_E_EMPTY;
        return 0;
    }
    size_t n = 0;
    return compress1(source, destination, size, flags, &n) ? 0 : n;
}

size_t qlz_decompress(const char *source, void *destination, char *scratch_decompress) {
    (void)scratch_decompress;
    size_t n = 0;
    if (decompress1(source, destination, &n)) die("qlz_decompress");
    return n;
}

size_t qlzx_go_decompress1(const char *source, size_t source_len, void *destination, size_t dst_cap) {
    t_last_status = QLZX_E_RUNTIME;  // replaced below; never left over from an earlier call
    if (!source || source_len == 0) {
        t_last_status = QLZX_E_HEADER;
        return QLZX_GO_ERROR;
    }
    const size_t hdr = (source[0] & 2) ? 9 : 3;
    const size_t dsize = source_len >= hdr ? qlz_size_decompressed(source) : 0;  // else the kernel: E_HEADER
    if (dsize > dst_cap) {
        t_last_status = QLZX_E_DST_CAP;
        fail(QLZX_R_BAD_ARG, "qlzx_go_decompress1: destination too small");
        return QLZX_GO_ERROR;
    }
    Ctx &c = t_ctx;
    if (c.init()) return QLZX_GO_ERROR;
    const size_t src_b = align_up(source_len, 256), dst_b = align_up(dsize + 1, 256);
    const size_t ws_b = qlzx_go_decompress_workspace_size(1);
    if (c.reserve(256 + src_b + dst_b + ws_b, 256 + std::max(src_b, dst_b))) return QLZX_GO_ERROR;
    uint8_t *d_meta = c.d_buf, *d_src = d_meta + 256, *d_dst = d_src + src_b, *d_ws = d_dst + dst_b;
    Meta *m = (Meta *)c.h_buf;
    uint8_t *h_data = c.h_buf + 256;
    memset(m, 0, sizeof(Meta));
    m->src_len = (uint32_t)source_len;
    m->dst_cap = (uint32_t)dsize;
    memcpy(h_data, source, source_len);
    if (hipMemcpyAsync(d_meta, c.h_buf, 256 + source_len, hipMemcpyHostToDevice, c.s) != hipSuccess)
        return fail(QLZX_R_HIP, "qlzx_go_decompress1: H2D"), QLZX_GO_ERROR;
    Meta *dm = (Meta *)d_meta;
    qlzx_blocks b{d_src, &dm->src_off, &dm->src_len, d_dst, &dm->dst_off, 1};
    if (qlzx_go_decompress_batch(&b, &dm->dst_cap, &dm->out_size, &dm->status, d_ws, ws_b, c.s)) return QLZX_GO_ERROR;
    if (hipMemcpyAsync(c.h_buf, d_meta, sizeof(Meta), hipMemcpyDeviceToHost, c.s) != hipSuccess ||
        (dsize && hipMemcpyAsync(h_data, d_dst, dsize, hipMemcpyDeviceToHost, c.s) != hipSuccess) ||
        hipStreamSynchronize(c.s) != hipSuccess)
        return fail(QLZX_R_HIP, "qlzx_go_decompress1: D2H"), QLZX_GO_ERROR;
    t_last_status = m->status;
    if (m->status != QLZX_OK) {
        char msg[64];
        snprintf(msg, sizeof msg, "qlzx_go_decompress1: status %d", (int)m->status);
        fail(QLZX_R_OK, msg);
        return QLZX_GO_ERROR;
    }
    memcpy(destination, h_data, dsize);
    return dsize;
}

uint32_t crc32_write(uint32_t crc, unsigned char *buf, int len) {
    if (len <= 0) return crc;  // store/crc32.go:65 loops zero times
    if ((size_t)len <= kCrcHostMax) {
        // readRecordAt / WriteRecord.getCRC pass header[4:24] and the key as slices of their own
        // (store/datafile.go:66-76); a request round trip (~20 us) costs more than the bytes, so
        // slices up to kCrcHostMax are folded on the calling thread.  The library still requires
        // its device: without one the call stops the process like every drop-in.
        if (!service()) die("crc32_write");
        return host_crc32(crc, buf, (size_t)len);
    }
    if ((size_t)len <= qlzx::kSvcIn - 64) {  // the request path (qlzx_service.hip)
        Service *S = service();
        if (!S) die("crc32_write");
        const uint32_t b = S->take_slot();
        memcpy(S->in(b), buf, (size_t)len);
        qlzx::SvcReq r{};
        r.slot = b, r.len = (uint32_t)len, r.arg = crc;
        const int rc = S->run(qlzx::kSvcCrc, r);
        const uint32_t v = ((const qlzx::SvcDone *)S->h_done)[b].crc;
        S->give_slot(b);
        if (rc != QLZX_R_OK) die("crc32_write");
        return v;
    }
    Ctx &c = t_ctx;
    if (c.init()) die("crc32_write");
    const size_t src_b = align_up((size_t)len, 256);
    if (c.reserve(256 + src_b, 256 + src_b)) die("crc32_write");
    uint8_t *d_meta = c.d_buf, *d_src = d_meta + 256;
    Meta *m = (Meta *)c.h_buf;
    memset(m, 0, sizeof(Meta));
    m->src_len = (uint32_t)len;
    m->crc_in = crc;
    memcpy(c.h_buf + 256, buf, (size_t)len);
    Meta *dm = (Meta *)d_meta;
    hipError_t e = hipMemcpyAsync(d_meta, c.h_buf, 256 + (size_t)len, hipMemcpyHostToDevice, c.s);
    if (e == hipSuccess &&
        qlzx_crc32_batch(d_src, &dm->src_off, &dm->src_len, 1, &dm->crc_in, 0, &dm->crc_out, c.s) != QLZX_R_OK)
        die("crc32_write");
    if (e == hipSuccess) e = hipMemcpyAsync(c.h_buf, d_meta, sizeof(Meta), hipMemcpyDeviceToHost, c.s);
    if (e == hipSuccess) e = hipStreamSynchronize(c.s);
    if (e != hipSuccess) {
        fail(QLZX_R_HIP, "crc32_write", e);
        die("crc32_write");
    }
    const uint32_t v = m->crc_out;
    c.trim();
    return v;
}

}  // extern "C"
