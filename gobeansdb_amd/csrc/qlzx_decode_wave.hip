// qlzx_decode_wave.hip -- fast batched level-3 decoder for blocks with
// dsize <= QLZX_FAST_MAX_DSIZE (the 4-64 KiB values of the BASELINE configs).
//
// Kernels per chunk of blocks: K1 k_dec_parse6 (one LANE per block: the serial
// control-word chain of quicklz.c:513-671, one 16-B GroupRec per control word) and K2
// k_dec_chunk4 (one WAVE per block: items 64 at a time, output 256 bytes at a time, every byte
// gathered from the position it copies; the record CRC is verified first when asked for,
// store/datafile.go:161-168).  Both are in qlzx_decode_v4.hip; this file holds the shared
// types, the block order, the header checks, K1's ring layout and the launcher.
//
// K1 of chunk c+1 runs on a side stream beside K2 of chunk c.
#include "qlzx_device.h"

#ifndef QLZX_FAST_MAX_DSIZE
#define QLZX_FAST_MAX_DSIZE 65536
#endif

namespace qlzx {

struct BlkInfo {
    uint32_t ngroups;
    uint32_t nitems;
    uint32_t kind;  // 0 skip (error / general path), 1 stored, 2 compressed
    uint32_t dsize;
};
struct GroupRec {
    uint32_t ip, m, a, b;
};

constexpr int32_t kPending = -1;  // status of blocks left to the general path
constexpr uint32_t kMaxDevices = 64;  // per-device side streams of the launcher
constexpr uint32_t kBlkSkip = 0, kBlkStored = 1, kBlkCompressed = 2;
// K1 workgroup: one wave (the 16 KiB LDS ring per wave bounds occupancy)
constexpr uint32_t kParseWG = 64;
#ifndef QLZX_CHUNK_BLOCKS  // blocks per K1/K2 chunk for batches of values up to 16 KiB
#define QLZX_CHUNK_BLOCKS 262144
#endif
#ifndef QLZX_CHUNK_BLOCKS_MIXED  // ... and for batches whose max_dsize exceeds 16 KiB
#define QLZX_CHUNK_BLOCKS_MIXED 131072
#endif
// Chunk size by the call's max_dsize (>= 256 CUs x 8 waves x 64 lanes: K1 fills the chip).  Same-box
// A/B (profiles/r04_c2_chunk_ab.txt, r04_chunk_c5_ab.txt): c2 (1 M x 16 KiB) 27.0 ms at 262144
// vs 27.35 at 131072; c5 (mixed 4-64 KiB, 64 GiB) 549 GiB/s at 262144 vs 621 at 131072.
__host__ __device__ inline uint32_t chunk_blocks(uint32_t max_dsize) {
    return max_dsize <= 16384 ? (uint32_t)QLZX_CHUNK_BLOCKS : (uint32_t)QLZX_CHUNK_BLOCKS_MIXED;
}
#ifndef QLZX_FIRST_CHUNK  // the first chunk's K1 is not hidden under a K2: a smaller first chunk (measured no gain)
#define QLZX_FIRST_CHUNK 0xffffffffu
#endif
__host__ __device__ inline uint32_t first_chunk_blocks(uint32_t max_dsize) {
    return QLZX_FIRST_CHUNK < chunk_blocks(max_dsize) ? (uint32_t)QLZX_FIRST_CHUNK : chunk_blocks(max_dsize);
}
constexpr uint32_t kRoundBytes = 32;  // bytes of a lane's stream per ring slot (16-B pieces)
constexpr uint32_t kPieces = kRoundBytes / 16;
// K1's LDS ring: kRingSlots rounds of kRoundBytes per lane (8 KiB per wave).  An 8-round ring
// for chunks of few waves gained 0.16 ms on c4's 4.4 ms chunk of long streams (their lanes are
// bound by the serial step chain, not by the load latency) and was dropped in round 5.
#ifndef QLZX_K1_SLOTS
#define QLZX_K1_SLOTS 4
#endif
constexpr uint32_t kRingSlots = QLZX_K1_SLOTS;
template <uint32_t S>
constexpr uint32_t kRingWaveS = S * kRoundBytes * 64;
__host__ __device__ inline uint32_t groups_max(uint32_t max_dsize) { return max_dsize / 31u + 2u; }

inline size_t rec_bytes_max(uint32_t md) { return (size_t)groups_max(md) * sizeof(GroupRec); }

inline size_t decode_wave_ws_bytes(uint32_t n, uint32_t max_dsize) {
    const uint32_t md = max_dsize > QLZX_FAST_MAX_DSIZE ? QLZX_FAST_MAX_DSIZE : max_dsize;
    const uint32_t cb = chunk_blocks(max_dsize);
    const uint32_t c = n < cb ? (n ? n : 1) : cb;
    return (((size_t)c * sizeof(BlkInfo) + 255) & ~(size_t)255) +
           ((((size_t)c * rec_bytes_max(md)) + 255) & ~(size_t)255) +
           ((((size_t)n * sizeof(uint32_t)) + 255) & ~(size_t)255) +              // block order, whole call
           1024 + 256;                                                            // order aux
}

// Workspace regions of a call (qlzx_decompress_workspace_size): 1 for a single chunk, 2 so K1 of
// chunk c+1 runs beside K2 of chunk c, and for calls of mixed sizes over three chunks or more one
// more region for each of the last QLZX_LAST_K1_EARLY chunks (the longest values, whose
// one-lane-per-block K1s are the longest): their K1s start with the first one.  One early chunk:
// c5 rounds of 15.4 GiB 616.8 GiB/s (two runs) against 610.0 with two and 606.3 with none; two
// early K1s hold enough LDS (8 KiB per K1 wave) to slow the first K2s 4x (profiles/r06_mixed_ab.txt).
#ifndef QLZX_LAST_K1_EARLY
#define QLZX_LAST_K1_EARLY 1
#endif
inline uint32_t decode_wave_early(uint32_t nchunks, uint32_t max_dsize) {
    if (max_dsize <= 16384 || nchunks < 3) return 0u;
    const uint32_t e = nchunks - 2;  // two regions stay for the chunks before
    return e < (uint32_t)QLZX_LAST_K1_EARLY ? e : (uint32_t)QLZX_LAST_K1_EARLY;
}
inline uint32_t decode_wave_chunks(uint32_t n, uint32_t max_dsize) {
    const uint32_t c0 = first_chunk_blocks(max_dsize), cb = chunk_blocks(max_dsize);
    return n <= c0 ? 1u : 1u + (n - c0 + cb - 1) / cb;
}
inline uint32_t decode_wave_halves(uint32_t n, uint32_t max_dsize) {
    const uint32_t nc = decode_wave_chunks(n, max_dsize);
    return nc == 1 ? 1u : 2u + decode_wave_early(nc, max_dsize);
}

// ---------------------------------------------------------- block order ----
// K1 runs one lane per block, so a wave lasts as long as its longest stream: with mixed
// 4-64 KiB values (c4, c5) most lanes would idle behind one 64 KiB block.  Two small
// kernels list ALL blocks of the call by compressed size, smallest first (counting sort on
// len / 512, 128 classes), and the chunks are cut from that list: K1 and K2 of chunk c take
// blocks list[c * chunk ..] and index their workspace by the place in the chunk.  So a K1
// wave's lanes have similar lengths, and K1(c+1), whose blocks are at most a class longer,
// hides under K2(c), whose chunk has as many blocks; the first, exposed K1 parses the
// smallest blocks.  Order within a class is arbitrary: outputs are indexed by the block.
// aux (zeroed before k_order_count): [0,128) class counts, [128,256) class cursors.
// One-wave workgroups (16 blocks per lane), launched before the first K1: a kernel queued
// between two K1s on the side stream delayed K1(c+1) until K2(c) had filled the CUs, and a
// 1024-thread workgroup waited for a whole CU to drain; both serialised K1 behind K2.
constexpr uint32_t kOrderClasses = 128, kOrderWG = 64, kOrderEPT = 16, kOrderPerWG = kOrderWG * kOrderEPT;
constexpr uint32_t kOrderAux = 2 * kOrderClasses;
__device__ __forceinline__ uint32_t order_class(uint32_t len) {
    const uint32_t c = len >> 9;
    return c < kOrderClasses - 1 ? c : kOrderClasses - 1;
}
#ifndef QLZX_K2_ONLY
__global__ void __launch_bounds__(kOrderWG) k_order_count(const uint32_t *src_len, uint32_t n, uint32_t *aux) {
    __shared__ uint32_t h[kOrderClasses];
    const uint32_t tid = threadIdx.x, i0 = blockIdx.x * kOrderPerWG + tid;
    for (uint32_t k = tid; k < kOrderClasses; k += kOrderWG) h[k] = 0;
    __syncthreads();
    uint32_t len[kOrderEPT];
#pragma unroll
    for (uint32_t e = 0; e < kOrderEPT; e++) {
        const uint32_t i = i0 + e * kOrderWG;
        len[e] = i < n ? src_len[i] : 0u;
    }
#pragma unroll
    for (uint32_t e = 0; e < kOrderEPT; e++)
        if (i0 + e * kOrderWG < n) atomicAdd(&h[order_class(len[e])], 1u);
    __syncthreads();
    for (uint32_t k = tid; k < kOrderClasses; k += kOrderWG)
        if (h[k]) atomicAdd(&aux[k], h[k]);
}
#endif  // QLZX_K2_ONLY
#ifndef QLZX_K2_ONLY
__global__ void __launch_bounds__(kOrderWG) k_order_scatter(const uint32_t *src_len, uint32_t n, uint32_t *aux,
                                                           uint32_t *list) {
    __shared__ uint32_t start[kOrderClasses], lc[kOrderClasses];
    const uint32_t tid = threadIdx.x, i0 = blockIdx.x * kOrderPerWG + tid;
    for (uint32_t k = tid; k < kOrderClasses; k += kOrderWG) start[k] = aux[k], lc[k] = 0;
    __syncthreads();
    if (tid == 0) {  // exclusive scan of the class counts (128 LDS words)
        uint32_t acc = 0;
        for (uint32_t k = 0; k < kOrderClasses; k++) {
            const uint32_t v = start[k];
            start[k] = acc;
            acc += v;
        }
    }
    uint32_t c[kOrderEPT], r[kOrderEPT];
#pragma unroll
    for (uint32_t e = 0; e < kOrderEPT; e++) {
        const uint32_t i = i0 + e * kOrderWG;
        c[e] = i < n ? order_class(src_len[i]) : 0u;
    }
#pragma unroll
    for (uint32_t e = 0; e < kOrderEPT; e++)
        r[e] = (i0 + e * kOrderWG < n) ? atomicAdd(&lc[c[e]], 1u) : 0u;  // rank in this workgroup's class
    __syncthreads();
    for (uint32_t k = tid; k < kOrderClasses; k += kOrderWG)
        if (lc[k]) start[k] += atomicAdd(&aux[kOrderClasses + k], lc[k]);
    __syncthreads();
#pragma unroll
    for (uint32_t e = 0; e < kOrderEPT; e++)
        if (i0 + e * kOrderWG < n) list[start[c[e]] + r[e]] = i0 + e * kOrderWG;
}
#endif  // QLZX_K2_ONLY

// ------------------------------------------------------------------ K1 ----
// Header checks of one block of `len` bytes (quicklz.c:780-811 and the batch API's bounds):
// the status, and for QLZX_OK its kind (kBlkStored / kBlkCompressed), sizes and header length.
__device__ __forceinline__ int classify_block(const uint8_t *src, uint32_t len, uint32_t cap, uint32_t max_dsize,
                                              uint32_t &kind, uint32_t &csize, uint32_t &dsize, uint32_t &hdr) {
    kind = kBlkSkip;
    if (len < 3) return QLZX_E_HEADER;
    hdr = (src[0] & 2u) ? 9u : 3u;
    if (len < hdr) return QLZX_E_HEADER;
    const Header h = parse_header(src);
    csize = h.csize;
    dsize = h.dsize;
    if (h.csize != len) return QLZX_E_SIZE_COMPRESSED;
    if (h.level != 3) return QLZX_E_LEVEL;
    if (h.dsize > cap) return QLZX_E_DST_CAP;
    if (h.dsize > max_dsize) return QLZX_E_MAX_DSIZE;     // the caller's bound is wrong
    if (h.dsize > QLZX_FAST_MAX_DSIZE) return kPending;  // general path owns it
    if (!h.compressed) {
        if (csize < hdr + dsize) return QLZX_E_CORRUPT;
        kind = kBlkStored;
    } else {
        kind = kBlkCompressed;
    }
    return QLZX_OK;
}

// Ring layout per wave: [slot][piece][lane][16 B]; stream byte p of a lane (q = p + shift,
// shift = src & 15) lives in round q / kRoundBytes, slot round % S, piece (q / 16) % kPieces,
// byte q % 16 -- i.e. at ((q / 16) % (kPieces S)) * 1 KiB + lane * 16 + q % 16.
template <uint32_t S>
__device__ __forceinline__ uint32_t ring_off(uint32_t q, uint32_t lane) {
    return (((q >> 4) & (kPieces * S - 1)) << 10) | (lane << 4) | (q & 15u);
}
template <uint32_t S>
__device__ __forceinline__ uint32_t ring_rd32(const uint8_t *ring, uint32_t q, uint32_t lane) {
    const uint32_t qa = q & ~3u;
    const uint32_t lo = *(const uint32_t *)(ring + ring_off<S>(qa, lane));
    const uint32_t hi = *(const uint32_t *)(ring + ring_off<S>(qa + 4, lane));
    return __builtin_amdgcn_alignbyte(hi, lo, q & 3u);
}

// ------------------------------------------------------------------- K2 helpers ----
// Per-lane coordinates of item I = 64 bt + lane: group g = I / 31, index k = I % 31.
// Advanced by one batch (64 = 2 * 31 + 2) without a division.
struct ItemCursor {
    uint32_t g, k;
    __device__ __forceinline__ void next() {
        k += 2;
        const bool wrap = k >= 31;
        k = wrap ? k - 31 : k;
        g += wrap ? 3 : 2;
    }
};

// Branch-free level-3 token decode (quicklz.c:579-610).  Token type
// ty = (t & 3) + ((t & 127) == 3) selects per-type bit fields from packed tables:
//   ty 0: 1 B, off = t[2:8),  len 3          ty 1: 2 B, off = t[2:16), len 3
//   ty 2: 2 B, off = t[6:16), len = t[2:6)+3  ty 3: 3 B, off = t[7:24), len = t[2:7)+2
//   ty 4: 4 B, off = t[15:32), len = t[7:15)+3
__device__ __forceinline__ void decode_tok_bf(uint32_t t, uint32_t &off, uint32_t &len, uint32_t &tl) {
    const uint32_t ty = (t & 3u) + ((t & 127u) == 3u ? 1u : 0u);
    const uint32_t f4 = ty * 4, f6 = ty * 6;
    const uint32_t osh = __builtin_amdgcn_ubfe(0xF7622u, f4, 4);
    const uint32_t ow = __builtin_amdgcn_ubfe((6u) | (14u << 6) | (10u << 12) | (17u << 18) | (17u << 24), f6, 6);
    const uint32_t lsh = __builtin_amdgcn_ubfe(0x72200u, f4, 4);
    const uint32_t lw = __builtin_amdgcn_ubfe(0x85400u, f4, 4);
    const uint32_t la = __builtin_amdgcn_ubfe(0x32333u, f4, 4);
    tl = __builtin_amdgcn_ubfe(0x43221u, f4, 4);
    off = __builtin_amdgcn_ubfe(t, osh, ow);
    len = __builtin_amdgcn_ubfe(t, lsh, lw) + la;
}

// Inclusive prefix sum over the 64 lanes with DPP (row shifts + row broadcasts).
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, true);   // row_shr:1
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, true);   // row_shr:2
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, true);   // row_shr:4
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, true);   // row_shr:8
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false);  // row_bcast:15
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false);  // row_bcast:31
    return v;
}

__device__ __forceinline__ uint32_t ff1_or(uint64_t m, uint32_t dflt) {
    return m ? (uint32_t)__builtin_ctzll(m) : dflt;
}

// Inclusive max over lanes 0..lane; DPP row shifts + row broadcasts.
__device__ __forceinline__ uint32_t wave_incl_max(uint32_t v) {
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false));  // row_shr:1
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false));  // row_shr:2
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false));  // row_shr:4
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false));  // row_shr:8
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false));  // row_bcast:15
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false));  // row_bcast:31
    return v;
}
// Value of lane - 1 (0 in lane 0): DPP wave_shr:1.
__device__ __forceinline__ uint32_t wave_shr1(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x138, 0xf, 0xf, false);
}

}  // namespace qlzx
#ifndef QLZX_K2_ONLY
#include "qlzx_decode_solo.hip"
#include "qlzx_decode_small.hip"
#endif
#include "qlzx_decode_v4.hip"
namespace qlzx {

#ifndef QLZX_K2_ONLY
// Set by an atexit handler registered once the runtime is in use (after HIP registered its own
// teardown; atexit runs in reverse order): per-thread HIP objects destroyed after that (threads
// exiting during process exit) are left to the runtime's teardown.
inline std::atomic<bool> g_hip_down{false};
inline void note_hip_up() {
    static std::once_flag once;
    std::call_once(once, [] { std::atexit([] { g_hip_down.store(true); }); });
}

#ifndef QLZX_K1_KMAX_UNI  // K1's step budget per iteration: uniform 16 KiB calls / mixed sizes (16 / 10 with the
                          // default scheduler; 12 / 10 under iterative-ILP: profiles/r05_sched_strategy_ab.txt)
#define QLZX_K1_KMAX_UNI 12
#endif
#ifndef QLZX_K1_KMAX_MIX
#define QLZX_K1_KMAX_MIX 10
#endif
#if QLZX_SPLIT_K1
int launch_k1_parse6(uint32_t grid, hipStream_t s, const qlzx_blocks &b, const uint32_t *dst_cap, uint32_t *dsize,
                     int32_t *status, uint32_t first, uint32_t cnt, BlkInfo *info, GroupRec *recs, uint32_t gmax,
                     const uint32_t *order, uint32_t max_dsize, uint32_t kmax);
#endif
#if QLZX_SPLIT_K2  // K2 without CRC lives in qlzx_k2.hip (its own scheduler strategy)
int launch_k2_nocrc(uint32_t grid, hipStream_t s, const qlzx_blocks &b, uint32_t *dsize, int32_t *status,
                    uint32_t first, uint32_t cnt, const BlkInfo *info, const GroupRec *recs, uint32_t gmax,
                    const uint32_t *order, bool big);
#endif
// Test hook (qlzx_service_test_fault modes 3 / 4, inert unless QLZX_TEST_HOOKS=1): the next K1 /
// K2 launch of a batch call is replaced by a launch failure, so the caller's error path runs.
inline std::atomic<int> g_batch_fault{0};
inline int batch_fault(int kernel) {
    int k = kernel;
    return g_batch_fault.load(std::memory_order_relaxed) == kernel && g_batch_fault.compare_exchange_strong(k, 0)
               ? (int)hipErrorLaunchFailure
               : 0;
}
// K1's grid: one wave per 64 blocks (persistent K1 waves, 512-2048 of them, made K1 the critical
// path: c2 24.2-35.7 ms against 23.8, DESIGN.md history, round 6)
inline uint32_t k1_grid(uint32_t cnt) { return (cnt + kParseWG - 1) / kParseWG; }
inline int launch_decode_wave(const qlzx_blocks &b, const uint32_t *dst_cap, uint32_t *dsize,
                              int32_t *status, const uint32_t *crc_state, const uint32_t *crc_expect,
                              uint32_t *crc_out, uint32_t max_dsize, void *ws, size_t ws_bytes,
                              hipStream_t s) {
    const uint32_t md = max_dsize > QLZX_FAST_MAX_DSIZE ? QLZX_FAST_MAX_DSIZE : max_dsize;
    const uint32_t gmax = groups_max(md);
    const uint32_t chunk = b.n < chunk_blocks(max_dsize) ? b.n : chunk_blocks(max_dsize);
    const uint32_t chunk0 = first_chunk_blocks(max_dsize);
    const size_t o_rec = ((size_t)chunk * sizeof(BlkInfo) + 255) & ~(size_t)255;
    const size_t one = decode_wave_ws_bytes(b.n, max_dsize);
    const size_t o_list = o_rec + ((((size_t)chunk * rec_bytes_max(md)) + 255) & ~(size_t)255);
    const size_t o_aux = o_list + ((((size_t)b.n * sizeof(uint32_t)) + 255) & ~(size_t)255);
    const bool sort = chunk > 64;
    // two workspace halves when the caller gave room for them: K1 of chunk c+1 runs on a
    // side stream while K2 of chunk c runs on `s` (K1 is latency-bound at low occupancy)
#ifndef QLZX_OVERLAP  // 0: K1 and K2 of all chunks on the caller's stream, one after another (timing)
#define QLZX_OVERLAP 1
#endif
    const bool overlap = QLZX_OVERLAP && ws_bytes >= 2 * one && b.n > chunk0;
    // per host thread (the batch API is re-entrant like the reference) and per device: the
    // side stream and events are created on the device that owns `s`
    struct Side {  // destroyed with the thread (Go runs cgo calls on many OS threads)
        hipStream_t st = nullptr, st2 = nullptr, st3 = nullptr;
        hipEvent_t k1[2] = {}, k2[2] = {}, order = nullptr, last[2] = {};
        ~Side() {
            if (!st || g_hip_down.load()) return;
            for (int j = 0; j < 2; j++) {
                if (k1[j]) (void)hipEventDestroy(k1[j]);
                if (k2[j]) (void)hipEventDestroy(k2[j]);
            }
            if (order) (void)hipEventDestroy(order);
            for (int j = 0; j < 2; j++)
                if (last[j]) (void)hipEventDestroy(last[j]);
            if (st3) (void)hipStreamDestroy(st3);
            if (st2) (void)hipStreamDestroy(st2);
            (void)hipStreamDestroy(st);
        }
    };
    thread_local Side sides[kMaxDevices];
    hipStream_t side = nullptr, side2 = nullptr, side3 = nullptr;
    hipEvent_t *ev_k1 = nullptr, *ev_k2 = nullptr, ev_order = nullptr, *ev_last = nullptr;
    if (overlap) {
        int dev = 0, cur = 0;
        if (s) {
            hipDevice_t hd;
            if (hipStreamGetDevice(s, &hd) != hipSuccess) return (int)hipErrorInvalidResourceHandle;
            dev = (int)hd;
        } else if (hipGetDevice(&dev) != hipSuccess) {
            return (int)hipErrorNoDevice;
        }
        if (dev < 0 || dev >= (int)kMaxDevices) return (int)hipErrorInvalidDevice;
        Side &sd = sides[dev];
        if (!sd.st) {
            note_hip_up();
            (void)hipGetDevice(&cur);
            if (cur != dev) (void)hipSetDevice(dev);
            hipError_t e = hipStreamCreateWithFlags(&sd.st, hipStreamNonBlocking);
            if (e == hipSuccess) e = hipStreamCreateWithFlags(&sd.st2, hipStreamNonBlocking);
            if (e == hipSuccess) e = hipStreamCreateWithFlags(&sd.st3, hipStreamNonBlocking);
            if (e == hipSuccess) e = hipEventCreateWithFlags(&sd.order, hipEventDisableTiming);
            for (int j = 0; j < 2 && e == hipSuccess; j++) e = hipEventCreateWithFlags(&sd.last[j], hipEventDisableTiming);
            for (int j = 0; j < 2 && e == hipSuccess; j++) {
                e = hipEventCreateWithFlags(&sd.k1[j], hipEventDisableTiming);
                if (e == hipSuccess) e = hipEventCreateWithFlags(&sd.k2[j], hipEventDisableTiming);
            }
            if (cur != dev) (void)hipSetDevice(cur);
            if (e != hipSuccess) return (int)e;
        }
        side = sd.st;
        side2 = sd.st2;
        side3 = sd.st3;
        ev_k1 = sd.k1;
        ev_k2 = sd.k2;
        ev_order = sd.order;
        ev_last = sd.last;
    }
    const bool crc = crc_state || crc_expect || crc_out;
    // A call of two chunks of mixed block sizes (smallest blocks first): K1 of the second chunk
    // runs on a second side stream, so it starts with the first K1 instead of after it.  It holds
    // the longest streams, and its K1 (one lane per block, latency-bound) was the critical path
    // (c4: 15.3 -> 11.7 ms per 4000 MiB chunk with k_rp_scan).  Calls of more chunks (c5's
    // rounds: 560 vs 620 GiB/s) and uniform 16 KiB chunks keep one side stream: there concurrent
    // K1s only compete with the K2s.
    const bool split_k1 = overlap && max_dsize > 16384 && b.n <= chunk0 + chunk;  // two chunks (c4's calls)
    // Calls of mixed sizes over three chunks or more (c5's rounds): the last chunks hold the
    // longest values, and their K1s (longest per lane, at low occupancy) ran after K2 of the chunk
    // two before had freed a workspace half, in front of their K2s (c5: the last K1 took 7.5 of
    // an 18.7 ms call).  With a region of their own, the K1s of the last `early` chunks start on
    // side streams 2 and 3 right after the block order, beside everything else.
    const uint32_t nchunks = decode_wave_chunks(b.n, max_dsize);
    uint32_t early = overlap ? decode_wave_early(nchunks, max_dsize) : 0u;
    while (early && ws_bytes < (2 + early) * one) early--;  // as many regions as the caller gave
    const uint32_t c_early = nchunks - early;                // first chunk whose K1 starts early
    if (overlap) (void)hipEventRecord(ev_k2[1], s), (void)hipStreamWaitEvent(side, ev_k2[1], 0);
    if (split_k1 || early) (void)hipStreamWaitEvent(side2, ev_k2[1], 0);
    if (early > 1) (void)hipStreamWaitEvent(side3, ev_k2[1], 0);
    if (sort) {  // block order of the whole call, ahead of the first K1 (workspace half 0)
        hipStream_t s1 = overlap ? side : s;
        uint32_t *aux = (uint32_t *)((uint8_t *)ws + o_aux);
        (void)hipMemsetAsync(aux, 0, kOrderAux * sizeof(uint32_t), s1);
        const dim3 g((b.n + kOrderPerWG - 1) / kOrderPerWG);
        hipLaunchKernelGGL(k_order_count, g, dim3(kOrderWG), 0, s1, b.src_len, b.n, aux);
        hipLaunchKernelGGL(k_order_scatter, g, dim3(kOrderWG), 0, s1, b.src_len, b.n, aux,
                           (uint32_t *)((uint8_t *)ws + o_list));
        if (split_k1 || early) {
            (void)hipEventRecord(ev_order, side), (void)hipStreamWaitEvent(side2, ev_order, 0);
            if (early > 1) (void)hipStreamWaitEvent(side3, ev_order, 0);
        }
    }
    for (uint32_t j = 0; j < early; j++) {  // the longest chunk first
        const uint32_t ce = nchunks - 1 - j;
        const uint32_t fe = chunk0 + (ce - 1) * chunk;
        const uint32_t cnt = (ce == nchunks - 1 ? b.n : fe + chunk) - fe;
        uint8_t *w = (uint8_t *)ws + (2 + (ce - c_early)) * one;
        uint32_t *order = sort ? (uint32_t *)((uint8_t *)ws + o_list) + fe : nullptr;
        hipStream_t se = j == 0 ? side2 : side3;
        if (const int ef = batch_fault(3)) return ef;
#if QLZX_SPLIT_K1
        if (const int e1 = launch_k1_parse6(k1_grid(cnt), se, b, dst_cap, dsize, status, fe, cnt, (BlkInfo *)w,
                                            (GroupRec *)(w + o_rec), gmax, order, max_dsize,
                                            (uint32_t)QLZX_K1_KMAX_MIX))
            return e1;
#else
        hipLaunchKernelGGL(k_dec_parse6, dim3(k1_grid(cnt)), dim3(kParseWG), 0, se, b, dst_cap, dsize, status, fe,
                           cnt, (BlkInfo *)w, (GroupRec *)(w + o_rec), gmax, order, max_dsize,
                           (uint32_t)QLZX_K1_KMAX_MIX);
#endif
        (void)hipEventRecord(ev_last[ce - c_early], se);
    }
    uint32_t c = 0;
    for (uint32_t first = 0, cnt = 0; first < b.n; first += cnt, c++) {
        const uint32_t cap = c == 0 ? chunk0 : chunk;
        cnt = b.n - first < cap ? b.n - first : cap;
        const bool last_early = c >= c_early;  // its K1 is already queued on side stream 2 or 3
        uint8_t *w = (uint8_t *)ws + (last_early ? (2 + (c - c_early)) * one : overlap ? (c & 1) * one : 0);
        BlkInfo *info = (BlkInfo *)w;
        GroupRec *recs = (GroupRec *)(w + o_rec);
        uint32_t *order = sort ? (uint32_t *)((uint8_t *)ws + o_list) + first : nullptr;
        hipStream_t s1 = overlap ? (split_k1 && (c & 1) ? side2 : side) : s;
        if (last_early) {
            (void)hipStreamWaitEvent(s, ev_last[c - c_early], 0);
        } else {
            if (overlap && c >= 2) (void)hipStreamWaitEvent(s1, ev_k2[c & 1], 0);  // K2(c-2) freed this half
            // K1's step budget per iteration: QLZX_K1_KMAX_UNI (12) for uniform 16 KiB calls,
            // QLZX_K1_KMAX_MIX (10) for mixed sizes (c4: 377 vs 363 GiB/s; c5 580 vs 560)
#if QLZX_SPLIT_K1
            // the helpers return hipGetLastError(), which also clears the error: keep it here
            if (const int ef = batch_fault(3)) return ef;
            if (const int e1 = launch_k1_parse6(k1_grid(cnt), s1, b, dst_cap, dsize, status, first, cnt, info, recs,
                                   gmax, order, max_dsize, max_dsize > 16384 ? (uint32_t)QLZX_K1_KMAX_MIX : (uint32_t)QLZX_K1_KMAX_UNI))
                return e1;
#else
            hipLaunchKernelGGL(k_dec_parse6, dim3(k1_grid(cnt)), dim3(kParseWG), 0, s1, b, dst_cap, dsize,
                               status, first, cnt, info, recs, gmax, order, max_dsize, max_dsize > 16384 ? (uint32_t)QLZX_K1_KMAX_MIX : (uint32_t)QLZX_K1_KMAX_UNI);
#endif
            if (overlap) (void)hipEventRecord(ev_k1[c & 1], s1), (void)hipStreamWaitEvent(s, ev_k1[c & 1], 0);
        }
        // one kernel for every block size: the LDS window slides over longer blocks
        if (const int ef = batch_fault(4)) return ef;
        if (crc)
            hipLaunchKernelGGL(k_dec_chunk4<true>, dim3(cnt), dim3(64), 0, s, b, dsize, status, first, cnt, info,
                               recs, gmax, (const uint32_t *)order, crc_state, crc_expect, crc_out);
        else
#if QLZX_SPLIT_K2
            if (const int e2 = launch_k2_nocrc(cnt, s, b, dsize, status, first, cnt, info, recs, gmax,
                                               (const uint32_t *)order, max_dsize > 16384))
                return e2;
#else
            hipLaunchKernelGGL(k_dec_chunk4<false>, dim3(cnt), dim3(64), 0, s, b, dsize, status, first, cnt, info,
                               recs, gmax, (const uint32_t *)order, nullptr, nullptr, nullptr);
#endif
        if (overlap) (void)hipEventRecord(ev_k2[c & 1], s);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return (int)e;
    }
    return 0;
}

#endif  // QLZX_K2_ONLY
}  // namespace qlzx
