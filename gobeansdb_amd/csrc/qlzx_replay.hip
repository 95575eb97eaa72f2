// qlzx_replay.hip -- batched replay of a .data chunk:
// record discovery with the nextValid resync of DataStreamReader
// (store/datafile.go:202-277), record CRC verify (store/datafile.go:66-76,
// 161-168) and the value hash Getvhash/Fnv1a (store/item.go:89-100,
// utils/hash.go:8-16).
//
// The sequential reader becomes data-parallel in four steps:
//   1. every 256-B slot is classified from its 24-B header; the plausible ones
//      (1 <= ksz <= max_key, vsz <= body_max, fits the file) are candidates;
//   2. one wave per candidate computes the record CRC: rsz[s] = the padded
//      record size when readRecordAt(256 s) would succeed, else 0 (steps 1 and 2
//      are one kernel, k_rp_scan, over 64-slot groups);
//   3. valid slots are compacted in order (A[]), and each gets its successor:
//      the reader, at the end p of record A[i], either hits an error (partial
//      header / truncated record with valid sizes: Next() returns an error),
//      reads the record at p (valid) or resyncs to the first valid slot >= p
//      (nextValid).  Because vidx[] is the exclusive count of valid slots,
//      "first valid slot >= p" is simply index vidx[p / 256];
//   4. the path from the start position is marked by pointer doubling
//      (log2 rounds) and compacted into the visited record list with each
//      record's sizeBroken.
#include "qlzx_device.h"

namespace qlzx {

constexpr uint32_t kRpSlot = 256;
constexpr uint32_t kRpHdr = 24;
enum : uint8_t { kSlotBadSize = 1, kSlotTrunc = 2, kSlotPartial = 3, kSlotCand = 4 };
constexpr uint32_t kScanTile = 1024;  // elements per scan tile (256 threads x 4)

struct RpCounters {
    uint32_t ncand, m, r0, nvis, end_kind, nlong, pad[2];
};

// 1-2. slot classification (readRecordAt's size checks, store/datafile.go:128-136) and the
// record CRC of every candidate, one wave each (wave_crc of qlzx_crc.hip).  A wave
// takes ~3 us per 4 KiB stripe, so a candidate longer than kRpLong (a false candidate can
// claim up to BodyMax = 50 MiB) would be one wave's serial tail for the whole launch: those go
// to a list (lng[], their per-list XOR accumulator and segment counter zeroed here) and are
// cut into kRpSeg segments that k_rp_crc_long spreads over every wave of the chip.
constexpr uint32_t kRpLong = 128u << 10;
constexpr uint32_t kRpSeg = 16u << 10;

__device__ __forceinline__ void rp_crc_verdict(const uint8_t *h, uint32_t s, uint32_t ksz, uint32_t vsz,
                                               uint32_t reg, uint32_t *rsz) {
    if ((reg ^ 0xffffffffu) == *(const uint32_t *)h) rsz[s] = ((kRpHdr + ksz + vsz + 255u) >> 8) << 8;
}

// k_rp_scan (round 5): a wave takes 64 consecutive slots (16 KiB of chunk) at a time, classifies
// them (one header load per lane, coalesced kind/rsz stores) and CRCs its candidates in slot
// order right away.  Round 4 ran the classification as a kernel of its own (one strided header
// load per thread and a candidate list behind one contended counter) before the CRC kernel:
// 2.2 + 1.5 ms per 4000 MiB chunk.  Long candidates still go to the k_rp_crc_long list.
__global__ void __launch_bounds__(256) k_rp_scan(const uint8_t *data, uint64_t size, uint32_t nslots, uint32_t max_key,
                                                 uint64_t body_max, uint8_t *kind, uint32_t *rsz, RpCounters *cnt,
                                                 uint32_t *lng, uint32_t *lacc, uint32_t *ldone) {
    __shared__ uint32_t tab[kCrcLdsWords];
    load_crc_lds(tab);
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t ngroups = (nslots + 63) / 64;
    uint32_t ncand = 0;
    for (uint32_t g = blockIdx.x * 4 + threadIdx.x / 64; g < ngroups; g += gridDim.x * 4) {
        const uint32_t s = g * 64 + lane;
        const bool in = s < nslots;
        const uint64_t off = (uint64_t)s * kRpSlot;
        uint8_t k = kSlotPartial;
        uint32_t ksz = 0, vsz = 0;
        if (in && off + kRpHdr <= size) {
            const uint2 kv = *(const uint2 *)(data + off + 16);
            ksz = kv.x, vsz = kv.y;
            if (ksz == 0 || ksz > max_key || (uint64_t)vsz > body_max) k = kSlotBadSize;
            else if (off + kRpHdr + ksz + vsz > size) k = kSlotTrunc;
            else k = kSlotCand;
        }
        if (in) {
            rsz[s] = 0;
            kind[s] = k;
        }
        uint64_t m = __ballot(in && k == kSlotCand);
        ncand += (uint32_t)__builtin_popcountll(m);
        while (m) {
            const uint32_t L = (uint32_t)__builtin_ctzll(m);
            m &= m - 1;
            const uint32_t sc = g * 64 + L;
            const uint32_t k2 = __shfl(ksz, L, 64), v2 = __shfl(vsz, L, 64);
            const uint32_t len = 20 + k2 + v2;  // header[4:24] ‖ key ‖ value
            const uint8_t *h = data + (uint64_t)sc * kRpSlot;
            if (len > kRpLong) {
                if (lane == 0) {
                    const uint32_t j = atomicAdd(&cnt->nlong, 1u);
                    lng[j] = sc;
                    lacc[j] = 0;
                    ldone[j] = 0;
                }
                continue;
            }
            const uint32_t reg = wave_crc(tab, h + 4, len, 0xffffffffu, lane);
            if (lane == 0) rp_crc_verdict(h, sc, k2, v2, reg, rsz);
        }
    }
    if (lane == 0 && ncand) atomicAdd(&cnt->ncand, ncand);
}

// long candidates: every wave walks the (normally empty or tiny) list 64 entries at a time
// (one load per lane, a wave scan of the segment counts) and takes the segments g of the
// global segment sequence with g = wave id (mod all waves).  A segment's raw CRC, shifted over
// the bytes after it, is XORed into its candidate's accumulator, and the wave that completes
// the last segment (counter == nseg) turns the sum into the verdict.
__global__ void __launch_bounds__(256) k_rp_crc_long(const uint8_t *data, const RpCounters *cnt,
                                                     uint32_t *rsz, const uint32_t *lng, uint32_t *lacc,
                                                     uint32_t *ldone) {
    __shared__ uint32_t tab[kCrcLdsWords];
    const uint32_t nl = cnt->nlong;
    if (nl == 0) return;
    load_crc_lds(tab);
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wid = blockIdx.x * 4 + threadIdx.x / 64, nw = gridDim.x * 4;
    uint64_t base = 0;  // global index of the batch's first segment
    for (uint32_t e0 = 0; e0 < nl; e0 += 64) {
        const uint32_t e = e0 + lane;
        uint32_t s = 0, len = 0;
        if (e < nl) {
            s = lng[e];
            const uint2 kv = *(const uint2 *)(data + (uint64_t)s * kRpSlot + 16);
            len = 20 + kv.x + kv.y;
        }
        const uint32_t ns = (len + kRpSeg - 1) / kRpSeg;
        uint32_t inc = ns;
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t y = __shfl_up(inc, d, 64);
            if (lane >= (uint32_t)d) inc += y;
        }
        const uint32_t total = __shfl(inc, 63, 64);
        for (uint32_t r = (uint32_t)((wid + nw - base % nw) % nw); r < total; r += nw) {
            const uint32_t L = (uint32_t)__builtin_ctzll(__ballot(inc > r));
            const uint32_t sl_s = __shfl(s, L, 64), sl_len = __shfl(len, L, 64);
            const uint32_t nseg = __shfl(ns, L, 64);
            const uint32_t o = (r - (__shfl(inc, L, 64) - nseg)) * kRpSeg;
            const uint32_t sl = sl_len - o < kRpSeg ? sl_len - o : kRpSeg;
            const uint8_t *h = data + (uint64_t)sl_s * kRpSlot;
            // segment 0 carries the initial state; each register is shifted over the rest
            const uint32_t raw = crc_shift(wave_crc(tab, h + 4 + o, sl, o ? 0u : 0xffffffffu, lane), sl_len - o - sl);
            if (lane == 0) {
                atomicXor(&lacc[e0 + L], raw);
                __threadfence();
                if (atomicAdd(&ldone[e0 + L], 1u) == nseg - 1) {
                    __threadfence();
                    const uint2 kv = *(const uint2 *)(h + 16);
                    rp_crc_verdict(h, sl_s, kv.x, kv.y, atomicOr(&lacc[e0 + L], 0u), rsz);
                }
            }
        }
        base += total;
    }
}

// ---- exclusive scan of per-element 0/1 flags over [0, n), three kernels ----
struct ValidFlag {  // slot s is a valid record start
    const uint32_t *rsz;
    __device__ uint32_t operator()(uint32_t i) const { return rsz[i] != 0; }
};
struct VisitFlag {  // valid index i < m lies on the reader's path (m, m+1 are the end markers)
    const uint8_t *flag;
    const RpCounters *cnt;
    __device__ uint32_t operator()(uint32_t i) const { return i < cnt->m ? flag[i] : 0u; }
};

template <class F>
__global__ void __launch_bounds__(256) k_scan_tiles(F f, uint32_t n, uint32_t *tile_sum) {
    __shared__ uint32_t part[4];
    const uint32_t base = blockIdx.x * kScanTile;
    uint32_t c = 0;
    for (uint32_t j = threadIdx.x; j < kScanTile; j += 256)
        if (base + j < n) c += f(base + j);
    for (int m = 32; m >= 1; m >>= 1) c += __shfl_xor(c, m, 64);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) tile_sum[blockIdx.x] = part[0] + part[1] + part[2] + part[3];
}

// single workgroup: exclusive scan of tile sums in place; *total = sum
__global__ void __launch_bounds__(1024) k_scan_top(uint32_t *tile_sum, uint32_t ntiles, uint32_t *total) {
    __shared__ uint32_t wsum[16];
    __shared__ uint32_t carry;
    if (threadIdx.x == 0) carry = 0;
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (uint32_t base = 0; base < ntiles; base += 1024) {
        const uint32_t i = base + threadIdx.x;
        const uint32_t v = i < ntiles ? tile_sum[i] : 0u;
        uint32_t x = v;  // inclusive wave scan
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t y = __shfl_up(x, d, 64);
            if (lane >= (uint32_t)d) x += y;
        }
        if (lane == 63) wsum[w] = x;
        __syncthreads();
        if (threadIdx.x == 0) {
            uint32_t acc = 0;
            for (int j = 0; j < 16; j++) { const uint32_t t = wsum[j]; wsum[j] = acc; acc += t; }
        }
        __syncthreads();
        const uint32_t excl = carry + wsum[w] + x - v;
        if (i < ntiles) tile_sum[i] = excl;
        __syncthreads();
        if (threadIdx.x == 1023) carry = excl + v;
        __syncthreads();
    }
    if (threadIdx.x == 0) *total = carry;
}

// per tile: local exclusive ranks + the tile's offset; g(i, idx, flag) scatters
template <class F, class G>
__global__ void __launch_bounds__(256) k_scan_apply(F f, G g, uint32_t n, const uint32_t *tile_sum) {
    __shared__ uint32_t wsum[4];
    const uint32_t base = blockIdx.x * kScanTile + threadIdx.x * 4;
    uint32_t v[4], c = 0;
#pragma unroll
    for (int j = 0; j < 4; j++) {
        v[j] = (base + j < n) ? f(base + j) : 0u;
        c += v[j];
    }
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint32_t x = c;
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(x, d, 64);
        if (lane >= (uint32_t)d) x += y;
    }
    if (lane == 63) wsum[w] = x;
    __syncthreads();
    uint32_t woff = 0;
    for (uint32_t j = 0; j < w; j++) woff += wsum[j];
    uint32_t idx = tile_sum[blockIdx.x] + woff + x - c;
#pragma unroll
    for (int j = 0; j < 4; j++) {
        if (base + j < n) g(base + j, idx, v[j]);
        idx += v[j];
    }
}

struct ScatterValid {  // vidx[s] = #valid slots before s; A[vidx] = s for valid s
    uint32_t *vidx, *A;
    __device__ void operator()(uint32_t s, uint32_t idx, uint32_t v) const {
        vidx[s] = idx;
        if (v) A[idx] = s;
    }
};
struct ScatterVisit {  // visited valid index i -> output position
    const uint32_t *A;
    uint32_t *vis;
    __device__ void operator()(uint32_t i, uint32_t idx, uint32_t v) const {
        if (v) vis[idx] = A[i];
    }
};

// Where the reader goes from byte position p (256-aligned): the index of the
// record it returns next (m = clean end, m + 1 = error).  Next() semantics,
// store/datafile.go:228-277.
__device__ __forceinline__ uint32_t rp_step(uint64_t p, uint64_t size, uint32_t nslots, const uint8_t *kind,
                                            const uint32_t *vidx, uint32_t m) {
    if (p >= size) return m;                           // io.EOF: err = nil, no record
    const uint32_t sp = (uint32_t)(p / kRpSlot);
    const uint8_t k = kind[sp];
    if (k == kSlotPartial || k == kSlotTrunc) return m + 1;  // io.ReadFull: unexpected EOF
    return sp < nslots ? vidx[sp] : m;                 // valid here, or nextValid's first valid slot >= p
}

__global__ void __launch_bounds__(256) k_rp_next(uint64_t size, uint32_t nslots, uint64_t start,
                                                 const uint8_t *kind, const uint32_t *rsz, const uint32_t *vidx,
                                                 const uint32_t *A, RpCounters *cnt, uint32_t *nxt, uint8_t *flag) {
    const uint32_t m = cnt->m;
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < m) {
        const uint32_t s = A[i];
        nxt[i] = rp_step((uint64_t)s * kRpSlot + rsz[s], size, nslots, kind, vidx, m);
        flag[i] = 0;
    } else if (i == m || i == m + 1) {
        nxt[i] = i;  // absorbing end / error
        flag[i] = 0;
    }
    if (i == 0) cnt->r0 = rp_step(start, size, nslots, kind, vidx, m);
}

__global__ void __launch_bounds__(256) k_rp_seed(RpCounters *cnt, uint8_t *flag) { flag[cnt->r0] = 1; }

// one pointer-doubling round: flag J(i) for flagged i; J2 = J o J
__global__ void __launch_bounds__(256) k_rp_double(const RpCounters *cnt, const uint32_t *J, uint32_t *J2,
                                                   uint8_t *flag) {
    const uint32_t m = cnt->m;
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m + 2) return;
    const uint32_t j = J[i];
    if (flag[i]) flag[j] = 1;
    J2[i] = J[j];
}

__global__ void __launch_bounds__(256) k_rp_emit(const uint32_t *vis, const RpCounters *cnt, const uint32_t *rsz,
                                                 uint64_t start, uint64_t *rec_off, uint32_t *rec_broken) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= cnt->nvis) return;
    const uint64_t off = (uint64_t)vis[k] * kRpSlot;
    const uint64_t prev_end = k == 0 ? start : (uint64_t)vis[k - 1] * kRpSlot + rsz[vis[k - 1]];
    rec_off[k] = off;
    rec_broken[k] = (uint32_t)(off - prev_end);  // sizeBroken: bytes nextValid skipped
}

__global__ void k_rp_finish(RpCounters *cnt, const uint8_t *flag, uint32_t *result) {
    const uint32_t m = cnt->m;
    result[0] = cnt->nvis;
    result[1] = flag[m + 1] ? 1u : 0u;  // the path ends in an error (unexpected EOF)
    result[2] = cnt->ncand;
    result[3] = m;
}

// ---- Getvhash (store/item.go:89-100) with the sign-extending Fnv1a (utils/hash.go:8-16) ----
__device__ __forceinline__ uint32_t fnv1a_bytes(const uint8_t *p, uint32_t n, uint32_t h) {
    for (uint32_t i = 0; i < n; i++) {
        h ^= (uint32_t)(int32_t)(int8_t)p[i];
        h *= 0x01000193u;
    }
    return h;
}

__global__ void __launch_bounds__(64) k_vhash(const uint8_t *src, const uint64_t *off, const uint32_t *len,
                                              uint32_t n, uint16_t *out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint8_t *v = src + off[i];
    const uint32_t l = len[i];
    uint32_t h = l * 97u;
    if (l <= 1024) {
        h += fnv1a_bytes(v, l, 0x811c9dc5u);
    } else {
        h += fnv1a_bytes(v, 512, 0x811c9dc5u);
        h *= 97u;
        h += fnv1a_bytes(v + l - 512, 512, 0x811c9dc5u);
    }
    out[i] = (uint16_t)h;
}

// ---- replay plan / finish (store/item.go:163-176 around the batch decoder, no host parse) ----
// Per record: its 24-B header, and for the FLAG_COMPRESS ones, in record order, the body's stream
// offset and length, its decompressed size (the QuickLZ header, quicklz.go:32-44; 0 when the body
// is shorter than a header, which the decoder reports) and a 256-B-aligned destination offset in
// one packed output buffer.  totals = {n, ncomp, max_dsize, out_bytes_lo, out_bytes_hi}.
constexpr uint32_t kFlagCompress = 0x00010000u;
constexpr uint32_t kBodyMax = 50u << 20;
struct CompFlag {
    const uint8_t *data;
    const uint64_t *off;
    const uint32_t *result;
    __device__ uint32_t operator()(uint32_t j) const {
        return j < result[0] && (((const uint32_t *)(data + off[j]))[2] & kFlagCompress) ? 1u : 0u;
    }
};
__device__ __forceinline__ uint32_t rp_body_dsize(const uint8_t *b, uint32_t len) {
    if (len < 3) return 0;
    if (b[0] & 2u) {
        if (len < 9) return 0;
        const uint32_t d = b[5] | (b[6] << 8) | (b[7] << 16) | ((uint32_t)b[8] << 24);
        return d < kBodyMax ? d : kBodyMax;
    }
    return b[2];
}
struct ScatterComp {
    const uint8_t *data;
    const uint64_t *off;
    uint32_t *comp_idx, *comp_len, *comp_dsize;
    uint64_t *comp_off;
    __device__ void operator()(uint32_t j, uint32_t idx, uint32_t v) const {
        if (!v) return;
        const uint32_t *h = (const uint32_t *)(data + off[j]);
        const uint64_t body = off[j] + 24 + h[4];
        comp_idx[idx] = j;
        comp_off[idx] = body;
        comp_len[idx] = h[5];
        comp_dsize[idx] = rp_body_dsize(data + body, h[5]);
    }
};
__global__ void __launch_bounds__(256) k_rp_headers(const uint8_t *data, const uint64_t *off, const uint32_t *result,
                                                    int32_t *hdr) {
    const uint32_t n = result[0];
    for (uint32_t j = blockIdx.x * 256 + threadIdx.x; j < n; j += gridDim.x * 256) {
        const uint32_t *h = (const uint32_t *)(data + off[j]);  // records are 256-B aligned
#pragma unroll
        for (int k = 0; k < 6; k++) hdr[6 * j + k] = (int32_t)h[k];
    }
}
// destination offsets: exclusive scan of the 256-B-rounded sizes (u64) by one workgroup.  Wave
// w owns the contiguous range [w P, (w + 1) P) and walks it twice, 64 coalesced sizes per step
// with the next step's load in flight: first its sum, then (after one scan of the 16 sums) the
// offsets by a wave scan with a carry -- no workgroup barrier per step (round 4 synchronised
// the workgroup four times per 1024 sizes: 265 us for 224 K records).
__global__ void __launch_bounds__(1024) k_rp_dstoff(const uint32_t *comp_dsize, const uint32_t *ncomp_p,
                                                     uint64_t *dst_off, uint32_t *totals, const uint32_t *result) {
    __shared__ uint64_t wsum[16];
    __shared__ uint32_t mx[16];
    const uint32_t nc = *ncomp_p, lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint32_t per = ((nc + 15) / 16 + 63) & ~63u;
    const uint32_t lo = w * per < nc ? w * per : nc, hi = lo + per < nc ? lo + per : nc;
    auto rnd = [](uint32_t d) { return ((uint64_t)d + 255) & ~(uint64_t)255; };
    uint64_t sum = 0;
    uint32_t mymax = 0;
    uint32_t nxt = lo + lane < hi ? comp_dsize[lo + lane] : 0u;
    for (uint32_t i = lo; i < hi; i += 64) {
        const uint32_t d = nxt;
        nxt = i + 64 + lane < hi ? comp_dsize[i + 64 + lane] : 0u;
        sum += rnd(d);
        mymax = max(mymax, d);
    }
    for (int k = 32; k >= 1; k >>= 1) {
        sum += __shfl_xor(sum, k, 64);
        mymax = max(mymax, (uint32_t)__shfl_xor(mymax, k, 64));
    }
    if (lane == 0) wsum[w] = sum, mx[w] = mymax;
    __syncthreads();
    uint64_t carry = 0, total = 0;
    for (uint32_t j = 0; j < 16; j++) {
        carry += j < w ? wsum[j] : 0;
        total += wsum[j];
    }
    nxt = lo + lane < hi ? comp_dsize[lo + lane] : 0u;
    for (uint32_t i = lo; i < hi; i += 64) {
        const uint64_t v = i + lane < hi ? rnd(nxt) : 0;
        nxt = i + 64 + lane < hi ? comp_dsize[i + 64 + lane] : 0u;
        uint64_t x = v;  // inclusive wave scan
        for (int k = 1; k < 64; k <<= 1) {
            const uint64_t y = __shfl_up(x, k, 64);
            if (lane >= (uint32_t)k) x += y;
        }
        if (i + lane < hi) dst_off[i + lane] = carry + x - v;
        carry += __shfl(x, 63, 64);
    }
    if (threadIdx.x == 0) {
        uint32_t m = 0;
        for (int j = 0; j < 16; j++) m = max(m, mx[j]);
        totals[0] = result[0];
        totals[1] = nc;
        totals[2] = m;
        totals[3] = (uint32_t)total;
        totals[4] = (uint32_t)(total >> 32);
    }
}
// After the batch decode of the compressed records: flag, value length, where the value lives
// (decompressed buffer or the raw body: Payload.Decompress errors are swallowed, store/item.go:
// 163-176) and Getvhash of every record.
__global__ void __launch_bounds__(256) k_rp_finish_vals(const uint8_t *data, const uint64_t *off, const uint32_t *result,
                                                       int32_t *flag, int32_t *value_len, uint8_t *in_out,
                                                       uint64_t *val_off) {
    for (uint32_t j = blockIdx.x * 256 + threadIdx.x; j < result[0]; j += gridDim.x * 256) {
        const uint32_t *h = (const uint32_t *)(data + off[j]);  // every record: the stored body first
        flag[j] = (int32_t)h[2];
        value_len[j] = (int32_t)h[5];
        in_out[j] = 0;
        val_off[j] = off[j] + 24 + h[4];
    }
}
__global__ void __launch_bounds__(256) k_rp_finish_comp(const uint32_t *ncomp_p, const uint32_t *comp_idx,
                                                       const int32_t *cstatus, const uint32_t *cdsize,
                                                       const uint64_t *cdst_off, int32_t *flag, int32_t *value_len,
                                                       uint8_t *in_out, uint64_t *val_off) {
    for (uint32_t k = blockIdx.x * 256 + threadIdx.x; k < *ncomp_p; k += gridDim.x * 256) {
        if (cstatus[k] != QLZX_OK) continue;
        const uint32_t j = comp_idx[k];
        flag[j] -= (int32_t)kFlagCompress;  // store/item.go:172-174
        value_len[j] = (int32_t)cdsize[k];
        in_out[j] = 1;
        val_off[j] = cdst_off[k];
    }
}
__global__ void __launch_bounds__(256) k_rp_vhash2(const uint8_t *data, const uint8_t *outbuf, const uint32_t *result,
                                                  const uint8_t *in_out, const uint64_t *val_off,
                                                  const int32_t *value_len, uint16_t *vh) {
    for (uint32_t j = blockIdx.x * 256 + threadIdx.x; j < result[0]; j += gridDim.x * 256) {
        const uint8_t *v = (in_out[j] ? outbuf : data) + val_off[j];
        const uint32_t l = (uint32_t)value_len[j];
        uint32_t h = l * 97u;
        if (l <= 1024) {
            h += fnv1a_bytes(v, l, 0x811c9dc5u);
        } else {
            h += fnv1a_bytes(v, 512, 0x811c9dc5u);
            h *= 97u;
            h += fnv1a_bytes(v + l - 512, 512, 0x811c9dc5u);
        }
        vh[j] = (uint16_t)h;
    }
}

inline size_t replay_plan_ws_bytes(uint32_t cap) { return 256 + (((size_t)cap / kScanTile + 2) * 4 + 255) / 256 * 256; }

inline int launch_replay_plan(const uint8_t *data, const uint64_t *off, const uint32_t *result, uint32_t cap,
                              int32_t *hdr, uint32_t *comp_idx, uint64_t *comp_off, uint32_t *comp_len,
                              uint32_t *comp_dsize, uint64_t *comp_dst_off, uint32_t *totals, void *ws,
                              hipStream_t s) {
    uint32_t *ncomp = (uint32_t *)ws, *tiles = (uint32_t *)((uint8_t *)ws + 256);
    const uint32_t ntiles = (cap + kScanTile - 1) / kScanTile;
    const uint32_t grid = std::min<uint32_t>((cap + 255) / 256, 4096);
    if (cap == 0) return (int)hipMemsetAsync(totals, 0, 5 * sizeof(uint32_t), s);
    hipLaunchKernelGGL(k_rp_headers, dim3(grid), dim3(256), 0, s, data, off, result, hdr);
    CompFlag cf{data, off, result};
    hipLaunchKernelGGL(k_scan_tiles<CompFlag>, dim3(ntiles), dim3(256), 0, s, cf, cap, tiles);
    hipLaunchKernelGGL(k_scan_top, dim3(1), dim3(1024), 0, s, tiles, ntiles, ncomp);
    hipLaunchKernelGGL((k_scan_apply<CompFlag, ScatterComp>), dim3(ntiles), dim3(256), 0, s, cf,
                       ScatterComp{data, off, comp_idx, comp_len, comp_dsize, comp_off}, cap, tiles);
    hipLaunchKernelGGL(k_rp_dstoff, dim3(1), dim3(1024), 0, s, (const uint32_t *)comp_dsize, (const uint32_t *)ncomp,
                       comp_dst_off, totals, result);
    return (int)hipGetLastError();
}

inline int launch_replay_finish(const uint8_t *data, const uint64_t *off, const uint32_t *result,
                                const uint32_t *totals, const uint32_t *comp_idx, const int32_t *cstatus,
                                const uint32_t *cdsize, const uint64_t *cdst_off, const uint8_t *outbuf,
                                uint32_t cap, int32_t *flag, int32_t *value_len, uint8_t *in_out, uint64_t *val_off,
                                uint16_t *vh, hipStream_t s) {
    if (cap == 0) return 0;
    const uint32_t grid = std::min<uint32_t>((cap + 255) / 256, 4096);
    hipLaunchKernelGGL(k_rp_finish_vals, dim3(grid), dim3(256), 0, s, data, off, result, flag, value_len, in_out,
                       val_off);
    hipLaunchKernelGGL(k_rp_finish_comp, dim3(grid), dim3(256), 0, s, totals + 1, comp_idx, cstatus, cdsize, cdst_off,
                       flag, value_len, in_out, val_off);
    hipLaunchKernelGGL(k_rp_vhash2, dim3(grid), dim3(256), 0, s, data, outbuf, result, (const uint8_t *)in_out,
                       (const uint64_t *)val_off, (const int32_t *)value_len, vh);
    return (int)hipGetLastError();
}

// ---- workspace layout ----
struct RpWs {
    RpCounters *cnt;
    uint8_t *kind, *flag;
    uint32_t *rsz, *vidx, *A, *J, *J2, *vis, *tiles;
};

inline size_t rp_align(size_t x) { return (x + 255) & ~(size_t)255; }

inline size_t replay_ws_layout(uint64_t size, uint8_t *base, RpWs *w) {
    const uint64_t ns = (size + kRpSlot - 1) / kRpSlot;
    const size_t n = (size_t)ns + 2;
    const size_t ntiles = (n + kScanTile - 1) / kScanTile;
    size_t o = 0;
    auto take = [&](size_t bytes) {
        uint8_t *p = base ? base + o : nullptr;
        o += rp_align(bytes);
        return p;
    };
    RpWs t;
    t.cnt = (RpCounters *)take(sizeof(RpCounters));
    t.kind = take(n);
    t.flag = take(n);
    t.rsz = (uint32_t *)take(4 * n);
    t.vidx = (uint32_t *)take(4 * n);
    t.A = (uint32_t *)take(4 * n);
    t.J = (uint32_t *)take(4 * n);
    t.J2 = (uint32_t *)take(4 * n);
    t.vis = (uint32_t *)take(4 * n);
    t.tiles = (uint32_t *)take(4 * (ntiles + 1));
    if (w) *w = t;
    return o;
}

inline int launch_replay_index(const uint8_t *data, uint64_t size, uint64_t start, uint32_t max_key,
                               uint64_t body_max, uint64_t *rec_off, uint32_t *rec_broken, uint32_t *result,
                               void *ws, hipStream_t s) {
    RpWs w;
    replay_ws_layout(size, (uint8_t *)ws, &w);
    const uint32_t nslots = (uint32_t)((size + kRpSlot - 1) / kRpSlot);
    const uint32_t n2 = nslots + 2;
    const uint32_t ntiles = (n2 + kScanTile - 1) / kScanTile;
    const uint32_t g256 = (n2 + 255) / 256;
    hipError_t e = hipMemsetAsync(w.cnt, 0, sizeof(RpCounters), s);
    if (e != hipSuccess) return (int)e;
    // slot classification + candidate CRCs in one pass: a grid-stride loop over 64-slot groups,
    // one table load per workgroup, 8 workgroups per CU; the long-candidate list and its
    // accumulators borrow vis, J and J2 (written later)
    const uint32_t ngroups = (nslots + 63) / 64;
    const uint32_t scan_grid = (ngroups + 3) / 4 < 2048 ? (ngroups + 3) / 4 : 2048;
    if (nslots)
        hipLaunchKernelGGL(k_rp_scan, dim3(scan_grid), dim3(256), 0, s, data, size, nslots, max_key, body_max, w.kind,
                           w.rsz, w.cnt, w.vis, w.J, w.J2);
    hipLaunchKernelGGL(k_rp_crc_long, dim3(2048), dim3(256), 0, s, data, w.cnt, w.rsz, w.vis, w.J, w.J2);
    // valid slots in order: vidx (exclusive count) and A
    ValidFlag vf{w.rsz};
    hipLaunchKernelGGL(k_scan_tiles<ValidFlag>, dim3(ntiles), dim3(256), 0, s, vf, nslots, w.tiles);
    hipLaunchKernelGGL(k_scan_top, dim3(1), dim3(1024), 0, s, w.tiles, ntiles, &w.cnt->m);
    hipLaunchKernelGGL((k_scan_apply<ValidFlag, ScatterValid>), dim3(ntiles), dim3(256), 0, s, vf,
                       ScatterValid{w.vidx, w.A}, nslots, w.tiles);
    // successors, start, and the path by pointer doubling
    hipLaunchKernelGGL(k_rp_next, dim3(g256), dim3(256), 0, s, size, nslots, start, w.kind, w.rsz, w.vidx, w.A,
                       w.cnt, w.J, w.flag);
    hipLaunchKernelGGL(k_rp_seed, dim3(1), dim3(1), 0, s, w.cnt, w.flag);
    uint32_t *J = w.J, *J2 = w.J2;
    for (uint64_t reach = 1; reach < (uint64_t)n2 + 1; reach <<= 1) {
        hipLaunchKernelGGL(k_rp_double, dim3(g256), dim3(256), 0, s, w.cnt, J, J2, w.flag);
        uint32_t *t = J; J = J2; J2 = t;
    }
    // visited records in order
    VisitFlag ff{w.flag, w.cnt};
    hipLaunchKernelGGL(k_scan_tiles<VisitFlag>, dim3(ntiles), dim3(256), 0, s, ff, nslots, w.tiles);
    hipLaunchKernelGGL(k_scan_top, dim3(1), dim3(1024), 0, s, w.tiles, ntiles, &w.cnt->nvis);
    hipLaunchKernelGGL((k_scan_apply<VisitFlag, ScatterVisit>), dim3(ntiles), dim3(256), 0, s, ff,
                       ScatterVisit{w.A, w.vis}, nslots, w.tiles);
    hipLaunchKernelGGL(k_rp_emit, dim3((nslots + 255) / 256 + 1), dim3(256), 0, s, w.vis, w.cnt, w.rsz, start,
                       rec_off, rec_broken);
    hipLaunchKernelGGL(k_rp_finish, dim3(1), dim3(1), 0, s, w.cnt, w.flag, result);
    e = hipGetLastError();
    return (int)e;
}

}  // namespace qlzx
