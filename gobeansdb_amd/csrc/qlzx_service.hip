// qlzx_service.hip -- the request path behind the quicklz.h drop-ins (qlz_decompress, qlz_compress,
// crc32_write), called once per GET / SET by store/item.go:140,151,167 and store/datafile.go:161-168.
//
// One service per device, shared by every calling thread (no per-thread GPU state):
//   * a pinned, fine-grained (host-coherent) arena of kSvcSlots request slots [in | out] and a
//     device arena of the same slots [src | dst | workspace];
//   * a caller takes a free slot, copies its bytes into the slot's `in`, and queues a request;
//   * requests are COALESCED: the first thread to find no leader becomes the leader and launches
//     everything queued as one batch per op (one workgroup per request), while later callers
//     simply queue behind it; there is no service thread and no lock held across a launch wait;
//   * each kernel stages its request in (host slot -> HBM), runs the op, stages the result out
//     (HBM -> host slot) and, after a system-scope release, stores the request's sequence number
//     into its host-visible completion word.  The caller spins on that word (no stream
//     synchronisation), copies its result out and frees the slot;
//   * every batch also records an event after its kernels; a spinning caller polls it now and then
//     (hipEventQuery), so a batch that ends without publishing, or a stream in error, fails its
//     requests with QLZX_R_HIP instead of leaving the callers spinning.
// Launches rotate over kSvcStreams streams, so a batch launched while an earlier one still runs
// does not queue behind it.  Values above kSvcMaxLen (and the Go-compat encoder modes) take the
// general per-call path in qlzx_api.hip.
#include <chrono>
#include <thread>
#include <vector>
#include <immintrin.h>

namespace qlzx {

constexpr uint32_t kSvcSlots = 64;        // concurrent requests (pinned + device arena)
constexpr uint32_t kSvcBatchMax = 32;     // requests per launch (kernel-argument descriptor)
constexpr uint32_t kSvcStreams = 4;
// Coalescing: with requests already on the GPU, a new batch waits for kSvcBatchTarget requests or
// kSvcDeadlineNs, whichever comes first (a lone caller finds nothing in flight and launches at once).
constexpr uint32_t kSvcBatchTarget = 8;
constexpr int64_t kSvcDeadlineNs = 20000;
constexpr uint32_t kSvcMaxLen = 65536;    // dsize / input length served here (solo decoder, WG encoder)
constexpr size_t kSvcIn = 80u << 10, kSvcOut = 80u << 10;
constexpr size_t kSvcHostSlot = kSvcIn + kSvcOut;
constexpr size_t kSvcRecs = ((size_t)kSoloGmax * sizeof(GroupRec) + 255) & ~(size_t)255;
constexpr size_t kSvcDevSlot = kSvcIn + kSvcOut + kSvcRecs;
static_assert(kSvcIn >= kSoloMaxCsize + 64 && kSvcOut >= kSvcMaxLen + 400 + 64, "slot sizes");

enum : uint32_t { kSvcDecode = 0, kSvcCompress = 1, kSvcCrc = 2, kSvcOps = 3 };

struct SvcReq {
    uint32_t slot, len, cap, seq;
    uint32_t arg;     // crc, and decode with kSvcVerify: the CRC state before the input bytes
    uint32_t expect;  // decode with kSvcVerify: the stored record CRC (~state after the input)
    uint32_t mode;    // decode: kSvcVerify and/or kSvcNoDecode (0: a plain qlz_decompress)
    uint32_t pad;
};
// decode request modes (qlzx_read_record1: readRecordAt's CRC check + Payload.Decompress, one request)
constexpr uint32_t kSvcVerify = 1, kSvcNoDecode = 2;
struct SvcBatch {
    uint32_t n, pad[3];
    SvcReq r[kSvcBatchMax];
};
struct alignas(16) SvcDone {
    uint32_t out;      // decompressed / compressed size
    int32_t status;    // enum qlzx_status
    uint32_t crc;      // crc32_write result
    uint32_t seq;      // written last: the request's sequence number
};

// host slot -> device slot, 16 B per thread (the slots are 16-B aligned; bytes past len are slack)
__device__ __forceinline__ void svc_copy(uint8_t *d, const uint8_t *s, uint32_t len, uint32_t tid, uint32_t nt) {
    for (uint32_t o = tid * 16; o < len; o += nt * 16) *(uint4 *)(d + o) = *(const uint4 *)(s + o);
}
// completion: every thread's stores are released to the system before thread 0 publishes
__device__ __forceinline__ void svc_publish(SvcDone *done, const SvcReq &r, uint32_t out, int32_t st, uint32_t crc) {
    __threadfence_system();
    __syncthreads();
    if (threadIdx.x == 0) {
        volatile SvcDone *d = done + r.slot;
        d->out = out;
        d->status = st;
        d->crc = crc;
        __threadfence_system();
        d->seq = r.seq;
    }
}

__global__ void __launch_bounds__(kSoloWG) k_svc_decode(SvcBatch B, const uint8_t *h_arena, uint8_t *d_arena,
                                                        SvcDone *done) {
    __shared__ __attribute__((aligned(16))) union {
        SoloLds solo;
        SmallLds small;
        uint32_t crc[kCrcLdsWords];
    } U;
    __shared__ int32_t st;
    __shared__ uint32_t ds, crc_s;
    const SvcReq r = B.r[blockIdx.x];
    const uint8_t *hin = h_arena + (size_t)r.slot * kSvcHostSlot;
    uint8_t *hout = (uint8_t *)hin + kSvcIn;
    uint32_t crc = 0;
    if (r.mode & kSvcVerify) {
        // readRecordAt (store/datafile.go:161-168): the record CRC over the value, continued from
        // the header[4:24] | key state, checked before anything is decoded
        load_crc_lds(U.crc);
        __syncthreads();
        if (threadIdx.x < 64) {
            const uint32_t c = wave_crc(U.crc, hin, r.len, r.arg, threadIdx.x);
            if (threadIdx.x == 0) crc_s = c;
        }
        __syncthreads();
        crc = crc_s;
        if ((~crc != r.expect) || (r.mode & kSvcNoDecode)) {
            svc_publish(done, r, 0, ~crc != r.expect ? QLZX_E_CRC : QLZX_OK, crc);
            return;
        }
    }
    // small blocks: stream from the host slot into LDS, result straight into the host slot
    if (small_decode(U.small, hin, r.len, hout, r.cap, r.cap, &st, &ds)) {
        __syncthreads();
        svc_publish(done, r, st == QLZX_OK ? ds : 0u, st, crc);
        return;
    }
    SoloLds &L = U.solo;
    uint8_t *dsrc = d_arena + (size_t)r.slot * kSvcDevSlot, *ddst = dsrc + kSvcIn;
    const uint32_t tid = threadIdx.x;
    svc_copy(dsrc, hin, r.len, tid, kSoloWG);
    __threadfence();
    __syncthreads();
    solo_decode(L, dsrc, r.len, ddst, r.cap, r.cap, (GroupRec *)(ddst + kSvcOut), &st, &ds);
    __threadfence();
    __syncthreads();
    const uint32_t n = st == QLZX_OK ? ds : 0u;
    svc_copy(hout, ddst, n, tid, kSoloWG);
    svc_publish(done, r, n, st, crc);
}

__global__ void __launch_bounds__(256) k_svc_crc(SvcBatch B, const uint8_t *h_arena, uint8_t *d_arena, SvcDone *done) {
    __shared__ uint32_t tab[kCrcLdsWords];
    load_crc_lds(tab);
    const SvcReq r = B.r[blockIdx.x];
    const uint8_t *hin = h_arena + (size_t)r.slot * kSvcHostSlot;
    uint8_t *dsrc = d_arena + (size_t)r.slot * kSvcDevSlot;
    svc_copy(dsrc, hin, r.len, threadIdx.x, 256);
    __threadfence();
    __syncthreads();
    uint32_t c = 0;
    if (threadIdx.x < 64) c = wave_crc(tab, dsrc, r.len, r.arg, threadIdx.x);
    svc_publish(done, r, 0, QLZX_OK, c);  // thread 0 holds lane 0's result
}

// compress: stage in and build the batch's block arrays, then k_encode_wg<65536>, then stage out
struct SvcEncDesc {
    uint64_t src_off[kSvcBatchMax], dst_off[kSvcBatchMax];
    uint32_t src_len[kSvcBatchMax], csize[kSvcBatchMax];
    int32_t status[kSvcBatchMax];
    uint32_t ticket;
};
__global__ void __launch_bounds__(256) k_svc_enc_in(SvcBatch B, const uint8_t *h_arena, uint8_t *d_arena,
                                                    SvcEncDesc *desc) {
    const SvcReq r = B.r[blockIdx.x];
    svc_copy(d_arena + (size_t)r.slot * kSvcDevSlot, h_arena + (size_t)r.slot * kSvcHostSlot, r.len, threadIdx.x, 256);
    if (threadIdx.x == 0) {
        desc->src_off[blockIdx.x] = (uint64_t)r.slot * kSvcDevSlot;
        desc->dst_off[blockIdx.x] = (uint64_t)r.slot * kSvcDevSlot + kSvcIn;
        desc->src_len[blockIdx.x] = r.len;
        if (blockIdx.x == 0) desc->ticket = 0;
    }
}
__global__ void __launch_bounds__(256) k_svc_enc_out(SvcBatch B, uint8_t *h_arena, const uint8_t *d_arena,
                                                     const SvcEncDesc *desc, SvcDone *done) {
    const SvcReq r = B.r[blockIdx.x];
    const int32_t st = desc->status[blockIdx.x];
    const uint32_t n = st == QLZX_OK ? desc->csize[blockIdx.x] : 0u;
    svc_copy(h_arena + (size_t)r.slot * kSvcHostSlot + kSvcIn, d_arena + (size_t)r.slot * kSvcDevSlot + kSvcIn, n,
             threadIdx.x, 256);
    svc_publish(done, r, n, st, 0);
}

// test hook (qlzx_service_test_fault): a batch that runs but never publishes its completions
__global__ void k_svc_nop(uint32_t *sink) {
    if (sink && threadIdx.x == 0) *sink = 0;
}

}  // namespace qlzx

namespace {

using qlzx::kSvcBatchMax;
using qlzx::kSvcSlots;
using qlzx::kSvcStreams;

inline int64_t now_ns() {
    return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
        .count();
}

struct SvcPending {
    uint32_t op;
    qlzx::SvcReq r;
};

struct Service {
    int dev = -1;
    bool ok = false;
    hipStream_t st[kSvcStreams] = {};
    uint8_t *h_arena = nullptr, *d_arena = nullptr;
    qlzx::SvcDone *h_done = nullptr;
    uint8_t *d_enc_ws[kSvcStreams] = {};  // encoder workspace + SvcEncDesc per stream
    size_t enc_ws_bytes = 0;
    std::atomic<uint64_t> free_mask{~0ull};
    uint32_t seq[kSvcSlots] = {};
    std::mutex mu;  // guards pending, leading, next_stream
    std::vector<SvcPending> pending;
    std::atomic<bool> leading{false};
    std::atomic<uint32_t> npending{0};
    std::atomic<uint32_t> inflight{0};     // launched, completion not yet seen by the caller
    std::atomic<int64_t> oldest_ns{0};     // when the oldest pending request was queued
    uint32_t next_stream = 0;
    // Batch events: a batch holds one from launch until every caller in it (and the leader) has
    // let go.  Each held event maps to a held slot, so kSvcSlots of them never run out for long.
    hipEvent_t ev[kSvcSlots] = {};
    std::atomic<int32_t> ev_refs[kSvcSlots] = {};
    std::atomic<uint64_t> ev_free{~0ull};
    std::atomic<uint64_t> slot_ev[kSvcSlots] = {};  // seq << 32 | (event index + 1), set after the record
    std::atomic<int> fault{0};                      // test hook, consumed by the next launch

    int init(int device) {
        dev = device;
        HIP_OK(hipSetDevice(device));
        for (auto &s : st) HIP_OK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
        for (auto &e : ev) HIP_OK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        HIP_OK(hipHostMalloc((void **)&h_arena, kSvcSlots * qlzx::kSvcHostSlot + kSvcSlots * sizeof(qlzx::SvcDone),
                             hipHostMallocCoherent | hipHostMallocMapped));
        h_done = (qlzx::SvcDone *)(h_arena + kSvcSlots * qlzx::kSvcHostSlot);
        memset(h_done, 0, kSvcSlots * sizeof(qlzx::SvcDone));
        HIP_OK(hipMalloc((void **)&d_arena, kSvcSlots * qlzx::kSvcDevSlot));
        enc_ws_bytes = align_up(sizeof(qlzx::SvcEncDesc), 256) + qlzx::encode_wg_ws_bytes(kSvcBatchMax, 65536);
        for (auto &w : d_enc_ws) HIP_OK(hipMalloc((void **)&w, enc_ws_bytes));
        ok = true;
        return 0;
    }
    // undo a partial init (service() keeps the failure, it never retries)
    void release() {
        for (auto &w : d_enc_ws)
            if (w) (void)hipFree(w), w = nullptr;
        if (d_arena) (void)hipFree(d_arena), d_arena = nullptr;
        if (h_arena) (void)hipHostFree(h_arena), h_arena = nullptr;
        for (auto &e : ev)
            if (e) (void)hipEventDestroy(e), e = nullptr;
        for (auto &s : st)
            if (s) (void)hipStreamDestroy(s), s = nullptr;
    }

    uint32_t take_ev() {
        for (uint32_t spins = 0;; spins++) {
            uint64_t m = ev_free.load(std::memory_order_relaxed);
            while (m) {
                const uint32_t b = (uint32_t)__builtin_ctzll(m);
                if (ev_free.compare_exchange_weak(m, m & ~(1ull << b), std::memory_order_acquire)) return b;
            }
            if (spins > 64) std::this_thread::yield(); else _mm_pause();
        }
    }
    void drop_ev(uint32_t e) {
        if (ev_refs[e].fetch_sub(1, std::memory_order_acq_rel) == 1) ev_free.fetch_or(1ull << e, std::memory_order_release);
    }

    uint32_t take_slot() {
        for (uint32_t spins = 0;; spins++) {
            uint64_t m = free_mask.load(std::memory_order_relaxed);
            while (m) {
                const uint32_t b = (uint32_t)__builtin_ctzll(m);
                if (free_mask.compare_exchange_weak(m, m & ~(1ull << b), std::memory_order_acquire)) return b;
            }
            if (spins > 64) std::this_thread::yield(); else _mm_pause();
        }
    }
    void give_slot(uint32_t b) { free_mask.fetch_or(1ull << b, std::memory_order_release); }
    uint8_t *in(uint32_t b) { return h_arena + (size_t)b * qlzx::kSvcHostSlot; }
    uint8_t *out(uint32_t b) { return in(b) + qlzx::kSvcIn; }

    // Launch everything queued (the caller is the leader).  Returns a qlzx_return code.
    int launch(std::vector<SvcPending> &batch) {
        const int inj = fault.exchange(0, std::memory_order_acq_rel);
        if (inj == 2) return fail(QLZX_R_HIP, "service launch (injected failure)");
        qlzx::SvcBatch B[qlzx::kSvcOps];
        for (auto &b : B) b.n = 0;
        for (const auto &p : batch) B[p.op].r[B[p.op].n++] = p.r;
        hipStream_t s;
        uint8_t *ws;
        {
            std::lock_guard<std::mutex> g(mu);
            const uint32_t k = next_stream++ % kSvcStreams;
            s = st[k];
            ws = d_enc_ws[k];
        }
        if (inj == 1) {  // the batch runs, publishes nothing and completes its event
            hipLaunchKernelGGL(qlzx::k_svc_nop, dim3(1), dim3(64), 0, s, (uint32_t *)nullptr);
            for (auto &b : B) b.n = 0;
        }
        if (B[qlzx::kSvcDecode].n)
            hipLaunchKernelGGL(qlzx::k_svc_decode, dim3(B[qlzx::kSvcDecode].n), dim3(qlzx::kSoloWG), 0, s,
                               B[qlzx::kSvcDecode], (const uint8_t *)h_arena, d_arena, h_done);
        if (B[qlzx::kSvcCrc].n)
            hipLaunchKernelGGL(qlzx::k_svc_crc, dim3(B[qlzx::kSvcCrc].n), dim3(256), 0, s, B[qlzx::kSvcCrc],
                               (const uint8_t *)h_arena, d_arena, h_done);
        if (const uint32_t n = B[qlzx::kSvcCompress].n) {
            auto *desc = (qlzx::SvcEncDesc *)ws;
            uint8_t *ews = ws + align_up(sizeof(qlzx::SvcEncDesc), 256);
            hipLaunchKernelGGL(qlzx::k_svc_enc_in, dim3(n), dim3(256), 0, s, B[qlzx::kSvcCompress],
                               (const uint8_t *)h_arena, d_arena, desc);
            qlzx_blocks bl{d_arena, desc->src_off, desc->src_len, d_arena, desc->dst_off, n};
            hipLaunchKernelGGL(qlzx::k_encode_wg<65536>, dim3(n), dim3(1024), 0, s, bl, desc->csize, desc->status,
                               (const uint32_t *)nullptr, (uint32_t *)nullptr, ews, &desc->ticket);
            hipLaunchKernelGGL(qlzx::k_svc_enc_out, dim3(n), dim3(256), 0, s, B[qlzx::kSvcCompress], h_arena,
                               (const uint8_t *)d_arena, (const qlzx::SvcEncDesc *)desc, h_done);
        }
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) {
            (void)hipStreamSynchronize(s);  // whatever did launch is done before its slots are failed
            return fail(QLZX_R_HIP, "service launch", e);
        }
        // the batch event: one reference per request plus the leader's until the slots know it
        const uint32_t k = take_ev();
        ev_refs[k].store((int32_t)batch.size() + 1, std::memory_order_relaxed);
        e = hipEventRecord(ev[k], s);
        if (e != hipSuccess) {
            ev_refs[k].store(1, std::memory_order_relaxed);
            drop_ev(k);
            (void)hipStreamSynchronize(s);
            return fail(QLZX_R_HIP, "service event record", e);
        }
        for (const auto &p : batch) slot_ev[p.r.slot].store(tag(p.r.seq, k), std::memory_order_release);
        drop_ev(k);
        return QLZX_R_OK;
    }
    static constexpr uint32_t kNoEv = 0xffffffffu;  // slot_ev for a batch that failed to launch
    static uint64_t tag(uint32_t seq, uint32_t k) { return (uint64_t)seq << 32 | (k == kNoEv ? kNoEv : k + 1); }

    // A caller's check on its own batch (every ~1K spins): 0 while it may still complete, else a
    // qlzx_return code.  `held` is the batch event this caller references (-1 until it is known).
    int check(uint32_t slot, uint32_t seq, volatile qlzx::SvcDone *d, int32_t *held) {
        if (*held < 0) {
            const uint64_t v = slot_ev[slot].load(std::memory_order_acquire);
            if ((uint32_t)(v >> 32) != seq || (uint32_t)v == 0 || (uint32_t)v == kNoEv) return 0;  // not yet
            *held = (int32_t)(uint32_t)v - 1;
        }
        const hipError_t q = hipEventQuery(ev[*held]);
        if (q == hipErrorNotReady) return 0;
        if (q != hipSuccess) return fail(QLZX_R_HIP, "service batch", q);
        std::atomic_thread_fence(std::memory_order_acquire);
        if (d->seq == seq) return 0;  // published after all; the loop sees it
        return fail(QLZX_R_HIP, "service batch ended without completing the request");
    }

    // Queue one request and wait for it.  On a launch failure every request of that batch is
    // completed with status -1 (the callers then report QLZX_R_HIP); a batch that ends without
    // publishing, or whose stream reports an error, fails the same way through its event.
    int run(uint32_t op, qlzx::SvcReq r) {
        r.seq = ++seq[r.slot];  // the slot is this thread's until give_slot
        volatile qlzx::SvcDone *d = h_done + r.slot;
        {
            std::lock_guard<std::mutex> g(mu);
            if (pending.empty()) oldest_ns.store(now_ns(), std::memory_order_relaxed);
            pending.push_back({op, r});
            npending.fetch_add(1, std::memory_order_release);
        }
        int rc = QLZX_R_OK;
        int32_t held = -1;  // this request's batch event, once launched
        for (uint32_t spins = 0; d->seq != r.seq; spins++) {
            if ((spins & 1023) == 1023 && (rc = check(r.slot, r.seq, d, &held)) != QLZX_R_OK) break;
            const uint32_t np = npending.load(std::memory_order_acquire);
            if (!leading.load(std::memory_order_acquire) && np &&
                (inflight.load(std::memory_order_acquire) == 0 || np >= qlzx::kSvcBatchTarget ||
                 now_ns() - oldest_ns.load(std::memory_order_relaxed) > qlzx::kSvcDeadlineNs)) {
                bool exp = false;
                if (leading.compare_exchange_strong(exp, true, std::memory_order_acq_rel)) {
                    std::vector<SvcPending> batch;
                    {
                        std::lock_guard<std::mutex> g(mu);
                        const size_t n = std::min<size_t>(pending.size(), kSvcBatchMax);
                        batch.assign(pending.begin(), pending.begin() + n);
                        pending.erase(pending.begin(), pending.begin() + n);
                        npending.fetch_sub((uint32_t)n, std::memory_order_release);
                        inflight.fetch_add((uint32_t)n, std::memory_order_acq_rel);
                        if (!pending.empty()) oldest_ns.store(now_ns(), std::memory_order_relaxed);
                    }
                    const int lr = batch.empty() ? QLZX_R_OK : launch(batch);
                    if (lr != QLZX_R_OK) {
                        bool mine = false;  // the leader's own request may belong to an earlier batch
                        for (const auto &p : batch) {
                            volatile qlzx::SvcDone *x = h_done + p.r.slot;
                            x->status = -1;
                            x->seq = p.r.seq;
                            slot_ev[p.r.slot].store(tag(p.r.seq, kNoEv), std::memory_order_release);
                            mine = mine || (p.r.slot == r.slot && p.r.seq == r.seq);
                        }
                        // only the failed batch's requests fail: one of an earlier, still running
                        // batch completes normally (the status -1 / kNoEv tags above fail the rest)
                        if (mine) rc = lr;
                    }
                    leading.store(false, std::memory_order_release);
                    continue;
                }
            }
            if (spins > 20000) std::this_thread::yield(); else _mm_pause();
        }
        // The leader always tags the request's slot after the launch (event or kNoEv); wait for
        // that, so the slot is not handed on while the leader may still write to it.  (A request
        // can be published before its leader gets there.)
        if (held < 0)
            for (uint32_t w = 0;; w++) {
                const uint64_t v = slot_ev[r.slot].load(std::memory_order_acquire);
                if ((uint32_t)(v >> 32) == r.seq && (uint32_t)v) {
                    if ((uint32_t)v != kNoEv) held = (int32_t)(uint32_t)v - 1;
                    break;
                }
                if (w > 64) std::this_thread::yield(); else _mm_pause();
            }
        if (held >= 0) drop_ev((uint32_t)held);
        std::atomic_thread_fence(std::memory_order_acquire);
        inflight.fetch_sub(1, std::memory_order_acq_rel);
        if (rc == QLZX_R_OK && d->status == -1) rc = fail(QLZX_R_HIP, "service launch failed (another caller's batch)");
        return rc;
    }
};

Service *service() {
    static Service *svc[qlzx::kMaxDevices] = {};
    static std::string init_err[qlzx::kMaxDevices];  // sticky: a failed init is not retried
    static std::mutex init_mu;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= (int)qlzx::kMaxDevices) {
        fail(QLZX_R_NO_DEVICE, "no HIP device");
        return nullptr;
    }
    if (Service *s = __atomic_load_n(&svc[dev], __ATOMIC_ACQUIRE)) return s;
    std::lock_guard<std::mutex> g(init_mu);
    if (!svc[dev]) {
        int ndev = 0;
        if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
            fail(QLZX_R_NO_DEVICE, "no HIP device");
            return nullptr;
        }
        if (!init_err[dev].empty()) {
            fail(QLZX_R_NO_DEVICE, init_err[dev].c_str());
            return nullptr;
        }
        auto *s = new Service();
        if (s->init(dev) != 0) {
            init_err[dev] = "service init failed earlier: " + t_last_error;
            s->release();
            delete s;
            fail(QLZX_R_NO_DEVICE, init_err[dev].c_str());
            return nullptr;
        }
        __atomic_store_n(&svc[dev], s, __ATOMIC_RELEASE);
    }
    return svc[dev];
}

}  // namespace
