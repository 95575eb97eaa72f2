// qlzx_k2.hip -- K2 of the batch decoder without the CRC prologue (k_dec_chunk4<false>) and, with
// QLZX_SPLIT_K1 (the release build), K1 (k_dec_parse6) in a translation unit of their own,
// compiled with the iterative-ilp machine scheduler
// (-mllvm -amdgpu-sched-strategy=iterative-ilp, gobeansdb_amd/build.py): that strategy speeds this
// kernel up but slows K2 with its CRC prologue, the encoder and the replay kernels, and the
// strategy is per translation unit (profiles/r05_sched_strategy_ab.txt).  Under QLZX_K2_ONLY the
// shared sources define no other kernel.  The rest of the library is qlzx_api.hip.
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdint>
#include <cstdlib>
#include <mutex>

#define QLZX_K2_ONLY 1
#include "qlzx_device.h"
namespace qlzx {  // defined in qlzx_tables.hip (qlzx_api.hip's unit); K2 without CRC reads none of them
constexpr int kMulTabs = 7;
extern __device__ uint32_t g_crc_mul[kMulTabs * 1024];
extern __device__ uint32_t g_crc_mul32[1024];
}  // namespace qlzx
#include "qlzx_crc.hip"
#include "qlzx_decode_wave.hip"

namespace qlzx {

int launch_k2_nocrc(uint32_t grid, hipStream_t s, const qlzx_blocks &b, uint32_t *dsize, int32_t *status,
                    uint32_t first, uint32_t cnt, const BlkInfo *info, const GroupRec *recs, uint32_t gmax,
                    const uint32_t *order, bool big) {
#if QLZX_K2_BIGW  // an 8 KiB window for calls of values over 16 KiB (fewer far loads, fewer waves per SIMD)
    if (big)
        hipLaunchKernelGGL((k_dec_chunk4<false, 8192>), dim3(grid), dim3(64), 0, s, b, dsize, status, first, cnt, info,
                           recs, gmax, order, nullptr, nullptr, nullptr);
    else
#endif
    hipLaunchKernelGGL(k_dec_chunk4<false>, dim3(grid), dim3(64), 0, s, b, dsize, status, first, cnt, info, recs,
                       gmax, order, nullptr, nullptr, nullptr);
    return (int)hipGetLastError();
}

#if QLZX_SPLIT_K1
int launch_k1_parse6(uint32_t grid, hipStream_t s, const qlzx_blocks &b, const uint32_t *dst_cap, uint32_t *dsize,
                     int32_t *status, uint32_t first, uint32_t cnt, BlkInfo *info, GroupRec *recs, uint32_t gmax,
                     const uint32_t *order, uint32_t max_dsize, uint32_t kmax) {
    hipLaunchKernelGGL(k_dec_parse6, dim3(grid), dim3(kParseWG), 0, s, b, dst_cap, dsize, status, first, cnt, info,
                       recs, gmax, order, max_dsize, kmax);
    return (int)hipGetLastError();
}
#endif

}  // namespace qlzx
