// qlzx_encode_wg.hip -- fast-path encoder (placeholder until the workgroup kernel lands).
#include "qlzx_device.h"
#ifndef QLZX_WG_MAX_LEN
#define QLZX_WG_MAX_LEN 65536
#endif
namespace qlzx {
inline bool encode_wg_enabled() { return false; }
inline size_t encode_wg_ws_bytes(uint32_t, uint32_t) { return 0; }
inline int launch_encode_wg(const qlzx_blocks &, uint32_t *, int32_t *, const uint32_t *, uint32_t *, uint32_t,
                            uint32_t, void *, hipStream_t) { return 0; }
}  // namespace qlzx
