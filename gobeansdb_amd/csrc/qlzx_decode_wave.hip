// qlzx_decode_wave.hip -- fast-path decoder (placeholder until the LDS kernel lands).
#include "qlzx_device.h"
#ifndef QLZX_FAST_MAX_DSIZE
#define QLZX_FAST_MAX_DSIZE 65536
#endif
namespace qlzx {
inline bool decode_wave_enabled() { return false; }
inline size_t decode_wave_ws_bytes(uint32_t n) { return 0; }
inline int launch_decode_wave(const qlzx_blocks &, const uint32_t *, uint32_t *, int32_t *, const uint32_t *,
                              const uint32_t *, uint32_t *, void *, hipStream_t) { return 0; }
}  // namespace qlzx
