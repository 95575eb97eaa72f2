"""Phase stamps of the single-call latency kernel k_dec_solo (csrc/qlzx_decode_solo.hip) from the
-DQLZX_PROFILE build, plus the host-side split of one qlz_decompress call.

usage: QLZX_LIB=gobeansdb_amd/libqlzx_prof.so python tools/solo_prof.py [calls]
"""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from gobeansdb_amd import _lib
from oracle import oracle as O

calls = int(sys.argv[1]) if len(sys.argv) > 1 else 200
L = _lib.lib()
L.qlzx_profile_set.argtypes = [ctypes.c_void_p]
dev = torch.device("cuda")
prof = torch.zeros(32, dtype=torch.int64, device=dev)
assert L.qlzx_profile_set(prof.data_ptr()) == 0
names = ["codes", "delta+j2", "walk", "recs", "items", "fill", "jumping", "gather"]
names_small = ["stage+info", "J2..J16", "walk+expand", "recs", "items", "fill", "jumping"]
for n in (4096, 16384, 32768, 65536):
    x = O.gen_text(0x5EED2026, n, n)
    c = O.compress(x)
    out = ctypes.create_string_buffer(n)
    assert L.qlz_decompress(c, out, None) == n and out.raw == x
    prof.zero_()
    torch.cuda.synchronize()
    ts = []
    for _ in range(calls):
        t0 = time.perf_counter_ns()
        L.qlz_decompress(c, out, None)
        ts.append(time.perf_counter_ns() - t0)
    p = prof.cpu().numpy().astype(np.float64)
    if p[31] > 0:  # the small-block LDS path (qlzx_decode_small.hip) took the calls
        k = p[31]
        ph = {nm: round(p[24 + j] / k) for j, nm in enumerate(names_small)}
        ph["(stage)"] = round(p[16] / k)
        ph["(stage+classify)"] = round(p[17] / k)
        if p[18]:
            ph["(.. +candidates)"] = round(p[18] / k)
    else:
        k = max(p[23], 1)
        ph = {nm: round(p[16 + j] / k) for j, nm in enumerate(names[:7])}
    print(f"{n} B (csize {len(c)}): call median {np.median(ts) / 1e3:.1f} us; kernel cycles {ph}, "
          f"sum {sum(ph.values())}", flush=True)
