"""Phase timing of the fast decode kernels from the -DQLZX_PROFILE build (s_memtime stamps).

usage: QLZX_LIB=gobeansdb_amd/libqlzx_prof.so python tools/phase_prof.py [nblocks] [block_size]
"""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from gobeansdb_amd import _lib, batch

n = int(sys.argv[1]) if len(sys.argv) > 1 else 131072
bs = int(sys.argv[2]) if len(sys.argv) > 2 else 16384
kind = sys.argv[3] if len(sys.argv) > 3 else "text"
L = _lib.lib()
L.qlzx_profile_set.argtypes = [ctypes.c_void_p]
dev = torch.device("cuda")
uniq = min(n, 16384)
plain = batch.synth(kind, 7, [bs] * uniq, device=dev)
comp, cs, st, _ = batch.compress(plain, max_len=bs)
torch.cuda.synchronize()
idx = np.arange(n) % uniq
src = batch.BlockBatch(comp.data, comp.off[torch.from_numpy(idx).to(dev)], cs[torch.from_numpy(idx).to(dev)])
out = batch.BlockBatch.empty_for([bs] * n, device=dev)
ws = batch.Workspace(dev)
batch.decompress(src, out, max_dsize=bs, workspace=ws)
torch.cuda.synchronize()
prof = torch.zeros(32, dtype=torch.int64, device=dev)
assert L.qlzx_profile_set(prof.data_ptr()) == 0
t0 = time.time()
dsz, st, _ = batch.decompress(src, out, max_dsize=bs, workspace=ws)
torch.cuda.synchronize()
t1 = time.time()
if not os.environ.get("QLZX_EXPERIMENT"):
    assert int((st != 0).sum()) == 0
p = prof.cpu().numpy().astype(np.float64)
csum = float(cs[torch.from_numpy(idx).to(dev)].double().sum())
items_est = n * 3817
waves_k1 = (n + 63) // 64
rounds = csum / n / 64
batches = n * 3817 / 64
print(f"blocks {n} x {bs} {kind}: wall {1e3 * (t1 - t0):.2f} ms, ratio {csum / (n * bs):.3f}")
# K1 k_dec_parse6 (slot 0): outer iterations, wave step trips, lane steps, cycles, waves
k1 = p[0:8]
w1 = max(k1[4], 1)
print("K1 per wave: iterations %.1f, wave step trips %.1f, lane steps per lane %.1f (lane efficiency %.2f), "
      "cycles %.0f" % (k1[0] / w1, k1[1] / w1, k1[2] / w1 / 64, k1[2] / max(64 * k1[1], 1), k1[3] / w1))
# K2 = k_dec_bytes: stamps 0..4 are phases, 5..7 counts (slot 1 = p[8:16])
names2 = ["item phase", "markers+fill", "pointer jumping", "gather", "store"]
k2 = p[8:16]
print("K2 per block (cycles):", {nm: round(k2[j] / n) for j, nm in enumerate(names2)}, "total", round(k2[:5].sum() / n))
print("K2 per block: batches %.1f, marker passes %.1f, pointer-jumping rounds %.1f" % (k2[5] / n, k2[6] / n, k2[7] / n))
