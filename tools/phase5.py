"""Phase cycles of the v5 ring K2 (dec_v5r_block) from the -DQLZX_PROFILE build (tools only).
usage: QLZX_LIB=gobeansdb_amd/libqlzx_prof.so python tools/phase5.py [nblocks] [block_size]"""
import ctypes, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from gobeansdb_amd import _lib, batch
n = int(sys.argv[1]) if len(sys.argv) > 1 else 131072
bs = int(sys.argv[2]) if len(sys.argv) > 2 else 16384
L = _lib.lib()
L.qlzx_profile_set.argtypes = [ctypes.c_void_p]
dev = torch.device("cuda")
uniq = min(n, 16384)
plain = batch.synth("text", 7, [bs] * uniq, device=dev)
comp, cs, st, _ = batch.compress(plain, max_len=bs)
idx = torch.from_numpy(np.arange(n) % uniq).to(dev)
src = batch.BlockBatch(comp.data, comp.off[idx], cs[idx])
out = batch.BlockBatch.empty_for([bs] * n, device=dev)
ws = batch.Workspace(dev)
batch.decompress(src, out, max_dsize=bs, workspace=ws)
torch.cuda.synchronize()
prof = torch.zeros(32, dtype=torch.int64, device=dev)
assert L.qlzx_profile_set(prof.data_ptr()) == 0
dsz, st, _ = batch.decompress(src, out, max_dsize=bs, workspace=ws)
torch.cuda.synchronize()
assert int((st != 0).sum()) == 0 and torch.equal(out.data[: uniq * bs], plain.data[: uniq * bs])
p = prof.cpu().numpy().astype(np.float64)[8:16]
names = ["items", "fill", "far", "gather1", "passes+store"]
print("K2 cycles per block:", {nm: round(p[j] / n) for j, nm in enumerate(names)}, "total", round(p[:5].sum() / n))
print("per block: batches %.1f, passes %.1f, far chunks %.1f" % (p[5] / n, p[6] / n, p[7] / n))
