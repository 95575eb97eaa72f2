"""Time qlzx_decompress_batch on n x bs synthetic text blocks (experiment builds via QLZX_LIB).

usage: QLZX_LIB=... python tools/exp_time.py [nblocks] [block_size] [reps]
Set QLZX_EXPERIMENT=1 for builds that produce wrong bytes on purpose (timing only).
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from gobeansdb_amd import batch

n = int(sys.argv[1]) if len(sys.argv) > 1 else 131072
bs = int(sys.argv[2]) if len(sys.argv) > 2 else 16384
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
dev = torch.device("cuda")
uniq = min(n, 65536)
plain = batch.synth("text", 7, [bs] * uniq, device=dev)
comp, cs, st, _ = batch.compress(plain, max_len=bs)
torch.cuda.synchronize()
idx = torch.from_numpy(np.arange(n) % uniq).to(dev)
src = batch.BlockBatch(comp.data, comp.off[idx], cs[idx])
out = batch.BlockBatch.empty_for([bs] * n, device=dev)
ws = batch.Workspace(dev)
kw = {}
if os.environ.get("QLZX_CRC"):   # time the fused record-CRC verify (K1) as well
    kw = dict(crc_state=torch.full((n,), -1, dtype=torch.int32, device=dev), crc_expect=batch.crc32(src))
dsz, st, _ = batch.decompress(src, out, max_dsize=bs, workspace=ws, **kw)
torch.cuda.synchronize()
exp = bool(os.environ.get("QLZX_EXPERIMENT"))
ok = int((st != 0).sum()) == 0 and torch.equal(out.data[: uniq * bs], plain.data[: uniq * bs])
if not exp and not ok:
    raise SystemExit("round trip FAILED")
ts = []
for _ in range(reps):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    batch.decompress(src, out, max_dsize=bs, workspace=ws, **kw)
    e1.record()
    torch.cuda.synchronize()
    ts.append(e0.elapsed_time(e1))
ms = float(np.median(ts))
print(f"{os.path.basename(os.environ.get('QLZX_LIB', 'libqlzx.so'))}{' +crc' if kw else ''}: {n} x {bs}: {ms:.3f} ms "
      f"({n * bs / ms / 1e6 / 1.073741824:.1f} GiB/s out) roundtrip={'ok' if ok else 'BAD'}")
