"""Debug: compress gen_text(5, n, n) through the 64 KiB encoder and save the GPU output next to
the oracle's (gpurun_out/rt_dump/)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from gobeansdb_amd import batch  # noqa: E402
from oracle import oracle as O  # noqa: E402

out = "gpurun_out/rt_dump"
os.makedirs(out, exist_ok=True)
for n in [int(a) for a in sys.argv[1:]] or [10000]:
    b = O.gen_text(5, n, n)
    src = batch.BlockBatch.from_bytes([b, b, b])
    dst, csize, status, crc = batch.compress(src, want_crc=True, max_len=65536)
    torch.cuda.synchronize()
    cs = csize.cpu().numpy()
    outs = dst.to_bytes(cs)
    exp = O.compress(b)
    for k, o in enumerate(outs):
        print(n, k, len(o), len(exp), o == exp)
        open(f"{out}/gpu_{n}_{k}.bin", "wb").write(o)
    open(f"{out}/orc_{n}.bin", "wb").write(exp)
    open(f"{out}/in_{n}.bin", "wb").write(b)
