"""Encoder cost by input class: k_encode_wg time per block for random, image-like, noisy text,
text and zero blocks (device-resident, fused CRC).  usage: python tools/enc_prof.py [nblocks] [bs]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from gobeansdb_amd import batch  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
bs = int(sys.argv[2]) if len(sys.argv) > 2 else 65536
dev = torch.device("cuda")
g = torch.Generator(device=dev).manual_seed(1)


def blocks(kind):
    if kind in ("text", "image"):
        return batch.synth(kind, 5, [bs] * n, device=dev)
    b = batch.BlockBatch.empty_for([bs] * n, device=dev)
    if kind == "random":
        b.data.copy_(torch.randint(0, 256, b.data.shape, dtype=torch.uint8, device=dev, generator=g))
    elif kind == "noisy":
        t = batch.synth("text", 6, [bs] * n, device=dev)
        r = torch.randint(0, 256, t.data.shape, dtype=torch.uint8, device=dev, generator=g)
        m = torch.rand(t.data.shape, device=dev, generator=g) < 0.42
        b.data.copy_(torch.where(m, r, t.data))
    return b


ws = batch.Workspace(dev)
if os.environ.get("ENC_ONE"):  # tools/enc_one.py: one class, REPS calls, no timing
    src = blocks(os.environ["ENC_ONE"])
    dst = batch.BlockBatch.empty_for([bs] * n, device=dev, pad=400)
    st0 = torch.full((n,), -1, dtype=torch.int32, device=dev)
    for _ in range(int(os.environ.get("REPS", "2"))):
        batch.compress(src, dst, crc_state=st0, max_len=bs, workspace=ws)
    torch.cuda.synchronize()
    sys.exit(0)
for kind in ("random", "image", "noisy", "text", "zeros"):
    src = blocks(kind)
    dst = batch.BlockBatch.empty_for([bs] * n, device=dev, pad=400)
    st0 = torch.full((n,), -1, dtype=torch.int32, device=dev)
    batch.compress(src, dst, crc_state=st0, max_len=bs, workspace=ws)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    _, cs, st, _ = batch.compress(src, dst, crc_state=st0, max_len=bs, workspace=ws)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1)
    stored = int((dst.data[dst.off] & 1 == 0).sum())
    print(f"{kind:7s} {n} x {bs}: {ms:8.2f} ms  {ms * 1e3 / n * 256:8.1f} us/block/WG-slot  "
          f"{n * bs / ms / 1e6:7.1f} GB/s in  stored {stored}/{n}  ratio {float(cs.double().sum()) / (n * bs):.3f}",
          flush=True)
