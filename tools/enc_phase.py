"""Per-phase cycles of k_encode_wg (profile build, s_memtime stamps), per input class.

usage: QLZX_LIB=gobeansdb_amd/libqlzx_prof.so python tools/enc_phase.py [nblocks] [bs]
"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from gobeansdb_amd import _lib, batch  # noqa: E402
sys.argv += [] if len(sys.argv) > 1 else []
import importlib.util  # noqa: E402

spec = importlib.util.spec_from_file_location("ep", os.path.join(os.path.dirname(__file__), "enc_prof.py"))
n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
bs = int(sys.argv[2]) if len(sys.argv) > 2 else 65536
L = _lib.lib()
L.qlzx_profile_set.argtypes = [ctypes.c_void_p]
dev = torch.device("cuda")
g = torch.Generator(device=dev).manual_seed(1)
names = ["setup", "proof+load", "sort", "match", "parse", "emit/stored", "crc"]
waves = bs // 64 // 64


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
prof = torch.zeros(40, dtype=torch.int64, device=dev)
for kind in os.environ.get("KINDS", "random,noisy,text,zeros").split(","):
    src = blocks(kind)
    dst = batch.BlockBatch.empty_for([bs] * n, device=dev, pad=int(os.environ.get("PAD", "400")))
    st0 = torch.full((n,), -1, dtype=torch.int32, device=dev)
    batch.compress(src, dst, crc_state=st0, max_len=bs, workspace=ws)
    torch.cuda.synchronize()
    prof.zero_()
    assert L.qlzx_profile_set(prof.data_ptr()) == 0
    batch.compress(src, dst, crc_state=st0, max_len=bs, workspace=ws)
    torch.cuda.synchronize()
    assert L.qlzx_profile_set(None) == 0
    p = prof.cpu().numpy()[16:24] / (n * max(waves, 1))
    print(f"{kind:7s} cycles/block:", {nm: int(p[j]) for j, nm in enumerate(names)}, "total", int(p[:7].sum()),
          flush=True)
    q = prof.cpu().numpy()[24:40] / (n * max(waves, 1))
    print("   sort passes (zero, count, scan, scatter):", [int(x) for x in q[0:4]], [int(x) for x in q[8:12]], flush=True)
