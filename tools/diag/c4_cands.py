"""Diagnostic: candidate statistics of the c4 chunk (how many slots pass the size checks and
how many CRC bytes they imply), to see what k_rp_crc spends its time on."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tools"))
import numpy as np, torch
import bench_replay as BR
from gobeansdb_amd import replay, batch
from gobeansdb_amd.replay import MAX_KEY_LEN, BODY_MAX
dev = torch.device("cuda", 0)
host, nrec, *_ , rec_off = BR.build_chunk(1000, 2026, dev)
ns = len(host) // 256
h = host[: ns * 256].reshape(ns, 256)
ksz = h[:, 16:20].copy().view(np.uint32)[:, 0].astype(np.int64)
vsz = h[:, 20:24].copy().view(np.uint32)[:, 0].astype(np.int64)
off = np.arange(ns, dtype=np.int64) * 256
cand = (ksz >= 1) & (ksz <= MAX_KEY_LEN) & (vsz <= BODY_MAX) & (off + 24 + ksz + vsz <= len(host))
real = np.zeros(ns, bool); real[(rec_off // 256).astype(np.int64)] = True
fl = (20 + ksz + vsz)[cand & ~real]
print("slots", ns, "records", nrec, "candidates", int(cand.sum()), "false", int((cand & ~real).sum()))
print("real crc bytes", int((20 + ksz + vsz)[real].sum()), "false crc bytes", int(fl.sum()), "max false", int(fl.max()) if len(fl) else 0)
print("false ksz sample", ksz[cand & ~real][:20], "vsz", vsz[cand & ~real][:20])
d = torch.from_numpy(host).to(dev); ws = batch.Workspace(dev)
for _ in range(3):
    torch.cuda.synchronize(); t = time.perf_counter()
    r = replay.index(d, workspace=ws); torch.cuda.synchronize()
    print("index ms", (time.perf_counter() - t) * 1e3, "ncand", r[3])
