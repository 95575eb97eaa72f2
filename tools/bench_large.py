"""Large values (> 64 KiB, up to BodyMax = 50 MiB, config/mc_config.go:7-8): decode and encode
time per value on the GPU against the reference quicklz.c on one host core (tools only).

TryCompress compresses whole bodies up to BodyMax (store/item.go:149-151) and Payload.Decompress
decodes them (store/item.go:167).  Per size (1, 8, 50 MiB text values):
  * gpu_batch_decode_ms   qlzx_decompress_batch on a device-resident value (the whole-GPU path,
                          qlzx_decode_huge.hip), event time;
  * gpu_single_decode_ms  qlz_decompress from host memory (H2D + decode + D2H), wall time;
  * gpu_batch_encode_ms / gpu_single_encode_ms   the same for compress (qlzx_encode_huge.hip);
  * ref_decode_ms / ref_encode_ms   reference qlz_decompress / qlz_compress, one core.
usage: python tools/bench_large.py [--out profiles/r04_large.json] [--reps 3]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

MIB = 1 << 20


def wall_ms(fn, reps):
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append((time.perf_counter() - t0) * 1e3)
    return round(float(np.median(ts)), 3)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--sizes", default="1,8,50")
    ap.add_argument("--no-encode", action="store_true")
    a = ap.parse_args()
    import torch
    from gobeansdb_amd import _lib, batch
    from oracle import oracle as O
    L = _lib.lib()
    ref = O.ref()
    dev = torch.device("cuda")
    rows = []
    for mib in [int(x) for x in a.sizes.split(",")]:
        n = mib * MIB
        plain = O.gen_text(0x1A46E, mib, n)
        comp = O.compress(plain)
        row = {"mib": mib, "bytes": n, "csize": len(comp), "ratio": round(len(comp) / n, 3)}
        # batch decode, device resident
        src = batch.BlockBatch.from_bytes([comp], device=dev)
        out = batch.BlockBatch.empty_for([n], device=dev)
        ws = batch.Workspace(dev)
        dsz, st, _ = batch.decompress(src, out, max_dsize=n, workspace=ws)
        torch.cuda.synchronize()
        assert int(st[0]) == 0 and out.to_bytes(dsz.cpu().numpy())[0] == plain, "batch decode mismatch"
        ts = []
        for _ in range(a.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            batch.decompress(src, out, max_dsize=n, workspace=ws)
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        row["gpu_batch_decode_ms"] = round(float(np.median(ts)), 3)
        # single call from host memory
        csrc = np.frombuffer(comp, np.uint8).copy()
        dst = np.zeros(n + 64, np.uint8)
        assert L.qlz_decompress(csrc.ctypes.data, dst.ctypes.data, None) == n and dst[:n].tobytes() == plain
        row["gpu_single_decode_ms"] = wall_ms(lambda: L.qlz_decompress(csrc.ctypes.data, dst.ctypes.data, None), a.reps)
        if ref is not None:
            Q = ref[0]
            sc = np.zeros(528400, np.uint8)
            row["ref_decode_ms"] = wall_ms(lambda: Q.qlz_decompress(csrc.ctypes.data, dst.ctypes.data, sc.ctypes.data),
                                           a.reps)
            row["decode_speedup_vs_ref_1core"] = round(row["ref_decode_ms"] / row["gpu_single_decode_ms"], 2)
        if not a.no_encode:
            psrc = np.frombuffer(plain, np.uint8).copy()
            cdst = np.zeros(n + 400, np.uint8)
            r = L.qlz_compress(psrc.ctypes.data, cdst.ctypes.data, n, None)
            assert cdst[:r].tobytes() == comp, "single-call encode differs from the oracle"
            row["gpu_single_encode_ms"] = wall_ms(lambda: L.qlz_compress(psrc.ctypes.data, cdst.ctypes.data, n, None),
                                                  a.reps)
            pb = batch.BlockBatch.from_bytes([plain], device=dev)
            cb = batch.BlockBatch.empty_for([n], device=dev, pad=400)
            batch.compress(pb, cb, max_len=n, workspace=ws)
            torch.cuda.synchronize()
            ts = []
            for _ in range(a.reps):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                batch.compress(pb, cb, max_len=n, workspace=ws)
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1))
            row["gpu_batch_encode_ms"] = round(float(np.median(ts)), 3)
            if ref is not None:
                row["ref_encode_ms"] = wall_ms(lambda: ref[0].qlz_compress(psrc.ctypes.data, cdst.ctypes.data, n,
                                                                           sc.ctypes.data), a.reps)
                row["encode_speedup_vs_ref_1core"] = round(row["ref_encode_ms"] / row["gpu_single_encode_ms"], 2)
        rows.append(row)
        print(json.dumps(row), flush=True)
    res = {"what": "large text values: GPU decode/encode per value vs reference quicklz.c on one core",
           "rows": rows}
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
