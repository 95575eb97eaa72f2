#!/usr/bin/env python3
"""Benchmark: device-resident batched QuickLZ decompress (BASELINE.json config c2).

One step = decompress every block of the rank's shard once (1 M x 16 KiB text-like
blocks by default, ~2x compressible), inputs already resident in HBM.  Blocks are
generated on the GPU (deterministic text) and compressed on the GPU
by this library's encoder; the round trip is verified on device before timing.

Multi-GPU: one process per GPU (torch.distributed.run); each rank owns an
independent shard of blocks (weak scaling, no data-path collective); timing is
barrier + synchronize bracketed and max-reduced over ranks.

Prints one JSON line (rank 0).  See DESIGN.md §6 for the roofline accounting.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)


def log(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print("[bench]", *a, file=sys.stderr, flush=True)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--blocks", type=int, default=1 << 20, help="blocks per GPU")
    p.add_argument("--block-size", type=int, default=16384)
    p.add_argument("--mode", choices=["decompress", "compress"], default="decompress")
    p.add_argument("--kind", choices=["text", "image"], default=None)
    p.add_argument("--unique", type=int, default=0,
                   help="distinct blocks generated+compressed (0 = all); the rest repeat them")
    p.add_argument("--gen-chunk", type=int, default=1 << 16)
    p.add_argument("--cpu-seconds", type=float, default=15.0)
    p.add_argument("--no-cpu", action="store_true")
    p.add_argument("--crc", action="store_true", help="fused record CRC verify in the timed pass")
    p.add_argument("--traffic-json", default=None,
                   help="PMC HBM bytes per block (tools/traffic.py output); default: the committed "
                        "profiles/r01_c2_traffic.json for the c2 workload")
    return p.parse_args()


def main():
    args = parse()
    from gobeansdb_amd import _lib, batch, shard

    rank, world, local = shard.env_rank()
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=dev)
    kind = args.kind or ("text" if args.mode == "decompress" else "image")
    if args.mode == "compress":
        return bench_compress(args, rank, world, dev, kind)
    n = args.blocks
    bs = args.block_size
    uniq = args.unique or n
    log(f"rank {rank}/{world}: {n} blocks x {bs} B {kind}, unique {uniq}; lib: {_lib.info()}")

    # ---- generate + compress the shard on the GPU, chunked, into one buffer ----
    t0 = time.time()
    ws = batch.Workspace(dev)
    coff, ctotal = batch.pack_offsets([bs] * uniq, pad=400)        # CCompress allocates len+400
    cbuf = torch.empty(ctotal, dtype=torch.uint8, device=dev)
    coff_t = torch.from_numpy(coff.view(np.int64)).to(dev)
    cs_parts = []
    first, _ = shard.weak_shard(rank, n)   # weak scaling: each rank owns its own block ids
    for c0 in range(0, uniq, args.gen_chunk):
        m = min(args.gen_chunk, uniq - c0)
        plain = batch.synth(kind, 0x5EED2026, [bs] * m, first_id=first + c0, device=dev)
        dst = batch.BlockBatch(cbuf, coff_t[c0:c0 + m], plain.length)
        _, cs, st, _ = batch.compress(plain, dst, max_len=bs, workspace=ws)
        if int((st != 0).sum().item()):
            raise SystemExit("compress failed on the GPU")
        cs_parts.append(cs)
        del plain
    torch.cuda.synchronize()
    log(f"generate+compress {uniq} blocks: {time.time() - t0:.1f}s")

    # blocks repeat the unique set when --unique < --blocks
    cs_all = torch.cat(cs_parts).cpu().numpy().view(np.uint32)
    idx = np.arange(n) % uniq
    src_off = torch.from_numpy(coff[idx].view(np.int64)).to(dev)
    src_len = torch.from_numpy(cs_all[idx].view(np.int32)).to(dev)
    src = batch.BlockBatch(cbuf, src_off, src_len)
    out = batch.BlockBatch.empty_for([bs] * n, device=dev)
    csum = int(cs_all[idx].astype(np.int64).sum())
    dsum = n * bs
    log(f"compressed {csum / 2**30:.2f} GiB, ratio {csum / dsum:.3f}")

    # ---- correctness gate on device: decompress once and compare ----
    dsz, st, _ = batch.decompress(src, out, max_dsize=bs, workspace=ws)
    torch.cuda.synchronize()
    assert int((st != 0).sum().item()) == 0, "decompress status"
    for c0 in range(0, uniq, args.gen_chunk):   # every unique block, chunk by chunk
        m = min(args.gen_chunk, uniq - c0)
        check = batch.synth(kind, 0x5EED2026, [bs] * m, first_id=first + c0, device=dev)
        if not torch.equal(out.data[c0 * bs:(c0 + m) * bs], check.data[:m * bs]):
            raise SystemExit(f"round trip mismatch in blocks {c0}..{c0 + m}")
        del check
    log("device round trip verified")

    crc_state = crc_expect = None
    if args.crc:
        crc_state = torch.full((n,), -1, dtype=torch.int32, device=dev)
        crc_expect = batch.crc32(src)

    # ---- timed region ----
    stream = torch.cuda.current_stream()

    def step():
        batch.decompress(src, out, crc_state=crc_state, crc_expect=crc_expect, max_dsize=bs,
                         workspace=ws, stream=stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    t_start = time.perf_counter()
    for e0, e1 in evs:
        e0.record(stream)
        step()
        e1.record(stream)
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t_start
    kern_ms = float(np.mean([e0.elapsed_time(e1) for e0, e1 in evs]))
    wall, kern_ms = shard.max_over_ranks([wall, kern_ms], device=dev)   # the slowest rank counts
    tot = shard.sum_over_ranks({"out_bytes": dsum, "in_bytes": csum}, device=dev)
    ms_per_step = wall * 1e3 / args.steps

    total_out = tot["out_bytes"] * args.steps
    value = total_out / wall / 2**30
    achieved = (csum + dsum) / (kern_ms * 1e-3) / 1e9
    traffic = None
    if args.traffic_json is None and args.mode == "decompress" and kind == "text" and bs == 16384 and not args.crc:
        args.traffic_json = os.path.join(ROOT, "profiles", "r01_c2_traffic.json")
    if args.traffic_json and os.path.exists(args.traffic_json):
        # PMC-measured HBM bytes per block (tools/traffic.py) x blocks per launch
        tj = json.load(open(args.traffic_json))
        traffic = round(tj["hbm_bytes_per_block"] * n)

    cpu = None
    if rank == 0 and not args.no_cpu:
        cpu = cpu_baseline(kind, bs, args.cpu_seconds)

    if rank == 0:
        rec = {
            "metric": "GiB/s device-resident QuickLZ decompress (+compress), batched 4-64 KiB values",
            "value": round(value, 3),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic",
            "config": {"workload": f"c2: decompress {n} x {bs} B {kind}-like blocks per GPU "
                                   f"(ratio {csum / dsum:.3f}), device-resident",
                       "blocks_per_gpu": n, "block_size": bs, "unique_blocks": uniq,
                       "fused_crc": bool(args.crc), "parallelism": f"shard{world}"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                         "kernel_ms": round(kern_ms, 4),
                         "algorithmic_bytes_per_launch": csum + dsum},
            "cpu_baseline": cpu,
        }
        print(json.dumps(rec), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


SEED = 0x5EED2026


def bench_compress(args, rank, world, dev, kind):
    """Config c3: compress every block of the rank's shard (1 M x 64 KiB image-like by default) with
    the fused record CRC, inputs resident in HBM.  Verified before timing by a device round trip
    (compress -> decompress == input) and a CRC recomputation over the outputs."""
    from gobeansdb_amd import batch, shard
    n, bs = args.blocks, args.block_size
    first, _ = shard.weak_shard(rank, n)
    t0 = time.time()
    plain = batch.BlockBatch.empty_for([bs] * n, device=dev)
    poff = plain.off.cpu().numpy().view(np.uint64)
    for c0 in range(0, n, args.gen_chunk):
        m = min(args.gen_chunk, n - c0)
        part = batch.synth(kind, SEED, [bs] * m, first_id=first + c0, device=dev)
        if bs % 256 == 0:   # contiguous packing: one copy per chunk
            o = int(poff[c0])
            plain.data[o:o + m * bs].copy_(part.data[:m * bs])
        else:
            for j in range(m):
                o, q = int(poff[c0 + j]), int(part.off[j])
                plain.data[o:o + bs].copy_(part.data[q:q + bs])
        del part
    dst = batch.BlockBatch.empty_for([bs] * n, device=dev, pad=400)   # CCompress allocates len+400
    ws = batch.Workspace(dev)
    crc_state = torch.full((n,), -1, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    log(f"rank {rank}: generated {n} x {bs} B {kind} in {time.time() - t0:.1f}s")

    # ---- correctness gate: round trip on the device, fused CRC == recomputed CRC ----
    _, cs, st, crc = batch.compress(plain, dst, crc_state=crc_state, max_len=bs, workspace=ws)
    torch.cuda.synchronize()
    if int((st != 0).sum().item()):
        raise SystemExit("compress status")
    comp = batch.BlockBatch(dst.data, dst.off, cs)
    if not torch.equal(batch.crc32(comp), crc):
        raise SystemExit("fused CRC != recomputed CRC")
    chk = 1 << 14
    tmp = batch.BlockBatch.empty_for([bs] * chk, device=dev)
    for c0 in range(0, n, chk):
        m = min(chk, n - c0)
        sub = batch.BlockBatch(dst.data, dst.off[c0:c0 + m], cs[c0:c0 + m])
        out = batch.BlockBatch(tmp.data, tmp.off[:m], tmp.length[:m])
        _, st2, _ = batch.decompress(sub, out, max_dsize=bs, workspace=ws)
        o0 = int(poff[c0])
        if int((st2 != 0).sum().item()) or not torch.equal(tmp.data[:m * bs], plain.data[o0:o0 + m * bs]):
            raise SystemExit(f"round trip mismatch in blocks {c0}..{c0 + m}")
    csum = int(cs.to(torch.int64).sum().item())
    stored = int((dst.data[dst.off] & 1 == 0).sum().item())
    log(f"device round trip verified; {stored}/{n} blocks stored, out/in {csum / (n * bs):.4f}")

    stream = torch.cuda.current_stream()

    def step():
        batch.compress(plain, dst, crc_state=crc_state, max_len=bs, workspace=ws, stream=stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    t_start = time.perf_counter()
    for e0, e1 in evs:
        e0.record(stream)
        step()
        e1.record(stream)
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t_start
    kern_ms = float(np.mean([e0.elapsed_time(e1) for e0, e1 in evs]))
    wall, kern_ms = shard.max_over_ranks([wall, kern_ms], device=dev)
    tot = shard.sum_over_ranks({"in_bytes": n * bs, "out_bytes": csum}, device=dev)
    value = tot["in_bytes"] * args.steps / wall / 2**30
    achieved = (n * bs + csum) / (kern_ms * 1e-3) / 1e9
    traffic = None
    tj = args.traffic_json or os.path.join(ROOT, "profiles", "r01_c3_traffic.json")
    if os.path.exists(tj) and kind == "image" and bs == 65536:
        traffic = round(json.load(open(tj))["hbm_bytes_per_block"] * n)
    cpu = None
    if rank == 0 and not args.no_cpu:
        cpu = cpu_baseline(kind, bs, args.cpu_seconds, mode="compress")
    if rank == 0:
        rec = {
            "metric": "GiB/s device-resident QuickLZ decompress (+compress), batched 4-64 KiB values",
            "value": round(value, 3), "unit": "GiB/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(wall * 1e3 / args.steps, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
            "data": "synthetic",
            "config": {"workload": f"c3: compress + fused CRC32 of {n} x {bs} B {kind}-like values per GPU "
                                   f"({stored} stored), device-resident; value = input GiB/s",
                       "blocks_per_gpu": n, "block_size": bs, "fused_crc": True,
                       "parallelism": f"shard{world}"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                         "kernel_ms": round(kern_ms, 4), "algorithmic_bytes_per_launch": n * bs + csum},
            "cpu_baseline": cpu,
        }
        print(json.dumps(rec), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


REF_WHAT = ("reference quicklz/quicklz.c {fn} (oracle/_ref/libqlzref.so, gcc -O2 as cgo builds it), "
            "per-thread scratch")


def cpu_baseline(kind: str, bs: int, seconds: float, mode: str = "decompress"):
    """Oracle decoder on the host cores over a bounded sample of the same workload."""
    from oracle import oracle as O
    threads = min(os.cpu_count() or 1, 16)
    L = O.lib()
    Q = O.ref_if_built()  # the reference quicklz.c (oracle/_ref) when built; else the C restatement
    kind_ = "reference" if Q is not None else "port"
    nblk = 2048 if mode == "decompress" else 256
    if mode == "compress":
        plain = [O.gen_text(SEED, i, bs) if kind == "text" else O.gen_image(SEED, i, bs) for i in range(nblk)]
        off_s, tot_s = _pack(plain)
        off_d, tot_d = _pack([b"\0" * (bs + 400)] * nblk)
        srcb = np.zeros(tot_s, np.uint8)
        for o, p_ in zip(off_s, plain):
            srcb[int(o): int(o) + len(p_)] = np.frombuffer(p_, np.uint8)
        lens = np.asarray([len(p_) for p_ in plain], np.uint32)
        dst = np.zeros(tot_d, np.uint8)
        reps, ns = 0, 0.0
        t_end = time.time() + seconds
        while time.time() < t_end or reps == 0:
            if Q is not None:
                ns += L.orc_bench_ref(ctypes.cast(Q.qlz_compress, ctypes.c_void_p).value, srcb.ctypes.data,
                                      off_s.ctypes.data, lens.ctypes.data, dst.ctypes.data, off_d.ctypes.data,
                                      nblk, threads, 1)
            else:
                ns += L.orc_bench_compress(srcb.ctypes.data, off_s.ctypes.data, lens.ctypes.data,
                                           dst.ctypes.data, off_d.ctypes.data, nblk, threads, 0)
            reps += 1
        gibs = reps * nblk * bs / (ns * 1e-9) / 2**30
        what = REF_WHAT.format(fn="qlz_compress") if Q is not None else "oracle/qlz_oracle.c orc_compress"
        return {"value": round(gibs, 3), "unit": "GiB/s", "cores": threads, "kind": kind_,
                "sample": f"{reps} passes over {nblk} x {bs} B {kind} blocks, {what} (no CRC), "
                          f"{threads} threads, -O2"}
    plain = [O.gen_text(0x5EED2026, i, bs) if kind == "text" else O.gen_image(0x5EED2026, i, bs)
             for i in range(nblk)]
    comp = [O.compress(p) for p in plain]
    off_c, tot_c = _pack(comp)
    off_d, tot_d = _pack(plain)
    srcb = np.zeros(tot_c, np.uint8)
    for o, c in zip(off_c, comp):
        srcb[int(o): int(o) + len(c)] = np.frombuffer(c, np.uint8)
    lens = np.asarray([len(c) for c in comp], np.uint32)
    dst = np.zeros(tot_d, np.uint8)
    reps, ns = 0, 0.0
    t_end = time.time() + seconds
    while time.time() < t_end or reps == 0:
        if Q is not None:
            ns += L.orc_bench_ref(ctypes.cast(Q.qlz_decompress, ctypes.c_void_p).value, srcb.ctypes.data,
                                  off_c.ctypes.data, lens.ctypes.data, dst.ctypes.data, off_d.ctypes.data,
                                  nblk, threads, 0)
        else:
            ns += L.orc_bench_decompress(srcb.ctypes.data, off_c.ctypes.data, lens.ctypes.data,
                                         dst.ctypes.data, off_d.ctypes.data, nblk, threads, 0)
        reps += 1
    if Q is not None and not all(dst[int(o): int(o) + bs].tobytes() == p_ for o, p_ in zip(off_d[:8], plain[:8])):
        raise RuntimeError("reference decompress baseline produced wrong bytes")
    gibs = reps * nblk * bs / (ns * 1e-9) / 2**30
    what = REF_WHAT.format(fn="qlz_decompress") if Q is not None else "oracle/qlz_oracle.c orc_decompress"
    return {"value": round(gibs, 3), "unit": "GiB/s", "cores": threads, "kind": kind_,
            "sample": f"{reps} passes over {nblk} x {bs} B {kind} blocks, {what}, {threads} threads, -O2"}


def _pack(blocks):
    ln = np.asarray([len(b) for b in blocks], np.int64)
    sz = (ln + 255) // 256 * 256
    off = np.zeros(len(ln), np.uint64)
    off[1:] = np.cumsum(sz)[:-1]
    return off, int(sz.sum())


if __name__ == "__main__":
    main()
