#!/usr/bin/env python3
"""Benchmark: device-resident batched QuickLZ decompress (BASELINE.json config c2).

One step = decompress every block of the rank's shard once (1 M x 16 KiB text-like
blocks by default, ~2x compressible), inputs already resident in HBM.  Blocks are
generated on the GPU (deterministic text) and compressed on the GPU
by this library's encoder; the round trip is verified on device before timing.

Multi-GPU: one process per GPU (torch.distributed.run); each rank owns an
independent shard of blocks (weak scaling, no data-path collective); timing is
barrier + synchronize bracketed and max-reduced over ranks.

Prints one JSON line (rank 0).  See DESIGN.md §3 for the roofline accounting.  The default c2
run (1 M x 16 KiB) also measures BASELINE config c3 -- compress + fused CRC32 of 1 M x 64 KiB
image-like values, the "(+compress)" of the metric -- after releasing the c2 buffers, and reports
it under "compress" in the same line (--no-c3 skips it; --config c3 runs it alone); then config c4
-- .data replay of one ~50 GiB corpus of chunk files split over the ranks on record boundaries,
device-resident and pipelined end to end -- under "replay" (--no-c4 skips it); then config c5
-- one 400 GiB corpus of distinct mixed 4-64 KiB values split over the ranks and streamed through
HBM in rounds, strong scaling -- under "mixed" (--no-c5 skips it; --config c5 runs it alone).
c4 and c5 carry a parity digest (XOR of output CRC32s, all-gathered) that is the same at every N.
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
    p.add_argument("--gpus", type=int, default=1,
                   help="ranks (one per GPU); > 1 without a torch.distributed.run environment "
                        "starts torch.distributed.run with that many ranks as a child process")
    p.add_argument("--config", choices=["c2", "c3", "c5"], default="c2",
                   help="c2: decompress 1 M x 16 KiB text (BASELINE metric); c3: compress 1 M x 64 KiB "
                        "image-like (= --mode compress); c5: 400 GiB of mixed values (tools/bench_c5.py)")
    p.add_argument("--standin", choices=["cpu"], default=None,
                   help="launcher test only: a CPU stand-in step on gloo instead of the GPU codec "
                        "(no measurement; used by tests/test_bench_launcher.py)")
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--blocks", type=int, default=1 << 20, help="blocks per GPU")
    p.add_argument("--block-size", type=int, default=None,
                   help="bytes per block (default: 16384; 65536 for --config c3 / --mode compress)")
    p.add_argument("--mode", choices=["decompress", "compress"], default="decompress")
    p.add_argument("--kind", choices=["text", "image"], default=None)
    p.add_argument("--unique", type=int, default=0,
                   help="distinct blocks generated+compressed (0 = all); the rest repeat them")
    p.add_argument("--gen-chunk", type=int, default=1 << 16)
    p.add_argument("--cpu-seconds", type=float, default=15.0)
    p.add_argument("--no-cpu", action="store_true")
    p.add_argument("--no-c3", action="store_true",
                   help="c2 run: skip the c3 compress leg reported under \"compress\" in the same line")
    p.add_argument("--c3-steps", type=int, default=3, help="timed steps of the c3 compress leg")
    p.add_argument("--legs-small", action="store_true",
                   help="rehearsal only: run the c3 and c5 legs at this run's --blocks and a 1 GiB c5 job")
    p.add_argument("--no-c5", action="store_true",
                   help="c2 run: skip the c5 leg (400 GiB of mixed values over the ranks, strong "
                        "scaling) reported under \"mixed\" in the same line")
    p.add_argument("--no-c4", action="store_true",
                   help="c2 run: skip the c4 .data replay leg reported under \"replay\" in the same line")
    p.add_argument("--c4-chunk-mib", type=int, default=4000, help="c4 leg: MiB per chunk file (two distinct)")
    p.add_argument("--c4-files", type=int, default=13, help="c4 leg: files in the corpus (~50 GiB)")
    p.add_argument("--no-record", action="store_true", help="c2 run: skip the f3 record-encode leg")
    p.add_argument("--record-values", type=int, default=1 << 18, help="f3 leg: values per GPU (16 KiB text)")
    p.add_argument("--crc", action="store_true", help="fused record CRC verify in the timed pass")
    p.add_argument("--no-crc-leg", action="store_true",
                   help="skip the \"crc\" leg (the c2 shard again with the fused CRC verify)")
    p.add_argument("--traffic-json", default=None,
                   help="PMC HBM bytes per block (tools/traffic.py output); default: the committed "
                        "profiles/r05_c2_traffic.json for the c2 workload")
    return p.parse_args()


def launch(n: int, argv: list[str]) -> int:
    """Run this script under torch.distributed.run with n ranks as a CHILD process (the parent
    has not touched the GPU and never execs), relay its output, return its exit code."""
    import socket
    import subprocess
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__), *argv]
    log(f"launching {n} ranks: {' '.join(cmd[1:])}")
    try:
        return subprocess.run(cmd).returncode
    except OSError as e:
        log(f"launch failed: {e}")
        return 1


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch(args.gpus, sys.argv[1:]))
    from gobeansdb_amd import shard
    rank, world, local = shard.env_rank()
    if world != args.gpus:
        log(f"WORLD_SIZE {world} != --gpus {args.gpus}: refusing to report a mislabelled line")
        sys.exit(2)
    if args.standin:
        return bench_standin(args, rank, world)
    if args.config == "c5":
        return bench_c5(args)
    if args.config == "c3":
        args.mode = "compress"
    if args.block_size is None:  # BASELINE configs: c2 1 M x 16 KiB, c3 1 M x 64 KiB
        args.block_size = 65536 if args.mode == "compress" else 16384
    from gobeansdb_amd import _lib, batch

    # one GPU per rank; on a box with fewer GPUs than ranks (a rehearsal, QLZX_BENCH_PG=gloo)
    # ranks share devices round-robin
    local = local % max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        import torch.distributed as dist
        backend = os.environ.get("QLZX_BENCH_PG", "nccl")  # nccl = RCCL; gloo only to rehearse N > 1
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
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

    crc_leg = None
    if not args.crc and not args.no_crc_leg:
        # the read path always verifies the record CRC (store/datafile.go:161-168): the same shard
        # decoded with the CRC fused into the pass and checked against the stored values' CRCs
        cst = torch.full((n,), -1, dtype=torch.int32, device=dev)
        cexp = batch.crc32(src)
        _, st3, _ = batch.decompress(src, out, crc_state=cst, crc_expect=cexp, max_dsize=bs, workspace=ws)
        torch.cuda.synchronize()
        assert int((st3 != 0).sum().item()) == 0, "fused CRC verify failed"
        for _ in range(args.warmup):
            batch.decompress(src, out, crc_state=cst, crc_expect=cexp, max_dsize=bs, workspace=ws, stream=stream)
        torch.cuda.synchronize()
        if world > 1:
            torch.distributed.barrier()
        torch.cuda.synchronize()
        t0c = time.perf_counter()
        for _ in range(args.steps):
            batch.decompress(src, out, crc_state=cst, crc_expect=cexp, max_dsize=bs, workspace=ws, stream=stream)
        torch.cuda.synchronize()
        if world > 1:
            torch.distributed.barrier()
        torch.cuda.synchronize()
        wall_c = shard.max_over_ranks([time.perf_counter() - t0c], device=dev)[0]
        crc_leg = {"value": round(tot["out_bytes"] * args.steps / wall_c / 2**30, 3), "unit": "GiB/s",
                   "ms_per_step": round(wall_c * 1e3 / args.steps, 4),
                   "vs_value": round((tot["out_bytes"] * args.steps / wall_c) / (tot["out_bytes"] * args.steps / wall), 4),
                   "what": "the c2 shard decoded with the record CRC32 of every block computed in the same "
                           "call (fused into the decode kernel K2) and verified against crc_expect before its "
                           "decode (read path of store/datafile.go:161-168)"}
        del cst, cexp

    total_out = tot["out_bytes"] * args.steps
    value = total_out / wall / 2**30
    achieved = (csum + dsum) / (kern_ms * 1e-3) / 1e9
    traffic = None
    if args.traffic_json is None and args.mode == "decompress" and kind == "text" and bs == 16384 and not args.crc:
        args.traffic_json = os.path.join(ROOT, "profiles", "r06_c2_traffic.json")
    traffic_src = None
    if args.traffic_json and os.path.exists(args.traffic_json):
        # PMC-measured HBM bytes per block (tools/traffic.py) x blocks per launch: a committed
        # measurement of this workload (FETCH_SIZE x 2 + WRITE_SIZE passes), not a counter of this run
        tj = json.load(open(args.traffic_json))
        per_block = tj.get("hbm_bytes_per_block")
        if per_block is None and tj.get("hbm_bytes_per_call") and tj.get("nblocks_per_call"):
            per_block = tj["hbm_bytes_per_call"] / tj["nblocks_per_call"]
        if per_block is not None:  # an unreadable profile leaves traffic null rather than no line
            traffic = round(per_block * n)
            traffic_src = (f"{os.path.relpath(args.traffic_json, ROOT)}: {per_block:.0f} B/block "
                           f"(PMC, committed) x {n} blocks")

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:  # the CPU leg: rank 0 at N = 1 only
        # the first 256 GPU-compressed blocks of rank 0 = blocks 0..255 of the CPU leg's sample
        ns = min(256, uniq)
        cb = cbuf[: int(coff[ns - 1]) + int(cs_all[ns - 1])].cpu().numpy()
        gpu_comp = [cb[int(coff[j]): int(coff[j]) + int(cs_all[j])].tobytes() for j in range(ns)]
        cpu = cpu_baseline(kind, bs, args.cpu_seconds, gpu_comp=gpu_comp)

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
                         "traffic_source": traffic_src, "kernel_ms": round(kern_ms, 4),
                         "algorithmic_bytes_per_launch": csum + dsum},
            "cpu_baseline": cpu,
        }
        if crc_leg is not None:
            rec["crc"] = crc_leg
    comp = None
    legs = args.mode == "decompress" and args.block_size == 16384 and (args.blocks == 1 << 20 or args.legs_small)
    if not args.no_c3 and legs:
        # BASELINE config c3 (the "+compress" of the metric) in the same driver run: the c2 buffers
        # are released first; value/roofline/cpu_baseline of c3 go under "compress"
        del src, out, cbuf, ws, coff_t, src_off, src_len
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
        a3 = argparse.Namespace(**vars(args))
        a3.mode, a3.block_size, a3.steps, a3.warmup = "compress", 65536, args.c3_steps, 1
        a3.traffic_json = None
        comp = bench_compress(a3, rank, world, dev, "image", emit=False)
    replay_rec = None
    if not args.no_c4 and legs:
        # BASELINE config c4: .data replay (scan + CRC + decompress + vhash) of one corpus split over
        # the ranks on record boundaries, device-resident and end to end from pinned host memory
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
        sys.path.insert(0, os.path.join(ROOT, "tools"))
        import bench_replay as c4mod
        a4 = argparse.Namespace(chunk_mib=256 if args.legs_small else args.c4_chunk_mib,
                                files=4 if args.legs_small else args.c4_files, steps=2, seed=2026,
                                cpu_seconds=max(2.0, args.cpu_seconds / 2), no_cpu=args.no_cpu,
                                pin_records=64 if args.legs_small else 1024)
        replay_rec = c4mod.run(a4, rank, world, dev)
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
    enc_rec = None
    if not args.no_record and legs:
        # write-side record encode (TryCompress + encodeHeader + CRC + padding) of distinct
        # 16 KiB text values, device-resident
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
        enc_rec = bench_record_encode(args, rank, world, dev)
    mixed = None
    if not args.no_c5 and legs:
        # BASELINE config c5 in the same run: one 400 GiB corpus of distinct mixed 4-64 KiB values
        # split over the ranks (strong scaling), so the driver's 1/2/4/8-GPU runs also measure it
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
        sys.path.insert(0, os.path.join(ROOT, "tools"))
        import bench_c5 as c5mod
        tg, rg = (1.0, 0.25) if args.legs_small else (400.0, 16.0)
        mixed = c5mod.run(argparse.Namespace(total_gib=tg, round_gib=rg, warmup=1, gen_chunk=1 << 15),
                             rank, world, dev)
    if rank == 0:
        if comp is not None:
            rec["compress"] = {k: comp[k] for k in ("value", "unit", "steps", "warmup", "ms_per_step", "config",
                                                    "roofline", "cpu_baseline")}
        if replay_rec is not None:
            rec["replay"] = replay_rec
        if enc_rec is not None:
            rec["record_encode"] = enc_rec
        if mixed is not None:
            rec["mixed"] = {k: mixed[k] for k in ("metric", "value", "unit", "scaling", "rounds_per_gpu", "wall_s",
                                                  "incl_h2d", "digest", "config", "roofline")}
            if world == 1 and not args.no_cpu:  # CPU leg at N = 1 only, like the other legs
                rec["mixed"]["cpu_baseline"] = cpu_baseline_mixed(max(2.0, args.cpu_seconds / 2))
        print(json.dumps(rec), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


SEED = 0x5EED2026


def bench_record_encode(args, rank, world, dev):
    """SURVEY f3 (store/item.go:114-161, store/datafile.go:66-88,307-330): record.encode of this
    rank's distinct 16 KiB text values with keys "key_%016x" -- the TryCompress trial (10 KiB) and
    full compress, the record CRC and the 256-B padded layout, all batched on the device.  Checked:
    the records replay (qlzx_replay_index + decompress) to the original values (an XOR of value
    CRCs).  Returns the leg's record on rank 0 (max-over-ranks time, summed bytes)."""
    from gobeansdb_amd import batch, record, replay, shard
    n = max(1, (args.record_values >> 4) if args.legs_small else args.record_values)
    bs = 16384
    first = rank * n
    vals = batch.synth("text", SEED + 3, [bs] * n, first_id=first, device=dev)
    keys = [b"key_%016x" % (first + i) for i in range(n)]
    ws = batch.Workspace(dev)
    enc = record.encode(keys, vals, workspace=ws)
    torch.cuda.synchronize()
    rr = replay.replay(enc.data, workspace=ws)
    torch.cuda.synchronize()
    assert rr.n == n and not rr.end_error and int(rr.size_broken.abs().sum()) == 0, (rr.n, n)
    assert int(((rr.flag & 0x10000) != 0).sum()) == 0, "a stored value failed to decode"
    want = shard.xor_of(batch.crc32(vals))
    got = shard.xor_of(rr.value_crcs())
    assert got == want, "record encode round trip: value digest differs"
    rec_bytes = int(enc.data.numel())
    ncomp = int((enc.flag & 0x10000 != 0).sum())
    del rr, enc
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    steps = max(1, min(args.steps, 3))
    t = time.perf_counter()
    for _ in range(steps):
        record.encode(keys, vals, workspace=ws)
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    sec = shard.max_over_ranks([(time.perf_counter() - t) / steps], device=dev)[0]
    tot = shard.sum_over_ranks({"values": n, "in": n * bs, "out": rec_bytes, "comp": ncomp}, device=dev)
    if rank != 0:
        return None
    alg = tot["in"] + tot["out"]
    return {"value": round(tot["in"] / sec / 2**30, 2), "unit": "GiB/s of values in",
            "records_per_s": round(tot["values"] / sec), "ms_per_call": round(sec * 1e3, 2), "steps": steps,
            "config": {"workload": f"f3: record.encode of {n} distinct {bs} B text values per GPU (keys key_%016x), "
                                   f"device-resident; {tot['comp']} stored compressed", "values_per_gpu": n},
            "digest_check": "the records replay to the original values (XOR of value crc32 equal)",
            "roofline": {"bound": "hbm", "achieved": round(alg / sec / 1e9, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(alg / sec / 1e9 / HBM_PEAK_GBS, 4), "traffic": None,
                         "what": "algorithmic bytes: every value byte read once + every record byte written once; "
                                 "the call also compresses a 10 KiB trial and the whole body (TryCompress) and "
                                 "syncs the host between its steps (sizes, flags)"}}


def bench_standin(args, rank, world):
    """Launcher test only (tests/test_bench_launcher.py): the contract's rank / barrier /
    max-over-ranks plumbing on gloo with a CPU stand-in step (a 4 MiB host copy).  It measures
    nothing about the codec and says so in its line."""
    import torch.distributed as dist
    from gobeansdb_amd import shard
    if world > 1:
        dist.init_process_group("gloo")
    a = np.random.default_rng(rank).integers(0, 256, 4 << 20, dtype=np.uint8)
    b = np.empty_like(a)
    for _ in range(args.warmup):
        b[:] = a
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        b[:] = a
    if world > 1:
        dist.barrier()
    wall = shard.max_over_ranks([time.perf_counter() - t0])[0]
    tot = shard.sum_over_ranks({"bytes": a.nbytes * args.steps})
    if rank == 0:
        print(json.dumps({"metric": "launcher stand-in (not a measurement)", "value": round(tot["bytes"] / wall / 2**30, 3),
                          "unit": "GiB/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                          "ms_per_step": round(wall * 1e3 / max(args.steps, 1), 4), "higher_is_better": True,
                          "scaling": "weak", "vs_baseline": None, "dtype": "u8",
                          "data": "cpu stand-in: 4 MiB host copy per rank per step",
                          "config": {"workload": "launcher test", "parallelism": f"shard{world}"}}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def bench_c5(args):
    """Config c5 (BASELINE configs[4]): tools/bench_c5.py under the same ranks."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import bench_c5
    sys.argv = [sys.argv[0], "--warmup", str(max(args.warmup, 1))]
    return bench_c5.main()


def bench_compress(args, rank, world, dev, kind, emit: bool = True):
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
    traffic_src = None
    tj = args.traffic_json or os.path.join(ROOT, "profiles", "r05_c3_traffic.json")
    if os.path.exists(tj) and kind == "image" and bs == 65536:
        tpb = json.load(open(tj)).get("hbm_bytes_per_block")
        if tpb is not None:
            traffic = round(tpb * n)
            traffic_src = f"{os.path.relpath(tj, ROOT)}: {tpb:.0f} B/block (PMC, committed) x {n} blocks"
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:  # the CPU leg: rank 0 at N = 1 only
        ns = min(256, n)
        dh = dst.data[: int(dst.off[ns - 1]) + bs + 400].cpu().numpy()
        doff = dst.off[:ns].cpu().numpy()
        csh = cs[:ns].cpu().numpy()
        gpu_comp = [dh[int(doff[j]): int(doff[j]) + int(csh[j])].tobytes() for j in range(ns)]
        gpu_crc = crc[:ns].cpu().numpy().view(np.uint32).tolist()
        cpu = cpu_baseline(kind, bs, args.cpu_seconds, mode="compress", gpu_comp=gpu_comp, gpu_crc=gpu_crc)
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
                         "traffic_source": traffic_src, "kernel_ms": round(kern_ms, 4),
                         "algorithmic_bytes_per_launch": n * bs + csum},
            "cpu_baseline": cpu,
        }
        if emit:
            print(json.dumps(rec), flush=True)
    if world > 1 and emit:
        torch.distributed.destroy_process_group()
    return rec if rank == 0 else None


REF_WHAT = ("reference quicklz/quicklz.c {fn} (oracle/_ref/libqlzref.so, gcc -O2 as cgo builds it)")


def host_cpus() -> tuple[int, int, str]:
    """(usable threads, nproc, CPU model).  Usable = the CPUs in this process's affinity mask,
    capped by the cgroup CPU quota (cpu.max) when one is set: on the GPU box the affinity
    mask shows the whole machine while the quota grants one GPU's share."""
    try:
        usable = len(os.sched_getaffinity(0))
    except AttributeError:
        usable = os.cpu_count() or 1
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            usable = max(1, min(usable, int(q) // int(per)))
    except (OSError, ValueError):
        pass
    model = "unknown"
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                model = ln.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return usable, os.cpu_count() or usable, model


def cpu_baseline(kind: str, bs: int, seconds: float, mode: str = "decompress", gpu_comp=None, gpu_crc=None):
    """The reference codec (oracle/_ref) -- else the C restatement -- on the host cores over a
    bounded sample of the same workload: every usable core (the process's affinity mask;
    nproc reported beside it), one core, and the cgo-faithful form that allocates the
    output and scratch per call as quicklz/cquicklz.go:24-49 does.

    gpu_comp: the GPU encoder's bytes for blocks 0.. of the same generator; each must equal
    the CPU codec's output for that block (sampled bit-exactness of the
    compressed bytes), else the bench fails.  gpu_crc: the fused CRC32 of those blocks (c3),
    checked against zlib.crc32 of the CPU codec's bytes (= store/crc32.go)."""
    from oracle import oracle as O
    threads, nproc, model = host_cpus()
    L = O.lib()
    Q = O.ref_if_built()  # the reference quicklz.c (oracle/_ref) when built; else the C restatement
    kind_ = "reference" if Q is not None else "port"
    comp_mode = mode == "compress"
    nblk = max(2048 if not comp_mode else 256, threads * (32 if not comp_mode else 4))
    nblk = min(nblk, 8192 if not comp_mode else 2048)
    gen = O.gen_text if kind == "text" else O.gen_image
    plain = [gen(SEED, i, bs) for i in range(nblk)]
    if comp_mode:
        src_list, out_len = plain, bs + 400
    else:
        src_list, out_len = [O.compress(p_) for p_ in plain], bs
    off_s, tot_s = _pack(src_list)
    off_d, tot_d = _pack([b"\0" * out_len] * nblk)
    srcb = np.zeros(tot_s, np.uint8)
    for o, c in zip(off_s, src_list):
        srcb[int(o): int(o) + len(c)] = np.frombuffer(c, np.uint8)
    lens = np.asarray([len(c) for c in src_list], np.uint32)
    dst = np.zeros(tot_d, np.uint8)
    fn = ctypes.cast(Q.qlz_compress if comp_mode else Q.qlz_decompress, ctypes.c_void_p).value if Q else None

    def run(nthr, secs, cgo):
        reps, ns = 0, 0.0
        t_end = time.time() + secs
        while time.time() < t_end or reps == 0:
            m = (1 if comp_mode else 0) | (2 if cgo else 0)
            if Q is not None:
                ns += L.orc_bench_ref(fn, srcb.ctypes.data, off_s.ctypes.data, lens.ctypes.data,
                                      dst.ctypes.data, off_d.ctypes.data, nblk, nthr, m)
            elif comp_mode:
                ns += L.orc_bench_compress(srcb.ctypes.data, off_s.ctypes.data, lens.ctypes.data,
                                           dst.ctypes.data, off_d.ctypes.data, nblk, nthr, int(cgo))
            else:
                ns += L.orc_bench_decompress(srcb.ctypes.data, off_s.ctypes.data, lens.ctypes.data,
                                             dst.ctypes.data, off_d.ctypes.data, nblk, nthr, int(cgo))
            reps += 1
        return reps * nblk * bs / (ns * 1e-9) / 2**30, reps

    parity = None
    if gpu_comp:
        for j, g in enumerate(gpu_comp):
            want = O.compress(plain[j]) if j < len(plain) else O.compress(gen(SEED, j, bs))
            if g != want:
                raise SystemExit(f"GPU-compressed block {j} differs from the CPU codec's bytes")
        parity = f"{len(gpu_comp)} GPU-compressed blocks == oracle/qlz_oracle.c bytes (pinned to quicklz.c)"
        if gpu_crc is not None:
            import zlib
            for j, c in enumerate(gpu_crc):
                if int(c) != zlib.crc32(gpu_comp[j]):
                    raise SystemExit(f"fused CRC of block {j} != zlib.crc32 of its bytes")
            parity += f"; their fused CRC32 == zlib.crc32 (store/crc32.go)"
    gibs, reps = run(threads, seconds, False)
    if not comp_mode and Q is not None and not all(
            dst[int(o): int(o) + bs].tobytes() == p_ for o, p_ in zip(off_d[:8], plain[:8])):
        raise RuntimeError("reference decompress baseline produced wrong bytes")
    one, _ = run(1, max(2.0, seconds / 5), False)
    cgo, _ = run(threads, max(2.0, seconds / 3), True)
    fn_name = "qlz_compress" if comp_mode else "qlz_decompress"
    what = REF_WHAT.format(fn=fn_name) if Q is not None else f"oracle/qlz_oracle.c orc_{mode}"
    unit_what = "input" if comp_mode else "output"
    return {"value": round(gibs, 3), "unit": "GiB/s", "cores": threads, "kind": kind_,
            "sample": f"{reps} passes over {nblk} x {bs} B {kind} blocks, {what}, {threads} threads "
                      f"(one scratch per thread), GiB/s of {unit_what}" + ("" if comp_mode else "; no CRC"),
            "threads": threads, "nproc": nproc, "cpu_model": model,
            "one_core": round(one, 3),
            "cgo_faithful": round(cgo, 3),
            "cgo_faithful_what": "per call: output + scratch malloc/free as quicklz/cquicklz.go:24-49",
            "compress_parity": parity}


def cpu_baseline_mixed(seconds: float):
    """c5's CPU leg: the reference qlz_decompress (oracle/_ref; else the C restatement) on the
    host cores over a bounded sample of the same value mix (log-uniform 4-64 KiB, 70 % text /
    30 % image-like, as tools/bench_c5.py draws them), GiB/s of output."""
    from oracle import oracle as O
    threads, nproc, model = host_cpus()
    L = O.lib()
    Q = O.ref_if_built()
    rng = np.random.default_rng(SEED)
    nblk = 2048
    sizes = [int(np.exp(rng.uniform(np.log(4096), np.log(65536)))) for _ in range(nblk)]
    is_text = rng.random(nblk) < 0.7
    plain = [(O.gen_text if t else O.gen_image)(SEED, i, n) for i, (t, n) in enumerate(zip(is_text, sizes))]
    comp = [O.compress(p_) for p_ in plain]
    off_s, tot_s = _pack(comp)
    off_d, tot_d = _pack(plain)
    srcb = np.zeros(tot_s, np.uint8)
    for o, c in zip(off_s, comp):
        srcb[int(o): int(o) + len(c)] = np.frombuffer(c, np.uint8)
    lens = np.asarray([len(c) for c in comp], np.uint32)
    dst = np.zeros(tot_d, np.uint8)
    out_bytes = sum(sizes)
    fn = ctypes.cast(Q.qlz_decompress, ctypes.c_void_p).value if Q else None

    def run(nthr, secs):
        reps, ns = 0, 0.0
        t_end = time.time() + secs
        while time.time() < t_end or reps == 0:
            if Q is not None:
                ns += L.orc_bench_ref(fn, srcb.ctypes.data, off_s.ctypes.data, lens.ctypes.data,
                                      dst.ctypes.data, off_d.ctypes.data, nblk, nthr, 0)
            else:
                ns += L.orc_bench_decompress(srcb.ctypes.data, off_s.ctypes.data, lens.ctypes.data,
                                             dst.ctypes.data, off_d.ctypes.data, nblk, nthr, 0)
            reps += 1
        return reps * out_bytes / (ns * 1e-9) / 2**30, reps

    gibs, reps = run(threads, seconds)
    if not all(dst[int(o): int(o) + len(p_)].tobytes() == p_ for o, p_ in zip(off_d[:16], plain[:16])):
        raise RuntimeError("mixed decompress baseline produced wrong bytes")
    one, _ = run(1, max(2.0, seconds / 5))
    what = REF_WHAT.format(fn="qlz_decompress") if Q is not None else "oracle/qlz_oracle.c orc_decompress"
    return {"value": round(gibs, 3), "unit": "GiB/s", "cores": threads, "kind": "reference" if Q else "port",
            "sample": f"{reps} passes over {nblk} log-uniform 4-64 KiB values (70 % text / 30 % image-like, "
                      f"{out_bytes / 2**20:.1f} MiB out), {what}, {threads} threads, GiB/s of output; no CRC",
            "threads": threads, "nproc": nproc, "cpu_model": model, "one_core": round(one, 3)}


def _pack(blocks):
    ln = np.asarray([len(b) for b in blocks], np.int64)
    sz = (ln + 255) // 256 * 256
    off = np.zeros(len(ln), np.uint64)
    off[1:] = np.cumsum(sz)[:-1]
    return off, int(sz.sum())


if __name__ == "__main__":
    main()
