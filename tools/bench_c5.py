#!/usr/bin/env python3
"""Config c5: 400 GiB of mixed 4-64 KiB values decompressed across N GPUs (strong scaling).

BASELINE.json configs[4] / SURVEY §8(d) c5.  The job is ONE corpus of distinct values: block i
(i = 0 .. ~19 M) has a log-uniform 4-64 KiB size and a kind (70 % text-like / 30 % image-like,
DESIGN.md §5) drawn from one seed, and its bytes are gen(kind, seed, i) -- the same on every
rank and at every N.  The corpus is split over the ranks by bytes (shard.partition_by_bytes);
each rank streams its share through HBM in rounds of at most --round-gib GiB of output:

  per round (untimed)  generate the round's values on the device, compress them with this
                       library's encoder, pack the streams densely and copy them to pinned host
                       memory; decode once and check every block's CRC32 against the plain
                       block's (the XOR of the output CRCs is the corpus digest)
  device-only (timed)  decode the round from the packed streams resident in HBM
  incl. H2D (timed)    H2D of the round's packed streams from pinned host memory, then the decode

So every round decodes distinct data (no value is decoded twice), and the rates are the corpus
output over the summed per-round times (HIP events), max over ranks.  One process per GPU under
torch.distributed.run; no data-path collective (max / sum / all-gather of the results only).

Prints one JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

HBM_PEAK_GBS = 8000.0
SEED = 0xC5C5_2026


def log(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print("[c5]", *a, file=sys.stderr, flush=True)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--total-gib", type=float, default=400.0, help="decompressed GiB for the whole job")
    p.add_argument("--round-gib", type=float, default=16.0, help="distinct decompressed GiB per round per rank")
    p.add_argument("--warmup", type=int, default=1, help="unused: each round's verifying decode warms the path")
    p.add_argument("--gen-chunk", type=int, default=1 << 15)
    args = p.parse_args()

    from gobeansdb_amd import shard

    rank, world, local = shard.env_rank()
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=dev)
    rec = run(args, rank, world, dev)
    if rank == 0:
        print(json.dumps(rec), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


def c5_traffic(round_out_bytes: int) -> dict:
    """PMC HBM bytes of one round (one batch decompress of the resident set): the committed
    per-output-byte figure (tools/traffic_call.py over a rocprofv3 FETCH_SIZE / WRITE_SIZE run)
    x this round's decompressed bytes; null when the profile is absent."""
    path = os.path.join(ROOT, "profiles", "r06_c5_traffic.json")
    if not os.path.exists(path):
        return {"traffic": None}
    tj = json.load(open(path))
    return {"traffic": round(tj["hbm_bytes_per_call_byte"] * round_out_bytes),
            "traffic_source": f"profiles/r06_c5_traffic.json: {tj['hbm_bytes_per_call_byte']:.3f} HBM B per output "
                              f"byte (PMC, one round of {tj['call_bytes'] / 2**30:.1f} GiB out) x bytes per round"}


def corpus(total_gib: float) -> tuple[np.ndarray, np.ndarray]:
    """(sizes, is_text) of the whole job's blocks, from SEED alone: log-uniform 4-64 KiB sizes
    until total_gib of output, 70 % text-like."""
    rng = np.random.default_rng(SEED)
    target = int(total_gib * 2**30)
    mean = (65536 - 4096) / math.log(16)
    sizes = np.zeros(0, np.int64)
    while int(sizes.sum()) < target:
        more = int((target - int(sizes.sum())) / mean * 1.05) + 64
        sizes = np.concatenate([sizes, np.exp(rng.uniform(np.log(4096), np.log(65536), more)).astype(np.int64)])
    n = int(np.searchsorted(np.cumsum(sizes), target, side="left")) + 1
    sizes = sizes[:n]
    is_text = np.random.default_rng([SEED, 1]).random(n) < 0.7
    return sizes, is_text


def plan_rounds(sizes: np.ndarray, lo: int, hi: int, round_gib: float) -> list[tuple[int, int]]:
    """Blocks [lo, hi) in ceil(bytes / round_gib) consecutive rounds of near-equal output bytes
    (each within one block of round_gib)."""
    from gobeansdb_amd import shard
    share = int(sizes[lo:hi].sum())
    k = max(1, math.ceil(share / (round_gib * 2**30)))
    return [(lo + a, lo + b) for a, b in shard.partition_by_bytes(sizes[lo:hi], k) if b > a]


def run(args, rank, world, dev):
    """The c5 job on this rank (process group, if any, already initialised); returns the
    record on rank 0, None elsewhere.  args: total_gib, round_gib, warmup, gen_chunk."""
    from gobeansdb_amd import _lib, batch, shard

    log(f"{world} rank(s); lib: {_lib.info()}")
    t_job = time.time()
    sizes, is_text = corpus(args.total_gib)
    lo, hi = shard.partition_by_bytes(sizes, world)[rank]
    rounds = plan_rounds(sizes, lo, hi, args.round_gib)
    log(f"corpus: {len(sizes)} blocks, {sizes.sum() / 2**30:.1f} GiB; rank {rank}: blocks [{lo}, {hi}) "
        f"in {len(rounds)} rounds")

    # buffers for the largest round: plain (text and image copies), staging, packed streams, output
    rmax = max([int(sizes[a:b].sum()) for a, b in rounds], default=0)
    nmax = max([b - a for a, b in rounds], default=0)
    plain_b = rmax + 256 * nmax
    ab = torch.empty(2 * plain_b + 256, dtype=torch.uint8, device=dev)
    staging = torch.empty(rmax + (400 + 256) * nmax + 256, dtype=torch.uint8, device=dev)
    packed = torch.empty(rmax + (400 + 256) * nmax + 256, dtype=torch.uint8, device=dev)
    outbuf = torch.empty(plain_b + 256, dtype=torch.uint8, device=dev)
    hpin = None   # pinned host copy of a round's packed streams, sized at the first round
    ws = batch.Workspace(dev)
    stream = torch.cuda.current_stream(dev)
    L = _lib.lib()

    digest, out_b, in_b, nblk = 0, 0, 0, 0
    t_dev, t_h2d, t_gen = 0.0, 0.0, 0.0
    for ri, (a, b) in enumerate(rounds):
        tg = time.time()
        n = b - a
        ln = sizes[a:b]
        off, tot = batch.pack_offsets(ln)
        off_t = torch.from_numpy(off.view(np.int64)).to(dev)
        len_t = torch.from_numpy(ln.astype(np.uint32).view(np.int32)).to(dev)
        # block a + k = gen(kind, SEED, a + k): both kinds generated, each block reads its own
        batch.synth("text", SEED, ln.tolist(), first_id=a, device=dev, out=batch.BlockBatch(ab, off_t, len_t))
        batch.synth("image", SEED, ln.tolist(), first_id=a, device=dev,
                    out=batch.BlockBatch(ab, off_t + plain_b, len_t))
        txt = torch.from_numpy(is_text[a:b]).to(dev)
        plain = batch.BlockBatch(ab, torch.where(txt, off_t, off_t + plain_b), len_t)
        soff, _ = batch.pack_offsets(ln, pad=400)   # CCompress allocates len + 400
        soff_t = torch.from_numpy(soff.view(np.int64)).to(dev)
        cs = torch.empty(n, dtype=torch.int32, device=dev)
        for c0 in range(0, n, args.gen_chunk):
            c1 = min(n, c0 + args.gen_chunk)
            sub = batch.BlockBatch(ab, plain.off[c0:c1], len_t[c0:c1])
            _, csc, st, _ = batch.compress(sub, batch.BlockBatch(staging, soff_t[c0:c1], len_t[c0:c1]),
                                           max_len=65536, workspace=ws)
            if int((st != 0).sum().item()):
                raise SystemExit("compress failed on the GPU")
            cs[c0:c1] = csc
        cs_h = cs.cpu().numpy().view(np.uint32)
        coff, ctot = batch.pack_offsets(cs_h)
        coff_t = torch.from_numpy(coff.view(np.int64)).to(dev)
        _lib.check(L.qlzx_copy_batch(staging.data_ptr(), soff_t.data_ptr(), cs.data_ptr(), packed.data_ptr(),
                                     coff_t.data_ptr(), n, batch._stream(stream)), "qlzx_copy_batch")
        src = batch.BlockBatch(packed, coff_t, cs)
        out = batch.BlockBatch(outbuf, off_t, len_t)
        _, st, _ = batch.decompress(src, out, max_dsize=65536, workspace=ws, stream=stream)
        got = batch.crc32(out)
        if int((st != 0).sum().item()) or not torch.equal(got, batch.crc32(plain)):
            raise SystemExit(f"round {ri}: round trip mismatch (blocks {a}..{b})")
        digest ^= shard.xor_of(got)
        if hpin is None or hpin.numel() < ctot:
            hpin = torch.empty(int(ctot * 1.1) + 4096, dtype=torch.uint8).pin_memory()
        hpin[:ctot].copy_(packed[:ctot])   # the host copy the H2D leg streams from
        torch.cuda.synchronize()
        t_gen += time.time() - tg
        # device-only: the packed streams resident in HBM
        e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
        e0.record(stream)
        batch.decompress(src, out, max_dsize=65536, workspace=ws, stream=stream)
        e1.record(stream)
        # incl. H2D: the streams come from pinned host memory first
        packed[:ctot].copy_(hpin[:ctot], non_blocking=True)
        batch.decompress(src, out, max_dsize=65536, workspace=ws, stream=stream)
        e2.record(stream)
        torch.cuda.synchronize()
        t_dev += e0.elapsed_time(e1) * 1e-3
        t_h2d += e1.elapsed_time(e2) * 1e-3
        out_b += int(ln.sum())
        in_b += int(cs_h.astype(np.int64).sum())
        nblk += n
        if ri == 0 or ri + 1 == len(rounds):
            log(f"rank {rank}: round {ri + 1}/{len(rounds)}: {n} blocks, {int(ln.sum()) / 2**30:.2f} GiB, "
                f"ratio {int(cs_h.astype(np.int64).sum()) / int(ln.sum()):.3f}, decode {e0.elapsed_time(e1):.2f} ms, "
                f"H2D + decode {e1.elapsed_time(e2):.2f} ms")
    if world > 1:
        torch.distributed.barrier()
    t_dev, t_h2d, t_gen = shard.max_over_ranks([t_dev, t_h2d, t_gen], device=dev)
    tot = shard.sum_over_ranks({"out": out_b, "in": in_b, "blocks": nblk, "rounds": len(rounds)}, device=dev)
    digest = shard.xor_digest_over_ranks(digest, device=dev)
    wall_job = shard.max_over_ranks([time.time() - t_job], device=dev)[0]
    if rank == 0:
        achieved = (tot["in"] + tot["out"]) / world / t_dev / 1e9   # per GPU, algorithmic bytes
        rmean = tot["out"] / max(tot["rounds"], 1)
        rec = {
            "metric": "GiB/s device-resident QuickLZ decompress, 400 GiB mixed 4-64 KiB values (c5)",
            "value": round(tot["out"] / t_dev / 2**30, 3),
            "unit": "GiB/s",
            "n_gpus": world,
            "rounds_per_gpu": math.ceil(tot["rounds"] / world),
            "wall_s": round(t_dev, 4),
            "higher_is_better": True,
            "scaling": "strong",
            "dtype": "u8",
            "data": "synthetic",
            "incl_h2d": {"value": round(tot["out"] / t_h2d / 2**30, 3), "unit": "GiB/s", "seconds": round(t_h2d, 4),
                         "what": "per round: H2D of the round's packed streams from pinned host memory, then the "
                                 "decode (one stream, not overlapped)"},
            "digest": {"blocks": tot["blocks"], "xor_output_crc32": f"{digest:08x}",
                       "what": "XOR over every block of the corpus of crc32 of its decoded bytes, per-rank XORs "
                               "all-gathered: equal at every N"},
            "config": {"workload": f"c5: one corpus of {tot['blocks']} distinct log-uniform 4-64 KiB values "
                                   f"({tot['out'] / 2**30:.0f} GiB, 70 % text / 30 % image-like) split over "
                                   f"{world} rank(s) by bytes; each rank streams its share through HBM in rounds of "
                                   f"<= {args.round_gib:g} GiB of distinct values (generated and compressed on the "
                                   "device, untimed); value = output / summed per-round decode time, max over ranks",
                       "rounds": tot["rounds"], "round_out_bytes_mean": round(rmean),
                       "ratio": round(tot["in"] / tot["out"], 3), "parallelism": f"shard{world}",
                       "job_wall_s": round(wall_job, 1), "generate_s": round(t_gen, 1)},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), **c5_traffic(round(rmean))},
        }
        return rec
    return None


if __name__ == "__main__":
    main()
