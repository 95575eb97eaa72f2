#!/usr/bin/env python3
"""Config c5: 400 GiB of mixed 4-64 KiB values decompressed across N GPUs (strong scaling).

BASELINE.json configs[4] / SURVEY §8(d) c5.  The job is a fixed total of decompressed
output (--total-gib, 400 by default) split evenly over the ranks.  400 GiB does not fit
one GPU, so each rank keeps ONE device-resident round of --round-gib GiB of output
(compressed inputs + output buffer in HBM, share / rounds bytes with rounds = ceil(share /
round-gib)) and decompresses it `rounds` times, so the job totals --total-gib at every N.
Every round replays the same resident blocks: refilling a round from host memory is the
PCIe leg that config c4 (tools/bench_replay.py) measures, not part of this number.

Values: log-uniform 4-64 KiB sizes, 70 % text-like / 30 % image-like,
generated and compressed on the GPU by this library; every block's round trip is
checked on device before timing.  One process per GPU under torch.distributed.run;
no data-path collective (barrier + max-over-ranks timing, RCCL sums of the counters).

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
    p.add_argument("--round-gib", type=float, default=16.0, help="resident decompressed GiB per rank")
    p.add_argument("--warmup", type=int, default=1, help="untimed rounds")
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
    path = os.path.join(ROOT, "profiles", "r04_c5_traffic.json")
    if not os.path.exists(path):
        return {"traffic": None}
    tj = json.load(open(path))
    return {"traffic": round(tj["hbm_bytes_per_call_byte"] * round_out_bytes),
            "traffic_source": f"profiles/r04_c5_traffic.json: {tj['hbm_bytes_per_call_byte']:.3f} HBM B per output "
                              f"byte (PMC, one round of {tj['call_bytes'] / 2**30:.1f} GiB out) x bytes per round"}


def plan_rounds(total_gib: float, round_gib: float, world: int) -> tuple[int, int]:
    """(rounds, resident bytes per rank): the rank's share of the job in whole rounds of at most
    round_gib, so rounds x resident x world = total_gib at every N (to a block)."""
    share = total_gib * 2**30 / world
    rounds = max(1, math.ceil(share / (round_gib * 2**30)))
    return rounds, int(share / rounds)


def run(args, rank, world, dev):
    """The c5 job on this rank (process group, if any, already initialised); returns the
    record on rank 0, None elsewhere.  args: total_gib, round_gib, warmup, gen_chunk."""
    from gobeansdb_amd import _lib, batch, shard

    log(f"{world} rank(s); lib: {_lib.info()}")

    # ---- this rank's resident round: mixed sizes and kinds, seeded per rank ----
    rng = np.random.default_rng([SEED, rank])
    rounds, target = plan_rounds(args.total_gib, args.round_gib, world)
    sizes = []
    tot = 0
    while tot < target:
        n = int(np.exp(rng.uniform(np.log(4096), np.log(65536))))
        sizes.append(n)
        tot += n
    sizes = np.asarray(sizes, np.int64)
    nblk = len(sizes)
    is_text = rng.random(nblk) < 0.7
    t0 = time.time()
    coff, ctotal = batch.pack_offsets(sizes.tolist(), pad=400)   # CCompress allocates len+400
    cbuf = torch.empty(ctotal, dtype=torch.uint8, device=dev)
    coff_t = torch.from_numpy(coff.view(np.int64)).to(dev)
    cs_all = np.zeros(nblk, np.int64)
    ws = batch.Workspace(dev)
    first = rank * (1 << 32)   # disjoint block ids per rank
    for kind, mask in (("text", is_text), ("image", ~is_text)):
        idx = np.nonzero(mask)[0]
        for c0 in range(0, len(idx), args.gen_chunk):
            sel = idx[c0:c0 + args.gen_chunk]
            plain = batch.synth(kind, SEED, sizes[sel].tolist(), first_id=first + int(sel[0]), device=dev)
            dst = batch.BlockBatch(cbuf, coff_t[torch.from_numpy(sel).to(dev)], plain.length)
            _, cs, st, _ = batch.compress(plain, dst, max_len=65536, workspace=ws)
            if int((st != 0).sum().item()):
                raise SystemExit("compress failed on the GPU")
            cs_all[sel] = cs.cpu().numpy().astype(np.int64)
            del plain
    torch.cuda.synchronize()
    src = batch.BlockBatch(cbuf, coff_t, torch.from_numpy(cs_all.astype(np.int32)).to(dev))
    out = batch.BlockBatch.empty_for(sizes.tolist(), device=dev)
    csum, dsum = int(cs_all.sum()), int(sizes.sum())
    log(f"rank {rank}: {nblk} blocks, {dsum / 2**30:.2f} GiB out, ratio {csum / dsum:.3f}, "
        f"generated+compressed in {time.time() - t0:.1f}s")

    # ---- device round trip of every block ----
    _, st, _ = batch.decompress(src, out, max_dsize=65536, workspace=ws)
    torch.cuda.synchronize()
    if int((st != 0).sum().item()):
        raise SystemExit("decompress status")
    # per-block CRC32 of the decompressed block == CRC32 of the regenerated plain block
    for kind, mask in (("text", is_text), ("image", ~is_text)):
        idx = np.nonzero(mask)[0]
        for c0 in range(0, len(idx), args.gen_chunk):
            sel = idx[c0:c0 + args.gen_chunk]
            sel_t = torch.from_numpy(sel).to(dev)
            check = batch.synth(kind, SEED, sizes[sel].tolist(), first_id=first + int(sel[0]), device=dev)
            got = batch.crc32(batch.BlockBatch(out.data, out.off[sel_t], out.length[sel_t]))
            if not torch.equal(got, batch.crc32(check)):
                raise SystemExit(f"round trip mismatch ({kind}, blocks from {sel[0]})")
            del check
    log("device round trip verified (per-block CRC32)")

    # ---- timed: this rank's share of the job, in rounds over the resident set ----
    stream = torch.cuda.current_stream()

    def one_round():
        batch.decompress(src, out, max_dsize=65536, workspace=ws, stream=stream)

    for _ in range(args.warmup):
        one_round()
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t_start = time.perf_counter()
    e0.record(stream)
    for _ in range(rounds):
        one_round()
    e1.record(stream)
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t_start
    kern_s = e0.elapsed_time(e1) * 1e-3
    wall, kern_s = shard.max_over_ranks([wall, kern_s], device=dev)
    tot = shard.sum_over_ranks({"out": dsum * rounds, "in": csum * rounds}, device=dev)
    if rank == 0:
        achieved = (tot["in"] + tot["out"]) / world / kern_s / 1e9   # per GPU, algorithmic bytes
        rec = {
            "metric": "GiB/s device-resident QuickLZ decompress, 400 GiB mixed 4-64 KiB values (c5)",
            "value": round(tot["out"] / wall / 2**30, 3),
            "unit": "GiB/s",
            "n_gpus": world,
            "rounds_per_gpu": rounds,
            "wall_s": round(wall, 4),
            "higher_is_better": True,
            "scaling": "strong",
            "dtype": "u8",
            "data": "synthetic",
            "config": {"workload": f"c5: {tot['out'] / 2**30:.0f} GiB of log-uniform 4-64 KiB values "
                                   f"(70 % text / 30 % image-like), {world} rank(s), {rounds} rounds of a "
                                   f"resident {dsum / 2**30:.1f} GiB set per rank",
                       "blocks_per_round": nblk, "round_out_bytes": dsum, "ratio": round(csum / dsum, 3),
                       "parallelism": f"shard{world}"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), **c5_traffic(dsum)},
        }
        return rec
    return None


if __name__ == "__main__":
    main()
