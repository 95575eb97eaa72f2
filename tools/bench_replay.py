#!/usr/bin/env python3
"""Config c4: replay a synthetic .data corpus on one GPU, device-only and end-to-end.

A chunk file (store/datafile.go layout: 24-B header, key, value, 256-B padding)
of --chunk-mib MiB is built from synthetic values (log-uniform 4-64 KiB,
70 % text / 30 % image-like).  Values pass the TryCompress policy of store/item.go:120-161:
the MIME sniff of the first 512 B (gobeansdb_amd.record.need_compress), a trial compress
of the first 10 KiB kept when float32(clen)/float32(tlen) <= 0.7, then the whole body.
Keys are "key_%016x".
Two such chunks are built from distinct seeds; the corpus is --files files alternating them
(13 x 4000 MiB ~ 50 GiB by default), split over the ranks on record boundaries:

  device-only   the chunks are resident in HBM; one step = every rank replays its share
                (qlzx_replay_index + decompress of FLAG_COMPRESS values + Getvhash,
                gobeansdb_amd.replay) once
  end-to-end    pipelined per piece: pinned H2D of the piece, the same replay, D2H of
                the decompressed values into pinned host memory, three streams

The CPU leg runs the reference record loop (crc32_write + qlz_decompress + Getvhash from
oracle/_ref) over the first chunk.  bench.py runs this as its "replay" leg (run()); run
alone it prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import struct
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from gobeansdb_amd.record import COMPRESS_RATIO_LIMIT, TRY_COMPRESS_SIZE, need_compress  # noqa: E402


def log(*a):
    print("[replay]", *a, file=sys.stderr, flush=True)


def build_chunk(mib: int, seed: int, dev):
    from gobeansdb_amd import batch
    rng = np.random.default_rng(seed)
    target = mib << 20
    sizes, total = [], 0
    while True:   # raw sizes for ~1.7x the target; records are cut at the target after compression
        n = int(np.exp(rng.uniform(np.log(4096), np.log(65536))))
        rs = (24 + 20 + n + 255) // 256 * 256
        if total + rs > 1.7 * target:
            break
        sizes.append(n)
        total += rs
    nrec = len(sizes)
    kinds = rng.random(nrec) < 0.7
    log(f"chunk: {nrec} records, raw values {sum(sizes) / 2**30:.2f} GiB")
    values = [None] * nrec
    flags = np.zeros(nrec, np.uint32)
    step = 8192
    t0 = time.time()
    for kind, mask in (("text", kinds), ("image", ~kinds)):
        idx = np.nonzero(mask)[0]
        for c0 in range(0, len(idx), step):
            ids = idx[c0:c0 + step]
            ln = [sizes[i] for i in ids]
            plain = batch.synth(kind, seed, ln, first_id=int(ids[0]) * 7919, device=dev)
            comp, cs, st, _ = batch.compress(plain, max_len=max(ln))
            tl = [min(n, TRY_COMPRESS_SIZE) for n in ln]   # store/item.go:133-140: the 10 KiB trial
            trial = batch.BlockBatch(plain.data, plain.off, torch.tensor(tl, dtype=torch.int32, device=dev))
            _, tcs, tst, _ = batch.compress(trial, max_len=max(tl))
            torch.cuda.synchronize()
            assert int((st != 0).sum()) == 0 and int((tst != 0).sum()) == 0
            ph = plain.to_bytes()
            ch = comp.to_bytes(cs)
            tcs_h = tcs.cpu().numpy()
            for j, i in enumerate(ids):
                # TryCompress (store/item.go:137-156): sniff, float32 trial ratio, whole body
                keep = need_compress(ph[j][:512]) and \
                    np.float32(tcs_h[j]) / np.float32(tl[j]) <= np.float32(COMPRESS_RATIO_LIMIT)
                if keep:
                    values[i], flags[i] = ch[j], 0x10000
                else:
                    values[i] = ph[j]
    log(f"values generated+compressed in {time.time() - t0:.1f}s, "
        f"{int((flags != 0).sum())} compressed")
    buf = np.zeros(target, np.uint8)
    off = 0
    crc_off, crc_len, rec_off = [], [], []
    for i in range(nrec):
        key = b"key_%016x" % (seed * 1000003 + i)
        v = values[i]
        hdr = struct.pack("<IIIiII", 0, 1700000000 + i, int(flags[i]), i % 7, len(key), len(v))
        rec = hdr + key + v
        if off + len(rec) > target:   # the chunk file is full (DataFileMax, store/config_default.go:39)
            nrec = i
            break
        buf[off: off + len(rec)] = np.frombuffer(rec, np.uint8)
        rec_off.append(off)
        crc_off.append(off + 4)
        crc_len.append(20 + len(key) + len(v))
        off += (len(rec) + 255) // 256 * 256
    buf = buf[:off]   # compressed values made the file shorter than the raw-size bound
    # record CRCs (store/datafile.go:66-76) on the GPU, patched into the headers
    from gobeansdb_amd import batch as B
    d = torch.from_numpy(buf).to(dev)
    crc = B.crc32(B.BlockBatch(d, torch.tensor(crc_off, dtype=torch.int64, device=dev),
                               torch.tensor(crc_len, dtype=torch.int32, device=dev)))
    c = crc.cpu().numpy().view(np.uint32)
    for o, v in zip(rec_off, c):
        buf[o: o + 4] = np.frombuffer(struct.pack("<I", int(v)), np.uint8)
    del d
    return buf, nrec, int(sum(len(v) for v in values[:nrec])), int(sum(sizes[:nrec])), np.asarray(rec_off, np.uint64)


def _value_digest(res, lo: int, f: int) -> int:
    """Device-only parity digest of one replayed piece: XOR over its records of crc32 of the value
    after Payload.Decompress, keyed by the record's place (file f, offset lo + offset) since the
    corpus repeats its two chunk files (a repeated record must not cancel itself out)."""
    from gobeansdb_amd import shard
    pos = res.offset.to(torch.int64) + lo
    key = (pos * 0x85EBCA77 + (f + 1) * 0x9E3779B1) & 0xFFFFFFFF
    return shard.xor_of((res.value_crcs().to(torch.int64) & 0xFFFFFFFF) ^ key)


def pin_sample(c, res, k: int) -> int:
    """Full-size parity: every record offset against the chunk's layout, and k sampled records
    (offset, flag after Payload.Decompress, value bytes, Getvhash) against the oracle's
    readRecordAt / CDecompressSafe / Getvhash restatements (oracle/replay.py, store/datafile.go:
    114-170, store/item.go:89-100,163-176) on the host copy of the same chunk."""
    from oracle import oracle as O
    from oracle import replay as R
    n = res.n
    assert np.array_equal(res.offset.cpu().numpy().view(np.uint64), c["rec_off"][:n].astype(np.uint64)), "offsets"
    host = c["host"]
    hb = memoryview(host)
    rng = np.random.default_rng(20260)
    picks = sorted(set(rng.integers(0, n, min(k, n)).tolist()))
    flag = res.flag.cpu().numpy().view(np.uint32)
    vlen = res.value_len.cpu().numpy()
    vh = res.vhash.cpu().numpy()
    in_out = res.in_out.cpu().numpy()
    voff = res.val_off.cpu().numpy().view(np.uint64)
    out = res.values.data
    for j in picks:
        off = int(c["rec_off"][j])
        ksz, vsz = struct.unpack_from("<II", host, off + 16)
        r = R.read_record_at(bytes(hb[off:off + 24 + ksz + vsz]), 0)
        assert r is not None, j
        eflag, ebody = r.flag, bytes(r.body)
        if eflag & R.FLAG_COMPRESS:
            st, dec = O.decompress(ebody)
            if st == O.OK:
                eflag, ebody = eflag - R.FLAG_COMPRESS, dec
        o, L = int(voff[j]), int(vlen[j])
        got = out[o:o + L].cpu().numpy().tobytes() if in_out[j] else bytes(hb[o:o + L])
        assert int(flag[j]) == eflag and got == ebody and int(vh[j]) == R.getvhash(ebody), f"record {j} differs"
    return len(picks)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--chunk-mib", type=int, default=4000)
    p.add_argument("--files", type=int, default=13)
    p.add_argument("--steps", type=int, default=4)
    p.add_argument("--seed", type=int, default=2026)
    p.add_argument("--cpu-seconds", type=float, default=8.0)
    p.add_argument("--no-cpu", action="store_true")
    p.add_argument("--pipe-mib", type=int, default=4096,
                   help="end-to-end legs: pieces cut at record starts into parts of about this size (smaller "
                        "parts shorten the exposed first H2D, but each replay call reads its record counts "
                        "back to size its outputs: 512 MiB parts gave 36 GiB/s for the hints leg, 128 MiB 21, "
                        "whole 4000 MiB pieces 46)")
    p.add_argument("--no-gc", action="store_true", help="skip the f4 GC leg (e.g. for a PMC pass over the replay)")
    p.add_argument("--pin-records", type=int, default=1024,
                   help="records per chunk compared with the oracle inside the correctness gate")
    a = p.parse_args()
    rec = run(a, 0, 1, torch.device("cuda", 0))
    print(json.dumps(rec), flush=True)


HBM_PEAK_GBS = 8000.0
C4_TRAFFIC = os.path.join(ROOT, "profiles", "r06_c4_traffic.json")


def committed_traffic(step_chunk_bytes: float, path: str = C4_TRAFFIC) -> dict:
    """PMC HBM bytes of one replay step: the committed per-chunk-byte figure of a rocprofv3
    FETCH_SIZE / WRITE_SIZE run over one replay call (tools/traffic_call.py) x this step's chunk
    bytes; null when the profile is absent."""
    if not os.path.exists(path):
        return {"traffic": None}
    tj = json.load(open(path))
    return {"traffic": round(tj["hbm_bytes_per_call_byte"] * step_chunk_bytes),
            "traffic_source": f"{os.path.relpath(path, ROOT)}: {tj['hbm_bytes_per_call_byte']:.3f} HBM B per chunk "
                              f"byte (PMC, one replay call of {tj['call_bytes'] / 2**20:.0f} MiB) x chunk bytes per step"}


def run(a, rank: int, world: int, dev):
    """c4 on this rank.  The job is ONE corpus: a.files .data files alternating two distinct
    chunk files (seeds a.seed and a.seed + 1, the same on every rank), ~50 GiB at the defaults.
    It is split over the ranks on record boundaries by bytes (shard.partition_data_files, SURVEY
    §8(e)); a rank replays only its byte ranges, each a .data stream of its own.
    * gate (untimed): both chunks replayed whole against their expected record sets and
      `pin_records` sampled records against the oracle; then every piece of this rank replayed
      once: its record count, no resync, and the XOR of its value CRCs (all-gathered into the
      corpus digest, the same at every N);
    * device-only: the rank's pieces from the resident chunks, a.steps passes;
    * end to end (replay.replay_pipelined): the same pieces in parts pipelined from pinned host
      memory (H2D of part i+1, replay of part i, D2H of part i-1's decompressed values and
      per-record fields on three streams), and again with only the hint fields going back
      (buildHintFromData frees each body after Getvhash).  Checked: an untimed pass of the values
      pipeline CRCs every value in host memory (zlib) against the device-only digest, the timed
      pass's last two parts likewise, and every part of the timed hints pass by a hint digest.
    Returns the record on rank 0 (max-over-ranks times, summed bytes; CPU leg at N = 1 only)."""
    from gobeansdb_amd import replay, batch, shard
    t0 = time.time()
    chunks = []
    for j in range(2):
        host, nrec, stored_bytes, raw_bytes, rec_off = build_chunk(a.chunk_mib, a.seed + j, dev)
        chunks.append(dict(host=host, nrec=nrec, raw=raw_bytes, rec_off=rec_off,
                           pinned=torch.from_numpy(host).pin_memory()))
    log(f"rank {rank}: two chunks built in {time.time() - t0:.1f}s: "
        f"{[len(c['host']) >> 20 for c in chunks]} MiB, {[c['nrec'] for c in chunks]} records")
    ws = batch.Workspace(dev)
    for c in chunks:
        c["dev"] = c["pinned"].to(dev, non_blocking=False)
        # correctness gate: every record found, no resync, values decompressed to their raw sizes
        res = replay.replay(c["dev"], workspace=ws)
        torch.cuda.synchronize()
        assert res.n == c["nrec"] and not res.end_error, (res.n, c["nrec"], res.end_error)
        assert int(res.size_broken.abs().sum()) == 0
        assert int(res.value_len.to(torch.int64).sum()) == c["raw"], "decompressed sizes"
        assert int(((res.flag & 0x10000) != 0).sum()) == 0, "a compressed value failed to decode"
        c["compressed"] = int(((res.header[:, 2] & 0x10000) != 0).sum())
        c["pinned_sample"] = pin_sample(c, res, getattr(a, "pin_records", 1024))
        del res
    log("replay verified: all records, all values decoded, both chunks")

    # ---- the corpus and this rank's share (the generated files have no gaps: every record
    # start is a cut point) ----
    corpus = [f & 1 for f in range(a.files)]
    plan = shard.partition_data_files([(chunks[k]["rec_off"], len(chunks[k]["host"])) for k in corpus], world)
    pieces = [(corpus[f], lo, hi) for f, lo, hi in plan[rank]]
    digest, hdigest, nrec_mine, out_mine, out_cap = 0, 0, 0, 0, 0
    for f, lo, hi in plan[rank]:
        c = chunks[corpus[f]]
        ro = c["rec_off"].astype(np.int64)
        want = int(np.searchsorted(ro, hi) - np.searchsorted(ro, lo))
        res = replay.replay(c["dev"][lo:hi], workspace=ws)
        torch.cuda.synchronize()
        assert res.n == want and not res.end_error and int(res.size_broken.abs().sum()) == 0, (res.n, want)
        digest ^= _value_digest(res, lo, f)
        hdigest ^= replay.hint_digest(res.offset, res.header, res.vhash, lo, f)
        nrec_mine += res.n
        out_mine += int(res.value_len.to(torch.int64).sum())
        out_cap = max(out_cap, int(res.values.data.numel()))
        del res
    digest_mine = digest
    digest = shard.xor_digest_over_ranks(digest, device=dev)
    stream = torch.cuda.current_stream(dev)

    def sync_all():
        torch.cuda.synchronize()
        if world > 1:
            torch.distributed.barrier()
        torch.cuda.synchronize()

    # ---- device-only: the rank's pieces from the resident chunks ----
    if pieces:
        k, lo, hi = pieces[0]
        replay.replay(chunks[k]["dev"][lo:hi], workspace=ws)
    sync_all()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t = time.perf_counter()
    e0.record(stream)
    for _ in range(a.steps):
        for k, lo, hi in pieces:
            replay.replay(chunks[k]["dev"][lo:hi], workspace=ws, stream=stream)
    e1.record(stream)
    sync_all()
    dev_wall = time.perf_counter() - t
    dev_ev = e0.elapsed_time(e1) * 1e-3
    share = sum(hi - lo for _, lo, hi in pieces)

    # ---- end to end from pinned host memory (replay.replay_pipelined): H2D of part i+1 ||
    # replay of part i || D2H of part i-1's results, three streams.  The pieces move in parts of
    # about --pipe-mib cut at record starts (every record start of the generated chunks is a cut
    # point; a part is a .data stream of its own) ----
    parts = []   # (file, chunk, lo, hi)
    step_b = max(getattr(a, "pipe_mib", 4096), 1) << 20
    for f, lo, hi in plan[rank]:
        k = corpus[f]
        ro = chunks[k]["rec_off"].astype(np.int64)
        x = lo
        while x < hi:
            want = x + step_b
            idx = int(np.searchsorted(ro, want, side="left"))  # first record start at or past want
            y = int(ro[idx]) if want < hi and idx < len(ro) else hi
            y = min(y, hi)
            parts.append((f, k, x, y))
            x = y
    host_parts = [chunks[k]["pinned"][lo:hi] for _, k, lo, hi in parts]
    want_n = [int(np.searchsorted(chunks[k]["rec_off"].astype(np.int64), hi)
                  - np.searchsorted(chunks[k]["rec_off"].astype(np.int64), lo)) for _, k, lo, hi in parts]

    def check_part(i, hp):
        assert hp.n == want_n[i] and not hp.end_error, ("part", i, hp.n, want_n[i], hp.end_error)

    # checking pass (untimed): every value as it lands in host memory, CRC'd on the host (zlib),
    # the keyed XOR over the rank's share equal to the device-only digest
    t = time.perf_counter()
    hd = [0]

    def sink(i, hp):
        check_part(i, hp)
        f, _, lo, _ = parts[i]
        hd[0] ^= replay.host_value_digest(hp, host_parts[i], lo, f)

    part_cap = max([hi - lo for _, _, lo, hi in parts], default=1)
    pipe_v = replay.ReplayPipeline(part_cap, "values", dev, ws, values_cap=out_cap)
    pipe_v.run(host_parts, sink=sink)
    assert hd[0] == digest_mine, f"end-to-end values: host digest {hd[0]:08x} != device-only {digest_mine:08x}"
    log(f"rank {rank}: end-to-end values checked on the host ({len(parts)} parts, {time.perf_counter() - t:.1f}s)")

    # the timed pass: the same pipeline with no host wait; the parts still in the two host slots
    # at its end are checked against device-only replays of the same parts
    sync_all()
    t = time.perf_counter()
    got = pipe_v.run(host_parts)
    sync_all()
    pipe_s = time.perf_counter() - t
    tail_checked = 0
    for i, hp in enumerate(got):
        if hp is None:
            continue
        check_part(i, hp)
        f, k, lo, hi = parts[i]
        res = replay.replay(chunks[k]["dev"][lo:hi], workspace=ws)
        assert replay.host_value_digest(hp, host_parts[i], lo, f) == _value_digest(res, lo, f), ("timed part", i)
        tail_checked += 1
        del res
    del got

    # ---- end to end as buildHintFromData needs it (store/bucket.go:89-117): the decompressed
    # body only feeds Getvhash and is freed (p.Free()), so per record only the hint fields travel
    # back -- offset, the stored header (ver, ksz, vsz: the record size) and vhash.  Every part's
    # hints stay in host memory: the timed pass itself is checked ----
    pipe_h = replay.ReplayPipeline(part_cap, "hints", dev, ws, nparts=len(parts))
    sync_all()
    t = time.perf_counter()
    hints = pipe_h.run(host_parts)
    sync_all()
    hint_s = time.perf_counter() - t
    hh = 0
    for i, hp in enumerate(hints):
        check_part(i, hp)
        f, _, lo, _ = parts[i]
        hh ^= replay.hint_digest(hp.offset, hp.header, hp.vhash, lo, f)
    assert hh == hdigest, f"end-to-end hints: host digest {hh:08x} != device-only {hdigest:08x}"
    del hints, pipe_v, pipe_h
    e2e_values = shard.xor_digest_over_ranks(hd[0], device=dev)
    e2e_hints = shard.xor_digest_over_ranks(hh, device=dev)
    hdigest = shard.xor_digest_over_ranks(hdigest, device=dev)
    # ---- f4: GC rewrite (store/gc.go:268-353) of the first chunk, device-resident: the records
    # the reader returns, a liveness mask keeping ~70 %, appended with re-encoded headers and
    # recomputed CRCs (gobeansdb_amd.gc.rewrite).  Checked: every rewritten CRC equals the stored
    # one, and the rewritten chunk replays to exactly the kept records ----
    from gobeansdb_amd import gc as gcmod
    do_gc = not getattr(a, "no_gc", False)
    c0 = chunks[0]
    ro_t = torch.from_numpy(c0["rec_off"].astype(np.int64)).to(dev)
    keep = torch.from_numpy(np.random.default_rng(a.seed).random(c0["nrec"]) < 0.7).to(dev)
    nk, kept_bytes, gc_s = int(keep.sum()), 0, 1.0
    if do_gc:
        g = gcmod.rewrite(c0["dev"], ro_t, keep)
        torch.cuda.synchronize()
        assert g.crc_mismatch == 0, f"gc: {g.crc_mismatch} rewritten CRCs differ"
        rr = replay.replay(g.chunks[0], workspace=ws)
        assert len(g.chunks) == 1 and rr.n == nk and not rr.end_error, (len(g.chunks), rr.n, nk)
        kept_bytes = int(g.chunks[0].numel())
        del rr, g
        sync_all()
        t = time.perf_counter()
        for _ in range(a.steps):
            g = gcmod.rewrite(c0["dev"], ro_t, keep)
        sync_all()
        gc_s = (time.perf_counter() - t) / a.steps
        del g
    dev_wall, dev_ev, pipe_s, hint_s, gc_s = shard.max_over_ranks([dev_wall, dev_ev, pipe_s, hint_s, gc_s], device=dev)
    tot = shard.sum_over_ranks({"chunk": share, "out": out_mine, "records": nrec_mine, "pieces": len(pieces),
                                "parts": len(parts), "tail_checked": tail_checked},
                               device=dev)
    cpu = None
    if rank == 0 and world == 1 and not a.no_cpu:
        cpu = cpu_baseline(chunks[0]["host"], chunks[0]["rec_off"], a.cpu_seconds)
    if rank != 0:
        return None
    achieved = (tot["chunk"] + tot["out"]) / world / (dev_ev / a.steps) / 1e9
    corpus_b = sum(len(chunks[k]["host"]) for k in corpus)
    return {
        "metric": "GiB/s .data replay (record scan + CRC + decompress + vhash), c4",
        "value": round(tot["chunk"] * a.steps / dev_wall / 2**30, 2), "unit": "GiB/s of chunk, device-resident",
        "ms_per_step": round(dev_wall * 1e3 / a.steps, 3), "steps": a.steps,
        "scaling": "strong",
        "config": {"workload": f"c4: one corpus of {a.files} .data files ({corpus_b / 2**30:.1f} GiB: two distinct "
                               f"{a.chunk_mib} MiB chunk files alternating; store/datafile.go layout, log-uniform "
                               "4-64 KiB values, 70 % text, TryCompress policy) split over the ranks on record "
                               "boundaries (shard.partition_data_files), replayed as buildHintFromData reads them "
                               "(store/bucket.go:89-117); a step = every rank replays its share once",
                   "records_per_chunk": [c["nrec"] for c in chunks],
                   "oracle_pinned_records": [c["pinned_sample"] for c in chunks],
                   "compressed_values": [c["compressed"] for c in chunks],
                   "chunk_bytes": [len(c["host"]) for c in chunks], "corpus_bytes": corpus_b,
                   "pieces": tot["pieces"], "parallelism": f"shard{world}"},
        "digest": {"records": tot["records"], "value_bytes": tot["out"],
                   "xor_value_crc32": f"{digest:08x}",
                   "what": "XOR over every record of the corpus of crc32 (store/crc32.go) of its value after "
                           "Payload.Decompress, keyed by the record's place ((offset * 0x85EBCA77 + (file + 1) * "
                           "0x9E3779B1) mod 2^32, XORed in) since the corpus repeats its two chunk files; per-rank "
                           "XORs all-gathered: equal at every N"},
        "values_out_gib_per_s": round(tot["out"] * a.steps / dev_wall / 2**30, 2),
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), **committed_traffic(tot["chunk"] / world),
                     "what": "per rank and step: every chunk byte of its share read once (scan + CRC) + every "
                             "value byte written",
                     "kernel_ms": round(dev_ev * 1e3 / a.steps, 3)},
        "end_to_end_pipelined": {"total_gib": round(tot["chunk"] / 2**30, 2),
                                 "gib_per_s_chunk": round(tot["chunk"] / pipe_s / 2**30, 2),
                                 "seconds": round(pipe_s, 2),
                                 "parts": tot["parts"], "part_mib": getattr(a, "pipe_mib", 4096),
                                 "digest": {"xor_value_crc32": f"{e2e_values:08x}",
                                            "equals_device_only": e2e_values == digest,
                                            "timed_parts_checked": tot["tail_checked"],
                                            "what": "an untimed pass of the same pipeline CRCs every value on the host "
                                                    "(zlib) as it lands in pinned memory, keyed like the device-only "
                                                    "digest; the timed pass's last two parts (still in the host slots) "
                                                    "are checked against device-only replays of the same parts; every "
                                                    "part's record count and end state are asserted"},
                                 "note": "replay.replay_pipelined: each rank's pieces in parts cut at record starts; "
                                         "pinned H2D of part i+1, replay of part i and pinned D2H of part i-1's "
                                         "decompressed values and per-record fields on three streams"},
        "end_to_end_hints": {"gib_per_s_chunk": round(tot["chunk"] / hint_s / 2**30, 2),
                             "seconds": round(hint_s, 2),
                             "digest": {"xor_hint": f"{e2e_hints:08x}", "equals_device_only": e2e_hints == hdigest,
                                        "what": "XOR over every record of a keyed mix of (offset, stored header, vhash) "
                                                "as the timed pass left them in host memory, against the device-only "
                                                "replay's"},
                             "note": "as buildHintFromData (store/bucket.go:89-117): the same pipeline, but the "
                                     "decompressed bodies stay on the device (they only feed Getvhash, p.Free()); "
                                     "per record offset, stored header and vhash go back (pinned D2H)"},
        "gc": None if not do_gc else {"value": round(kept_bytes / gc_s / 2**30, 2), "unit": "GiB/s of rewritten records",
               "ms_per_call": round(gc_s * 1e3, 2), "records_kept": nk, "records": chunks[0]["nrec"],
               "roofline": {"bound": "hbm", "achieved": round(2 * kept_bytes / gc_s / 1e9, 1), "peak": HBM_PEAK_GBS,
                            "unit": "GB/s", "frac": round(2 * kept_bytes / gc_s / 1e9 / HBM_PEAK_GBS, 4),
                            "traffic": None,
                            "what": "algorithmic bytes: every kept record read once and written once (the CRC "
                                    "pass re-reads the written records; the header gather is 24 B per record)"},
               "check": "every recomputed CRC equals the stored one; the rewritten chunk replays to the kept records",
               "what": "SURVEY f4, store/gc.go:268-353: gc.rewrite of one chunk file (rank 0's first), ~70 % of "
                       "its records kept, host planning + qlzx_copy_batch + qlzx_crc32_batch; one call per step"},
        "data": "synthetic",
        "cpu_baseline": cpu,
    }


def cpu_baseline(host: np.ndarray, rec_off: np.ndarray, seconds: float):
    """The reference record loop (store/bucket.go:89-117 over store/datafile.go:228-277) on the
    host cores over the same chunk: CRC verify with the reference crc32_write, the reference
    qlz_decompress for FLAG_COMPRESS values, Getvhash (oracle/qlz_oracle.c orc_bench_replay,
    reference code from oracle/_ref).  Records are split into contiguous ranges, one per
    thread (buckets replay independently in the reference)."""
    import ctypes
    from bench import host_cpus
    from oracle import oracle as O
    Q, C = O.ref_if_built(), O.crc_ref_if_built()
    if Q is None or C is None:
        return None
    L = O.lib()
    threads, nproc, model = host_cpus()
    dec = ctypes.cast(Q.qlz_decompress, ctypes.c_void_p).value
    crc = ctypes.cast(C.crc32_write, ctypes.c_void_p).value
    bad = ctypes.c_uint64(0)

    def run(nthr, nbytes_cap, secs, cgo):
        n = len(rec_off)
        # records [0, last): all of them, or those starting before the byte cap
        last = n if nbytes_cap is None else max(1, int(np.searchsorted(rec_off, nbytes_cap, side="left")))
        end = len(host) if last == n else int(rec_off[last])
        cuts = np.asarray([int(rec_off[last * t // nthr]) for t in range(nthr)] + [end], np.uint64)
        span = int(cuts[-1] - cuts[0])
        reps, ns = 0, 0.0
        t_end = time.time() + secs
        while time.time() < t_end or reps == 0:
            ns += L.orc_bench_replay(dec, crc, host.ctypes.data, cuts.ctypes.data, nthr, int(cgo), ctypes.byref(bad))
            reps += 1
            if bad.value:
                raise RuntimeError(f"reference replay: {bad.value} records failed CRC/decompress")
        return reps * span / (ns * 1e-9) / 2**30, reps, span

    gibs, reps, span = run(threads, None, seconds, True)
    one, _, one_span = run(1, 256 << 20, max(2.0, seconds / 4), True)
    return {"value": round(gibs, 3), "unit": "GiB/s of chunk", "cores": threads, "kind": "reference",
            "sample": f"{reps} passes over the whole {span / 2**20:.0f} MiB chunk, {threads} threads on contiguous "
                      f"record ranges; per record: reference crc32_write over header[4:24]|key|value, "
                      f"reference qlz_decompress (output malloc per value, cgo-faithful) if FLAG_COMPRESS, Getvhash",
            "threads": threads, "nproc": nproc, "cpu_model": model, "one_core": round(one, 3),
            "one_core_sample": f"first {one_span / 2**20:.0f} MiB of the chunk"}


if __name__ == "__main__":
    main()
