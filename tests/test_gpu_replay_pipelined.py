"""GPU: the c4 end-to-end path (replay.replay_pipelined) checked against oracle/replay.py.

Two distinct 64 MiB chunk files of the c4 leg (tools/bench_replay.build_chunk: store/datafile.go
layout, log-uniform 4-64 KiB values, 70 % text, TryCompress policy) are cut at record starts
into parts and replayed from pinned host memory through the three-stream pipeline (pinned H2D,
replay, pinned D2H).  What lands in host memory -- every record's offset, stored header, flag
and value after Payload.Decompress, and Getvhash -- must equal the oracle's buildHintFromData
restatement (store/bucket.go:89-117, store/datafile.go:228-277) on the same bytes; the host-side
digest must equal the device-only replay's.
"""
import os
import sys

import numpy as np
import pytest
import torch

from oracle import replay as R

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def chunks(cuda):
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from bench_replay import build_chunk
    out = []
    for seed in (77, 78):
        host, nrec, _, _, rec_off = build_chunk(64, seed, cuda)
        rows, err = R.replay(host.tobytes())
        assert err is None and len(rows) == nrec
        out.append(dict(host=host, rec_off=rec_off.astype(np.int64), rows=rows,
                        pinned=torch.from_numpy(host).pin_memory()))
    return out


def _parts(chunks, part_bytes):
    parts = []
    for f, c in enumerate(chunks):
        ro, lo = c["rec_off"], 0
        while lo < len(c["host"]):
            idx = int(np.searchsorted(ro, lo + part_bytes, side="left"))
            hi = int(ro[idx]) if idx < len(ro) else len(c["host"])
            parts.append((f, lo, hi))
            lo = hi
    return parts


def _expect(c, lo, hi):
    return [r for r in c["rows"] if lo <= r[0] < hi]


@pytest.mark.parametrize("part_mib", [64, 20, 7])
def test_values_land_in_host_memory_like_the_oracle(cuda, chunks, part_mib):
    from gobeansdb_amd import replay
    parts = _parts(chunks, part_mib << 20)
    host_parts = [chunks[f]["pinned"][lo:hi] for f, lo, hi in parts]
    seen = []

    def sink(i, hp):
        f, lo, hi = parts[i]
        rows = _expect(chunks[f], lo, hi)
        assert hp.n == len(rows) and not hp.end_error
        off = hp.offset.numpy()
        hdr = hp.header.numpy()
        for j, (o, broken, key, ver, flag, body, vh) in enumerate(rows):
            assert broken == 0 and int(off[j]) + lo == o
            assert int(hdr[j, 3]) == ver and int(hp.flag[j]) == flag
            assert bytes(hp.value(host_parts[i], j)) == body, (i, j)
            assert int(hp.vhash[j]) & 0xFFFF == vh
        seen.append(i)

    replay.replay_pipelined(host_parts, "values", device=cuda, sink=sink)
    assert seen == list(range(len(parts)))

    # the timed form (no host wait): the last two parts are intact at the end and equal the
    # device-only replay's digest
    got = replay.replay_pipelined(host_parts, "values", device=cuda)
    live = [i for i, hp in enumerate(got) if hp is not None]
    assert live == list(range(max(0, len(parts) - 2), len(parts)))
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from bench_replay import _value_digest
    for i in live:
        f, lo, hi = parts[i]
        res = replay.replay(chunks[f]["pinned"][lo:hi].to(cuda))
        assert replay.host_value_digest(got[i], host_parts[i], lo, f) == _value_digest(res, lo, f)


def test_hints_land_in_host_memory_like_the_oracle(cuda, chunks):
    from gobeansdb_amd import replay
    parts = _parts(chunks, 24 << 20)
    host_parts = [chunks[f]["pinned"][lo:hi] for f, lo, hi in parts]
    hints = replay.replay_pipelined(host_parts, "hints", device=cuda)
    dev_digest = host_digest = 0
    for (f, lo, hi), hp in zip(parts, hints):
        rows = _expect(chunks[f], lo, hi)
        assert hp.n == len(rows) and not hp.end_error
        assert [int(x) + lo for x in hp.offset.numpy()] == [r[0] for r in rows]
        assert [int(x) & 0xFFFF for x in hp.vhash.numpy()] == [r[6] for r in rows]
        res = replay.replay(chunks[f]["pinned"][lo:hi].to(cuda))
        dev_digest ^= replay.hint_digest(res.offset, res.header, res.vhash, lo, f)
        host_digest ^= replay.hint_digest(hp.offset, hp.header, hp.vhash, lo, f)
    assert host_digest == dev_digest
