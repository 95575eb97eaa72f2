"""GPU: Go quicklz level 1 (k_enc_go_l1 / k_dec_go_l1, qlzx_level1.hip) against the
level-1 oracle and the reference-level-1 fixtures (tests/golden/make_golden_l1.py)."""
import json
import os
import random

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module")
def l1():
    man = json.load(open(os.path.join(GOLDEN, "golden_l1.json")))
    blob = open(os.path.join(GOLDEN, "qlz_l1_vectors.bin"), "rb").read()
    get = lambda span: blob[span[0]:span[0] + span[1]]  # noqa: E731
    return [(v["name"], get(v["input"]), get(v["ref"])) for v in man["vectors"]]


def _decode_batch(streams, caps):
    import torch
    from gobeansdb_amd import batch
    src = batch.BlockBatch.from_bytes(streams)
    out = batch.BlockBatch.empty_for([max(c, 1) for c in caps])
    cap_t = torch.tensor(np.asarray(caps, np.uint32).view(np.int32), device="cuda")
    dsize, st = batch.go_decompress(src, out, dst_cap=cap_t)
    torch.cuda.synchronize()
    ds = dsize.cpu().numpy()
    return st.cpu().numpy().tolist(), out.to_bytes(ds)


def test_l1_decode_reference_streams(cuda, l1):
    """Every reference level-1 stream (one lane each, one launch) decodes to its input."""
    sizes = [len(d) for _, d, _ in l1]
    st, outs = _decode_batch([r for _, _, r in l1], sizes)
    for (name, data, _), s, o in zip(l1, st, outs):
        assert s == 0 and o == data, name


def test_l1_compress_matches_oracle(cuda, l1):
    """Go Compress(src, 1) on the GPU == the oracle byte for byte, and decodes on the GPU."""
    import torch
    from gobeansdb_amd import batch
    datas = [d for _, d, _ in l1]
    src = batch.BlockBatch.from_bytes(datas)
    dst, cs, st = batch.go_l1_compress(src)
    torch.cuda.synchronize()
    assert st.cpu().numpy().tolist() == [0] * len(datas)
    outs = dst.to_bytes(cs.cpu().numpy())
    for (name, data, _), o in zip(l1, outs):
        assert o == O.compress_go_l1(data), name
    st2, back = _decode_batch(outs, [len(d) for d in datas])
    assert st2 == [0] * len(datas) and back == datas


def test_l1_corrupt_status_matches_oracle(cuda, l1):
    """Byte flips and truncations of reference streams: the GPU status equals the oracle's
    (QLZX_E_CORRUPT exactly where Go Decompress panics), and so does an OK output."""
    rng = random.Random(77)
    cases, caps = [], []
    for name, data, ref in l1:
        if len(data) < 12:
            continue
        for _ in range(6):
            b = bytearray(ref)
            if rng.random() < 0.75:
                for _ in range(rng.randint(1, 3)):
                    b[rng.randrange(9, len(b))] ^= rng.randrange(1, 256)
            else:
                b = b[: rng.randrange(9, len(b) + 1)]
            cases.append(bytes(b))
            caps.append(O.lib().orc_size_decompressed(bytes(b)))
    st, outs = _decode_batch(cases, caps)
    nbad = 0
    for c, cap, s, o in zip(cases, caps, st, outs):
        ost, od = O.decompress_go_l1(c, cap=cap)
        assert s == ost
        nbad += ost != 0
        if ost == 0:
            assert o == od
    assert nbad > 0


def test_go_api_level1_round_trip(cuda, l1):
    """The quicklz.Compress / Decompress mirror at level 1 (single-call path), the stored
    zero-fill of Go's copy(), and the level checks."""
    from gobeansdb_amd import quicklz as Q
    for name, data, ref in l1[::5]:
        c = Q.Compress(data, 1)
        assert c == O.compress_go_l1(data), name
        assert Q.Decompress(c) == data, name
        assert Q.Decompress(ref) == data, name
    assert Q.Compress(b"", 1) is None
    short_stored = bytes([0x46]) + (20).to_bytes(4, "little") + (12).to_bytes(4, "little") + b"abc"
    assert Q.Decompress(short_stored) == b"abc" + bytes(9)
    with pytest.raises(Q.QuicklzError):
        Q.Decompress(bytes([0x49]) + bytes(8))
    bad = bytearray(Q.Compress(O.gen_text(1, 0, 5000), 1))
    del bad[40:]
    with pytest.raises(Q.QuicklzError):
        Q.Decompress(bytes(bad))


def test_go_l1_batches_past_one_launch(cuda):
    """More blocks than one level-1 launch takes (kL1Chunk = 65536, qlzx_api.hip): the chunks
    reuse one workspace with chunk-local indices.  Every block in both chunks equals the oracle
    byte for byte and decodes back through go_decompress."""
    import torch
    from gobeansdb_amd import batch
    rng = random.Random(5)
    words = [b"alpha ", b"beta ", b"gamma ", b"delta ", b"value:", b"0123", b"\x00\x01", b"key_"]
    datas = []
    for i in range(65536 + 37):
        n = rng.randrange(1, 160)
        d = b"".join(rng.choice(words) for _ in range(n // 4 + 1))[:n]
        datas.append(d)
    src = batch.BlockBatch.from_bytes(datas)
    dst, cs, st = batch.go_l1_compress(src)
    torch.cuda.synchronize()
    assert st.cpu().numpy().tolist() == [0] * len(datas)
    outs = dst.to_bytes(cs.cpu().numpy())
    for i, (d, o) in enumerate(zip(datas, outs)):
        assert o == O.compress_go_l1(d), i
    st2, back = _decode_batch(outs, [len(d) for d in datas])
    assert st2 == [0] * len(datas)
    assert back == datas
