"""CPU: the level-1 oracle (oracle/qlz_oracle_l1.c, Go quicklz.go level 1) against the
fixtures from the reference quicklz.c compiled at level 1 (tests/golden/make_golden_l1.py)."""
import json
import os
import random

import pytest

from oracle import oracle as O

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module")
def l1():
    man = json.load(open(os.path.join(GOLDEN, "golden_l1.json")))
    blob = open(os.path.join(GOLDEN, "qlz_l1_vectors.bin"), "rb").read()
    get = lambda span: blob[span[0]:span[0] + span[1]]  # noqa: E731
    return [(v["name"], get(v["input"]), get(v["ref"]), v["go_quirk"]) for v in man["vectors"]]


def test_oracle_decodes_reference_level1(l1):
    for name, data, ref, _ in l1:
        st, out = O.decompress_go_l1(ref)
        assert st == O.OK and out == data, name


def test_oracle_go_compress_matches_reference_core(l1):
    """Go Compress(src, 1) = the reference level-1 stream after the header, except the
    Go encoder's documented quirks (9-byte header always, no core minimum, bail-out
    counting the header), which must still decode."""
    for name, data, ref, quirk in l1:
        go = O.compress_go_l1(data)
        assert go[0] & 0x0C == 0x04 and go[0] & 2, name            # level 1, 9-byte header
        assert int.from_bytes(go[1:5], "little") == len(go), name
        assert int.from_bytes(go[5:9], "little") == len(data), name
        if not quirk:
            assert go[9:] == ref[(9 if ref[0] & 2 else 3):], name
        st, out = O.decompress_go_l1(go)
        assert st == O.OK and out == data, name


def test_oracle_l1_edges():
    assert O.compress_go_l1(b"") is None                             # quicklz.go:109-111
    # stored stream with a short body: Go copy() zero-fills the rest
    st, out = O.decompress_go_l1(bytes([0x46]) + (20).to_bytes(4, "little") + (12).to_bytes(4, "little") + b"abc")
    assert st == O.OK and out == b"abc" + bytes(9)
    st, _ = O.decompress_go_l1(bytes([0x49]) + bytes(8))              # level 2
    assert st == O.E_LEVEL
    st, _ = O.decompress_go_l1(bytes([0x47, 1]))                      # header past the buffer
    assert st == O.E_HEADER


def test_oracle_l1_corrupt_never_overruns(l1):
    """Random byte flips and truncations: every result is a status, never a crash; an OK
    result has exactly SizeDecompressed bytes."""
    rng = random.Random(5)
    for name, data, ref, _ in l1[::7]:
        for _ in range(20):
            b = bytearray(ref)
            if len(b) > 10 and rng.random() < 0.8:
                b[rng.randrange(9, len(b))] ^= rng.randrange(1, 256)
            else:
                b = b[: rng.randrange(1, len(b) + 1)]
            st, out = O.decompress_go_l1(bytes(b))
            assert st in (O.OK, O.E_CORRUPT, O.E_HEADER, O.E_LEVEL), (name, st)
            if st == O.OK:
                assert len(out) == O.lib().orc_size_decompressed(bytes(b))
