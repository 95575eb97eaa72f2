"""Write-side record encode: MIME sniff policy (CPU) and the GPU
encoder reproducing the golden .data records byte for byte (GPU)."""
import numpy as np
import pytest

from gobeansdb_amd import record

# store/item_test.go:7-22 (sniffTests): data, expected NeedCompress
SNIFF = [
    (b"MThd\x00\x00\x00\x06\x00\x01", True),
    (b"ID3\x03\x00\x00\x00\x00\x0f", False),
    (b"RIFFb\xb8\x00\x00WAVEfmt \x12\x00\x00\x00\x06", False),
    (b"RIFF,\x00\x00\x00WAVEfmt \x12\x00\x00\x00\x06", False),
    (b"FORM\x00\x00\x00\x00AIFFCOMM\x00\x00\x00\x12\x00\x01\x00\x00\x57\x55\x00\x10\x40\x0d\xf3\x34", True),
    (b"OggS\x00\x02\x00\x00\x00\x00\x00\x00\x00\x00\x7e\x46\x00\x00\x00\x00\x00\x00\x1f\xf6\xb4\xfc\x01\x1e\x01"
     b"\x76\x6f\x72", True),
    (b"ID3\x03\x00\x00\x00\x00\x04", False),
    (b"ID3\x03\x00\x00\x00\x00\x0a", False),
]


@pytest.mark.parametrize("data,expect", SNIFF)
def test_need_compress_sniff_table(data, expect):
    value = data + bytes(512 - len(data))          # ValueWithKind(st.data, 512), item_test.go:24-31
    assert record.need_compress(value[:512]) == expect


# the same sniffTests data under the shipped conf/global.yaml:29-33 set (adds audio/ogg and
# audio/midi): MIDI is now stored raw; Ogg still compresses because Go 1.13 answers
# "application/ogg" (store/item_test.go:19), never "audio/ogg".
SNIFF_SHIPPED = [(d, e and not d.startswith(b"MThd")) for d, e in SNIFF]


@pytest.mark.parametrize("data,expect", SNIFF_SHIPPED)
def test_need_compress_shipped_not_compress_set(data, expect):
    value = data + bytes(512 - len(data))
    assert record.need_compress(value[:512], record.NOT_COMPRESS_SHIPPED) == expect


def test_sniff_answers():
    assert record.sniff(b"MThd\x00\x00\x00\x06" + bytes(8)) == "audio/midi"
    assert record.sniff(b"MThd\x00\x00\x00\x07" + bytes(8)) is None        # header length must be 6
    assert record.sniff(b"OggS\x00" + bytes(8)) == "application/ogg"
    assert record.sniff(b"RIFF\x01\x02\x03\x04AVI " + bytes(8)) == "video/avi"
    assert record.sniff(b".snd" + bytes(8)) == "audio/basic"
    assert record.sniff(b"MTh") is None                                         # too short to match


def test_riff_webp_is_not_wave():
    assert record.need_compress(b"RIFF\x00\x00\x00\x00WEBPVP8 " + bytes(100))


@pytest.mark.gpu
def test_encode_reproduces_golden_records(cuda, golden):
    from gobeansdb_amd import batch
    recs = golden.records
    keys = [r["key"].encode() for r in recs]
    values = [golden.get(r["value"]) for r in recs]
    vb = batch.BlockBatch.from_bytes(values)
    enc = record.encode(keys, vb, vers=[r["ver"] for r in recs], ts=[r["ts"] for r in recs])
    got = enc.data.cpu().numpy().tobytes()
    assert list(enc.offset) == [r["offset"] for r in recs]
    assert list(enc.flag) == [r["flag"] for r in recs]
    assert list(enc.crc) == [r["crc"] for r in recs]
    assert got == golden.records_data


@pytest.mark.gpu
def test_encode_policy_edges(cuda):
    from gobeansdb_amd import batch
    from oracle import oracle as O
    from oracle import replay as R
    vals = [b"ID3\x03" + O.gen_text(1, 0, 20000),      # audio/mpeg: never compressed
            O.gen_text(1, 1, 20000),                     # compressible, > 10 KiB: whole body recompressed
            O.gen_text(1, 2, 300),                        # small but padded size > 256
            b"x" * 200,                                   # record fits one slot: skipped
            O.gen_image(5, 0, 30000),                     # random: trial ratio > 0.7, kept raw
            O.gen_text(1, 3, 5000)]                       # ver < 0: skipped
    flags = [0, 0, 0, 0, 0, 0]
    vers = [1, 1, 1, 1, 1, -1]
    keys = [b"k%d" % i for i in range(len(vals))]
    enc = record.encode(keys, batch.BlockBatch.from_bytes(vals), flags=flags, vers=vers)
    exp, exp_flags = b"", []
    for k, v, f, ver in zip(keys, vals, flags, vers):
        body, fl = v, f
        if ver >= 0 and (24 + len(k) + len(v) + 255) // 256 * 256 > 256 and not v.startswith(b"ID3"):
            t = v[:10240]
            c = O.compress(t)
            if np.float32(len(c)) / np.float32(len(t)) <= np.float32(0.7):
                body, fl = (O.compress(v) if len(v) > len(t) else c), f | 0x10000
        exp += R.make_record(k, body, flag=fl, ver=ver)
        exp_flags.append(fl)
    assert enc.data.cpu().numpy().tobytes() == exp
    assert [int(f) for f in enc.flag] == exp_flags
    assert exp_flags[1] == 0x10000 and exp_flags[0] == exp_flags[3] == exp_flags[4] == exp_flags[5] == 0


def test_sniff_many_matches_sniff():
    """The vectorised policy record.encode uses (sniff_many) answers need_compress exactly,
    per row and in row order, for crafted signatures, near misses and random heads."""
    import numpy as np
    rng = np.random.default_rng(5)
    heads = [sig[1] + bytes(16) for sig in record._AV_SIGS]
    heads += [b"MThd\x00\x00\x00\x07" + bytes(8), b"MTh", b"", b"RIFF\x01\x02\x03\x04WAVE" + bytes(4), b"ID3",
              b"RIFF\x00\x00\x00\x00WEBPVP8 " + bytes(4), b"FORM\x01\x02\x03\x04AIFF"]
    heads += [rng.integers(0, 256, 20, dtype=np.uint8).tobytes() for _ in range(300)]
    H = np.zeros((len(heads), 16), np.uint8)
    L = np.zeros(len(heads), np.int64)
    for i, h in enumerate(heads):
        b = np.frombuffer(h[:16], np.uint8)
        H[i, :len(b)] = b
        L[i] = len(h)
    for nc in (record.NOT_COMPRESS, record.NOT_COMPRESS_SHIPPED, frozenset(),
               frozenset({"video/avi", "audio/basic", "application/ogg", "audio/aiff"})):
        got = record.sniff_many(H, L, nc)
        want = np.array([record.need_compress(h, nc) for h in heads])
        assert (got == want).all()
