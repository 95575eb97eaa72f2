"""GPU parity: the HIP codec through the C ABI vs the reference golden vectors and the oracle."""
import ctypes
import zlib

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu

KAT = (b"LZ compression is based on finding repeated strings: Five, six, seven, eight, nine, "
       b"fifteen, sixteen, seventeen, fifteen, sixteen, seventeen.")


def _dsize(c: bytes) -> int:
    """quicklz.go:39-44 on the host (header only)."""
    if len(c) < 3:
        return 0
    if c[0] & 2:
        return int.from_bytes((c + bytes(9))[5:9], "little")
    return c[2]


def _gpu_compress(blocks, **kw):
    import torch
    from gobeansdb_amd import batch
    src = batch.BlockBatch.from_bytes(blocks)
    dst, csize, status, crc = batch.compress(src, **kw)
    torch.cuda.synchronize()
    cs = csize.cpu().numpy().view(np.uint32)
    return dst.to_bytes(cs), status.cpu().numpy(), (None if crc is None else crc.cpu().numpy().view(np.uint32))


def _gpu_decompress(comp, caps=None, **kw):
    import torch
    from gobeansdb_amd import batch
    src = batch.BlockBatch.from_bytes(comp)
    sizes = [_dsize(c) for c in comp]
    caps_arr = sizes if caps is None else caps
    out = batch.BlockBatch.empty_for([max(s, 1) for s in caps_arr])
    cap_t = torch.tensor(np.asarray(caps_arr, dtype=np.uint32).view(np.int32), device="cuda")
    dsize, status, crc = batch.decompress(src, out, dst_cap=cap_t, max_dsize=max(caps_arr + [1]), **kw)
    torch.cuda.synchronize()
    ds = dsize.cpu().numpy().view(np.uint32)
    return out.to_bytes(ds), status.cpu().numpy(), (None if crc is None else crc.cpu().numpy().view(np.uint32))


def test_compress_golden_bit_exact(cuda, golden):
    vs = golden.vectors
    outs, st, crc = _gpu_compress([golden.get(v["input"]) for v in vs], want_crc=True)
    assert (st == 0).all()
    for v, o, c in zip(vs, outs, crc):
        assert o == golden.get(v["c_out"]), v["name"]
        assert int(c) == v["crc_c_out"], v["name"]   # fused CRC over the compressed value


# general=True: every block through the general lane-per-block kernel (values over 64 KiB)
@pytest.mark.parametrize("general", [False, True])
def test_decompress_golden(cuda, golden, general):
    vs = golden.vectors
    outs, st, crc = _gpu_decompress([golden.get(v["c_out"]) for v in vs], want_crc=True, general=general)
    assert (st == 0).all(), [(v["name"], s) for v, s in zip(vs, st) if s]
    for v, o, c in zip(vs, outs, crc):
        assert o == golden.get(v["input"]), v["name"]
        assert int(c) == v["crc_c_out"]


def test_quicklz_go_api_kat(cuda):
    """quicklz/quicklz_test.go:7-34, against the GPU-backed mirror."""
    from gobeansdb_amd.quicklz import (CCompress, CDecompress, Compress, Decompress,
                                       SizeCompressed, SizeDecompressed)
    orig = KAT
    compressed = Compress(orig, 3)
    l, lc = len(orig), len(compressed)
    assert lc == 116
    s, sc = SizeDecompressed(compressed), SizeCompressed(compressed)
    assert s == l and sc == lc
    assert len(Decompress(compressed)) == l
    compressed2, ok = CCompress(orig)
    assert ok
    decompressed2, err = CDecompress(compressed2.Body, s)
    assert err is None and decompressed2.Body == orig


def test_single_call_symbols(cuda, golden):
    from gobeansdb_amd import _lib
    L = _lib.lib()
    for v in golden.vectors[::7]:
        data, c = golden.get(v["input"]), golden.get(v["c_out"])
        dst = ctypes.create_string_buffer(len(data) + 400)
        n = L.qlz_compress(data, dst, len(data), ctypes.create_string_buffer(528400))
        assert dst.raw[:n] == c, v["name"]
        out = ctypes.create_string_buffer(len(data) + 1)
        assert L.qlz_decompress(c, out, ctypes.create_string_buffer(16)) == len(data)
        assert out.raw[:len(data)] == data
        assert L.crc32_write(0xFFFFFFFF, data, len(data)) ^ 0xFFFFFFFF == v["crc_in"]
    assert L.qlz_compress(b"", ctypes.create_string_buffer(400), 0, None) == 0   # quicklz.c:705


def test_cdecompress_safe_errors(cuda, golden):
    from gobeansdb_amd.quicklz import CDecompressSafe
    c = golden.get([v for v in golden.vectors if v["name"] == "text_4096"][0]["c_out"])
    arr, err = CDecompressSafe(c[:-1])
    assert err is not None and "bad sizeCompressed" in str(err)
    arr, err = CDecompressSafe(c)
    assert err is None and len(arr.Body) == 4096


@pytest.mark.parametrize("general", [False, True])
def test_corrupt_status_matches_oracle(cuda, golden, general):
    rng = np.random.default_rng(5)
    base = [golden.get(v["c_out"]) for v in golden.vectors if v["cls"] in ("text", "runs", "kat") and v["n"] >= 100]
    cases = []
    for c in base:
        for _ in range(6):
            b = bytearray(c)
            hdr = 9 if b[0] & 2 else 3
            k = int(rng.integers(hdr, len(b)))
            b[k] = int(rng.integers(0, 256))
            cases.append(bytes(b))
        cases.append(c[:-1])
    caps = [_dsize(c) for c in cases]
    caps = [min(x, 1 << 20) for x in caps]
    outs, st, _ = _gpu_decompress(cases, caps=caps, general=general)
    for c, cap, o, s in zip(cases, caps, outs, st):
        ost, od = O.decompress(c, cap=cap)
        assert s == ost
        if s == 0:
            assert o == od


def test_crc_batch(cuda, golden):
    import torch
    from gobeansdb_amd import batch
    datas = [golden.get(v["input"]) for v in golden.vectors]
    src = batch.BlockBatch.from_bytes(datas)
    out = batch.crc32(src).cpu().numpy().view(np.uint32)
    for d, v, c in zip(datas, golden.vectors, out):
        assert int(c) == (zlib.crc32(d) if d else 0), v["name"]
    init = torch.tensor(np.full(len(datas), 0x12345678, np.uint32).view(np.int32), device="cuda")
    raw = batch.crc32(src, init=init, final_xor=0).cpu().numpy().view(np.uint32)
    for d, c in zip(datas, raw):
        assert int(c) == O.crc32_write(0x12345678, d)


def test_crc_unaligned_and_stripe_edges(cuda):
    """wave_crc: every length 0..300 and the 4 KiB stripe edges (4095/4096/4097, 8191, ...,
    1 MiB + 3) at every start alignment 0..3 of one shared buffer, with a non-default init."""
    import torch
    from gobeansdb_amd import batch
    rng = np.random.default_rng(3)
    buf = rng.integers(0, 256, (2 << 20) + 64, dtype=np.uint8)
    lens = list(range(0, 301)) + [4092, 4095, 4096, 4097, 4100, 8191, 8192, 8193, 12345, 65536 + 7, (1 << 20) + 3]
    offs, ls = [], []
    for k, n in enumerate(lens):
        for m in range(4):
            offs.append(8 * k + m)
            ls.append(n)
    d = torch.from_numpy(buf).cuda()
    src = batch.BlockBatch(d, torch.tensor(offs, dtype=torch.int64, device="cuda"),
                           torch.tensor(ls, dtype=torch.int32, device="cuda"))
    init = torch.tensor(np.full(len(ls), 0x9E3779B9, np.uint32).view(np.int32), device="cuda")
    got = batch.crc32(src, init=init, final_xor=0).cpu().numpy().view(np.uint32)
    std = batch.crc32(src).cpu().numpy().view(np.uint32)
    for o, n, g, s in zip(offs, ls, got, std):
        b = buf[o:o + n].tobytes()
        assert int(g) == O.crc32_write(0x9E3779B9, b), (o, n)
        assert int(s) == zlib.crc32(b), (o, n)


@pytest.mark.parametrize("kind", ["text", "image"])
def test_synth_matches_oracle(cuda, kind):
    import torch
    from gobeansdb_amd import batch
    lens = [16384, 65536, 5, 4096, 777]
    b = batch.synth(kind, 1234, lens, first_id=100)
    torch.cuda.synchronize()
    got = b.to_bytes()
    gen = O.gen_text if kind == "text" else O.gen_image
    for i, n in enumerate(lens):
        assert got[i] == gen(1234, 100 + i, n)


def test_go_compat_compress(cuda):
    blocks = [O.gen_text(99, n, n) for n in (1, 4, 5, 215, 216, 4096)] + [O.gen_image(3, 0, 4096), KAT]
    outs, st, _ = _gpu_compress(blocks, go_compat=True)
    assert (st == 0).all()
    for b, o in zip(blocks, outs):
        assert o == O.compress_go(b)


@pytest.mark.parametrize("general", [False, True])
def test_record_fused_crc_verify(cuda, golden, general):
    """store/datafile.go:161-168: CRC over header[4:24] ‖ key ‖ value, fused with decompress."""
    import struct
    import torch
    data = golden.records_data
    comp, states, expect, values = [], [], [], []
    for r in golden.records:
        if not r["flag"] & 0x10000:
            continue
        o = r["offset"]
        crc, ts, flag, ver, ksz, vsz = struct.unpack_from("<IIIiII", data, o)
        key = data[o + 24:o + 24 + ksz]
        body = data[o + 24 + ksz:o + 24 + ksz + vsz]
        st = O.crc32_write(O.crc32_write(0xFFFFFFFF, data[o + 4:o + 24]), key)
        comp.append(body), states.append(st), expect.append(crc), values.append(golden.get(r["value"]))
    # flip one byte of one record's value to force a CRC failure
    bad = bytearray(comp[1])
    bad[len(bad) // 2] ^= 0x40
    comp[1] = bytes(bad)
    s_t = torch.tensor(np.asarray(states, np.uint32).view(np.int32), device="cuda")
    e_t = torch.tensor(np.asarray(expect, np.uint32).view(np.int32), device="cuda")
    outs, st, crc = _gpu_decompress(comp, crc_state=s_t, crc_expect=e_t, general=general)
    for i, (o, s, v) in enumerate(zip(outs, st, values)):
        if i == 1:
            assert s == 5   # QLZX_E_CRC
        else:
            assert s == 0 and o == v


# max_dsize 16384 and 65536: the two chunk regimes of the batch decoder (uniform / mixed sizes),
# both with the record-CRC prologue of k_dec_chunk4<true>.
@pytest.mark.parametrize("max_dsize", [16384, 65536])
def test_batch_crc_verify_every_length(cuda, max_dsize):
    """store/datafile.go:161-168 through qlzx_decompress_batch: the CRC continued from a per-block
    state over blocks of every length 0..699 and 300 longer ones (to 17,000 B), packed at unaligned
    offsets; every 7th stored CRC is wrong and must give QLZX_E_CRC, the others must not."""
    import torch
    from gobeansdb_amd import _lib, batch
    rng = np.random.default_rng(5)
    lens = list(range(700)) + [int(x) for x in rng.integers(700, 17000, 300)]
    blocks = []
    for n in lens:
        b = bytearray(rng.integers(0, 256, n, dtype=np.uint8).tobytes())
        if n >= 3:  # a short level-3 stored header with dsize 16: no block goes to the general path
            b[0], b[1], b[2] = 0x0C, n & 0xFF, 16
        blocks.append(bytes(b))
    states = rng.integers(0, 2 ** 32, len(lens), dtype=np.uint64).astype(np.uint32)
    want = np.array([O.crc32_write(int(s), b) ^ 0xFFFFFFFF for s, b in zip(states, blocks)], np.uint32)
    bad = np.arange(len(lens)) % 7 == 3
    expect = want ^ np.where(bad, np.uint32(0x1000), np.uint32(0))
    src = batch.BlockBatch.from_bytes(blocks)
    out = batch.BlockBatch.empty_for([256] * len(lens))
    cap_t = torch.full((len(lens),), 256, dtype=torch.int32, device="cuda")
    s_t = torch.tensor(states.view(np.int32), device="cuda")
    e_t = torch.tensor(expect.view(np.int32), device="cuda")
    _, st, crc = batch.decompress(src, out, dst_cap=cap_t, crc_state=s_t, crc_expect=e_t, max_dsize=max_dsize)
    torch.cuda.synchronize()
    crc = crc.cpu().numpy().view(np.uint32)
    st = st.cpu().numpy()
    assert (crc == want).all(), np.nonzero(crc != want)[0][:10]
    assert (st[bad] == _lib.E_CRC).all()
    assert (st[~bad] != _lib.E_CRC).all()


# (crc, max_dsize): the uniform regime (chunks of 262144 blocks, two workspace halves) and the
# mixed one (max_dsize > 16 KiB: chunks of 131072; at three chunks the last chunk's K1 starts
# first in a third workspace region)
@pytest.mark.parametrize("crc,mixed", [(False, False), (True, False), (False, True), (True, True), (False, 4)])
def test_multi_chunk_overlap_round_trip(cuda, crc, mixed):
    """More blocks than one decode chunk (chunk_blocks in qlzx_decode_wave.hip): K1 of chunk c+1
    runs on the side stream while K2 of chunk c runs.  Every block must round-trip, and with crc
    the fused record CRC must equal a separate CRC pass over the compressed values."""
    import torch
    from gobeansdb_amd import _lib, batch
    n = (393216 if mixed == 4 else 262144) + 9000
    lens = [256 + (i * 37) % 1800 for i in range(n)]
    max_dsize = 32768 if mixed else max(lens)
    if mixed:  # three (four) chunks: a region more for the last (two) chunks' early K1s
        L = _lib.lib()
        regions = 3  # one early chunk (QLZX_LAST_K1_EARLY) at three chunks and at four
        assert L.qlzx_decompress_workspace_size(n, max_dsize) > \
            (regions + 0.2) * L.qlzx_decompress_workspace_size(100000, max_dsize)
    plain = batch.synth("text", 77, lens)
    comp, cs, st, _ = batch.compress(plain, max_len=max(lens))
    assert int((st != 0).sum()) == 0
    src = batch.BlockBatch(comp.data, comp.off, cs)
    out = batch.BlockBatch.empty_for(lens)
    kw = {}
    if crc:
        kw = dict(crc_state=torch.full((n,), -1, dtype=torch.int32, device="cuda"), want_crc=True)
    dsz, st2, crc_out = batch.decompress(src, out, max_dsize=max_dsize, **kw)
    torch.cuda.synchronize()
    assert int((st2 != 0).sum()) == 0
    assert torch.equal(dsz, plain.length)
    # every valid byte (same lengths -> same packing; the padding between blocks is not compared)
    ln = plain.length.to(torch.int64)
    starts = torch.cumsum(ln, 0) - ln
    rel = torch.arange(int(ln.sum()), device="cuda") - torch.repeat_interleave(starts, ln)
    pos = torch.repeat_interleave(plain.off, ln) + rel
    assert torch.equal(out.data[pos], plain.data[pos])
    if crc:
        assert torch.equal(crc_out, batch.crc32(src))


def test_mixed_sizes_block_order_round_trip(cuda):
    """Log-uniform 1-64 KiB text and image-like blocks over two decode chunks: K1 and K2 take
    their blocks from the size-ordered list (k_order_count / k_order_scatter), so every block's
    output must still land at its own offset.  Compared by per-block CRC32 of output vs plain."""
    import numpy as np
    import torch
    from gobeansdb_amd import batch
    n = 131072 + 3000
    rng = np.random.default_rng(5)
    lens = np.exp(rng.uniform(np.log(1024), np.log(65536), n)).astype(np.int64)
    n_img = n * 3 // 10    # image-like blocks: mostly stored in the mix
    parts = [batch.synth("text", 91, lens[n_img:].tolist()), batch.synth("image", 92, lens[:n_img].tolist())]
    comps = []
    for plain in parts:
        comp, cs, st, _ = batch.compress(plain, max_len=65536)
        assert int((st != 0).sum()) == 0
        comps.append((comp, cs))
    perm = torch.from_numpy(rng.permutation(n)).cuda()
    data = torch.cat([comps[0][0].data, comps[1][0].data])
    off = torch.cat([comps[0][0].off, comps[1][0].off + comps[0][0].data.numel()])
    src = batch.BlockBatch(data, off[perm], torch.cat([comps[0][1], comps[1][1]])[perm])
    plen = torch.cat([parts[0].length, parts[1].length])[perm]
    out = batch.BlockBatch.empty_for(plen.cpu().numpy().astype(np.int64).tolist())
    expect = torch.cat([batch.crc32(parts[0]), batch.crc32(parts[1])])[perm]
    dsz, st2, _ = batch.decompress(src, out, max_dsize=65536)
    torch.cuda.synchronize()
    assert int((st2 != 0).sum()) == 0
    assert torch.equal(dsz, plen)
    assert torch.equal(batch.crc32(out), expect)


def test_max_dsize_contract(cuda):
    """A block whose header dsize exceeds the batch's max_dsize argument is reported as
    QLZX_E_MAX_DSIZE (not left pending, not misreported as corrupt); the others decode."""
    import torch
    from gobeansdb_amd import _lib, batch
    sizes = [4000, 20000, 70000, 16000]
    plain = [O.gen_text(3, i, n) for i, n in enumerate(sizes)]
    comp = [O.compress(p) for p in plain]
    src = batch.BlockBatch.from_bytes(comp)
    for md in (16384, 65536):
        out = batch.BlockBatch.empty_for(sizes)
        dsz, st, _ = batch.decompress(src, out, max_dsize=md)
        torch.cuda.synchronize()
        st = st.cpu().numpy().tolist()
        assert st == [0 if n <= md else _lib.E_MAX_DSIZE for n in sizes], (md, st)
        got = out.to_bytes(dsz.cpu().numpy())
        for n, p, g, s in zip(sizes, plain, got, st):
            if s == 0:
                assert g == p


@pytest.mark.parametrize("general", [False, True])
@pytest.mark.parametrize("with_cap", [False, True])
def test_max_dsize_above_fast_limit(cuda, general, with_cap):
    """max_dsize above the fast-path limit: blocks over 64 KiB take the general kernel, which
    must also refuse a block whose dsize exceeds max_dsize (QLZX_E_MAX_DSIZE, nothing written),
    with and without dst_cap, and with no workspace at all (general=True)."""
    import torch
    from gobeansdb_amd import _lib, batch
    md = 100000
    sizes = [200000, 90000, 16000, 100000]
    plain = [O.gen_text(4, i, n) for i, n in enumerate(sizes)]
    comp = [O.compress(p) for p in plain]
    src = batch.BlockBatch.from_bytes(comp)
    out_sizes = [min(n, md) for n in sizes]   # destinations sized by max_dsize
    out = batch.BlockBatch.empty_for(out_sizes)
    guard = out.data.clone()
    cap = torch.tensor(out_sizes, dtype=torch.int32, device="cuda") if with_cap else None
    dsz, st, _ = batch.decompress(src, out, dst_cap=cap, max_dsize=md, general=general)
    torch.cuda.synchronize()
    st = st.cpu().numpy().tolist()
    # with dst_cap the capacity check comes first (K1's order: cquicklz.go:45 sizes by dsize)
    assert st == [_lib.E_DST_CAP if with_cap else _lib.E_MAX_DSIZE, 0, 0, 0], st
    got = out.to_bytes(dsz.cpu().numpy())
    for p, g, s in zip(plain, got, st):
        if s == 0:
            assert g == p
    # the refused block's destination is untouched
    o0 = int(out.off[0])
    assert torch.equal(out.data[o0:o0 + out_sizes[0]], guard[o0:o0 + out_sizes[0]])


def test_go_decompress1_error_channel(cuda):
    """A compressed level-1 stream with dsize 0 whose first control word has a match bit: Go
    panics on destination[0]; qlzx_go_decompress1 must report QLZX_GO_ERROR (not 0 == a valid
    empty result) and the Decompress mirror must raise."""
    import struct
    from gobeansdb_amd import _lib
    from gobeansdb_amd.quicklz import Decompress, QuicklzError
    L = _lib.lib()
    for cw, want in ((0x80000001, _lib.E_CORRUPT), (0x80000000, _lib.OK)):
        s = bytes([0x47]) + struct.pack("<II", 17, 0) + struct.pack("<I", cw) + bytes([0, 1, 2, 3])
        assert O.decompress_go_l1(s)[0] == want
        dst = ctypes.create_string_buffer(1)
        r = L.qlzx_go_decompress1(s, len(s), dst, 0)
        if want == _lib.OK:
            assert r == 0 and L.qlzx_last_status() == _lib.OK
            assert Decompress(s) == b""
        else:
            assert r == _lib.GO_ERROR and L.qlzx_last_status() == want
            with pytest.raises(QuicklzError):
                Decompress(s)


def test_decompress_inflated_header_csize_decodes_like_go(cuda):
    """Go's Decompress never reads SizeCompressed (quicklz.go:291-431): a valid stream whose header
    csize is larger than the buffer decodes, and one whose tokens run past the buffer panics.
    The mirror bounds the decoder by len(s) (the header is rewritten), pinned by the oracle on
    the same rewritten stream."""
    import struct
    from gobeansdb_amd.quicklz import Decompress, QuicklzError
    for n in (100, 5000, 70000):
        v = O.gen_text(31, n, n)
        c = O.compress(v)
        assert c[0] & 1
        hdr = 9 if c[0] & 2 else 3
        if hdr == 9:
            inflated = c[:1] + struct.pack("<I", len(c) + 1000) + c[5:]
        else:
            inflated = c[:1] + bytes([min(255, len(c) + 50)]) + c[2:]
        assert O.decompress(c)[1] == v  # the oracle on the stream bounded by its length
        assert Decompress(inflated) == v
        cut = inflated[:len(c) - 7]  # tokens run past the buffer: Go panics
        with pytest.raises(QuicklzError):
            Decompress(cut)


def test_decompress_deflated_header_csize_decodes_like_go(cuda):
    """The other direction: a valid stream whose header csize is SMALLER than the
    buffer its tokens use.  Go never reads the field, so it decodes; the mirror rewrites csize to
    len(s) and decodes the same bytes.  A stream with bytes after its last item is the one
    documented difference (check C5 rejects it; Go ignores them)."""
    import struct
    from gobeansdb_amd.quicklz import Decompress, QuicklzError
    for n in (100, 5000, 70000):
        v = O.gen_text(37, n, n)
        c = O.compress(v)
        assert c[0] & 1
        if c[0] & 2:
            small = c[:1] + struct.pack("<I", len(c) - 5) + c[5:]
        else:
            small = c[:1] + bytes([len(c) - 5]) + c[2:]
        assert Decompress(small) == v
        with pytest.raises(QuicklzError):
            Decompress(c + b"\0\0\0")  # trailing bytes after the last item: C5


def test_crc32_write_drop_in_every_length_to_600(cuda):
    """crc32_write (store/crc32.go:61-68, a raw table update with no inversions) at every length
    0..600 -- slices up to the library's host threshold (256 B) and the request path above it --
    from several states, and chained over header[4:24] | key | value as readRecordAt does
    (store/datafile.go:161-168): equal to the oracle's."""
    from gobeansdb_amd import _lib
    L = _lib.lib()
    rng = np.random.default_rng(600)
    data = rng.integers(0, 256, 600, dtype=np.uint8).tobytes()
    for n in range(0, 601):
        for s0 in (0xFFFFFFFF, 0, 0x12345678):
            assert L.crc32_write(s0, data[:n], n) == O.crc32_write(s0, data[:n]), (n, s0)
    for klen, vlen in ((20, 4000), (250, 256), (3, 257), (100, 16384)):
        hdr, key, val = data[:20], data[20:20 + klen], O.gen_text(5, vlen, vlen)
        st = 0xFFFFFFFF
        for part in (hdr, key, val):
            st = L.crc32_write(st, part, len(part))
        assert st ^ 0xFFFFFFFF == O.record_crc(hdr, key, val)
