"""GPU parity for values far above 64 KiB, up to BodyMax (50 MiB, config/mc_config.go:8):
the whole-GPU encoder (qlzx_encode_huge.hip) and decoder (qlzx_decode_huge.hip, k_dec_lane8 without
a workspace) against the oracle, including long literal runs (the byte-serial loop of k_dec_lane8) and corrupted
streams of such values.  Offsets >= 131071 (quicklz.c:361 falls back to literals) occur at
these sizes."""
import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu

MIB = 1 << 20


def _noisy(seed: int, n: int, p: float) -> bytes:
    """Text with a fraction p of bytes replaced by random ones: compressed blocks full of
    literal runs (compressible enough to stay compressed at p ~ 0.3)."""
    t = np.frombuffer(O.gen_text(seed, 1, n), np.uint8).copy()
    rng = np.random.default_rng(seed)
    m = rng.random(n) < p
    t[m] = rng.integers(0, 256, int(m.sum()), dtype=np.uint8)
    return t.tobytes()


def _values():
    return {
        "text_1MiB": O.gen_text(21, 0, 1 * MIB),
        "noisy_8MiB": _noisy(22, 8 * MIB, 0.3),
        "mixed_50MiB": O.gen_text(23, 0, 20 * MIB) + bytes(10 * MIB) + _noisy(24, 20 * MIB, 0.25),
    }


@pytest.fixture(scope="module")
def large():
    vals = _values()
    return {k: (v, O.compress(v)) for k, v in vals.items()}


def test_large_decode_matches_oracle(cuda, large):
    """Oracle-compressed values through k_dec_lane8 (and the batch API's max_dsize routing)."""
    import torch
    from gobeansdb_amd import batch
    names = list(large)
    comp = [large[k][1] for k in names]
    src = batch.BlockBatch.from_bytes(comp)
    sizes = [len(large[k][0]) for k in names]
    out = batch.BlockBatch.empty_for(sizes)
    dsz, st, crc = batch.decompress(src, out, max_dsize=max(sizes), want_crc=True,
                                    crc_state=torch.full((len(names),), -1, dtype=torch.int32, device="cuda"))
    torch.cuda.synchronize()
    assert st.cpu().numpy().tolist() == [0] * len(names)
    got = out.to_bytes(dsz.cpu().numpy())
    for k, g in zip(names, got):
        assert g == large[k][0], k
    # fused record CRC over the compressed value == CRC of the compressed bytes
    for k, c in zip(names, crc.cpu().numpy().view(np.uint32)):
        assert int(c) == O.crc32_write(0xFFFFFFFF, large[k][1]) ^ 0xFFFFFFFF, k


def test_large_encode_matches_oracle(cuda, large):
    """The whole-GPU encoder's output bytes == the oracle (== reference quicklz.c) for 1, 8 and
    50 MiB values."""
    import torch
    from gobeansdb_amd import batch
    names = ["text_1MiB", "noisy_8MiB", "mixed_50MiB"]
    src = batch.BlockBatch.from_bytes([large[k][0] for k in names])
    dst, cs, st, _ = batch.compress(src, max_len=max(len(large[k][0]) for k in names))
    torch.cuda.synchronize()
    assert st.cpu().numpy().tolist() == [0] * len(names)
    outs = dst.to_bytes(cs.cpu().numpy())
    for k, o in zip(names, outs):
        assert o == large[k][1], k


def test_large_corrupt_status_matches_oracle(cuda, large):
    """Corrupted control words, tokens and literal bytes, and truncations, of the 1 MiB and
    8 MiB streams: the GPU status (and output when OK) equals the oracle's."""
    import torch
    from gobeansdb_amd import batch
    rng = np.random.default_rng(7)
    cases = []
    for k in ("text_1MiB", "noisy_8MiB"):
        c = large[k][1]
        for _ in range(6):
            b = bytearray(c)
            pos = int(rng.integers(9, len(b)))
            b[pos] ^= int(rng.integers(1, 256))
            cases.append(bytes(b))
        b = bytearray(c)
        b[-1] ^= 0x5A                    # last literal byte
        cases.append(bytes(b))
        cases.append(c[: len(c) // 2])   # truncated: csize mismatch
    caps = [len(large["noisy_8MiB"][0])] * len(cases)
    src = batch.BlockBatch.from_bytes(cases)
    out = batch.BlockBatch.empty_for(caps)
    cap_t = torch.tensor(np.asarray(caps, np.uint32).view(np.int32), device="cuda")
    dsz, st, _ = batch.decompress(src, out, dst_cap=cap_t, max_dsize=max(caps))
    torch.cuda.synchronize()
    st = st.cpu().numpy()
    got = out.to_bytes(dsz.cpu().numpy())
    for c, cap, s, g in zip(cases, caps, st, got):
        ost, od = O.decompress(c, cap=cap)
        assert int(s) == ost
        if ost == 0:
            assert g == od


def test_large_values_mixed_with_small_and_record_crc(cuda, large):
    """Large values (the whole-GPU decoder, qlzx_decode_huge.hip) in one batch with 4-64 KiB
    values (K1/K2) and a stored large value, with the fused record-CRC verify: a wrong expected
    CRC on a large value gives QLZX_E_CRC and writes nothing (store/datafile.go:161-168)."""
    import torch
    from gobeansdb_amd import batch, _lib
    big = large["text_1MiB"]
    stored_plain = np.random.default_rng(3).integers(0, 256, 300_000, dtype=np.uint8).tobytes()
    stored = O.compress(stored_plain)
    assert not stored[0] & 1
    plains = [O.gen_text(31, 0, 16384), big[0], O.gen_text(31, 1, 4096), stored_plain, big[0],
              O.gen_text(31, 2, 65536)]
    comps = [O.compress(p) if p is not big[0] else big[1] for p in plains]
    comps[3] = stored
    src = batch.BlockBatch.from_bytes(comps)
    out = batch.BlockBatch.empty_for([len(p) for p in plains])
    exp = [O.crc32_write(0xFFFFFFFF, c) ^ 0xFFFFFFFF for c in comps]
    exp[4] ^= 1  # the second copy of the large value: a record whose CRC does not match
    crc_expect = torch.tensor(np.asarray(exp, np.uint32).view(np.int32), device="cuda")
    dsz, st, crc = batch.decompress(src, out, max_dsize=max(len(p) for p in plains), want_crc=True,
                                    crc_state=torch.full((len(plains),), -1, dtype=torch.int32, device="cuda"),
                                    crc_expect=crc_expect)
    torch.cuda.synchronize()
    st = st.cpu().numpy().tolist()
    assert st == [0, 0, 0, 0, _lib.E_CRC, 0], st
    dz = dsz.cpu().numpy()
    assert int(dz[4]) == 0
    got = out.to_bytes(dz)
    for k in (0, 1, 2, 3, 5):
        assert got[k] == plains[k], k
    c = crc.cpu().numpy().view(np.uint32)
    assert [int(x) for x in c] == [O.crc32_write(0xFFFFFFFF, x) ^ 0xFFFFFFFF for x in comps]


def test_large_all_literal_and_periodic(cuda):
    """Large values whose groups are all literals (no shortcut needed beyond the sentinel) or all
    long matches (deep pointer-jumping chains: a period-3 pattern), against the oracle."""
    import torch
    from gobeansdb_amd import batch
    rng = np.random.default_rng(11)
    lit = (rng.integers(0, 256, 200_000, dtype=np.uint8) & 0x3F).tobytes()  # barely compressible
    per = np.resize(np.frombuffer(b"xyz", np.uint8), 3 * MIB + 7).tobytes()
    plains = [lit, per, O.gen_text(5, 0, 65537)]
    comps = [O.compress(p) for p in plains]
    src = batch.BlockBatch.from_bytes(comps)
    out = batch.BlockBatch.empty_for([len(p) for p in plains])
    dsz, st, _ = batch.decompress(src, out, max_dsize=max(len(p) for p in plains))
    torch.cuda.synchronize()
    assert st.cpu().numpy().tolist() == [0, 0, 0]
    assert out.to_bytes(dsz.cpu().numpy()) == plains


def _encode_cases():
    rng = np.random.default_rng(31)
    return {
        "zeros_300K": bytes(300_000),  # one bucket: hash_counter wraps every 256 positions (quicklz.c:316)
        "period7_200K": (bytes(range(7)) * 40_000)[:200_000],
        "random_100K": rng.integers(0, 256, 100_000, dtype=np.uint8).tobytes(),  # bails out: stored
        "low6_150K": (rng.integers(0, 256, 150_000, dtype=np.uint8) & 0x3F).tobytes(),
        "text_65537": O.gen_text(32, 0, 65537),
        "text_70000": O.gen_text(33, 1, 70_000),
        "noisy_3M": _noisy(34, 3 * MIB, 0.5),
        "text_zero_text_2M": O.gen_text(35, 2, MIB) + bytes(50_000) + O.gen_text(35, 3, MIB),
    }


def test_large_encode_edge_cases_match_oracle(cuda):
    """The whole-GPU encoder (qlzx_encode_huge.hip) on values just past 64 KiB, one-bucket data
    (the hash counter's byte wrap), periodic and barely compressible data, a value that bails out
    to stored, mixed with a small block in one batch; bytes == oracle/qlz_oracle.c (pinned to
    quicklz.c), fused CRC of the output == crc32_write."""
    import torch
    from gobeansdb_amd import batch
    cases = _encode_cases()
    names = list(cases) + ["small"]
    plains = [cases[k] for k in cases] + [O.gen_text(36, 0, 5000)]
    src = batch.BlockBatch.from_bytes(plains)
    dst, cs, st, crc = batch.compress(src, max_len=max(map(len, plains)),
                                      crc_state=torch.full((len(plains),), -1, dtype=torch.int32, device="cuda"))
    torch.cuda.synchronize()
    assert st.cpu().numpy().tolist() == [0] * len(plains)
    outs = dst.to_bytes(cs.cpu().numpy())
    for k, p, o, c in zip(names, plains, outs, crc.cpu().numpy().view(np.uint32)):
        want = O.compress(p)
        assert o == want, (k, len(o), len(want))
        assert int(c) == O.crc32_write(0xFFFFFFFF, want) ^ 0xFFFFFFFF, k
    assert outs[names.index("random_100K")][0] & 1 == 0  # stored


def test_large_encode_go_compat_matches_oracle(cuda):
    """QLZX_F_GO_COMPAT (Go quicklz.Compress, quicklz.go:80-289: the bail-out counts the header)
    through the whole-GPU encoder == oracle compress_go."""
    import torch
    from gobeansdb_amd import batch
    plains = [O.gen_text(37, 0, 90_000), bytes(200_000), _noisy(38, 400_000, 0.45)]
    src = batch.BlockBatch.from_bytes(plains)
    dst, cs, st, _ = batch.compress(src, go_compat=True, max_len=max(map(len, plains)))
    torch.cuda.synchronize()
    assert st.cpu().numpy().tolist() == [0] * len(plains)
    for p, o in zip(plains, dst.to_bytes(cs.cpu().numpy())):
        assert o == O.compress_go(p)


def test_large_single_call_compress(cuda):
    """qlz_compress on a 6 MiB value (the per-call path over the batch encoder) == the oracle."""
    import ctypes
    from gobeansdb_amd import _lib
    L = _lib.lib()
    p = O.gen_text(39, 0, 6 * MIB)
    out = ctypes.create_string_buffer(len(p) + 400)
    n = L.qlz_compress(p, out, len(p), None)
    assert out.raw[:n] == O.compress(p)
