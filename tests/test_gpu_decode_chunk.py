"""GPU parity for the byte-parallel K2 (k_dec_chunk4, qlzx_decode_v4.hip) on inputs built to
stress its three mechanisms, against the oracle-compressed stream of the same input:

* in-chunk sources resolved by pointer jumping: periodic data (short periods give chains of
  dozens of bytes inside one 256-B chunk; 255/256/257 straddle the chunk size);
* the 4 KiB LDS window boundary: periods and back-references just below / at / above the
  window size and the window minus a chunk (near vs far source);
* far sources read back from HBM, ragged block ends (dsize not a multiple of 4 or 256) and
  tiny blocks.
"""
import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _periodic(rng, n, period):
    base = rng.integers(0, 256, period, dtype=np.uint8)
    return np.resize(base, n).tobytes()


def _backref(rng, n, dist, seg=64):
    """Text with segments copied from exactly `dist` bytes earlier."""
    text = bytearray(O.gen_text(int(rng.integers(1 << 30)), 0, n))
    p = dist
    while p + seg <= n:
        text[p:p + seg] = text[p - dist:p - dist + seg]
        p += seg + int(rng.integers(seg, 8 * seg))
    return bytes(text)


def _cases():
    rng = np.random.default_rng(17)
    out = []
    for period in (3, 4, 5, 7, 16, 31, 64, 100, 255, 256, 257, 511, 1000):
        out.append(_periodic(rng, 16384 + period, period))
    for dist in (3000, 3583, 3584, 3585, 3600, 4095, 4096, 4097, 7000, 12000, 30000):
        out.append(_backref(rng, 40000 + dist % 977, dist))
    out += [bytes(65536), bytes(16384 + 3), b"a" * 4097, b"ab" * 3000 + b"c"]
    out += [O.gen_text(5, k, n) for k, n in enumerate((1, 2, 3, 5, 9, 13, 64, 255, 256, 257, 1023, 1025,
                                                        4095, 4097, 16383, 16385, 65535, 65536))]
    return out


def test_decode_bytes_stress_round_trip(cuda):
    import torch
    from gobeansdb_amd import batch
    plain = _cases()
    comp = [O.compress(p) for p in plain]
    assert any(c[0] & 1 for c in comp)
    src = batch.BlockBatch.from_bytes(comp)
    out = batch.BlockBatch.empty_for([len(p) for p in plain])
    dsz, st, _ = batch.decompress(src, out, max_dsize=65536)
    torch.cuda.synchronize()
    st = st.cpu().numpy()
    assert (st == 0).all(), [(k, int(s)) for k, s in enumerate(st) if s]
    got = out.to_bytes(dsz.cpu().numpy())
    for k, (p, g) in enumerate(zip(plain, got)):
        assert g == p, (k, len(p))


def test_decode_bytes_unaligned_destinations(cuda):
    """Destinations at every byte alignment (the chunk stores are unaligned dword stores)."""
    import torch
    from gobeansdb_amd import batch
    rng = np.random.default_rng(3)
    plain = [_backref(rng, 20000 + k, 4000 + 37 * k) for k in range(8)]
    comp = [O.compress(p) for p in plain]
    src = batch.BlockBatch.from_bytes(comp)
    lens = [len(p) for p in plain]
    offs = []
    pos = 0
    for k, n in enumerate(lens):
        pos = (pos + 255) // 256 * 256 + k   # alignment k mod 256
        offs.append(pos)
        pos += n
    data = torch.zeros(pos + 64, dtype=torch.uint8, device="cuda")
    out = batch.BlockBatch(data, torch.tensor(offs, dtype=torch.int64, device="cuda"),
                           torch.tensor(lens, dtype=torch.int32, device="cuda"))
    dsz, st, _ = batch.decompress(src, out, max_dsize=65536)
    torch.cuda.synchronize()
    assert (st.cpu().numpy() == 0).all()
    host = data.cpu().numpy().tobytes()
    for o, n, p in zip(offs, lens, plain):
        assert host[o:o + n] == p
    # nothing written between the blocks
    mask = np.ones(len(host), bool)
    for o, n in zip(offs, lens):
        mask[o:o + n] = False
    assert not np.frombuffer(host, np.uint8)[mask].any()
