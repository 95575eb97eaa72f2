"""GPU: reference-held vectors pinned through the C ABI (What's missing #5).

* Getvhash (store/item.go:89-100) over the buggy sign-extending Fnv1a (utils/hash.go:8-16):
  qlzx_vhash_batch against the reference KAT Fnv1a("test") == 2949673445
  (store/htree_test.go:18-23) and against oracle/replay.getvhash on values at and around the
  1024-byte switch, with bytes >= 0x80 (the sign-extension).
* BASELINE configs[0]: quicklz/quicklz_test.go:27-34 (CCompress -> CDecompressSafe round trip)
  at 1,024 x 4 KiB text values through the Go-API mirror, the compressed bytes equal to the
  reference-pinned oracle's.
"""
import numpy as np
import pytest
import torch

from oracle import oracle as O
from oracle import replay as R

pytestmark = pytest.mark.gpu


def _vhash_gpu(values):
    from gobeansdb_amd import _lib, batch
    L = _lib.lib()
    lens = [len(v) for v in values]
    offs = np.zeros(len(values), np.int64)
    offs[1:] = np.cumsum([(n + 255) & ~255 for n in lens])[:-1]
    buf = np.zeros(int(offs[-1]) + max(256, (lens[-1] + 255) & ~255), np.uint8)
    for o, v in zip(offs, values):
        buf[o:o + len(v)] = np.frombuffer(v, np.uint8)
    d = torch.from_numpy(buf).cuda()
    o = torch.from_numpy(offs).cuda()
    n = torch.tensor(lens, dtype=torch.int32).cuda()
    out = torch.zeros(len(values), dtype=torch.int16, device="cuda")
    rc = L.qlzx_vhash_batch(d.data_ptr(), o.data_ptr(), n.data_ptr(), len(values), out.data_ptr(),
                            batch._stream(None))
    _lib.check(rc, "qlzx_vhash_batch")
    torch.cuda.synchronize()
    return [int(x) & 0xFFFF for x in out.cpu().numpy()]


def test_vhash_reference_kat(cuda):
    """Getvhash("test") = (4 * 97 + Fnv1a("test")) mod 2^16 with the reference's own Fnv1a value."""
    want = (4 * 97 + 2949673445) & 0xFFFF
    assert _vhash_gpu([b"test"]) == [want]


def test_vhash_batch_matches_oracle_around_1024(cuda):
    rng = np.random.default_rng(606)
    values = [b"", b"\x80", b"\xff" * 3]
    for n in (1, 7, 511, 512, 513, 1000, 1023, 1024, 1025, 1026, 1535, 1536, 4096, 16384, 65536):
        values.append(rng.integers(0x80, 0x100, n, dtype=np.uint8).tobytes())   # all sign-extended
        values.append(rng.integers(0, 0x100, n, dtype=np.uint8).tobytes())
        values.append(O.gen_text(606, n, n))
    got = _vhash_gpu(values)
    want = [R.getvhash(v) for v in values]
    assert got == want


def test_c1_go_api_round_trip_1k_x_4k(cuda):
    """BASELINE configs[0] (quicklz/quicklz_test.go:27-34 at 1 k x 4 KiB): CCompress then
    CDecompressSafe through the Go-API mirror, every value through the GPU drop-ins."""
    from gobeansdb_amd.quicklz import CCompress, CDecompressSafe, SizeCompressed, SizeDecompressed
    for i in range(1024):
        v = O.gen_text(1, i, 4096)
        c, ok = CCompress(v)
        assert ok
        assert c.Body == O.compress(v), i
        assert SizeDecompressed(c.Body) == 4096 and SizeCompressed(c.Body) == len(c.Body)
        d, err = CDecompressSafe(c.Body)
        assert err is None and d.Body == v, i
