"""GPU parity of the position-parallel workgroup encoder (k_encode_wg, csrc/qlzx_encode_wg.hip).

Every output is compared byte for byte with the oracle (oracle/qlz_oracle.c, itself pinned to
the reference quicklz.c by tests/golden) and the fused CRC with zlib.crc32 of the output.  The
cases aim at the places where a position-parallel restatement of quicklz.c:197-494 could drift
from the serial loop:
  * hash-counter wrap at 256 insertions and the 16-slot ring (zero runs: one bucket for all)
  * ties between equal-length candidates (small alphabets; quicklz.c:344 prefers the larger o)
  * same-bucket positions inside one 64-position batch (periodic data)
  * matches that jump over whole 64-position walker segments (long runs)
  * the bail-out test at control-word boundaries (noisy text, quicklz.c:218)
  * the stored-block proof on incompressible input (random bytes) and its near misses
  * the 9-byte core minimum, the 3/9-byte header switch at 216 B and all three size classes
"""
import zlib

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu

SIZES = [1, 2, 3, 4, 5, 8, 9, 10, 11, 12, 13, 20, 31, 32, 33, 63, 64, 65, 100, 215, 216, 217, 255, 256,
         257, 300, 1000, 4095, 4096, 4097, 10000, 16383, 16384, 16385, 30000, 65535, 65536]


def _noisy(rng, base: bytes, frac: float) -> bytes:
    a = np.frombuffer(base, np.uint8).copy()
    hit = rng.random(len(a)) < frac
    a[hit] = rng.integers(0, 256, int(hit.sum()), dtype=np.uint8)
    return a.tobytes()


def _patterns(rng, n):
    out = [O.gen_text(5, n, n), O.gen_image(9, n, n), rng.integers(0, 256, n, dtype=np.uint8).tobytes(),
           bytes(n)]
    for per in (1, 2, 3, 4, 5, 7, 64, 300):
        unit = rng.integers(0, 256, per, dtype=np.uint8).tobytes()
        out.append((unit * (n // per + 1))[:n])
    out.append(_noisy(rng, O.gen_text(6, n, n), 0.42))
    out.append(_noisy(rng, O.gen_text(7, n, n), 0.15))
    out.append(rng.integers(0, 3, n, dtype=np.uint8).tobytes())           # many equal-length ties
    out.append(rng.choice(np.frombuffer(b"ab", np.uint8), n).tobytes())
    # random with a repeated stretch: the stored proof must not fire on a compressible tail
    r = bytearray(rng.integers(0, 256, n, dtype=np.uint8).tobytes())
    if n >= 64:
        k = n // 3
        r[n - k:] = r[:k]
    out.append(bytes(r))
    return out


def _gpu_compress(blocks, crc_state=None, **kw):
    import torch
    from gobeansdb_amd import batch
    src = batch.BlockBatch.from_bytes(blocks)
    cs_t = None if crc_state is None else torch.tensor(np.asarray(crc_state, np.uint32).view(np.int32),
                                                       device="cuda")
    dst, csize, status, crc = batch.compress(src, crc_state=cs_t, want_crc=True, **kw)
    torch.cuda.synchronize()
    cs = csize.cpu().numpy().view(np.uint32)
    return dst.to_bytes(cs), status.cpu().numpy(), crc.cpu().numpy().view(np.uint32)


def _check(blocks, crc_state=None, **kw):
    outs, st, crc = _gpu_compress(blocks, crc_state=crc_state, **kw)
    for i, (b, o) in enumerate(zip(blocks, outs)):
        assert st[i] == 0, (i, len(b), st[i])
        exp = O.compress(b)
        assert o == exp, (i, len(b), len(o), len(exp), o[:16].hex(), exp[:16].hex())
        s = 0xFFFFFFFF if crc_state is None else crc_state[i]
        assert int(crc[i]) == O.crc32_write(s, o) ^ 0xFFFFFFFF, i
    return outs


@pytest.mark.parametrize("cls", [4096, 16384, 65536])
def test_wg_encoder_matches_oracle(cuda, cls):
    rng = np.random.default_rng(cls)
    blocks = []
    for n in SIZES:
        if n <= cls:
            blocks += _patterns(rng, n)
    _check(blocks, max_len=max(len(b) for b in blocks))


def test_wg_encoder_mixed_batch_and_reuse(cuda):
    """More 64 KiB blocks than persistent workgroups (each one encodes several), mixed sizes,
    empty values and a custom CRC state."""
    rng = np.random.default_rng(11)
    blocks = []
    for k in range(300):
        n = [65536, 65536, 40000, 777, 16384][k % 5]
        kind = k % 4
        if kind == 0:
            blocks.append(O.gen_text(21, k, n))
        elif kind == 1:
            blocks.append(O.gen_image(21, k, n))
        elif kind == 2:
            blocks.append(rng.integers(0, 256, n, dtype=np.uint8).tobytes())
        else:
            blocks.append(_noisy(rng, O.gen_text(22, k, n), 0.3))
    states = [int(x) for x in rng.integers(0, 2**32, len(blocks), dtype=np.uint64)]
    _check(blocks, crc_state=states)
    outs, st, crc = _gpu_compress([b"", b"x" * 300, b""])
    assert list(st) == [7, 0, 7]   # QLZX_E_EMPTY (cquicklz.go:36 panics on an empty value)
    assert outs[1] == O.compress(b"x" * 300)


def test_wg_encoder_round_trip_on_device(cuda):
    """compress -> decompress on the GPU at a larger count (size-independent property)."""
    import torch
    from gobeansdb_amd import batch
    n, bs = 2048, 65536
    plain = batch.synth("image", 77, [bs] * n)
    comp, cs, st, _ = batch.compress(plain, max_len=bs)
    torch.cuda.synchronize()
    assert int((st != 0).sum()) == 0
    src = batch.BlockBatch(comp.data, comp.off, cs)
    out = batch.BlockBatch.empty_for([bs] * n)
    dsz, st2, _ = batch.decompress(src, out, max_dsize=bs)
    torch.cuda.synchronize()
    assert int((st2 != 0).sum()) == 0
    assert torch.equal(out.data, plain.data)
    # spot-check bytes against the oracle
    h = comp.to_bytes(cs)
    for i in (0, 1, 2, 3, 1000, 2047):
        assert h[i] == O.compress(O.gen_image(77, i, bs))



def _copy_block(rng, n, frac):
    """Random bytes with one earlier stretch of frac * n bytes repeated once: few repeated
    3-grams (so the prefix-first pass is tried) but long matches, so the first bail-out test
    past 3/4 of the input may pass and the block takes the full pass after all."""
    a = bytearray(rng.integers(0, 256, n, dtype=np.uint8).tobytes())
    k = int(n * frac)
    a[k:2 * k] = a[:k]
    return bytes(a)


@pytest.mark.parametrize("n", [16384, 40000, 65536])
def test_wg_encoder_prefix_first_pass(cuda, n):
    """The prefix-first pass (phase 4 of k_encode_wg): poorly compressible blocks parse only the
    positions below 3/4 of the input + 1 KiB first and are stored if the first bail-out test
    fails there (quicklz.c:216-219); otherwise the whole block is encoded.  Noise fractions
    around the bail-out boundary and the repeat-count threshold, and blocks whose first test
    passes (long copies) or that never bail, all against the oracle."""
    rng = np.random.default_rng(n + 5)
    blocks = []
    for frac in (0.2, 0.3, 0.35, 0.38, 0.4, 0.42, 0.44, 0.46, 0.5, 0.6):
        for seed in range(3):
            blocks.append(_noisy(rng, O.gen_text(40 + seed, int(frac * 1000), n), frac))
    for frac in (0.1, 0.14, 0.17, 0.2, 0.25):
        blocks.append(_copy_block(rng, n, frac))
    outs = _check(blocks, max_len=65536)
    kinds = [o[0] & 1 for o in outs]  # header bit 0: compressed
    assert 0 < sum(kinds) < len(kinds), kinds  # both stored and compressed outcomes are covered


def test_wg_encoder_unaligned_source_and_destination(cuda):
    """Source and destination offsets off the 16-B grid.  An unaligned source skips the stored
    proof (the block then runs the full parse); an unaligned destination turns off the proof's
    speculative stored copy, so a bail-out after the parse must write the whole stored value
    itself.  Every output equals the oracle and its fused CRC equals zlib's."""
    import torch
    from gobeansdb_amd import batch
    rng = np.random.default_rng(31)
    n = 65536
    blocks = [_noisy(rng, O.gen_text(6, n, n), 0.42), rng.integers(0, 256, n, dtype=np.uint8).tobytes(),
              O.gen_text(5, n, n), _noisy(rng, O.gen_text(8, 30000, 30000), 0.42), O.gen_image(9, n, n),
              _noisy(rng, O.gen_text(10, n, n), 0.42)]
    src_shift = [0, 5, 0, 3, 0, 0]
    dst_shift = [3, 8, 1, 0, 12, 4]
    so, do, tot_s, tot_d = [], [], 0, 0
    for b, ss, ds in zip(blocks, src_shift, dst_shift):
        so.append(tot_s + ss)
        tot_s += ss + len(b) + 256
        do.append(tot_d + ds)
        tot_d += ds + len(b) + 400 + 256
    host = np.zeros(tot_s, np.uint8)
    for o, b in zip(so, blocks):
        host[o:o + len(b)] = np.frombuffer(b, np.uint8)
    lens = torch.tensor(np.asarray([len(b) for b in blocks], np.uint32).view(np.int32), device="cuda")
    src = batch.BlockBatch(torch.from_numpy(host).cuda(), torch.tensor(so, dtype=torch.int64, device="cuda"), lens)
    dst = batch.BlockBatch(torch.zeros(tot_d, dtype=torch.uint8, device="cuda"),
                           torch.tensor(do, dtype=torch.int64, device="cuda"), lens.clone())
    _, cs, st, crc = batch.compress(src, dst, want_crc=True, max_len=n)
    torch.cuda.synchronize()
    assert st.cpu().numpy().tolist() == [0] * len(blocks)
    outs = dst.to_bytes(cs.cpu().numpy())
    crc = crc.cpu().numpy().view(np.uint32)
    for i, (b, o) in enumerate(zip(blocks, outs)):
        assert o == O.compress(b), i
        assert int(crc[i]) == zlib.crc32(o), i
    stored = [o[0] & 1 == 0 for o in outs]
    assert stored[1] and not stored[2]  # the random block is stored, the text block is not
