"""GPU parity at the BASELINE block shapes against the oracle (pinned to the reference
quicklz.c by tests/golden): c2-shaped 16 KiB text blocks, c3-shaped 64 KiB image-like blocks
and c5-shaped mixed 4-64 KiB values, a few thousand each.  Compressed bytes must equal the
oracle's; decompressing the oracle's streams (every K2 kernel) must give the inputs back."""
import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _sizes(kind, n, rng):
    if kind == "mixed":
        return [int(np.exp(rng.uniform(np.log(4096), np.log(65536)))) for _ in range(n)]
    return [16384 if kind == "text" else 65536] * n


@pytest.mark.parametrize("kind,n", [("text", 2048), ("image", 512), ("mixed", 1024)])
def test_compress_bytes_equal_oracle(cuda, kind, n):
    import torch
    from gobeansdb_amd import batch
    rng = np.random.default_rng(len(kind))
    lens = _sizes(kind, n, rng)
    synth_kind = "image" if kind == "image" else "text"
    plain = batch.synth(synth_kind, 99, lens, first_id=5000)
    dst, cs, st, _ = batch.compress(plain, max_len=max(lens))
    torch.cuda.synchronize()
    assert st.cpu().numpy().tolist() == [0] * n
    got = dst.to_bytes(cs.cpu().numpy())
    gen = O.gen_image if synth_kind == "image" else O.gen_text
    for i, (g, ln) in enumerate(zip(got, lens)):
        assert g == O.compress(gen(99, 5000 + i, ln)), (kind, i, ln)


@pytest.mark.parametrize("kind,n", [("text", 2048), ("mixed", 1024)])
def test_decompress_oracle_streams(cuda, kind, n):
    import torch
    from gobeansdb_amd import batch
    rng = np.random.default_rng(7 + len(kind))
    lens = _sizes(kind, n, rng)
    plains = [O.gen_text(123, 9000 + i, ln) for i, ln in enumerate(lens)]
    src = batch.BlockBatch.from_bytes([O.compress(p) for p in plains])
    out = batch.BlockBatch.empty_for(lens)
    dsz, st, _ = batch.decompress(src, out, max_dsize=max(lens))
    torch.cuda.synchronize()
    assert st.cpu().numpy().tolist() == [0] * n
    assert out.to_bytes(dsz.cpu().numpy()) == plains
