"""GPU: the request service under concurrent callers (qlzx_service.hip).

The single-call drop-ins (qlz_decompress, qlz_compress, crc32_write) of values up to 64 KiB go
through a pinned slot arena and a leader that coalesces the calls in flight into one launch.
Sixteen threads call all three at once (ctypes releases the GIL for the foreign call), on
values of many sizes and kinds, and every result must equal the oracle's: a slot or a batch
index mixed up between callers would show as another caller's bytes.
"""
import ctypes
import os
import threading

# arms qlzx_service_test_fault (read once by the library, at its first call)
os.environ.setdefault("QLZX_TEST_HOOKS", "1")

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _values():
    rng = np.random.default_rng(44)
    vals = []
    for i, n in enumerate([1, 2, 9, 100, 215, 216, 300, 1000, 4095, 4096, 5000, 12000, 16384, 16385,
                           30000, 40000, 65535, 65536]):
        vals.append(O.gen_text(100 + i, n, n))
        vals.append(rng.integers(0, 256, n, dtype=np.uint8).tobytes())
        a = np.frombuffer(O.gen_text(200 + i, n, n), np.uint8).copy()
        hit = rng.random(n) < 0.3
        a[hit] = rng.integers(0, 256, int(hit.sum()), dtype=np.uint8)
        vals.append(a.tobytes())
    return vals


def test_service_concurrent_callers(cuda):
    from gobeansdb_amd import _lib
    L = _lib.lib()
    vals = _values()
    comp = [O.compress(v) for v in vals]
    crcs = [O.crc32_write(0x1234567 * (i + 1) & 0xFFFFFFFF, v) for i, v in enumerate(vals)]
    errors = []

    def worker(seed):
        rng = np.random.default_rng(seed)
        try:
            for _ in range(120):
                i = int(rng.integers(0, len(vals)))
                v, c = vals[i], comp[i]
                op = int(rng.integers(0, 3))
                if op == 0:
                    out = ctypes.create_string_buffer(len(v) + 1)
                    n = L.qlz_decompress(c, out, None)
                    if n != len(v) or out.raw[:n] != v:
                        errors.append(("decompress", i, n))
                elif op == 1:
                    dst = ctypes.create_string_buffer(len(v) + 400)
                    n = L.qlz_compress(v, dst, len(v), None)
                    if dst.raw[:n] != c:
                        errors.append(("compress", i, n))
                else:
                    r = L.crc32_write(0x1234567 * (i + 1) & 0xFFFFFFFF, v, len(v))
                    if r != crcs[i]:
                        errors.append(("crc32_write", i, r))
        except Exception as e:  # noqa: BLE001 -- reported below with the thread's seed
            errors.append(("exception", seed, repr(e)))

    threads = [threading.Thread(target=worker, args=(s,)) for s in range(16)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=240)
    assert not any(t.is_alive() for t in threads), "a caller did not return"
    assert errors == [], errors[:5]


@pytest.mark.parametrize("mode,msg", [(1, "ended without completing"), (2, "injected failure")])
def test_service_batch_failure_is_reported(cuda, mode, msg):
    """A batch whose kernel runs but publishes nothing (mode 1, caught through the batch event)
    or whose launch fails (mode 2) fails its request with QLZX_R_HIP instead of leaving the
    caller spinning; the next request is served normally (no slot or event left behind)."""
    from gobeansdb_amd import _lib
    L = _lib.lib()
    v = O.gen_text(7, 0, 3000)
    dst = ctypes.create_string_buffer(len(v) + 400)
    assert L.qlzx_compress1(v, dst, len(v), 0) == len(O.compress(v))  # the service is up
    assert L.qlzx_service_test_fault(mode) == 0
    result = []
    t = threading.Thread(target=lambda: result.append(L.qlzx_compress1(v, dst, len(v), 0)))
    t.start()
    t.join(timeout=60)
    assert not t.is_alive(), "the failed request did not return"
    assert result == [0]
    # qlzx_last_error is per thread: repeat on this thread for the message
    assert L.qlzx_service_test_fault(mode) == 0
    assert L.qlzx_compress1(v, dst, len(v), 0) == 0
    assert msg in L.qlzx_last_error().decode()
    for _ in range(3 * 64):  # more than the slot and event pools: nothing leaked
        n = L.qlzx_compress1(v, dst, len(v), 0)
        assert dst.raw[:n] == O.compress(v)
    assert L.qlzx_service_test_fault(5) != 0


@pytest.mark.parametrize("mode", [3, 4])
def test_batch_launch_failure_is_returned(cuda, mode):
    """qlzx_decompress_batch returns QLZX_R_HIP when its K1 (mode 3) or K2 (mode 4) launch fails
    (the split build's launch helpers report through their return value), and the next call on
    the same workspace decodes normally."""
    import torch
    from gobeansdb_amd import _lib, batch
    L = _lib.lib()
    lens = [16384] * 3000
    plain = batch.synth("text", 11, lens)
    comp, cs, st, _ = batch.compress(plain, max_len=16384)
    torch.cuda.synchronize()
    src = batch.BlockBatch(comp.data, comp.off, cs)
    out = batch.BlockBatch.empty_for(lens)
    ws = batch.Workspace(torch.device("cuda"))
    assert L.qlzx_service_test_fault(mode) == 0
    with pytest.raises(_lib.QlzxError, match="decode_wave launch"):
        batch.decompress(src, out, max_dsize=16384, workspace=ws)
    torch.cuda.synchronize()
    dsz, st, _ = batch.decompress(src, out, max_dsize=16384, workspace=ws)
    torch.cuda.synchronize()
    assert int((st != 0).sum()) == 0
    assert torch.equal(out.data, plain.data)
