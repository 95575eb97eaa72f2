"""CPU check of the stored-block proof used by the workgroup encoder (csrc/qlzx_encode_wg.hip,
stored_proof): whenever its two inequalities hold for D = number of positions whose 3-gram
repeats an earlier one, the oracle (pinned to quicklz.c) emits a stored block.  Brute force
over random and near-random inputs, including sizes where the bound is tight."""
import numpy as np

from oracle import oracle as O


def _proof(n, D):
    T = 3 * (n >> 2)
    return 2 * D + 31 + T + 11 <= n and 70 * D < 4 * (T + 1) + 31 * ((T + 1) >> 5)


def _repeats(b):
    seen, D = set(), 0
    for y in range(len(b) - 2):
        g = b[y:y + 3]
        D += g in seen
        seen.add(g)
    return D


def test_stored_proof_implies_stored():
    rng = np.random.default_rng(3)
    fired = 0
    for n in (256, 300, 1000, 4096, 20000):
        for trial in range(12):
            a = rng.integers(0, 256, n, dtype=np.uint8)
            # sprinkle copies so D approaches the bound from below
            for _ in range(trial * (n // 512)):
                L = int(rng.integers(3, 12))
                s, d = int(rng.integers(0, n - L)), int(rng.integers(0, n - L))
                a[d:d + L] = a[s:s + L]
            b = a.tobytes()
            if _proof(n, _repeats(b)):
                fired += 1
                assert O.compress(b)[0] & 1 == 0, (n, trial)   # stored (header bit C = 0)
    assert fired > 20


def test_stored_proof_rejects_small_and_compressible():
    assert not _proof(100, 0)          # no control word past 3n/4 inside the main loop
    assert not _proof(65536, 4000)
    assert _proof(65536, 3000)
