"""Deterministic synthetic workloads for the QuickLZ hot path.

Host-side tables only: the 3000-word vocabulary and the integer Zipf(α=1)
CDF.  The generators themselves run on the GPU (``qlzx_synth_*`` in
``csrc/qlzx_synth.hip``); the oracle restates them on the CPU
(``oracle/qlz_oracle.c: orc_gen_text / orc_gen_image``) so tests can check
both produce identical bytes.  Spec: DESIGN.md §5.
"""
from __future__ import annotations

import numpy as np

CONSONANTS = b"bcdfghjklmnprstv"   # 16
VOWELS = b"aeiou"                  # 5
NWORDS = 3000
VOCAB_SEED = 0x5EED
MASK64 = (1 << 64) - 1


def _sm64(state: int) -> tuple[int, int]:
    state = (state + 0x9E3779B97F4A7C15) & MASK64
    z = state
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & MASK64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & MASK64
    return state, z ^ (z >> 31)


def block_seed(seed: int, block_id: int) -> int:
    s = (seed ^ (block_id * 0xD1B54A32D192ED03)) & MASK64
    return _sm64(s)[1]


def vocabulary() -> tuple[np.ndarray, np.ndarray]:
    """Return (bytes u8[total], offsets u32[NWORDS+1])."""
    s = VOCAB_SEED
    words = []
    for _ in range(NWORDS):
        s, r = _sm64(s)
        nsyl = 1 + r % 4
        w = bytearray()
        for _ in range(nsyl):
            s, r2 = _sm64(s)
            w.append(CONSONANTS[r2 % 16])
            w.append(VOWELS[(r2 >> 8) % 5])
        words.append(bytes(w))
    off = np.zeros(NWORDS + 1, dtype=np.uint32)
    off[1:] = np.cumsum([len(w) for w in words])
    return np.frombuffer(b"".join(words), dtype=np.uint8).copy(), off


def zipf_cdf(nwords: int = NWORDS) -> np.ndarray:
    """Integer Zipf(1) CDF scaled to 2^32 (exact integer arithmetic)."""
    w = [(1 << 48) // (k + 1) for k in range(nwords)]
    total = sum(w)
    cdf = np.zeros(nwords, dtype=np.uint32)
    acc = 0
    for k in range(nwords):
        acc += w[k]
        cdf[k] = min((acc << 32) // total, 0xFFFFFFFF)
    cdf[-1] = 0xFFFFFFFF
    return cdf


_TABLES = None


def tables():
    global _TABLES
    if _TABLES is None:
        v, o = vocabulary()
        _TABLES = (v, o, zipf_cdf())
    return _TABLES


def key_for(i: int) -> bytes:
    """Record keys: "key_%016x" (20 B), SURVEY.md §8(d)."""
    return b"key_%016x" % i
