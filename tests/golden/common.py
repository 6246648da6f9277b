"""Deterministic input generators shared by the golden script, the tests and
bench.py (so the CPU can regenerate any device-generated buffer).

splitmix64: 64-bit word k (little-endian at byte 8k) of a buffer with seed s
is mix(s + (k + 1) * 0x9E3779B97F4A7C15) -- the same rule the library's
device fill kernel uses (hcrc_fill_splitmix64_async).
"""
from __future__ import annotations

import numpy as np

_GAMMA = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)


def splitmix64_words(seed: int, first_word: int, nwords: int) -> np.ndarray:
    k = np.arange(first_word + 1, first_word + 1 + nwords, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = np.uint64(seed) + k * _GAMMA
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
        z = z ^ (z >> np.uint64(31))
    return z


def splitmix64_bytes(seed: int, nbytes: int, start: int = 0) -> np.ndarray:
    """Bytes [start, start+nbytes) of the seeded stream."""
    w0 = start // 8
    w1 = (start + nbytes + 7) // 8
    words = splitmix64_words(seed, w0, w1 - w0)
    b = words.view(np.uint8)
    s = start - 8 * w0
    return b[s:s + nbytes].copy()
