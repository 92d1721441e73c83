"""Host restatement of the synthetic input the device writes
(rbc_dev_fill_random): 64-bit word w of global row r of a [rows][pitch]
buffer is splitmix64(seed * 0x9E3779B97F4A7C15 + r * pitch / 8 + w),
little-endian.  bench.py fills multi-GiB inputs on the GPU and rebuilds the
few rows it checks against the oracle here, so nothing large crosses PCIe."""
from __future__ import annotations

import numpy as np

GOLDEN = np.uint64(0x9E3779B97F4A7C15)


def splitmix64(z: np.ndarray) -> np.ndarray:
    z = z.astype(np.uint64, copy=True)
    with np.errstate(over="ignore"):
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def row(seed: int, r: int, pitch: int, nbytes: int) -> np.ndarray:
    """The first nbytes of global row r."""
    assert pitch % 16 == 0 and nbytes <= pitch
    words = (nbytes + 7) // 8
    with np.errstate(over="ignore"):
        base = np.uint64(seed) * GOLDEN + np.uint64(r) * np.uint64(pitch // 8)
        z = base + np.arange(words, dtype=np.uint64)
    return splitmix64(z).astype("<u8").view(np.uint8)[:nbytes]
