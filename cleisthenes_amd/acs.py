"""Multi-GPU partitioning of independent RBC instances and ACS output-set
assembly (BASELINE north_star (5)).

RBC instances (proposer x epoch) are independent, so they are partitioned
over the GPUs of a node in contiguous blocks (instance i -> GPU
floor(i * G / I)) with no data-path collective.  The one exchange step is the
ACS output set: every rank all-gathers the per-instance {root[32],
digest[32]} records over xGMI (RCCL, rbc_dev_allgather_roots) and assembles
the ordered set -- the part of ACS (absent in the reference, see
honeybadger.go:19-21 and img/cleisthenes-module-view.png) that consumes RBC
outputs.
"""
from __future__ import annotations

from typing import Dict, List, Sequence, Tuple

import numpy as np

RECORD = 64  # root[32] || digest[32]


def partition(total: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous block of instance ids for `rank`: (first, count)."""
    if world < 1 or not (0 <= rank < world) or total < 0:
        raise ValueError("bad partition arguments")
    first = (rank * total) // world
    last = ((rank + 1) * total) // world
    return first, last - first


def max_share(total: int, world: int) -> int:
    """Per-rank slot count of the all-gather buffer (ranks pad to it)."""
    return max(partition(total, world, r)[1] for r in range(world)) if world else 0


def pack_records(roots: np.ndarray, digests: np.ndarray, slots: int) -> np.ndarray:
    """[count][32] + [count][32] -> [slots][64] zero padded (host mirror of
    the device packing done by rbc_dev_allgather_roots)."""
    count = roots.shape[0]
    out = np.zeros((slots, RECORD), dtype=np.uint8)
    out[:count, :32] = roots
    out[:count, 32:] = digests
    return out


def assemble_output_set(gathered: np.ndarray, total: int, world: int,
                        status: Sequence[int] = None) -> List[Dict]:
    """gathered: [world][slots][64] all-gathered records -> ordered ACS set
    [{instance, root, digest}] for every instance id 0..total-1 whose
    interpolate succeeded (status[i] == 0 when a status vector is given)."""
    slots = gathered.shape[1]
    out = []
    for r in range(world):
        first, count = partition(total, world, r)
        if count > slots:
            raise ValueError("gather buffer smaller than a rank's share")
        for t in range(count):
            inst = first + t
            if status is not None and status[inst] != 0:
                continue
            rec = gathered[r, t]
            out.append({"instance": inst, "root": bytes(rec[:32]), "digest": bytes(rec[32:])})
    return out
