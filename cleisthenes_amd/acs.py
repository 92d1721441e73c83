"""Multi-GPU partitioning of independent RBC instances and ACS output-set
assembly (BASELINE north_star (5)).

RBC instances (proposer x epoch) are independent, so they are partitioned
over the GPUs of a node in contiguous blocks (rank r owns
[r*total/G, (r+1)*total/G)) with no data-path collective.  The one exchange
step is the ACS output set: every rank all-gathers its per-instance
{root[32], digest[32]} records over xGMI (RCCL, rbc_dev_allgather_records;
ragged shares padded to max_share slots, a failed instance carries a zero
digest) and assembles the ordered set -- the part of ACS (absent in the
reference: honeybadger.go:19-21 TODO, sendBatch panics at
honeybadger.go:57-59) that consumes RBC outputs.

The functions here are thin bindings of the C ABI (rbc_acs_*, host code in
librbc_gpu.so, callable without a GPU), so a Go or C++ host gets the same
assembly through cgo.
"""
from __future__ import annotations

from ctypes import byref, c_int
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from ._lib import check, lib

RECORD = 64  # root[32] || digest[32]


def partition(total: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous block of instance ids for `rank`: (first, count)."""
    first, count = c_int(0), c_int(0)
    rc = lib.rbc_acs_partition(total, world, rank, byref(first), byref(count))
    if rc:
        raise ValueError("bad partition arguments")
    return first.value, count.value


def max_share(total: int, world: int) -> int:
    """Per-rank slot count of the all-gather buffer (ranks pad to it)."""
    s = c_int(0)
    check(lib.rbc_acs_max_share(total, world, byref(s)), "rbc_acs_max_share")
    return s.value


def pack_records(roots: np.ndarray, digests: np.ndarray, slots: int,
                 status: Optional[Sequence[int]] = None) -> np.ndarray:
    """[count][32] + [count][32] -> [slots][64], zero padded, zero digest
    where status != 0: the host mirror of rbc_dev_allgather_records' device
    packing (used to check the gathered bytes)."""
    count = roots.shape[0]
    out = np.zeros((slots, RECORD), dtype=np.uint8)
    out[:count, :32] = roots
    out[:count, 32:] = digests
    if status is not None:
        out[:count][np.asarray(status) != 0, 32:] = 0
    return out


def assemble_output_set(gathered: np.ndarray, total: int, world: int) -> List[Dict]:
    """gathered: [world][slots][64] all-gathered records -> the ordered ACS set
    [{instance, root, digest}] of every instance id 0..total-1 whose
    interpolate succeeded (non-zero digest), via rbc_acs_assemble."""
    g = np.ascontiguousarray(gathered, dtype=np.uint8)
    slots = g.shape[1] if g.ndim == 3 else 0
    ids = np.zeros(max(total, 1), dtype=np.int32)
    recs = np.zeros((max(total, 1), RECORD), dtype=np.uint8)
    m = c_int(0)
    rc = lib.rbc_acs_assemble(g.ctypes.data if g.size else None, world, slots, total, ids.ctypes.data,
                              recs.ctypes.data, byref(m))
    if rc:
        raise ValueError("gather buffer does not match the partition")
    return [{"instance": int(ids[t]), "root": bytes(recs[t, :32]), "digest": bytes(recs[t, 32:])}
            for t in range(m.value)]
