"""C-ABI boundary checks that need no GPU: the library loads, exports every
function include/rbc_gpu.h declares, and reports status strings; host-only
entry points behave (no compute calls are made here)."""
import ctypes
import subprocess

import numpy as np


def test_library_exports_every_header_symbol():
    from cleisthenes_amd import _lib
    names = _lib.header_functions()
    assert len(names) >= 40
    nm = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True,
                        check=True).stdout
    exported = {line.split()[-1] for line in nm.splitlines() if " T " in line}
    missing = [n for n in names if n not in exported]
    assert not missing, missing
    for n in names:
        assert hasattr(_lib.lib, n)


def test_abi_version_and_strerror():
    from cleisthenes_amd import _lib
    assert _lib.lib.rbc_abi_version() == 7
    assert _lib.lib.rbc_strerror(-3) == b"too few shards given"
    assert _lib.lib.rbc_strerror(-8).startswith(b"interpolated merkle root")
    assert _lib.lib.rbc_strerror(12345) == b"unknown rbc status"


def test_invalid_arguments_rejected_without_gpu():
    from cleisthenes_amd import _lib
    lib = _lib.lib
    p = ctypes.c_void_p()
    # reedsolomon.New argument checks happen before any device call
    assert lib.rbc_rs_new(0, 1, 0, ctypes.byref(p)) == _lib.RBC_ERR_INV_SHARD_NUM
    assert lib.rbc_rs_new(2, -1, 0, ctypes.byref(p)) == _lib.RBC_ERR_INV_SHARD_NUM
    assert lib.rbc_rs_new(200, 57, 0, ctypes.byref(p)) == _lib.RBC_ERR_MAX_SHARD_NUM
    assert lib.rbc_ctx_create(4, 2, 0, ctypes.byref(p)) == _lib.RBC_ERR_INV_SHARD_NUM
    assert lib.rbc_ctx_create(300, 10, 0, ctypes.byref(p)) == _lib.RBC_ERR_MAX_SHARD_NUM
    assert lib.rbc_ctx_create(4, 1, 0, None) == _lib.RBC_ERR_INVALID_ARG
    n = ctypes.c_int(-1)
    assert lib.rbc_device_count(ctypes.byref(n)) == 0 and n.value >= 0


def test_acs_partition_covers_all_instances():
    from cleisthenes_amd import acs
    for total in (0, 1, 7, 8192, 8193):
        for world in (1, 2, 3, 8):
            seen = []
            for r in range(world):
                first, cnt = acs.partition(total, world, r)
                seen.extend(range(first, first + cnt))
            assert seen == list(range(total))
            assert acs.max_share(total, world) == max(acs.partition(total, world, r)[1] for r in range(world))
    g = np.zeros((2, 3, 64), dtype=np.uint8)
    g[0, :2, 0] = [1, 2]
    g[1, :3, 0] = [3, 4, 5]
    g[0, :2, 32] = 1
    g[1, [0, 2], 40] = 9  # instance 3 (rank 1, slot 1) failed: zero digest
    out = acs.assemble_output_set(g, 5, 2)
    assert [o["instance"] for o in out] == [0, 1, 2, 4]
    assert [o["root"][0] for o in out] == [1, 2, 3, 5]
