#!/usr/bin/env python3
"""Raw pinned host<->device copy bandwidth (hipMemcpy through the C ABI), the
ceiling of the PCIe-inclusive host path (bench.py's pcie_inclusive key)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cleisthenes_amd as ca  # noqa: E402


def main():
    out = {}
    for mb in (64, 256, 1024):
        n = mb << 20
        h = ca.pinned_empty(n)
        h[:] = 7
        d = ca.DeviceBuffer(n)
        d.upload(h)
        for name, fn in (("h2d", lambda: d.upload(h)), ("d2h", lambda: ca.rbc.lib.rbc_memcpy_d2h(
                ca.rbc._ptr(h), d.ptr, n))):
            fn()
            t0 = time.perf_counter()
            reps = 5
            for _ in range(reps):
                fn()
            dt = time.perf_counter() - t0
            out[f"{name}_{mb}MiB_GBps"] = round(n * reps / dt / 1e9, 2)
    # 2D copies of shard rows (the host batch API's direct path): rows of
    # S = 23832 bytes (C2) between a device pitch and a host pitch
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so.7")
    hip.hipMemcpy2D.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t,
                                ctypes.c_size_t, ctypes.c_size_t, ctypes.c_int]
    S, rows = 23832, 64 * 128
    for dp, hp in ((23936, 23832), (23936, 23936), (23832, 23832)):
        h = ca.pinned_empty(rows * hp)
        d = ca.DeviceBuffer(rows * dp)
        for kind, name in ((1, "h2d"), (2, "d2h")):
            args = ((d.ptr.value, dp, h.ctypes.data, hp) if kind == 1 else (h.ctypes.data, hp, d.ptr.value, dp))
            assert hip.hipMemcpy2D(args[0], args[1], args[2], args[3], S, rows, kind) == 0
            t0 = time.perf_counter()
            for _ in range(5):
                hip.hipMemcpy2D(args[0], args[1], args[2], args[3], S, rows, kind)
            dt = time.perf_counter() - t0
            out[f"{name}_2d_dev{dp}_host{hp}_GBps"] = round(S * rows * 5 / dt / 1e9, 2)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
