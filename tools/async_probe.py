#!/usr/bin/env python3
"""Does a HIP copy call return before the copy is done?  Host-side call time
vs completion for hipMemcpyAsync / hipMemcpy2DAsync between device memory and
pinned host memory (the host batch API's direct paths)."""
import ctypes
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cleisthenes_amd as ca  # noqa: E402


def main():
    hip = ctypes.CDLL("libamdhip64.so.7")
    vp, sz = ctypes.c_void_p, ctypes.c_size_t
    hip.hipMemcpyAsync.argtypes = [vp, vp, sz, ctypes.c_int, vp]
    hip.hipMemcpy2DAsync.argtypes = [vp, sz, vp, sz, sz, sz, ctypes.c_int, vp]
    hip.hipStreamSynchronize.argtypes = [vp]
    s = ca.Stream(0)
    S, rows = 23832, 64 * 128
    h = ca.pinned_empty(rows * 23936)
    d = ca.DeviceBuffer(rows * 23936)
    out = {}
    cases = {
        "d2h_1d": lambda: hip.hipMemcpyAsync(h.ctypes.data, d.ptr.value, S * rows, 2, s.ptr),
        "h2d_1d": lambda: hip.hipMemcpyAsync(d.ptr.value, h.ctypes.data, S * rows, 1, s.ptr),
        "d2h_2d_pitch_diff": lambda: hip.hipMemcpy2DAsync(h.ctypes.data, S, d.ptr.value, 23936, S, rows, 2, s.ptr),
        "h2d_2d_pitch_diff": lambda: hip.hipMemcpy2DAsync(d.ptr.value, 23936, h.ctypes.data, S, S, rows, 1, s.ptr),
        "d2h_2d_same_pitch": lambda: hip.hipMemcpy2DAsync(h.ctypes.data, 23936, d.ptr.value, 23936, S, rows, 2,
                                                           s.ptr),
        "h2d_64x1MiB": lambda: [hip.hipMemcpyAsync(d.ptr.value + i * (1 << 20), h.ctypes.data + i * (1 << 20),
                                                   1 << 20, 1, s.ptr) for i in range(64)],
    }
    for name, fn in cases.items():
        fn()
        hip.hipStreamSynchronize(s.ptr)
        t0 = time.perf_counter()
        fn()
        t1 = time.perf_counter()
        hip.hipStreamSynchronize(s.ptr)
        t2 = time.perf_counter()
        out[name] = {"call_ms": round((t1 - t0) * 1e3, 3), "done_ms": round((t2 - t0) * 1e3, 3)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
