"""cleisthenes_amd -- MI355X-native Reliable Broadcast data path.

Drop-in for joomanzi/cleisthenes' rbc package data path (rbc/rbc.go:86-100:
shard / validateMessage / interpolate, and the klauspost reedsolomon.Encoder
held at rbc/rbc.go:20), served by hand-written gfx950 HIP kernels through the
C ABI in include/rbc_gpu.h.  This Python package is a thin host binding
(tests, bench, tooling); the Go side binds the same C ABI through cgo
(INTEGRATION.md).
"""
from .rbc import (  # noqa: F401
    Batcher,
    Context,
    DeviceBuffer,
    Encoder,
    RBCError,
    Stream,
    Event,
    device_count,
    pinned_empty,
)

__all__ = ["Batcher", "Context", "DeviceBuffer", "Encoder", "RBCError", "Stream", "Event", "device_count", "pinned_empty"]
