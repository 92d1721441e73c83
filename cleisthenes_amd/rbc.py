"""Host binding of the RBC data path (include/rbc_gpu.h), mirroring the
reference's interfaces:

* ``Context.shard(data)``            -> rbc/rbc.go:97-100 ``shard(enc, data)`` (+ Merkle commit, rbc.go:42)
* ``Context.validate_message(...)``  -> rbc/rbc.go:92-95 ``validateMessage(echo)``
* ``Context.interpolate(root, shards)`` -> rbc/rbc.go:86-90 ``interpolate(rootHash, shards)``
* ``Encoder(k, p)``                  -> ``reedsolomon.New`` / ``reedsolomon.Encoder`` (rbc/rbc.go:20)
* ``Context.dev_*``                  -> batched device-resident stages (the Go batcher's path)

Missing shards are ``None`` or empty (Go ``len == 0``); errors raise
``RBCError`` carrying the klauspost v1.9.1 error value as ``code``.
"""
from __future__ import annotations

import ctypes
from ctypes import byref, c_float, c_int, c_size_t, c_uint8, c_uint32, c_uint64, c_void_p
from typing import List, Optional, Sequence

import numpy as np

from . import _lib
from ._lib import RBCError, check, lib

__all__ = ["Context", "Encoder", "DeviceBuffer", "Stream", "Event", "RBCError", "device_count"]


def device_count() -> int:
    n = c_int(0)
    check(lib.rbc_device_count(byref(n)), "rbc_device_count")
    return n.value


def _ptr(a: np.ndarray) -> c_void_p:
    return c_void_p(a.ctypes.data)


def mem_info(device: int = 0) -> tuple:
    """(free, total) device memory in bytes (hipMemGetInfo)."""
    free, total = c_size_t(0), c_size_t(0)
    check(lib.rbc_device_mem_info(device, byref(free), byref(total)), "rbc_device_mem_info")
    return free.value, total.value


def pci_bus_id(device: int) -> str:
    buf = ctypes.create_string_buffer(64)
    check(lib.rbc_device_pci_bus_id(device, buf, 64), "rbc_device_pci_bus_id")
    return buf.value.decode().lower()


def fill_random(device: int, stream, dst, first_row: int, rows: int, pitch: int, seed: int) -> None:
    """Synthetic bytes on the device (cleisthenes_amd.synth restates them)."""
    check(lib.rbc_dev_fill_random(device, _dv(stream), _dv(dst), first_row, rows, pitch, seed),
          "rbc_dev_fill_random")


def count_mismatch(device: int, stream, a, a_pitch: int, b, b_pitch: int, rows: int, length: int, counter) -> None:
    """Device counter <- 16-byte chunks where rows of a and b differ in
    their first `length` bytes (read it after the stream completes)."""
    check(lib.rbc_dev_count_mismatch(device, _dv(stream), _dv(a), a_pitch, _dv(b), b_pitch, rows, length,
                                     _dv(counter)), "rbc_dev_count_mismatch")


def count_mismatch_rows(device: int, stream, shards, inst_pitch: int, row_pitch: int, k: int, shard_len: int,
                        values, value_pitch: int, value_len: int, count: int, counter) -> None:
    """Device counter <- 16-byte chunks where the k data rows of each instance
    (the row-view value of interpolate) differ from its value bytes."""
    check(lib.rbc_dev_count_mismatch_rows(device, _dv(stream), _dv(shards), inst_pitch, row_pitch, k, shard_len,
                                          _dv(values), value_pitch, value_len, count, _dv(counter)),
          "rbc_dev_count_mismatch_rows")


def poison_rows(device: int, stream, shards, inst_pitch: int, row_pitch: int, n: int, present, corrupt, count: int,
                seed: int) -> None:
    """Overwrite every absent row (present == 0) and the corrupt[i] row of
    each instance with seeded garbage over the whole row pitch: the receive
    guard's input, so that only a real regeneration restores them."""
    check(lib.rbc_dev_poison_rows(device, _dv(stream), _dv(shards), inst_pitch, row_pitch, n, _dv(present),
                                  _dv(corrupt), count, seed), "rbc_dev_poison_rows")


def library_path() -> str:
    """The file librbc_gpu.so was actually mapped from (dladdr inside the library)."""
    buf = ctypes.create_string_buffer(4096)
    check(lib.rbc_library_path(buf, 4096), "rbc_library_path")
    return buf.value.decode()


def _bytes_array(x) -> np.ndarray:
    if x is None:
        return np.zeros(0, dtype=np.uint8)
    if isinstance(x, np.ndarray):
        return np.ascontiguousarray(x, dtype=np.uint8)
    return np.frombuffer(bytes(x), dtype=np.uint8)


class DeviceBuffer:
    """A device allocation made by the library (hipMalloc)."""

    def __init__(self, nbytes: int, device: int = 0):
        self.nbytes = int(nbytes)
        self.device = device
        p = c_void_p()
        check(lib.rbc_dev_malloc(device, self.nbytes, byref(p)), "rbc_dev_malloc")
        self.ptr = p

    @property
    def value(self) -> int:
        return self.ptr.value

    def upload(self, a: np.ndarray, offset: int = 0) -> None:
        a = np.ascontiguousarray(a)
        assert offset + a.nbytes <= self.nbytes
        check(lib.rbc_memcpy_h2d(c_void_p(self.ptr.value + offset), _ptr(a), a.nbytes), "h2d")

    def download(self, nbytes: Optional[int] = None, offset: int = 0) -> np.ndarray:
        n = self.nbytes - offset if nbytes is None else nbytes
        out = np.empty(n, dtype=np.uint8)
        check(lib.rbc_memcpy_d2h(_ptr(out), c_void_p(self.ptr.value + offset), n), "d2h")
        return out

    def zero(self) -> None:
        check(lib.rbc_dev_memset(self.ptr, 0, self.nbytes), "memset")

    def free(self) -> None:
        if self.ptr is not None and self.ptr.value:
            lib.rbc_dev_free(self.ptr)
        self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class Stream:
    def __init__(self, device: int = 0, priority: Optional[str] = None):
        """priority None: default stream priority; "high" / "low": the device's
        greatest / least (rbc_stream_create_priority)."""
        p = c_void_p()
        if priority is None:
            check(lib.rbc_stream_create(device, byref(p)), "rbc_stream_create")
        else:
            check(lib.rbc_stream_create_priority(device, 1 if priority == "high" else 0, byref(p)),
                  "rbc_stream_create_priority")
        self.ptr = p

    def sync(self) -> None:
        check(lib.rbc_stream_sync(self.ptr), "rbc_stream_sync")

    def wait(self, event: "Event") -> None:
        check(lib.rbc_stream_wait_event(self.ptr, event.ptr), "rbc_stream_wait_event")

    def __del__(self):
        try:
            if self.ptr:
                lib.rbc_stream_destroy(self.ptr)
        except Exception:
            pass


def pinned_empty(shape, dtype=np.uint8) -> np.ndarray:
    """numpy array over C-owned pinned host memory (rbc_host_alloc).  The batch
    entry points copy to and from such buffers directly (no staging memcpy):
    what a Go batcher gets by keeping its rings in rbc_host_alloc memory."""
    import ctypes
    import weakref
    nbytes = int(np.prod(shape)) * np.dtype(dtype).itemsize
    p = c_void_p()
    check(lib.rbc_host_alloc(max(nbytes, 1), byref(p)), "rbc_host_alloc")
    buf = (ctypes.c_uint8 * max(nbytes, 1)).from_address(p.value)
    weakref.finalize(buf, lib.rbc_host_free, p)
    return np.frombuffer(buf, dtype=dtype, count=int(np.prod(shape))).reshape(shape)


class Event:
    def __init__(self):
        p = c_void_p()
        check(lib.rbc_event_create(byref(p)), "rbc_event_create")
        self.ptr = p

    def record(self, stream: Optional[Stream] = None) -> None:
        check(lib.rbc_event_record(self.ptr, stream.ptr if stream else None), "rbc_event_record")

    def elapsed_ms(self, end: "Event") -> float:
        ms = c_float(0)
        check(lib.rbc_event_elapsed_ms(self.ptr, end.ptr, byref(ms)), "rbc_event_elapsed_ms")
        return ms.value

    def __del__(self):
        try:
            if self.ptr:
                lib.rbc_event_destroy(self.ptr)
        except Exception:
            pass


def _dv(x) -> Optional[c_void_p]:
    """DeviceBuffer / int / None -> c_void_p."""
    if x is None:
        return None
    if isinstance(x, DeviceBuffer):
        return x.ptr
    if isinstance(x, int):
        return c_void_p(x)
    return x


class HostTicket:
    """An in-flight host-API submission; the caller's arrays stay referenced
    until wait() completes it."""

    def __init__(self, ctx, ticket, result, keep=()):
        self.ctx, self.ticket, self.result, self._keep = ctx, ticket, result, keep

    def done(self) -> bool:
        d = c_int(0)
        check(lib.rbc_poll(self.ctx._p, self.ticket, byref(d)), "rbc_poll")
        return bool(d.value)

    def wait(self) -> dict:
        if self._keep is not None:
            check(lib.rbc_wait(self.ctx._p, self.ticket), "rbc_wait")
            self._keep = None
        return self.result


class Context:
    """One (N, f) RBC geometry on one GPU (rbc/rbc.go:9-20)."""

    def __init__(self, n: int, f: int, device: int = 0):
        p = c_void_p()
        check(lib.rbc_ctx_create(n, f, device, byref(p)), "rbc_ctx_create")
        self._p = p
        self.n, self.f, self.device = n, f, device
        k, par, d = c_int(), c_int(), c_int()
        check(lib.rbc_ctx_params(p, byref(k), byref(par), byref(d)))
        self.k, self.p, self.depth = k.value, par.value, d.value

    def close(self) -> None:
        if getattr(self, "_p", None):
            lib.rbc_ctx_destroy(self._p)
            self._p = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def handle(self) -> c_void_p:
        return self._p

    CODEC_AUTO, CODEC_MATRIX, CODEC_FFT = 0, 1, 2

    @property
    def codec(self) -> str:
        """Effective GF(2^8) codec: "fft" (additive FFT) or "matrix"."""
        c = c_int()
        check(lib.rbc_ctx_codec(self._p, byref(c)))
        return "fft" if c.value == self.CODEC_FFT else "matrix"

    def set_wave_priority(self, commit: int, receive: int) -> None:
        """s_setprio level (0..3) of the commit-side / receive-side kernels."""
        check(lib.rbc_ctx_set_wave_priority(self._p, commit, receive), "rbc_ctx_set_wave_priority")

    def set_decode_priority(self, gemv: int, reencode: int) -> None:
        """s_setprio level (0..3, -1 = the commit level) of interpolate's GF transforms."""
        check(lib.rbc_ctx_set_decode_priority(self._p, gemv, reencode), "rbc_ctx_set_decode_priority")

    def set_recheck(self, mode: str) -> None:
        """The receive step's root recheck: "reuse" (default; only the subtrees
        with no valid ECHO leaf are hashed) or "full" (the whole tree)."""
        check(lib.rbc_ctx_set_recheck(self._p, {"reuse": 0, "full": 1}[mode]), "rbc_ctx_set_recheck")

    def verify_form(self, shard_len: int) -> str:
        """"walk" or "shared_path": the ECHO-verify form for rows of shard_len
        bytes (rbc_ctx_verify_form)."""
        f = c_int(0)
        check(lib.rbc_ctx_verify_form(self._p, shard_len, ctypes.byref(f)), "rbc_ctx_verify_form")
        return ("walk", "shared_path")[f.value]

    def set_codec(self, codec: str) -> None:
        check(lib.rbc_ctx_set_codec(self._p, {"auto": 0, "matrix": 1, "fft": 2}[codec]), "rbc_ctx_set_codec")

    def encode_matrix(self) -> np.ndarray:
        m = np.zeros(self.n * self.k, dtype=np.uint8)
        check(lib.rbc_ctx_encode_matrix(self._p, _ptr(m)))
        return m.reshape(self.n, self.k)

    # ---- single-call drop-ins -------------------------------------------
    def shard(self, data) -> dict:
        """shard(enc, data) + Merkle commit -> {shards, root, branches (flat, Go form)}"""
        d = _bytes_array(data)
        S = (len(d) + self.k - 1) // self.k if len(d) else 0
        out = np.zeros(max(self.n * S, 1), dtype=np.uint8)
        br = np.zeros(max(self.n * self.depth * 32, 1), dtype=np.uint8)
        root = np.zeros(32, dtype=np.uint8)
        slen = c_size_t(0)
        check(lib.rbc_shard(self._p, _ptr(d) if len(d) else None, len(d), _ptr(out), out.nbytes, byref(slen),
                            _ptr(root), _ptr(br)), "rbc_shard")
        S = slen.value
        shards = [out[j * S:(j + 1) * S].copy() for j in range(self.n)]
        brs = br[: self.n * self.depth * 32].reshape(self.n, self.depth, 32) if self.depth else None
        flat = []
        for j in range(self.n):
            parts = []
            for lvl in range(self.depth):
                if lvl == 0 and (j ^ 1) >= self.n:
                    continue
                parts.append(bytes(brs[j, lvl]))
            flat.append(b"".join(parts))
        return {"shards": shards, "shard_len": S, "root": bytes(root), "branches": flat}

    def validate_message(self, root: bytes, branch: bytes, shard, index: int) -> bool:
        s = _bytes_array(shard)
        b = _bytes_array(branch)
        r = _bytes_array(root)
        if len(r) != 32:
            return False
        ok = c_int(0)
        check(lib.rbc_validate_message(self._p, _ptr(r), _ptr(b) if len(b) else None, len(b),
                                       _ptr(s) if len(s) else None, len(s), index, byref(ok)),
              "rbc_validate_message")
        return bool(ok.value)

    def interpolate(self, root: bytes, shards: Sequence) -> dict:
        arrs = [_bytes_array(s) for s in shards]
        if len(arrs) != self.n:
            raise RBCError(_lib.RBC_ERR_TOO_FEW_SHARDS, "interpolate")
        lens = (c_size_t * self.n)(*[len(a) for a in arrs])
        ptrs = (c_void_p * self.n)(*[(a.ctypes.data if len(a) else None) for a in arrs])
        S = max(len(a) for a in arrs)
        value = np.zeros(max(self.k * S, 1), dtype=np.uint8)
        vlen = c_size_t(0)
        dig = np.zeros(32, dtype=np.uint8)
        r = _bytes_array(root)
        check(lib.rbc_interpolate(self._p, _ptr(r), ptrs, lens, _ptr(value), value.nbytes, byref(vlen), _ptr(dig)),
              "rbc_interpolate")
        return {"value": bytes(value[: vlen.value]), "digest": bytes(dig)}

    # ---- host batch API ---------------------------------------------------
    def shard_commit_batch(self, values: Sequence[bytes]) -> dict:
        return self.shard_commit_submit(values).wait()

    def shard_commit_submit(self, values: Sequence[bytes], out: Optional[dict] = None) -> "HostTicket":
        """Asynchronous rbc_shard_commit: returns at once; .wait() completes
        it (the context pipelines consecutive submissions through its slots).
        `out` may hold preallocated (e.g. pinned_empty) "shards" [count][N][Smax],
        "roots" [count][32] and "branches" [count][N][max(d,1)][32] arrays."""
        count = len(values)
        arrs = [v if isinstance(v, np.ndarray) and v.dtype == np.uint8 and v.flags.c_contiguous
                else _bytes_array(v) for v in values]
        Smax = max((len(a) + self.k - 1) // self.k for a in arrs)
        pitch = Smax
        bshape = (count, self.n, max(self.depth, 1), 32)
        if out is not None:  # out["shards"] may be [count][N][pitch >= Smax] (a 64-B pitch: one D2H copy)
            shards, roots, br = out["shards"], out["roots"], out["branches"]
            pitch = shards.shape[2]
            assert shards.shape[:2] == (count, self.n) and pitch >= Smax and shards.flags.c_contiguous
            assert roots.shape == (count, 32) and br.shape == bshape
        else:
            shards = np.zeros((count, self.n, pitch), dtype=np.uint8)
            roots = np.zeros((count, 32), dtype=np.uint8)
            br = np.zeros(bshape, dtype=np.uint8)
        slens = np.zeros(count, dtype=np.uint32)
        vlens = (c_size_t * count)(*[len(a) for a in arrs])
        vptrs = (c_void_p * count)(*[a.ctypes.data if len(a) else None for a in arrs])
        t = c_uint64(0)
        check(lib.rbc_shard_commit(self._p, count, vptrs, vlens, _ptr(shards), pitch,
                                   slens.ctypes.data_as(_lib.u32p), _ptr(roots), _ptr(br), byref(t)),
              "rbc_shard_commit")
        out = {"shards": shards[:, :, :Smax] if pitch != Smax else shards, "shard_lens": slens, "roots": roots,
               "branches": br[:, :, : self.depth]}
        return HostTicket(self, t.value, out, keep=(arrs, vlens, vptrs, br))

    def shard_commit_val(self, values: Sequence[bytes], ring: Optional[np.ndarray] = None) -> dict:
        """rbc_shard_commit_val: shard + commit and the N per-recipient VAL
        pb.Messages of every proposal, handed over in one D2H.  `ring` may be
        a preallocated (e.g. pinned_empty) uint8 array [count][n][msg_pitch]."""
        return self.shard_commit_val_submit(values, ring).wait()

    def shard_commit_val_submit(self, values: Sequence[bytes], ring: Optional[np.ndarray] = None) -> "HostTicket":
        """Asynchronous rbc_shard_commit_val (see shard_commit_submit)."""
        count = len(values)
        arrs = [v if isinstance(v, np.ndarray) and v.dtype == np.uint8 and v.flags.c_contiguous
                else _bytes_array(v) for v in values]
        Smax = max((len(a) + self.k - 1) // self.k for a in arrs)
        need = max(lib.rbc_val_message_size(self.n, Smax, 0, 0), lib.rbc_val_message_size(self.n, Smax, self.n - 1, 0))
        pitch = (need + 15) // 16 * 16
        if ring is None:
            ring = np.zeros((count, self.n, pitch), dtype=np.uint8)
        assert ring.shape[:2] == (count, self.n) and ring.shape[2] % 16 == 0 and ring.shape[2] >= pitch
        lens = np.zeros((count, self.n), dtype=np.uint32)
        roots = np.zeros((count, 32), dtype=np.uint8)
        vlens = (c_size_t * count)(*[len(a) for a in arrs])
        vptrs = (c_void_p * count)(*[a.ctypes.data if len(a) else None for a in arrs])
        t = c_uint64(0)
        check(lib.rbc_shard_commit_val(self._p, count, vptrs, vlens, _ptr(ring), ring.shape[2],
                                       lens.ctypes.data_as(_lib.u32p), _ptr(roots), byref(t)), "rbc_shard_commit_val")
        out = {"msgs": ring, "lens": lens, "roots": roots, "message": lambda i, j: bytes(ring[i, j, : lens[i, j]])}
        return HostTicket(self, t.value, out, keep=(arrs, vlens, vptrs))

    def validate_batch(self, shards, indices, branches, roots) -> np.ndarray:
        count = len(shards)
        sh = [_bytes_array(s) for s in shards]
        br = [_bytes_array(b) for b in branches]
        rt = [_bytes_array(r) for r in roots]
        slens = (c_size_t * count)(*[len(s) for s in sh])
        blens = (c_size_t * count)(*[len(b) for b in br])
        sp = (c_void_p * count)(*[s.ctypes.data if len(s) else None for s in sh])
        bp = (c_void_p * count)(*[b.ctypes.data if len(b) else None for b in br])
        rp = (c_void_p * count)(*[r.ctypes.data for r in rt])
        idx = (c_uint32 * count)(*[int(i) for i in indices])
        ok = np.zeros(count, dtype=np.uint8)
        t = c_uint64(0)
        check(lib.rbc_validate_batch(self._p, count, sp, slens, idx, bp, blens, rp, _ptr(ok), byref(t)),
              "rbc_validate_batch")
        check(lib.rbc_wait(self._p, t.value))
        return ok.astype(bool)

    def validate_packed(self, arena: np.ndarray, offs, lens, idx, branches: np.ndarray, roots: np.ndarray,
                        arena_bytes: Optional[int] = None, leaves: bool = False):
        """rbc_validate_packed: message i is arena[offs[i] : offs[i] + lens[i]]
        (offs[i] % 64 == 0), its branch branches[i] in the device form
        [depth][32], its root roots[i], its leaf index idx[i]; waits and returns
        the verdicts (and, leaves=True, the [count][32] message leaves of
        rbc_validate_packed_leaves)."""
        return self.validate_packed_submit(arena, offs, lens, idx, branches, roots, arena_bytes, leaves).wait()

    def validate_packed_submit(self, arena: np.ndarray, offs, lens, idx, branches: np.ndarray, roots: np.ndarray,
                               arena_bytes: Optional[int] = None, leaves: bool = False,
                               out: Optional[dict] = None, keep: Optional["DeviceBuffer"] = None) -> "HostTicket":
        """Asynchronous rbc_validate_packed_leaves; .wait() returns the verdicts
        (bool array) or, leaves=True, (verdicts, leaves [count][32]).  `out` may
        hold preallocated (pinned) "ok" [count] and "leaves" [count][32] arrays.
        keep (a DeviceBuffer >= the arena): rbc_validate_packed_keep -- message i
        then stays at keep.value + offs[i] for interpolate_kept_submit."""
        count = len(offs)
        arena = arena if (isinstance(arena, np.ndarray) and arena.dtype == np.uint8 and arena.flags.c_contiguous) \
            else np.ascontiguousarray(arena, dtype=np.uint8)
        o = np.ascontiguousarray(offs, dtype=np.uint64)
        ln = np.ascontiguousarray(lens, dtype=np.uint32)
        ix = np.ascontiguousarray(idx, dtype=np.uint8)
        br = np.ascontiguousarray(branches, dtype=np.uint8)
        rt = np.ascontiguousarray(roots, dtype=np.uint8)
        ok = out["ok"] if out else np.zeros(max(count, 1), dtype=np.uint8)
        lv = (out["leaves"] if out else np.zeros((max(count, 1), 32), dtype=np.uint8)) if leaves else None
        t = c_uint64(0)
        nb = arena.nbytes if arena_bytes is None else arena_bytes
        if keep is not None:
            check(lib.rbc_validate_packed_keep(self._p, count, _ptr(arena), nb, _ptr(o), _ptr(ln), _ptr(ix), _ptr(br),
                                               _ptr(rt), _ptr(ok), _ptr(lv) if leaves else None, keep.ptr,
                                               keep.nbytes, byref(t)), "rbc_validate_packed_keep")
        else:
            check(lib.rbc_validate_packed_leaves(self._p, count, _ptr(arena), nb, _ptr(o), _ptr(ln), _ptr(ix),
                                                 _ptr(br), _ptr(rt), _ptr(ok), _ptr(lv) if leaves else None,
                                                 byref(t)), "rbc_validate_packed_leaves")

        class _V(HostTicket):
            def wait(self_):
                if self_.ticket and self_._keep is not None:
                    check(lib.rbc_wait(self._p, self_.ticket), "rbc_wait")
                self_._keep = None
                v = ok[:count].astype(bool)
                return (v, lv[:count]) if leaves else v
        return _V(self, t.value, None, keep=(arena, o, ln, ix, br, rt, ok, lv))

    def interpolate_batch(self, shards: np.ndarray, shard_lens, present: np.ndarray, roots: np.ndarray,
                          values_out: Optional[np.ndarray] = None, leaves: Optional[np.ndarray] = None) -> dict:
        return self.interpolate_submit(shards, shard_lens, present, roots, values_out, leaves).wait()

    def interpolate_submit(self, shards: np.ndarray, shard_lens, present: np.ndarray, roots: np.ndarray,
                           values_out: Optional[np.ndarray] = None, leaves: Optional[np.ndarray] = None,
                           digests_out: Optional[np.ndarray] = None,
                           status_out: Optional[np.ndarray] = None) -> "HostTicket":
        """Asynchronous rbc_interpolate_batch: returns at once; .wait()
        completes it (values, digests, status land in the returned arrays).
        leaves [count][n][32] (the present rows' SHA-256 from
        validate_packed(leaves=True)) selects rbc_interpolate_batch_verified."""
        shards = np.ascontiguousarray(shards, dtype=np.uint8)
        count, n, pitch = shards.shape
        assert n == self.n
        present = np.ascontiguousarray(present, dtype=np.uint8)
        roots = np.ascontiguousarray(roots, dtype=np.uint8)
        sl = (c_size_t * count)(*[int(x) for x in shard_lens])
        Smax = int(max(shard_lens))
        vp = self.k * Smax
        if values_out is not None:
            values = values_out
            assert values.shape[0] == count and values.shape[1] >= max(vp, 1) and values.dtype == np.uint8
        else:
            values = np.zeros((count, max(vp, 1)), dtype=np.uint8)
        digests = np.zeros((count, 32), dtype=np.uint8) if digests_out is None else digests_out
        status = np.zeros(count, dtype=np.int32) if status_out is None else status_out
        lv = None
        if leaves is not None:
            lv = leaves if (leaves.dtype == np.uint8 and leaves.flags.c_contiguous) else \
                np.ascontiguousarray(leaves, dtype=np.uint8)
            assert lv.size == count * self.n * 32
        t = c_uint64(0)
        check(lib.rbc_interpolate_batch_verified(self._p, count, _ptr(shards), pitch, sl, _ptr(present),
                                                 _ptr(lv) if lv is not None else None, _ptr(roots), _ptr(values),
                                                 values.shape[1], _ptr(digests), status.ctypes.data_as(_lib.i32p),
                                                 byref(t)), "rbc_interpolate_batch_verified")
        out = {"values": values, "digests": digests, "status": status}
        return HostTicket(self, t.value, out, keep=(shards, present, roots, sl, lv))

    def interpolate_kept_submit(self, rows: np.ndarray, shard_lens, roots: np.ndarray,
                                leaves: Optional[np.ndarray] = None, values_out: Optional[np.ndarray] = None,
                                digests_out: Optional[np.ndarray] = None,
                                status_out: Optional[np.ndarray] = None) -> "HostTicket":
        """Asynchronous rbc_interpolate_batch_kept: rows [count][n] uint64 device
        addresses of the shards (0 = missing), e.g. keep.value + offs of a
        validate_packed_submit(keep=...); leaves [count][n][32] as
        interpolate_submit's.  .wait() returns values / digests / status."""
        rows = np.ascontiguousarray(rows, dtype=np.uint64)
        count, n = rows.shape
        assert n == self.n
        roots = np.ascontiguousarray(roots, dtype=np.uint8)
        sl = (c_size_t * count)(*[int(x) for x in shard_lens])
        vp = self.k * int(max(shard_lens))
        values = values_out if values_out is not None else np.zeros((count, max(vp, 1)), dtype=np.uint8)
        assert values.shape[0] == count and values.shape[1] >= vp and values.dtype == np.uint8
        digests = np.zeros((count, 32), dtype=np.uint8) if digests_out is None else digests_out
        status = np.zeros(count, dtype=np.int32) if status_out is None else status_out
        lv = None if leaves is None else np.ascontiguousarray(leaves, dtype=np.uint8)
        assert lv is None or lv.size == count * self.n * 32
        t = c_uint64(0)
        check(lib.rbc_interpolate_batch_kept(self._p, count, _ptr(rows), sl, _ptr(lv) if lv is not None else None,
                                             _ptr(roots), _ptr(values), values.shape[1], _ptr(digests),
                                             status.ctypes.data_as(_lib.i32p), byref(t)),
              "rbc_interpolate_batch_kept")
        out = {"values": values, "digests": digests, "status": status}
        return HostTicket(self, t.value, out, keep=(rows, roots, sl, lv))

    def receive_batch(self, shards, shard_lens, present, branches, roots, **kw) -> dict:
        return self.receive_submit(shards, shard_lens, present, branches, roots, **kw).wait()

    def receive_submit(self, shards: np.ndarray, shard_lens, present: np.ndarray, branches: np.ndarray,
                       roots: np.ndarray, values_out: Optional[np.ndarray] = None,
                       valid_out: Optional[np.ndarray] = None, digests_out: Optional[np.ndarray] = None,
                       status_out: Optional[np.ndarray] = None) -> "HostTicket":
        """Asynchronous rbc_receive_batch: ECHO verify of every present row
        (branches [count][n][depth][32], device form) and interpolate of the
        valid ones, the present rows crossing PCIe once; .wait() gives
        {"valid", "values", "digests", "status"}."""
        shards = shards if (shards.dtype == np.uint8 and shards.flags.c_contiguous) else \
            np.ascontiguousarray(shards, dtype=np.uint8)
        count, n, pitch = shards.shape
        assert n == self.n
        present = np.ascontiguousarray(present, dtype=np.uint8)
        br = branches if (branches.dtype == np.uint8 and branches.flags.c_contiguous) else \
            np.ascontiguousarray(branches, dtype=np.uint8)
        assert br.size == count * n * max(self.depth, 1) * 32
        roots = np.ascontiguousarray(roots, dtype=np.uint8)
        sl = (c_size_t * count)(*[int(x) for x in shard_lens])
        vp = self.k * int(max(shard_lens))
        values = np.zeros((count, max(vp, 1)), np.uint8) if values_out is None else values_out
        assert values.shape == (count, max(vp, 1))
        valid = np.zeros((count, n), np.uint8) if valid_out is None else valid_out
        digests = np.zeros((count, 32), np.uint8) if digests_out is None else digests_out
        status = np.zeros(count, np.int32) if status_out is None else status_out
        t = c_uint64(0)
        check(lib.rbc_receive_batch(self._p, count, _ptr(shards), pitch, sl, _ptr(present), _ptr(br), _ptr(roots),
                                    _ptr(valid), _ptr(values), values.shape[1], _ptr(digests),
                                    status.ctypes.data_as(_lib.i32p), byref(t)), "rbc_receive_batch")
        out = {"valid": valid, "values": values, "digests": digests, "status": status}
        return HostTicket(self, t.value, out, keep=(shards, present, br, roots, sl))

    # ---- device-resident stages --------------------------------------------
    def dev_encode(self, stream, count, values, value_pitch, value_lens, uniform_len, shards, shard_pitch):
        check(lib.rbc_dev_encode(self._p, _dv(stream), count, _dv(values), value_pitch, _dv(value_lens),
                                 uniform_len, _dv(shards), shard_pitch), "rbc_dev_encode")

    def dev_leaves(self, stream, count, shards, shard_pitch, shard_lens, uniform_len, leaves):
        check(lib.rbc_dev_leaves(self._p, _dv(stream), count, _dv(shards), shard_pitch, _dv(shard_lens),
                                 uniform_len, _dv(leaves)), "rbc_dev_leaves")

    def dev_merkle_build(self, stream, count, leaves, roots, branches):
        check(lib.rbc_dev_merkle_build(self._p, _dv(stream), count, _dv(leaves), _dv(roots), _dv(branches)),
              "rbc_dev_merkle_build")

    def dev_shard_commit(self, stream, count, values, value_pitch, value_lens, uniform_len, shards, shard_pitch,
                         shard_lens, leaves, roots, branches):
        check(lib.rbc_dev_shard_commit(self._p, _dv(stream), count, _dv(values), value_pitch, _dv(value_lens),
                                       uniform_len, _dv(shards), shard_pitch, _dv(shard_lens), _dv(leaves),
                                       _dv(roots), _dv(branches)), "rbc_dev_shard_commit")

    def dev_verify(self, stream, count, shards, shard_pitch, shard_lens, uniform_len, branches, roots, present,
                   valid, leaves):
        check(lib.rbc_dev_verify(self._p, _dv(stream), count, _dv(shards), shard_pitch, _dv(shard_lens),
                                 uniform_len, _dv(branches), _dv(roots), _dv(present), _dv(valid), _dv(leaves)),
              "rbc_dev_verify")

    def dev_interpolate(self, stream, count, shards, shard_pitch, shard_lens, uniform_len, valid, leaves,
                        leaves_verified, roots, values_out, value_pitch, digests, status):
        check(lib.rbc_dev_interpolate(self._p, _dv(stream), count, _dv(shards), shard_pitch, _dv(shard_lens),
                                      uniform_len, _dv(valid), _dv(leaves), int(leaves_verified), _dv(roots),
                                      _dv(values_out), value_pitch, _dv(digests), _dv(status)),
              "rbc_dev_interpolate")

    @staticmethod
    def rx_batch(count, shards, shard_pitch, shard_lens, uniform_len, branches, roots, present, valid, leaves,
                 values_out, value_pitch, digests, status, verified=False) -> "_lib.RxBatch":
        """An rbc_rx_batch of device buffers (DeviceBuffer / int / None);
        verified=True: valid / leaves already hold rbc_dev_verify's output."""
        def v(x):
            p = _dv(x)
            return p.value if isinstance(p, c_void_p) else p
        return _lib.RxBatch(count, v(shards), shard_pitch, v(shard_lens), uniform_len, v(branches), v(roots),
                            v(present), v(valid), v(leaves), v(values_out), value_pitch, v(digests), v(status),
                            1 if verified else 0)

    def dev_receive_step(self, stream, cur=None, prev=None, hashed=None, decode_begin=None, decoded=None,
                         hash_begin=None, rows_hashed=None, prev_released=None) -> None:
        """Pipelined receiver: verify(cur) + rehash(prev) in one SHA launch,
        prev's recheck + digest, cur's decode (rbc_dev_receive_step).  hashed /
        decode_begin / decoded (Events, optional) are recorded after the
        hashing launch (and the shared-path verify), before cur's decode and
        after it; hash_begin / rows_hashed right before and after the
        row-hashing launch alone; prev_released once nothing of the call reads
        prev's shard set any more (rbc_rx_marks)."""
        marks = None
        evs = (hashed, decode_begin, decoded, hash_begin, rows_hashed, prev_released)
        if any(e is not None for e in evs):
            ev = lambda e: e.ptr.value if e is not None else None  # noqa: E731
            marks = ctypes.byref(_lib.RxMarks(*(ev(e) for e in evs)))
        check(lib.rbc_dev_receive_step(self._p, _dv(stream), ctypes.byref(cur) if cur is not None else None,
                                       ctypes.byref(prev) if prev is not None else None, marks),
              "rbc_dev_receive_step")

    def dev_marshal_val(self, stream, count, msg_type, shards, shard_pitch, shard_lens, uniform_len, branches,
                        roots, out, out_pitch, out_lens):
        """Per-recipient VAL / ECHO pb.Message bytes in HBM (include/rbc_protocol.h)."""
        check(lib.rbc_dev_marshal_val(self._p, _dv(stream), count, msg_type, _dv(shards), shard_pitch,
                                      _dv(shard_lens), uniform_len, _dv(branches), _dv(roots), _dv(out), out_pitch,
                                      _dv(out_lens)), "rbc_dev_marshal_val")

    def val_message_size(self, shard_len: int, index: int = 0, msg_type: int = 0) -> int:
        return lib.rbc_val_message_size(self.n, shard_len, index, msg_type)

    def dev_inject_faults(self, stream, count, shards, shard_pitch, corrupt):
        check(lib.rbc_dev_inject_faults(self._p, _dv(stream), count, _dv(shards), shard_pitch, _dv(corrupt)),
              "rbc_dev_inject_faults")

    # ---- multi-GPU ------------------------------------------------------------
    @staticmethod
    def comm_unique_id() -> bytes:
        buf = np.zeros(128, dtype=np.uint8)
        check(lib.rbc_comm_unique_id(_ptr(buf)), "rbc_comm_unique_id")
        return bytes(buf)

    def comm_init(self, nranks: int, rank: int, uid: bytes) -> None:
        b = np.frombuffer(uid, dtype=np.uint8).copy()
        check(lib.rbc_comm_init(self._p, nranks, rank, _ptr(b)), "rbc_comm_init")

    def dev_allgather_roots(self, stream, count, roots, digests, gathered) -> None:
        check(lib.rbc_dev_allgather_roots(self._p, _dv(stream), count, _dv(roots), _dv(digests), _dv(gathered)),
              "rbc_dev_allgather_roots")

    def dev_allgather_records(self, stream, count, slots, roots, digests, status, gathered) -> None:
        """Ragged-share ACS all-gather: [nranks][slots][64] records, zero
        padded; a failed instance (status != 0) carries a zero digest."""
        check(lib.rbc_dev_allgather_records(self._p, _dv(stream), count, slots, _dv(roots), _dv(digests),
                                            _dv(status), _dv(gathered)), "rbc_dev_allgather_records")

    def comm_info(self, with_comm: bool = True) -> dict:
        """RCCL as it reports itself: nranks / rank of the communicator, the
        library version and the files RCCL and the HIP runtime were mapped from."""
        nr, rk, ver, hver = c_int(0), c_int(0), c_int(0), c_int(0)
        rp, hp = ctypes.create_string_buffer(4096), ctypes.create_string_buffer(4096)
        check(lib.rbc_comm_info(self._p, byref(nr) if with_comm else None, byref(rk) if with_comm else None,
                                byref(ver), rp, 4096, byref(hver), hp, 4096), "rbc_comm_info")
        v = ver.value
        out = {"version": v, "version_str": f"{v // 10000}.{(v // 100) % 100}.{v % 100}",
               "lib": rp.value.decode(), "hip_runtime_version": hver.value, "hip_lib": hp.value.decode()}
        if with_comm:
            out.update(nranks=nr.value, rank=rk.value)
        return out


class Encoder:
    """reedsolomon.Encoder mirror (klauspost v1.9.1 semantics), GPU-backed."""

    def __init__(self, data_shards: int, parity_shards: int, device: int = 0):
        p = c_void_p()
        check(lib.rbc_rs_new(data_shards, parity_shards, device, byref(p)), "reedsolomon.New")
        self._p = p
        self.data_shards, self.parity_shards = data_shards, parity_shards
        self.shards = data_shards + parity_shards

    def __del__(self):
        try:
            if self._p:
                lib.rbc_rs_free(self._p)
        except Exception:
            pass

    @staticmethod
    def _pack(shards):
        arrs = [None if s is None else _bytes_array(s).copy() for s in shards]
        n = len(arrs)
        lens = (c_size_t * n)(*[0 if a is None else len(a) for a in arrs])
        ptrs = (c_void_p * n)(*[(a.ctypes.data if (a is not None and len(a)) else None) for a in arrs])
        return arrs, lens, ptrs

    def encode(self, shards: List) -> None:
        arrs, lens, ptrs = self._pack(shards)
        check(lib.rbc_rs_encode(self._p, ptrs, lens, len(arrs)), "Encode")
        for i in range(self.data_shards, min(len(arrs), self.shards)):
            shards[i] = arrs[i]

    def verify(self, shards) -> bool:
        arrs, lens, ptrs = self._pack(shards)
        ok = c_int(0)
        check(lib.rbc_rs_verify(self._p, ptrs, lens, len(arrs), byref(ok)), "Verify")
        return bool(ok.value)

    def _reconstruct(self, shards: List, data_only: bool) -> None:
        arrs = [None if s is None else _bytes_array(s).copy() for s in shards]
        size = max([len(a) for a in arrs if a is not None] + [0])
        n = len(arrs)
        bufs = [a if (a is not None and len(a)) else np.zeros(max(size, 1), dtype=np.uint8) for a in arrs]
        lens = (c_size_t * n)(*[0 if (a is None) else len(a) for a in arrs])
        ptrs = (c_void_p * n)(*[b.ctypes.data for b in bufs])
        fn = lib.rbc_rs_reconstruct_data if data_only else lib.rbc_rs_reconstruct
        check(fn(self._p, ptrs, lens, n), "ReconstructData" if data_only else "Reconstruct")
        for i in range(n):
            if lens[i]:
                shards[i] = bufs[i][: lens[i]].copy()

    def update(self, shards: List, new_data: List) -> None:
        """Update(shards, newDatashards): parity shards in `shards` are updated
        for the changed data shards (None / empty = unchanged); as in Go, each
        changed old data shard is left holding old ^ new."""
        arrs = [None if s is None else _bytes_array(s).copy() for s in shards]
        news = [None if s is None else _bytes_array(s) for s in new_data]
        n, m = len(arrs), len(news)
        lens = (c_size_t * n)(*[0 if a is None else len(a) for a in arrs])
        ptrs = (c_void_p * n)(*[(a.ctypes.data if (a is not None and len(a)) else None) for a in arrs])
        nlens = (c_size_t * m)(*[0 if a is None else len(a) for a in news])
        nptrs = (c_void_p * m)(*[(a.ctypes.data if (a is not None and len(a)) else None) for a in news])
        check(lib.rbc_rs_update(self._p, ptrs, lens, n, nptrs, nlens, m), "Update")
        for i in range(n):
            if arrs[i] is not None:
                shards[i] = arrs[i]

    def reconstruct(self, shards: List) -> None:
        self._reconstruct(shards, False)

    def reconstruct_data(self, shards: List) -> None:
        self._reconstruct(shards, True)

    def split(self, data) -> List[np.ndarray]:
        d = _bytes_array(data)
        per = c_size_t(0)
        per_est = (len(d) + self.data_shards - 1) // self.data_shards if len(d) else 0
        out = np.zeros(max(self.shards * per_est, 1), dtype=np.uint8)
        check(lib.rbc_rs_split(self._p, _ptr(d) if len(d) else None, len(d), _ptr(out), out.nbytes, byref(per)),
              "Split")
        p = per.value
        return [out[i * p:(i + 1) * p].copy() for i in range(self.shards)]

    def join(self, shards, out_size: int) -> bytes:
        arrs = [None if s is None else _bytes_array(s) for s in shards]
        n = len(arrs)
        lens = (c_size_t * n)(*[0 if a is None else len(a) for a in arrs])
        ptrs = (c_void_p * n)(*[(None if a is None else (a.ctypes.data if len(a) else 1)) for a in arrs])
        out = np.zeros(max(out_size, 1), dtype=np.uint8)
        check(lib.rbc_rs_join(self._p, ptrs, lens, n, out_size, _ptr(out)), "Join")
        return bytes(out[:out_size])


def _by_ref(x) -> np.ndarray:
    """A contiguous uint8 ndarray as it is (the caller keeps it unchanged until
    the request completes), anything else copied into one."""
    if isinstance(x, np.ndarray) and x.dtype == np.uint8 and x.flags.c_contiguous and x.ndim == 1:
        return x
    return _bytes_array(x).copy()


class Batcher:
    """Request coalescing (include/rbc_gpu.h rbc_batcher_*): single-instance
    shard / validate / interpolate submissions from any number of threads are
    merged into batched launches.  ``submit_*`` return a handle that keeps the
    request's buffers alive; ``wait`` completes it."""

    def __init__(self, ctx: Context, max_batch: int = 256, max_wait_us: int = 200):
        p = c_void_p()
        check(lib.rbc_batcher_create(ctx.handle, max_batch, max_wait_us, byref(p)), "rbc_batcher_create")
        self._p = p
        self.ctx = ctx

    def close(self) -> None:
        if getattr(self, "_p", None):
            lib.rbc_batcher_destroy(self._p)
            self._p = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def submit_shard(self, data) -> dict:
        d = _bytes_array(data).copy()
        k, n = self.ctx.k, self.ctx.n
        S = (len(d) + k - 1) // k if len(d) else 0
        h = {"kind": "shard", "data": d, "out": np.zeros(max(n * S, 1), np.uint8), "root": np.zeros(32, np.uint8),
             "br": np.zeros(max(n * self.ctx.depth * 32, 1), np.uint8), "slen": c_size_t(0), "t": c_uint64(0)}
        check(lib.rbc_batcher_shard(self._p, _ptr(d) if len(d) else None, len(d), _ptr(h["out"]), h["out"].nbytes,
                                    byref(h["slen"]), _ptr(h["root"]), _ptr(h["br"]), byref(h["t"])),
              "rbc_batcher_shard")
        return h

    def submit_validate(self, root, branch, shard, index, leaf: bool = False) -> dict:
        """validateMessage through the lane; leaf=True also returns the shard's
        SHA-256 leaf (rbc_batcher_validate_leaf) for submit_interpolate(leaves=).
        A contiguous uint8 ndarray shard is passed by reference (not copied):
        with set_keep, interpolate finds it kept when handed the same array."""
        r, b, s = _bytes_array(root).copy(), _bytes_array(branch).copy(), _by_ref(shard)
        h = {"kind": "validate", "r": r, "b": b, "s": s, "ok": c_int(0), "t": c_uint64(0),
             "leaf": np.zeros(32, np.uint8) if leaf else None}
        check(lib.rbc_batcher_validate_leaf(self._p, _ptr(r), _ptr(b) if len(b) else None, len(b),
                                            _ptr(s) if len(s) else None, len(s), index, byref(h["ok"]),
                                            _ptr(h["leaf"]) if leaf else None, byref(h["t"])),
              "rbc_batcher_validate_leaf")
        return h

    def submit_interpolate(self, root, shards, leaves=None) -> dict:
        """interpolate through the coalescer; leaves (n x 32, the leaves of the
        present shards from submit_validate(leaf=True)) selects
        rbc_batcher_interpolate_verified: only regenerated rows are hashed."""
        n, k = self.ctx.n, self.ctx.k
        arrs = [_by_ref(x) for x in shards]
        S = max(len(a) for a in arrs)
        lens = (c_size_t * n)(*[len(a) for a in arrs])
        ptrs = (c_void_p * n)(*[(a.ctypes.data if len(a) else None) for a in arrs])
        r = _bytes_array(root).copy()
        h = {"kind": "interp", "arrs": arrs, "lens": lens, "ptrs": ptrs, "r": r,
             "value": np.zeros(max(k * S, 1), np.uint8), "vlen": c_size_t(0), "dig": np.zeros(32, np.uint8),
             "t": c_uint64(0)}
        if leaves is None:
            check(lib.rbc_batcher_interpolate(self._p, _ptr(r), ptrs, lens, _ptr(h["value"]), h["value"].nbytes,
                                              byref(h["vlen"]), _ptr(h["dig"]), byref(h["t"])),
                  "rbc_batcher_interpolate")
        else:
            lv = np.ascontiguousarray(leaves, dtype=np.uint8).reshape(n, 32).copy()
            h["lv"] = lv
            check(lib.rbc_batcher_interpolate_verified(self._p, _ptr(r), ptrs, lens, _ptr(lv), _ptr(h["value"]),
                                                       h["value"].nbytes, byref(h["vlen"]), _ptr(h["dig"]),
                                                       byref(h["t"])), "rbc_batcher_interpolate_verified")
        return h

    def wait(self, h: dict):
        st = lib.rbc_batcher_wait(self._p, h["t"].value)
        if h["kind"] == "validate":
            check(st, "validate")
            if h["leaf"] is not None:
                return bool(h["ok"].value), bytes(h["leaf"])
            return bool(h["ok"].value)
        check(st, h["kind"])
        if h["kind"] == "shard":
            S = h["slen"].value
            return {"shards": [h["out"][j * S:(j + 1) * S].copy() for j in range(self.ctx.n)],
                    "root": bytes(h["root"]), "shard_len": S}
        return {"value": bytes(h["value"][: h["vlen"].value]), "digest": bytes(h["dig"])}

    def set_keep(self, device_bytes: int) -> None:
        """rbc_batcher_set_keep: validated shards stay in a device ring of
        device_bytes for their instance's interpolate (before the first validate)."""
        check(lib.rbc_batcher_set_keep(self._p, int(device_bytes)), "rbc_batcher_set_keep")

    def keep_stats(self) -> dict:
        v = [c_uint64(0) for _ in range(4)]
        check(lib.rbc_batcher_keep_stats(self._p, *[byref(x) for x in v]), "rbc_batcher_keep_stats")
        return dict(zip(("kept_interps", "host_interps", "kept_launches", "unkept_launches"), (x.value for x in v)))

    def set_validate(self, max_msgs: int, max_bytes: int) -> None:
        """The validate lane's arena size (rbc_batcher_set_validate; before the first validate)."""
        check(lib.rbc_batcher_set_validate(self._p, max_msgs, max_bytes), "rbc_batcher_set_validate")

    def stats(self):
        b, r = c_uint64(0), c_uint64(0)
        check(lib.rbc_batcher_stats(self._p, byref(b), byref(r)))
        return b.value, r.value
