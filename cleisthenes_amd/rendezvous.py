"""Host-side coordination of a one-process-per-GPU run without torch.

bench.py (and any host runtime above the C ABI) needs a handful of tiny
host collectives: broadcast RCCL's 128-byte unique id, a barrier around the
timed region, the max over ranks of the elapsed time and an all-gather of
small check records.  Doing them through torch.distributed would import
torch, whose bundled libamdhip64 / librccl would then be the ones the
process maps -- not the ROCm runtime librbc_gpu.so is linked against.  This
module does them over loopback TCP instead: rank 0 listens on an ephemeral
127.0.0.1 port and publishes it through a file keyed by the launch (every
rank of one launch -- torch.distributed.run's agent or bench.py's own
parent -- shares a parent process), the other ranks connect, and every
collective is a star through rank 0.  Single node only, which is what the
bench contract launches.
"""
from __future__ import annotations

import os
import pickle
import socket
import struct
import tempfile
import time
from typing import Any, List, Optional


def _parent_start_time(pid: int) -> str:
    try:
        with open(f"/proc/{pid}/stat") as f:
            return f.read().rsplit(")", 1)[1].split()[19]  # field 22: starttime
    except OSError:
        return "0"


def launch_key() -> str:
    """Identifies one launch: RBC_RDZV_KEY if the launcher set it, else the
    shared parent process (pid + start time) and MASTER_PORT."""
    k = os.environ.get("RBC_RDZV_KEY")
    if k:
        return k
    ppid = os.getppid()
    return f"{ppid}_{_parent_start_time(ppid)}_{os.environ.get('MASTER_PORT', '0')}"


def _send(sock: socket.socket, payload: bytes) -> None:
    sock.sendall(struct.pack("<Q", len(payload)) + payload)


def _recv_exact(sock: socket.socket, n: int) -> bytes:
    buf = bytearray()
    while len(buf) < n:
        chunk = sock.recv(min(n - len(buf), 1 << 20))
        if not chunk:
            raise ConnectionError("rendezvous peer closed the connection")
        buf += chunk
    return bytes(buf)


def _recv(sock: socket.socket) -> bytes:
    (n,) = struct.unpack("<Q", _recv_exact(sock, 8))
    return _recv_exact(sock, n)


class Rendezvous:
    """world ranks of one launch; all collectives are blocking and must be
    called by every rank in the same order."""

    def __init__(self, world: int, rank: int, key: Optional[str] = None, timeout: float = 300.0):
        if world < 1 or not (0 <= rank < world):
            raise ValueError(f"bad rank {rank} of {world}")
        self.world, self.rank = world, rank
        self.peers = {}          # rank 0: rank -> socket
        self.sock = None         # other ranks: socket to rank 0
        if world == 1:
            return
        key = key or launch_key()
        path = os.path.join(tempfile.gettempdir(), f"rbc_rdzv_{key}")
        deadline = time.monotonic() + timeout
        if rank == 0:
            srv = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
            srv.bind(("127.0.0.1", 0))
            srv.listen(world)
            srv.settimeout(max(1.0, deadline - time.monotonic()))
            tmp = f"{path}.{os.getpid()}.tmp"
            with open(tmp, "w") as f:
                f.write(str(srv.getsockname()[1]))
            os.replace(tmp, path)
            try:
                while len(self.peers) < world - 1:
                    c, _ = srv.accept()
                    c.settimeout(None)
                    c.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
                    (r,) = struct.unpack("<i", _recv_exact(c, 4))
                    if not (0 < r < world) or r in self.peers:
                        raise ConnectionError(f"unexpected rank {r} at rendezvous")
                    self.peers[r] = c
            finally:
                srv.close()
                try:
                    os.unlink(path)
                except OSError:
                    pass
        else:
            while True:
                try:
                    with open(path) as f:
                        port = int(f.read())
                    s = socket.create_connection(("127.0.0.1", port), timeout=10)
                    break
                except (OSError, ValueError):
                    if time.monotonic() > deadline:
                        raise TimeoutError(f"rank {rank}: no rendezvous at {path}")
                    time.sleep(0.05)
            s.settimeout(None)
            s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
            s.sendall(struct.pack("<i", rank))
            self.sock = s

    # ---- collectives -------------------------------------------------------
    def allgather_bytes(self, payload: bytes) -> List[bytes]:
        if self.world == 1:
            return [payload]
        if self.rank == 0:
            parts = [payload] + [_recv(self.peers[r]) for r in range(1, self.world)]
            blob = b"".join(struct.pack("<Q", len(p)) + p for p in parts)
            for r in range(1, self.world):
                _send(self.peers[r], blob)
            return parts
        _send(self.sock, payload)
        blob = _recv(self.sock)
        parts, off = [], 0
        for _ in range(self.world):
            (n,) = struct.unpack_from("<Q", blob, off)
            parts.append(blob[off + 8: off + 8 + n])
            off += 8 + n
        return parts

    def allgather(self, obj: Any) -> List[Any]:
        # trusted peers only: the ranks of one local launch, over loopback
        return [pickle.loads(p) for p in self.allgather_bytes(pickle.dumps(obj))]

    def broadcast(self, obj: Any, root: int = 0) -> Any:
        return self.allgather(obj if self.rank == root else None)[root]

    def barrier(self) -> None:
        self.allgather_bytes(b"")

    def max(self, x: float) -> float:
        return max(self.allgather(x))

    def sum(self, x):
        return sum(self.allgather(x))

    def all(self, flag: bool) -> bool:
        return all(self.allgather(bool(flag)))

    def close(self) -> None:
        for s in list(self.peers.values()) + ([self.sock] if self.sock else []):
            try:
                s.close()
            except OSError:
                pass
        self.peers, self.sock = {}, None

    def __del__(self):
        self.close()
