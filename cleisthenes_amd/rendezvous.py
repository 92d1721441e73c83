"""Host-side coordination of a one-process-per-GPU run without torch.

bench.py (and any host runtime above the C ABI) needs a handful of tiny
host collectives: broadcast RCCL's 128-byte unique id, a barrier around the
timed region, the max over ranks of the elapsed time and an all-gather of
small check records.  Doing them through torch.distributed would import
torch, whose bundled libamdhip64 / librccl would then be the ones the
process maps -- not the ROCm runtime librbc_gpu.so is linked against.  This
module does them over loopback TCP instead; every collective is a star
through rank 0.  Single node only, which is what the bench contract launches.

Trust and failure model:
* Rank 0 publishes its ephemeral port and a fresh random secret in a file
  created with O_EXCL inside a directory only this user can enter
  (<tmp>/rbc_rdzv_<uid>, mode 0700, ownership checked; a pre-existing file is
  refused).  Other ranks read it and present rank + secret on connect; rank 0
  drops any connection that does not, so another local user can neither claim
  a rank nor learn the port's secret.
* Payloads are bytes or JSON -- nothing is unpickled.
* Every receive has a deadline (RBC_RDZV_TIMEOUT seconds, default 600): a
  peer that died closes its socket (ConnectionError at once), a peer that
  hangs raises TimeoutError naming the operation and the peer.
"""
from __future__ import annotations

import hmac
import json
import os
import secrets
import socket
import stat
import struct
import tempfile
import time
from typing import Any, List, Optional

_SECRET_LEN = 32  # bytes, sent hex-encoded (64 characters)


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


def private_dir() -> str:
    """<tmp>/rbc_rdzv_<uid>: created 0700 if absent; refused unless it is a
    real directory owned by this user that nobody else can enter."""
    d = os.path.join(tempfile.gettempdir(), f"rbc_rdzv_{os.getuid()}")
    try:
        os.mkdir(d, 0o700)
    except FileExistsError:
        pass
    st = os.lstat(d)
    if not stat.S_ISDIR(st.st_mode) or st.st_uid != os.getuid() or st.st_mode & 0o077:
        raise PermissionError(f"rendezvous directory {d} is not private to uid {os.getuid()}")
    return d


def _send(sock: socket.socket, payload: bytes) -> None:
    sock.sendall(struct.pack("<Q", len(payload)) + payload)


def _recv_exact(sock: socket.socket, n: int, what: str) -> bytes:
    buf = bytearray()
    while len(buf) < n:
        try:
            chunk = sock.recv(min(n - len(buf), 1 << 20))
        except socket.timeout:
            raise TimeoutError(f"rendezvous: no data from {what} within {sock.gettimeout():.0f} s") from None
        if not chunk:
            raise ConnectionError(f"rendezvous: {what} closed the connection (the rank exited)")
        buf += chunk
    return bytes(buf)


def _recv(sock: socket.socket, what: str, limit: int = 1 << 30) -> bytes:
    (n,) = struct.unpack("<Q", _recv_exact(sock, 8, what))
    if n > limit:
        raise ConnectionError(f"rendezvous: {what} announced {n} bytes")
    return _recv_exact(sock, n, what)


class Rendezvous:
    """world ranks of one launch; all collectives are blocking and must be
    called by every rank in the same order."""

    def __init__(self, world: int, rank: int, key: Optional[str] = None, timeout: Optional[float] = None,
                 connect_timeout: float = 300.0):
        if world < 1 or not (0 <= rank < world):
            raise ValueError(f"bad rank {rank} of {world}")
        self.world, self.rank = world, rank
        self.timeout = float(os.environ.get("RBC_RDZV_TIMEOUT", "600")) if timeout is None else timeout
        self.peers = {}          # rank 0: rank -> socket
        self.sock = None         # other ranks: socket to rank 0
        if world == 1:
            return
        key = key or launch_key()
        if not key.replace("_", "").isalnum():
            raise ValueError(f"bad rendezvous key {key!r}")
        path = os.path.join(private_dir(), key)
        deadline = time.monotonic() + connect_timeout
        if rank == 0:
            self._serve(path, deadline)
        else:
            self._join(path, deadline)

    def _serve(self, path: str, deadline: float) -> None:
        secret = secrets.token_hex(_SECRET_LEN).encode()
        srv = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
        srv.bind(("127.0.0.1", 0))
        srv.listen(self.world)
        tmp = f"{path}.{os.getpid()}.tmp"
        fd = os.open(tmp, os.O_WRONLY | os.O_CREAT | os.O_EXCL, 0o600)
        with os.fdopen(fd, "w") as f:
            f.write(f"{srv.getsockname()[1]} {secret.decode()}")
        try:
            os.link(tmp, path)  # atomic and exclusive: never replaces an existing file
        except FileExistsError:
            srv.close()
            raise FileExistsError(f"rendezvous file {path} already exists (another launch with this key?)") from None
        finally:
            os.unlink(tmp)
        try:
            while len(self.peers) < self.world - 1:
                left = deadline - time.monotonic()
                if left <= 0:
                    raise TimeoutError(f"rank 0: {len(self.peers)} of {self.world - 1} ranks joined the rendezvous")
                srv.settimeout(left)
                try:
                    c, _ = srv.accept()
                except socket.timeout:
                    continue
                c.settimeout(10.0)
                try:
                    hello = _recv_exact(c, 4 + 2 * _SECRET_LEN, "a connecting peer")
                except (TimeoutError, ConnectionError):
                    c.close()
                    continue
                (r,) = struct.unpack_from("<i", hello)
                if not hmac.compare_digest(hello[4:], secret) or not (0 < r < self.world) or r in self.peers:
                    c.close()  # not one of this launch's ranks
                    continue
                c.settimeout(self.timeout)
                c.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
                self.peers[r] = c
        finally:
            srv.close()
            try:
                os.unlink(path)
            except OSError:
                pass

    def _join(self, path: str, deadline: float) -> None:
        while True:
            try:
                with open(path) as f:
                    port_s, secret = f.read().split()
                s = socket.create_connection(("127.0.0.1", int(port_s)), timeout=10)
                break
            except (OSError, ValueError):
                if time.monotonic() > deadline:
                    raise TimeoutError(f"rank {self.rank}: no rendezvous at {path}") from None
                time.sleep(0.05)
        s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        s.sendall(struct.pack("<i", self.rank) + secret.encode())
        s.settimeout(self.timeout)
        self.sock = s

    # ---- collectives -------------------------------------------------------
    def allgather_bytes(self, payload: bytes) -> List[bytes]:
        if self.world == 1:
            return [payload]
        if self.rank == 0:
            parts = [payload] + [_recv(self.peers[r], f"rank {r}") for r in range(1, self.world)]
            blob = b"".join(struct.pack("<Q", len(p)) + p for p in parts)
            for r in range(1, self.world):
                _send(self.peers[r], blob)
            return parts
        _send(self.sock, payload)
        blob = _recv(self.sock, "rank 0")
        parts, off = [], 0
        for _ in range(self.world):
            (n,) = struct.unpack_from("<Q", blob, off)
            parts.append(blob[off + 8: off + 8 + n])
            off += 8 + n
        return parts

    def allgather(self, obj: Any) -> List[Any]:
        """JSON values only (numbers, strings, lists, dicts, bools, None)."""
        return [json.loads(p) for p in self.allgather_bytes(json.dumps(obj).encode())]

    def broadcast_bytes(self, payload: Optional[bytes], root: int = 0) -> bytes:
        return self.allgather_bytes(payload if self.rank == root else b"")[root]

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
