"""One process per GPU: launching the ranks, placing them, and failing loudly.

BASELINE north_star (5) partitions independent RBC instances over the GPUs
of a node.  The host side of that is small but has to
be right the first time it runs on eight GPUs:

* ``spawn_ranks``  -- start N ranks with the torch.distributed.run
  environment (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_*) before anything
  touches a GPU, and return the first failure; when one rank fails the others
  are terminated (they would wait at the rendezvous), and killed if they do
  not exit within a grace period.
* ``Watchdog``     -- names the stage a rank is in (rendezvous, RCCL init,
  warmup, timed loop, checks).  A stage that outlives its deadline -- a hung
  RCCL collective, a peer that stopped answering -- or a SIGTERM from the
  launcher makes the rank print rank, stage, elapsed time and its context
  (device, PCI bus, RCCL) as one JSON line on stderr and exit non-zero.
  SIGTERM reaches the watchdog thread through the interpreter's wakeup fd
  (the C-level handler writes it from whichever thread takes the signal), so
  the report comes out even while the main thread sits inside a HIP call.
* ``host_info`` / ``numa_place`` -- the cores a rank may use (cgroup quota,
  affinity) and the CPUs local to its GPU.

No torch import anywhere here: bench.py must map the HIP runtime and RCCL
that librbc_gpu.so links (cleisthenes_amd/rendezvous.py).
"""
from __future__ import annotations

import json
import os
import select
import signal
import socket
import subprocess
import sys
import threading
import time
import uuid
from contextlib import contextmanager
from typing import Dict, List, Optional, Sequence

EXIT_DEADLINE = 4     # a stage outlived its deadline
EXIT_TERMINATED = 143  # SIGTERM from the launcher (128 + 15)


def spawn_ranks(n: int, argv: Sequence[str], script: str, grace_s: float = 10.0) -> int:
    """Run ranks 0..n-1 of `script` with the torch.distributed.run
    environment on loopback; return the first non-zero exit status, else 0.
    After the first failure the other ranks get SIGTERM, then SIGKILL once
    `grace_s` has passed (a stopped or wedged rank ignores SIGTERM)."""
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    key = uuid.uuid4().hex
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RBC_RDZV_KEY=key)
        procs.append(subprocess.Popen([sys.executable, script] + list(argv), env=env))
    rc, kill_at = 0, None
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 128 - code  # -9 (SIGKILL) -> 137, as a shell reports it
                for q in live:
                    q.terminate()
                kill_at = time.monotonic() + grace_s
        if kill_at is not None and time.monotonic() > kill_at:
            for q in live:
                q.kill()
            kill_at = None
        time.sleep(0.05)
    return rc


class Watchdog:
    """Stage tracker with deadlines for one rank (see the module docstring)."""

    def __init__(self, rank: int, world: int, scale: float = 1.0):
        self.rank, self.world, self.scale = rank, world, scale
        self.info: Dict = {}
        self._stage: Optional[str] = None
        self._t0 = time.monotonic()
        self._deadline: Optional[float] = None
        self._lock = threading.Lock()
        self._wake = None
        if threading.current_thread() is threading.main_thread():
            # the C handler behind signal.signal writes the signal number to
            # the wakeup fd at once, whatever the main thread is doing; the
            # Python-level handler does the same report if it runs first
            r, w = os.pipe()
            os.set_blocking(w, False)
            signal.signal(signal.SIGTERM, lambda *_: self._terminated())
            self._old_wakeup = signal.set_wakeup_fd(w)
            self._wake = (r, w)
        self._stop = False
        self._thread = threading.Thread(target=self._run, name="rbc-watchdog", daemon=True)
        self._thread.start()

    def enter(self, stage: str, seconds: float) -> None:
        with self._lock:
            self._stage, self._t0 = stage, time.monotonic()
            self._deadline = self._t0 + seconds * self.scale

    def leave(self) -> None:
        with self._lock:
            self._deadline = None

    @contextmanager
    def stage(self, name: str, seconds: float):
        self.enter(name, seconds)
        try:
            yield
        except BaseException as e:
            if not isinstance(e, SystemExit) or e.code not in (0, None):
                self.report(f"error: {type(e).__name__}: {e}")
            raise
        self.leave()

    def report(self, why: str) -> None:
        with self._lock:
            stage, t0 = self._stage, self._t0
        line = {"watchdog": why, "rank": self.rank, "world": self.world, "stage": stage,
                "elapsed_s": round(time.monotonic() - t0, 2), **self.info}
        os.write(2, (json.dumps(line, default=str) + "\n").encode())

    def close(self) -> None:
        self._stop = True
        self._thread.join(timeout=2)
        if self._wake:
            signal.set_wakeup_fd(self._old_wakeup)
            signal.signal(signal.SIGTERM, signal.SIG_DFL)
            for fd in self._wake:
                os.close(fd)
            self._wake = None

    def _terminated(self) -> None:
        with self._lock:
            first, self._dying = not getattr(self, "_dying", False), True
        if first:
            self.report("terminated by the launcher (another rank failed)")
        os._exit(EXIT_TERMINATED)

    def _run(self) -> None:
        while not self._stop:
            if self._wake:
                ready, _, _ = select.select([self._wake[0]], [], [], 0.25)
                if ready and signal.SIGTERM in os.read(self._wake[0], 64):
                    self._terminated()
            else:
                time.sleep(0.25)
            with self._lock:
                late = self._deadline is not None and time.monotonic() > self._deadline
            if late:
                self.report("deadline exceeded")
                os._exit(EXIT_DEADLINE)


# ----------------------------------------------------------------- host facts
def host_info() -> Dict:
    info = {"logical_cpus": os.cpu_count()}
    try:
        info["affinity_cpus"] = len(os.sched_getaffinity(0))
    except AttributeError:
        info["affinity_cpus"] = os.cpu_count()
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            quota = int(q) / int(per)
    except (OSError, ValueError):
        try:
            q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            if q > 0:
                quota = q / per
        except (OSError, ValueError):
            pass
    info["cgroup_cpu_quota"] = quota
    try:
        info["nproc"] = int(subprocess.run(["nproc"], capture_output=True, text=True, timeout=10).stdout)
    except Exception:  # noqa: BLE001
        info["nproc"] = None
    model = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    info["cpu_model"] = model
    usable = info["affinity_cpus"]
    if quota:
        usable = min(usable, int(quota))
    info["usable_cores"] = max(1, usable)
    return info


def _cpulist(text: str) -> List[int]:
    cpus = []
    for part in text.strip().split(","):
        if part:
            a, _, b = part.partition("-")
            cpus.extend(range(int(a), int(b or a) + 1))
    return cpus


def numa_place(bus_id: str) -> Dict:
    """Bind this process's host threads to the CPUs local to the GPU at PCI
    `bus_id` (best effort: placement is an optimisation only)."""
    try:
        base = f"/sys/bus/pci/devices/{bus_id}"
        node = int(open(f"{base}/numa_node").read())
        allowed = os.sched_getaffinity(0) & set(_cpulist(open(f"{base}/local_cpulist").read()))
        if allowed:
            os.sched_setaffinity(0, allowed)
        return {"numa_node": node, "cpus": len(allowed)}
    except Exception as e:  # noqa: BLE001
        return {"numa_error": type(e).__name__}
