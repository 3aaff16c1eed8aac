"""``client``: the pull-based worker (one process per GPU).

Reference (client.go:21-81): dial ``SERVER_IP:SERVER_PORT`` with a 10 s timeout,
block on a <=100-byte read for ``dir;idx;args``, download ``<idx>.mp4`` with wget,
run ffmpeg, upload log + output over FTP, write ``success;idx`` /
``fail;idx[;reason]`` on the same connection, close, redial; sleep 10 s after a
dial error.  One job at a time.

MI355X-first changes:

* ``leases`` (K) connections are held at once; the jobs that arrive together are
  encoded as ONE batched GPU call (backends/gpu.py), so a single worker keeps
  all 256 CUs busy.  With K=1 the behaviour is exactly the reference's.
* v1 extras: a ``hello;<id>;<gpu>`` greeting (a v0 server ignores it,
  server.go:301-302), and ``heart;<idx>`` every ``heartbeat_s`` while encoding so
  the coordinator can tell a slow job from a dead worker.
* failures carry reasons (bad args, fetch, decode, encode, store) instead of
  being noticed only at upload (D11); malformed jobs are answered, not crashed on (D10/D14).
* fault injection for tests: ``MIVC_FAULT`` =
  ``kind[:idx=N][,kind...]`` with kind in crash_after_fetch | fail | hang | garbage |
  short | disconnect; each fires once per process.
"""
from __future__ import annotations

import os
import queue
import shutil
import socket
import sys
import tempfile
import threading
import time
from dataclasses import dataclass, field

from ..obs import get_logger
from . import protocol as proto
from .coordinator import out_dir_name
from .transport import TransportError


@dataclass(eq=False)
class _Lease:
    sock: socket.socket
    job: proto.Job
    done: threading.Event = field(default_factory=threading.Event)
    reply: proto.Reply | None = None
    lock: threading.Lock = field(default_factory=threading.Lock)
    silent: bool = False          # fault injection: never answer


def parse_faults(spec: str | None) -> list[dict]:
    out = []
    for item in (spec or "").split(","):
        item = item.strip()
        if not item:
            continue
        kind, _, rest = item.partition(":")
        f = {"kind": kind, "idx": None, "fired": False}
        for kv in rest.split(":") if rest else []:
            k, _, v = kv.partition("=")
            if k == "idx":
                f["idx"] = v
        out.append(f)
    return out


class Worker:
    def __init__(self, server_ip: str, port: int, backend, transport, leases: int = 1, worker_id: str | None = None,
                 gpu: str = "", scratch: str | None = None, retry_s: float = 10.0, dial_timeout: float = 10.0,
                 heartbeat_s: float = 5.0, idle_exit_s: float | None = None, max_jobs: int | None = None,
                 batch_wait_s: float = 0.2, out_ext: str = "mp4", faults: str | None = None, log=None):
        self.addr = (server_ip, int(port))
        self.backend = backend
        self.transport = transport
        self.leases = max(1, int(leases))
        self.worker_id = worker_id or f"{socket.gethostname()}-{os.getpid()}"
        self.gpu = gpu
        self.scratch = scratch or tempfile.mkdtemp(prefix="mivc_worker_")
        self.retry_s = retry_s
        self.dial_timeout = dial_timeout
        self.heartbeat_s = heartbeat_s
        self.idle_exit_s = idle_exit_s
        self.max_jobs = max_jobs
        self.batch_wait_s = batch_wait_s
        self.out_ext = out_ext
        self.faults = parse_faults(faults if faults is not None else os.environ.get("MIVC_FAULT"))
        self.log = log or (lambda *a: None)
        self.jobs_q: queue.Queue[_Lease] = queue.Queue()
        self.active: set[_Lease] = set()
        self.active_lock = threading.Lock()
        self.stop = threading.Event()
        self.last_job = time.monotonic()
        self.n_jobs = 0
        self.n_jobs_lock = threading.Lock()
        self.completed: list[proto.Reply] = []

    # ------------------------------------------------------------------ faults
    def _fault(self, kind: str, idx: str) -> bool:
        for f in self.faults:
            if f["kind"] == kind and not f["fired"] and (f["idx"] is None or f["idx"] == idx):
                f["fired"] = True
                return True
        return False

    # ------------------------------------------------------------------ lease threads
    def _claim_slot(self) -> bool:
        with self.n_jobs_lock:
            if self.max_jobs is not None and self.n_jobs >= self.max_jobs:
                return False
            self.n_jobs += 1
            return True

    def _release_slot(self):
        with self.n_jobs_lock:
            self.n_jobs -= 1

    def _lease_loop(self):
        while not self.stop.is_set():
            if not self._claim_slot():
                return
            try:
                sock = socket.create_connection(self.addr, timeout=self.dial_timeout)
            except OSError as e:
                self._release_slot()
                self.log(f"dial {self.addr[0]}:{self.addr[1]} failed: {e}")
                self.stop.wait(self.retry_s)
                continue
            try:
                sock.settimeout(None)
                sock.sendall(f"hello;{self.worker_id};{self.gpu}\n".encode())
                lines = proto.LineSocket(sock)
                while True:
                    data = lines.recv_message(timeout=None)
                    if not data:
                        raise ConnectionError("server closed the connection")
                    if proto.is_heartbeat(data) or data.strip() == b"idle":
                        continue
                    break
            except (OSError, ConnectionError, proto.ProtocolError) as e:
                self._release_slot()
                sock.close()
                self.log(f"read failed: {e}")
                self.stop.wait(min(self.retry_s, 1.0))
                continue
            self.last_job = time.monotonic()
            try:
                job = proto.parse_job(data)
            except proto.ProtocolError as e:
                # reply on the connection instead of blocking forever (D14)
                try:
                    sock.sendall(proto.Reply(False, "?", str(e)).encode())
                finally:
                    sock.close()
                continue
            lease = _Lease(sock, job)
            with self.active_lock:
                self.active.add(lease)
            self.jobs_q.put(lease)
            lease.done.wait()
            with self.active_lock:
                self.active.discard(lease)
            try:
                if lease.silent:
                    while sock.recv(4096):          # hold the lease until the server drops it
                        pass
                elif lease.reply is not None:
                    with lease.lock:
                        sock.sendall(lease.reply.encode())
                    self.completed.append(lease.reply)
            except OSError as e:
                self.log(f"reply failed: {e}")
            finally:
                sock.close()

    def _heartbeat_loop(self):
        while not self.stop.wait(self.heartbeat_s):
            with self.active_lock:
                leases = list(self.active)
            for ls in leases:
                if ls.silent:
                    continue
                try:
                    with ls.lock:
                        ls.sock.sendall(f"heart;{ls.job.idx}\n".encode())
                except OSError:
                    pass

    # ------------------------------------------------------------------ jobs
    def _finish(self, lease: _Lease, ok: bool, reason: str = ""):
        lease.reply = proto.Reply(ok, lease.job.idx, reason)
        lease.done.set()

    def _run_batch(self, batch: list[_Lease]):
        from ..backends import PieceJob
        by_args: dict[str, list[_Lease]] = {}
        for ls in batch:
            by_args.setdefault(ls.job.args, []).append(ls)
        for args, group in by_args.items():
            if not args.strip():
                for ls in group:   # client.go:87-90 ("转换参数为空")
                    self._finish(ls, False, "conversion arguments are empty")
                continue
            jobs, temps, ready = [], [], []
            for ls in group:
                j = ls.job
                if self._fault("hang", j.idx):
                    ls.silent = True                # never answered: lease timeout on the server
                    ls.done.set()
                    continue
                try:
                    local, tmp = self.transport.fetch(j.dir, j.idx, os.path.join(self.scratch, "in"))
                except TransportError as e:
                    self._finish(ls, False, str(e))
                    continue
                if self._fault("crash_after_fetch", j.idx):
                    self.log(f"fault: crash after fetching {j.idx}")
                    os._exit(17)
                if tmp:
                    temps.append(local)
                odir = os.path.join(self.scratch, "out", out_dir_name(j.dir))
                os.makedirs(odir, exist_ok=True)
                jobs.append(PieceJob(j.idx, local, os.path.join(odir, f"{j.idx}.{self.out_ext}"),
                                     os.path.join(odir, f"c{j.idx}.{self.out_ext}.log")))
                ready.append(ls)
            t0 = time.perf_counter()
            results = self.backend.run(jobs, args) if jobs else []
            get_logger("worker").event("batch", worker=self.worker_id, pieces=[j.idx for j in jobs],
                                       seconds=round(time.perf_counter() - t0, 4),
                                       ok=[r.ok for r in results])
            for ls, pj, r in zip(ready, jobs, results):
                j = ls.job
                try:
                    if not r.ok:
                        self._finish(ls, False, r.reason)
                        continue
                    if self._fault("fail", j.idx):
                        self._finish(ls, False, "injected failure")
                        continue
                    if self._fault("garbage", j.idx):
                        ls.reply = None
                        with ls.lock:
                            ls.sock.sendall(b"\x00\xffgarbage\n")
                        ls.done.set()
                        continue
                    if self._fault("short", j.idx):
                        ls.reply = None
                        with ls.lock:
                            ls.sock.sendall(b"su")
                        ls.done.set()
                        continue
                    if self._fault("disconnect", j.idx):
                        ls.reply = None
                        ls.done.set()
                        continue
                    odir = out_dir_name(j.dir)
                    try:
                        if pj.log_path and os.path.exists(pj.log_path):   # log first, as client.go:153-161
                            self.transport.store(pj.log_path, odir, os.path.basename(pj.log_path))
                        self.transport.store(pj.out_path, odir, f"{j.idx}.{self.out_ext}")
                    except (TransportError, OSError) as e:
                        self._finish(ls, False, f"store: {e}")
                        continue
                    self._finish(ls, True)
                finally:
                    for pth in (pj.out_path, pj.log_path):   # client.go:133-139 cleanup
                        if pth and os.path.exists(pth):
                            os.remove(pth)
            for t in temps:
                if os.path.exists(t):
                    os.remove(t)

    def run(self) -> int:
        threads = [threading.Thread(target=self._lease_loop, daemon=True) for _ in range(self.leases)]
        hb = threading.Thread(target=self._heartbeat_loop, daemon=True)
        for t in threads:
            t.start()
        hb.start()
        try:
            while True:
                try:
                    first = self.jobs_q.get(timeout=0.1)
                except queue.Empty:
                    if not any(t.is_alive() for t in threads):
                        break
                    if self.idle_exit_s is not None and time.monotonic() - self.last_job > self.idle_exit_s:
                        with self.active_lock:
                            busy = bool(self.active)
                        if not busy:
                            break
                    continue
                batch = [first]
                deadline = time.monotonic() + self.batch_wait_s
                while len(batch) < self.leases:
                    left = deadline - time.monotonic()
                    if left <= 0:
                        break
                    try:
                        batch.append(self.jobs_q.get(timeout=left))
                    except queue.Empty:
                        break
                try:
                    self._run_batch(batch)
                except Exception as e:  # noqa: BLE001 - never leave a lease unanswered
                    for ls in batch:
                        if not ls.done.is_set():
                            self._finish(ls, False, f"worker error: {e}")
                for ls in batch:
                    if not ls.done.is_set() and not ls.silent:
                        self._finish(ls, False, "worker error")
                self.last_job = time.monotonic()
        finally:
            self.stop.set()
            for t in threads:
                t.join(timeout=1.0)
            shutil.rmtree(self.scratch, ignore_errors=True)
            try:
                self.backend.close()
            except Exception:  # noqa: BLE001
                pass
        return 0


def env_config(env: dict | None = None) -> dict:
    """The reference's environment contract (client.go:22-36): SERVER_IP required,
    SERVER_PORT optional (8055); FTP_USERNAME/FTP_PASSWORD required by the http
    transport (the FTP replacement).  A missing variable prints ``<NAME> NIL``."""
    env = os.environ if env is None else env
    missing = []
    if not env.get("SERVER_IP"):
        missing.append("SERVER_IP")
    if env.get("MIVC_TRANSPORT", "localfs") == "http":
        missing += [k for k in ("FTP_USERNAME", "FTP_PASSWORD") if not env.get(k)]
    if missing:
        for k in missing:
            print(f"{k} NIL", file=sys.stderr)
        raise SystemExit(1)
    return {"server_ip": env["SERVER_IP"], "port": int(env.get("SERVER_PORT", "8055"))}
