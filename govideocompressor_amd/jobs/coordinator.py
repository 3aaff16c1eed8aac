"""``server c``: hand out pieces to pull-based workers, track leases, finish.

Reference (server.go:65-121, 161-191, 267-308): a goroutine per connection,
a dispatcher that writes ``dir;idx;args`` to each queued connection in
*descending* piece-table order, deletes the source piece on ``success`` and
``os.Exit(0)`` when the remain map is empty.  Its defects are fixed here
(SURVEY.md App. B):

* D5  -- single-threaded asyncio: every state change happens on one event loop;
* D6  -- ``fail`` / disconnect / lease timeout re-queue the piece (up to
  ``max_retries``); the server finishes even if a piece is abandoned and says which;
* D7  -- framed reads (protocol.py), no busy-spin on errors, short messages are errors;
* D8  -- restart without ``-p`` enumerates the *actual* remaining piece names and a
  state file (``<dir>/.mivc_state.json``) remembers finished pieces;
* D4  -- the listen error is reported, not dereferenced.

Leases are renewed by ``heart;<idx>`` messages from v1 workers; v0 workers (which
never send them) are covered by ``lease_timeout``, which should then exceed the
longest piece's encode time.
"""
from __future__ import annotations

import asyncio
import json
import os
import time
from collections import deque
from dataclasses import asdict, dataclass, field

from ..obs import get_logger
from ..segment import merge as M
from ..segment.split import piece_files
from . import protocol as proto


def now_str() -> str:
    return time.strftime("%Y-%m-%d %H:%M:%S")


def out_dir_name(d: str) -> str:
    """Output sub-directory for split dir ``d`` (the reference used /home/vuser/<d>)."""
    return os.path.basename(d.rstrip("/")) or d


@dataclass
class Piece:
    idx: str
    state: str = "queued"        # queued | leased | done | failed
    attempts: int = 0
    worker: str = ""
    leased_at: float = 0.0
    last_beat: float = 0.0
    reason: str = ""
    stats: dict = field(default_factory=dict)


class _Conn:
    _ids = 0

    def __init__(self, reader, writer):
        _Conn._ids += 1
        self.id = _Conn._ids
        self.reader = reader
        self.writer = writer
        peer = writer.get_extra_info("peername")
        self.peer = f"{peer[0]}:{peer[1]}" if peer else "?"
        self.worker = ""
        self.gpu = ""
        self.lease: str | None = None
        self.closed = False
        self.v1 = False

    def close(self):
        if not self.closed:
            self.closed = True
            try:
                self.writer.close()
            except Exception:  # noqa: BLE001
                pass


class Coordinator:
    def __init__(self, split_dir: str, args: str, pieces: list[str] | None = None, port: int = 8055,
                 host: str = "0.0.0.0", out_root: str = "out", lease_timeout: float = 600.0, max_retries: int = 3,
                 delete_source: bool = True, merge: bool = False, http_port: int | None = None,
                 http_auth: tuple[str, str] | None = None, log=print, state_file: bool = True,
                 hello_wait: float = 0.25, src_root: str | None = None):
        # the split directory on this host, and the token workers receive: its path relative to
        # the shared source root (the reference's nginx root = the coordinator's CWD, client.go:92)
        self.src_root = os.path.abspath(src_root or os.getcwd())
        self.dir = os.path.abspath(split_dir)
        rel = os.path.relpath(self.dir, self.src_root)
        if rel == "." or rel.startswith(".."):
            raise ValueError(f"split directory {split_dir} is not inside the source root {self.src_root}")
        self.token = rel.replace(os.sep, "/")
        from .ffargs import expand_preset
        self.args = expand_preset(args)   # "264"/"265" shorthands (server.go:67-71)
        self.port = port
        self.host = host
        self.out_root = out_root
        self.lease_timeout = lease_timeout
        self.max_retries = max_retries
        self.delete_source = delete_source
        self.merge = merge
        self.http_port = http_port
        self.http_auth = http_auth
        self.log = log
        self.hello_wait = hello_wait
        self.partial = bool(pieces)
        self.state_path = os.path.join(self.dir, ".mivc_state.json") if state_file else None
        self.out_dir = os.path.join(out_root, out_dir_name(self.dir))
        prior = self._load_state()
        files = piece_files(self.dir)
        if pieces:
            order = list(pieces)
        else:
            order = sorted(files, key=lambda s: int(s))
        self.all_pieces = sorted(set(files) | set(prior.get("done", {})), key=lambda s: int(s))
        self.pieces: dict[str, Piece] = {}
        for idx in order:
            p = Piece(idx)
            if idx in prior.get("done", {}) and idx not in files:
                p.state, p.stats = "done", prior["done"][idx]
            self.pieces[idx] = p
        # dispatch order: the reference walks its table from the end (server.go:170-185)
        self.queue: deque[str] = deque(i for i in order if self.pieces[i].state == "queued")
        self.waiting: deque[_Conn] = deque()
        self.conns: set[_Conn] = set()
        self.workers: dict[str, dict] = {}
        self.done_event: asyncio.Event | None = None
        self.t_start = time.time()
        self.http = None
        self.jlog = get_logger("coordinator")

    # ------------------------------------------------------------------ state file
    def _load_state(self) -> dict:
        if self.state_path and os.path.exists(self.state_path):
            try:
                with open(self.state_path) as f:
                    return json.load(f)
            except (OSError, ValueError):
                return {}
        return {}

    def _save_state(self):
        if not self.state_path:
            return
        st = {"dir": self.dir, "args": self.args,
              "done": {i: p.stats for i, p in self.pieces.items() if p.state == "done"},
              "failed": {i: p.reason for i, p in self.pieces.items() if p.state == "failed"}}
        prior = self._load_state().get("done", {})
        for k, v in prior.items():
            st["done"].setdefault(k, v)
        tmp = self.state_path + ".tmp"
        with open(tmp, "w") as f:
            json.dump(st, f, indent=1, default=float)
        os.replace(tmp, self.state_path)

    # ------------------------------------------------------------------ bookkeeping
    def remaining(self) -> list[str]:
        return [i for i, p in self.pieces.items() if p.state in ("queued", "leased")]

    def _remain_line(self) -> str:
        rem = sorted(self.remaining(), key=lambda s: int(s))
        return f"[{len(rem)}]remain job[map[{' '.join(f'{int(i)}:{i}' for i in rem)}]]"

    def _check_done(self):
        if not self.remaining() and self.done_event is not None:
            self.done_event.set()

    def _requeue(self, idx: str, reason: str):
        p = self.pieces[idx]
        self.jlog.event("requeue", piece=idx, reason=reason, attempts=p.attempts)
        p.worker, p.reason = "", reason
        if p.attempts > self.max_retries:
            p.state = "failed"
            self.log(f"@@[{idx}]piece abandoned after {p.attempts} attempts: {reason}")
            self._save_state()
        else:
            p.state = "queued"
            self.queue.append(idx)
        self._check_done()

    # ------------------------------------------------------------------ dispatch
    def _dispatch(self):
        while self.waiting and self.queue:
            c = self.waiting.popleft()
            if c.closed:
                continue
            idx = self.queue.pop()
            job = proto.Job(self.token, idx, self.args)
            try:
                c.writer.write(job.encode(v1=c.v1))
            except Exception as e:  # noqa: BLE001
                self.log(f"!!!send error[{e}]")
                self.queue.append(idx)
                c.close()
                continue
            p = self.pieces[idx]
            p.state, p.attempts, p.worker = "leased", p.attempts + 1, c.worker or c.peer
            p.leased_at = p.last_beat = time.monotonic()
            c.lease = idx
            self.log(f"[{now_str()}]OnConnect send success[{self.token};{idx}]")
            self.jlog.event("dispatch", piece=idx, worker=p.worker, attempt=p.attempts)

    def _on_reply(self, c: _Conn, r: proto.Reply):
        idx = r.idx
        if c.lease is None or idx != c.lease:
            self.log(f"!!!unexpected reply for piece [{idx}] from {c.peer}")
            c.close()
            return
        c.lease = None
        c.close()
        p = self.pieces[idx]
        if r.ok:
            p.state, p.reason = "done", ""
            stats_path = os.path.join(self.out_dir, f"c{idx}.mp4.log")
            if os.path.exists(stats_path):
                try:
                    with open(stats_path) as f:
                        p.stats = json.load(f)
                except (OSError, ValueError):
                    p.stats = {}
            self.log(f"###[{now_str()}] [{idx}]piece convert success")
            self.jlog.event("success", piece=idx, worker=c.worker or c.peer,
                            lease_s=round(time.monotonic() - p.leased_at, 3), stats=p.stats)
            if self.delete_source:
                files = piece_files(self.dir)
                if idx in files:
                    try:
                        os.remove(os.path.join(self.dir, files[idx]))
                    except OSError:
                        pass
            self._save_state()
            if self.remaining():
                self.log(self._remain_line())
            self._check_done()
        else:
            self.log(f"@@[{idx}]piece convert fail")
            if r.reason:
                self.log(f"@@reason[{r.reason}]")
            self._requeue(idx, r.reason or "fail")
            self._dispatch()

    def _on_hello(self, c: _Conn, line: str):
        parts = line.split(";")
        c.v1 = True
        c.worker = parts[1] if len(parts) > 1 else ""
        c.gpu = parts[2] if len(parts) > 2 else ""
        self.workers[c.worker or c.peer] = {"peer": c.peer, "gpu": c.gpu, "seen": time.time()}
        if c.lease:
            self.pieces[c.lease].worker = c.worker

    async def _serve_conn(self, reader, writer):
        c = _Conn(reader, writer)
        self.conns.add(c)
        try:
            # v1 workers greet first; a v0 worker stays silent until it has a job
            try:
                first = await proto.read_message(reader, timeout=self.hello_wait)
            except asyncio.TimeoutError:
                first = None
            except (proto.ProtocolError, ConnectionError, OSError):
                first = b""
            if first == b"":
                return
            if first is not None:
                line = first.decode(errors="replace").rstrip("\r\n")
                if line.startswith("hello;"):
                    self._on_hello(c, line)
            self.waiting.append(c)
            self._dispatch()
            while not c.closed:
                try:
                    data = await proto.read_message(reader)
                except (proto.ProtocolError, ConnectionError, OSError):
                    data = b""
                if not data:
                    break
                line = data.decode(errors="replace").rstrip("\r\n")
                if line.startswith("hello;"):
                    self._on_hello(c, line)
                    continue
                if proto.is_heartbeat(line):
                    if c.lease:
                        self.pieces[c.lease].last_beat = time.monotonic()
                    continue
                if line.startswith(("success", "fail")):
                    try:
                        r = proto.parse_reply(line)
                    except proto.ProtocolError as e:
                        self.log(f"!!!bad reply from {c.peer}: {e}")
                        break
                    self._on_reply(c, r)
                    break
                # anything else: ignored, as the reference does (server.go:301-302)
        finally:
            self.conns.discard(c)
            if c in self.waiting:
                self.waiting.remove(c)
            if c.lease is not None:
                idx, c.lease = c.lease, None
                self.log(f"@@[{idx}]piece lost: worker {c.worker or c.peer} disconnected")
                self._requeue(idx, "worker disconnected")
                self._dispatch()
            c.close()

    async def _watchdog(self):
        period = max(0.05, min(1.0, self.lease_timeout / 4))
        while True:
            await asyncio.sleep(period)
            t = time.monotonic()
            for c in list(self.conns):
                if c.lease is not None and t - self.pieces[c.lease].last_beat > self.lease_timeout:
                    idx, c.lease = c.lease, None
                    self.log(f"@@[{idx}]piece lease timed out on {c.worker or c.peer}")
                    c.close()
                    self._requeue(idx, "lease timeout")
            self._dispatch()

    # ------------------------------------------------------------------ lifecycle
    def _prepare_outputs(self):
        os.makedirs(self.out_dir, exist_ok=True)
        if not self.partial:
            M.make_filelist(self.all_pieces, self.out_dir, "mp4")
            M.make_concat_script(self.out_dir)

    async def run_async(self) -> int:
        self.log(f"c:[{self.token}] [{self.args}] [{';'.join(self.pieces) if self.partial else ''}]")
        if not self.args.strip():
            self.log("warning: empty conversion arguments -- every worker will fail the job")
        try:
            proto.Job(self.token, "0", self.args).encode()
        except proto.ProtocolError as e:
            self.log(f"bad input argument: {e}")
            return 2
        self._prepare_outputs()
        self.log(f"pieceNum[{len(self.pieces)}]")
        self.done_event = asyncio.Event()
        try:
            server = await asyncio.start_server(self._serve_conn, self.host, self.port, reuse_address=True)
        except OSError as e:
            self.log(f"Failure to listen: {e}")
            return 2
        self.port = server.sockets[0].getsockname()[1]
        if self.http_port is not None:
            from .transport import PieceHttpServer
            user, pw = self.http_auth or (None, None)
            self.http = PieceHttpServer(self.src_root, self.out_root, self.host, self.http_port, user, pw).start()
            self.http_port = self.http.port
        self.listening()
        self._check_done()
        wd = asyncio.create_task(self._watchdog())
        async with server:
            await self.done_event.wait()
            wd.cancel()
            server.close()
            for c in list(self.conns):
                c.close()
        if self.http:
            self.http.stop()
        failed = [i for i, p in self.pieces.items() if p.state == "failed"]
        self._save_state()
        if failed:
            self.log(f"!!!{len(failed)} piece(s) failed: {';'.join(sorted(failed, key=int))} "
                     f"(re-run with -p \"{';'.join(sorted(failed, key=int))}\")")
            return 1
        self.log("------Convert All Done-----")
        if self.merge and not self.partial:
            out = M.merge_dir(self.out_dir)
            self.log(f"merged [{out}]")
        return 0

    def listening(self):
        """Hook called once the sockets are bound (tests read self.port here)."""
        self.log(f"listening on {self.host}:{self.port}" +
                 (f" (pieces over http :{self.http_port})" if self.http_port else ""))

    def run(self) -> int:
        return asyncio.run(self.run_async())

    def summary(self) -> dict:
        return {"dir": self.dir, "pieces": {i: asdict(p) for i, p in self.pieces.items()},
                "workers": self.workers, "elapsed_s": time.time() - self.t_start}
