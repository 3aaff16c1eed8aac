"""Coordinator <-> worker wire protocol (one TCP connection = one job lease).

Reference semantics:

    worker connects                       == "give me work"              client.go:38
    server -> worker : <dir>;<idx>;<args>  one unframed write            server.go:179
    worker -> server : success;<idx>                                     client.go:173
                     | fail;<idx>[;<reason>]                             client.go:89,144-170
    both close; the worker reconnects for the next job                   client.go:67,76-79

The reference reads at most 100 bytes per message (client.go:43, server.go:271)
and has no framing, so long directory names or argument strings were silently
truncated (defect D9), ``;`` inside args broke parsing (D10) and a 2-field
message crashed the worker (D10).  This implementation keeps the same tokens
but terminates every message with ``\\n`` (v1).  A v1 reader accepts unterminated
v0 messages (EOF or the 100-byte window ends them); a v1 writer never emits a
message a v0 peer could not parse, so old and new peers interoperate.

v1 additions (all optional): ``heart;<idx>`` lease renewal from a busy worker
(the reference's unused ``heart`` at server.go:310-323), ``hello;<worker>;<gpu>``
census greeting (`server t`), and ``idle`` from the server when no work is left.
"""
from __future__ import annotations

import asyncio
import socket
from dataclasses import dataclass

V0_READ = 100  # bytes: the reference's fixed read window
MAX_LINE = 64 * 1024


class ProtocolError(ValueError):
    pass


@dataclass(frozen=True)
class Job:
    dir: str
    idx: str
    args: str

    def encode(self, v1: bool = True) -> bytes:
        """v1 peers get a '\\n'-terminated line; a v0 peer (no ``hello``) gets the bare
        tokens, since the reference worker would pass a trailing newline on to ffmpeg."""
        if ";" in self.dir or ";" in self.idx:
            raise ProtocolError("';' is not allowed in the directory or piece index")
        if ";" in self.args or "\n" in self.args:
            raise ProtocolError("';' and newlines are not allowed in the conversion arguments")
        msg = f"{self.dir};{self.idx};{self.args}"
        if not v1 and len(msg.encode()) > V0_READ:
            raise ProtocolError(f"job message exceeds the {V0_READ}-byte v0 read window")
        return (msg + "\n").encode() if v1 else msg.encode()

    @property
    def piece_path(self) -> str:
        """dir/idx.mp4 -- the reference's piece naming (client.go:54)."""
        return f"{self.dir}/{self.idx}"


@dataclass(frozen=True)
class Reply:
    ok: bool
    idx: str
    reason: str = ""

    def encode(self) -> bytes:
        if self.ok:
            return f"success;{self.idx}\n".encode()
        r = self.reason.replace(";", ",").replace("\n", " ")
        return (f"fail;{self.idx};{r}\n" if r else f"fail;{self.idx}\n").encode()


def parse_job(data: bytes | str) -> Job:
    s = data.decode(errors="replace") if isinstance(data, bytes) else data
    s = s.rstrip("\r\n")
    parts = s.split(";", 2)
    if len(parts) < 2 or not parts[0] or not parts[1]:
        raise ProtocolError(f"malformed job message {s[:80]!r}")
    return Job(parts[0], parts[1], parts[2] if len(parts) > 2 else "")


def parse_reply(data: bytes | str) -> Reply:
    s = data.decode(errors="replace") if isinstance(data, bytes) else data
    s = s.rstrip("\r\n")
    parts = s.split(";", 2)
    if parts[0] == "success" and len(parts) >= 2 and parts[1]:
        return Reply(True, parts[1])
    if parts[0] == "fail" and len(parts) >= 2 and parts[1]:
        return Reply(False, parts[1], parts[2] if len(parts) > 2 else "")
    raise ProtocolError(f"malformed reply {s[:80]!r}")


def is_heartbeat(line: bytes | str) -> bool:
    s = line.decode(errors="replace") if isinstance(line, bytes) else line
    return s.startswith("heart")


async def read_message(reader: asyncio.StreamReader, timeout: float | None = None) -> bytes:
    """Read one message: up to and including '\\n' (v1), or whatever an unframed v0 peer
    wrote before closing.  Bytes after the newline stay buffered in ``reader``."""
    async def _read():
        try:
            return await reader.readuntil(b"\n")
        except asyncio.IncompleteReadError as e:
            return e.partial
        except asyncio.LimitOverrunError:
            raise ProtocolError("message too long") from None
    if timeout is None:
        return await _read()
    return await asyncio.wait_for(_read(), timeout)


class LineSocket:
    """Blocking line reader over a socket (the worker side); keeps bytes past '\\n'."""

    def __init__(self, sock: socket.socket):
        self.sock = sock
        self.buf = b""

    def recv_message(self, timeout: float | None = None) -> bytes:
        self.sock.settimeout(timeout)
        while b"\n" not in self.buf:
            if len(self.buf) > MAX_LINE:
                raise ProtocolError("message too long")
            chunk = self.sock.recv(4096)
            if not chunk:
                out, self.buf = self.buf, b""
                return out
            self.buf += chunk
        i = self.buf.index(b"\n") + 1
        out, self.buf = self.buf[:i], self.buf[i:]
        return out
