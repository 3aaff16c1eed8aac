"""Piece transports: how a worker gets ``<dir>/<idx>`` and returns its output.

Reference: input over HTTP from an external nginx rooted at the coordinator's
CWD (``wget http://SERVER_IP/<dir>/<idx>.mp4``, client.go:92-94; exit code
ignored, D11); output and log over FTP to ``/home/vuser/<dir>/`` with
plaintext credentials from the environment (client.go:132-175).

Here both directions go through one pluggable interface:

* :class:`LocalFs` -- shared filesystem (one node, or NFS): zero-copy read of the
  split directory, atomic rename into the output root.
* :class:`HttpTransport` + :class:`PieceHttpServer` -- a built-in HTTP server run by
  the coordinator: ``GET /piece/<dir>/<idx>`` (the server resolves the piece's
  container), ``GET /<dir>/<file>`` (nginx-style), ``PUT /out/<dir>/<name>``
  guarded by HTTP basic auth with ``FTP_USERNAME``/``FTP_PASSWORD`` (the reference's
  credential variables).  No external nginx/FTP daemon is needed.
"""
from __future__ import annotations

import base64
import http.server
import os
import shutil
import threading
import urllib.error
import urllib.parse
import urllib.request

from ..segment.split import PIECE_RE, piece_files


class TransportError(RuntimeError):
    pass


def _safe(*parts: str) -> str:
    """Join relative path parts, refusing absolute paths, backslashes and . / .. segments."""
    for p in parts:
        if p.startswith("/") or "\\" in p or any(s in ("", ".", "..") for s in p.split("/")):
            raise TransportError(f"unsafe path component {p!r}")
    return "/".join(parts)


def resolve_piece(src_root: str, d: str, idx: str) -> str:
    _safe(d, idx)
    pdir = os.path.join(src_root, d)
    files = piece_files(pdir)
    if idx not in files:
        raise TransportError(f"piece {d}/{idx} not found")
    return os.path.join(pdir, files[idx])


class LocalFs:
    name = "localfs"

    def __init__(self, src_root: str = ".", out_root: str = "out"):
        self.src_root = src_root
        self.out_root = out_root

    def fetch(self, d: str, idx: str, scratch: str) -> tuple[str, bool]:
        """Returns (local path, is_temporary)."""
        return resolve_piece(self.src_root, d, idx), False

    def store(self, local: str, d: str, name: str) -> None:
        _safe(d, name)
        dst_dir = os.path.join(self.out_root, d)
        os.makedirs(dst_dir, exist_ok=True)
        tmp = os.path.join(dst_dir, f".{name}.part{os.getpid()}")
        shutil.copyfile(local, tmp)
        os.replace(tmp, os.path.join(dst_dir, name))


class HttpTransport:
    name = "http"

    def __init__(self, host: str, port: int, user: str | None, password: str | None, timeout: float = 60.0):
        self.base = f"http://{host}:{port}"
        self.auth = None
        if user is not None and password is not None:
            self.auth = "Basic " + base64.b64encode(f"{user}:{password}".encode()).decode()
        self.timeout = timeout

    def fetch(self, d: str, idx: str, scratch: str) -> tuple[str, bool]:
        url = f"{self.base}/piece/{urllib.parse.quote(_safe(d, idx))}"
        try:
            with urllib.request.urlopen(url, timeout=self.timeout) as r:
                name = r.headers.get("X-Piece-Name") or f"{idx}.mp4"
                if not PIECE_RE.match(name):
                    raise TransportError(f"server returned a bad piece name {name!r}")
                os.makedirs(scratch, exist_ok=True)
                path = os.path.join(scratch, name)
                with open(path, "wb") as f:
                    shutil.copyfileobj(r, f)
        except urllib.error.HTTPError as e:
            raise TransportError(f"download failed: HTTP {e.code}") from None
        except (urllib.error.URLError, OSError) as e:
            raise TransportError(f"download failed: {e}") from None
        return path, True

    def store(self, local: str, d: str, name: str) -> None:
        url = f"{self.base}/out/{urllib.parse.quote(_safe(d, name))}"
        with open(local, "rb") as f:
            data = f.read()
        req = urllib.request.Request(url, data=data, method="PUT")
        if self.auth:
            req.add_header("Authorization", self.auth)
        try:
            with urllib.request.urlopen(req, timeout=self.timeout) as r:
                r.read()
        except urllib.error.HTTPError as e:
            raise TransportError(f"upload failed: HTTP {e.code}") from None
        except (urllib.error.URLError, OSError) as e:
            raise TransportError(f"upload failed: {e}") from None


class _Handler(http.server.BaseHTTPRequestHandler):
    server_version = "mivc-pieces/1"

    def log_message(self, fmt, *args):  # quiet
        pass

    def _path(self) -> list[str]:
        p = urllib.parse.unquote(urllib.parse.urlparse(self.path).path)
        parts = [x for x in p.split("/") if x]
        if any(x in (".", "..") or "\\" in x for x in parts):
            raise TransportError("bad path")
        return parts

    def _send_file(self, path: str, name: str):
        size = os.path.getsize(path)
        self.send_response(200)
        self.send_header("Content-Length", str(size))
        self.send_header("Content-Type", "application/octet-stream")
        self.send_header("X-Piece-Name", name)
        self.end_headers()
        with open(path, "rb") as f:
            shutil.copyfileobj(f, self.wfile)

    def do_GET(self):  # noqa: N802
        srv = self.server
        try:
            parts = self._path()
            if len(parts) >= 3 and parts[0] == "piece":
                path = resolve_piece(srv.src_root, "/".join(parts[1:-1]), parts[-1])
                return self._send_file(path, os.path.basename(path))
            path = os.path.join(srv.src_root, *parts)
            if parts and os.path.isfile(path):
                return self._send_file(path, parts[-1])
        except TransportError:
            pass
        self.send_error(404)

    def do_PUT(self):  # noqa: N802
        srv = self.server
        if srv.auth and self.headers.get("Authorization") != srv.auth:
            self.send_response(401)
            self.send_header("WWW-Authenticate", 'Basic realm="mivc"')
            self.end_headers()
            return
        try:
            parts = self._path()
        except TransportError:
            return self.send_error(400)
        if len(parts) < 3 or parts[0] != "out":
            return self.send_error(404)
        n = int(self.headers.get("Content-Length", "0"))
        dst_dir = os.path.join(srv.out_root, *parts[1:-1])
        os.makedirs(dst_dir, exist_ok=True)
        tmp = os.path.join(dst_dir, f".{parts[-1]}.part{threading.get_ident()}")
        with open(tmp, "wb") as f:
            left = n
            while left > 0:
                chunk = self.rfile.read(min(left, 1 << 20))
                if not chunk:
                    break
                f.write(chunk)
                left -= len(chunk)
        if left:
            os.unlink(tmp)
            return self.send_error(400)
        os.replace(tmp, os.path.join(dst_dir, parts[-1]))
        self.send_response(201)
        self.send_header("Content-Length", "0")
        self.end_headers()


class PieceHttpServer:
    """Threaded HTTP server replacing the reference's external nginx (GET) + FTP (STOR)."""

    def __init__(self, src_root: str, out_root: str, host: str = "0.0.0.0", port: int = 0,
                 user: str | None = None, password: str | None = None):
        self.httpd = http.server.ThreadingHTTPServer((host, port), _Handler)
        self.httpd.daemon_threads = True
        self.httpd.src_root = src_root
        self.httpd.out_root = out_root
        self.httpd.auth = ("Basic " + base64.b64encode(f"{user}:{password}".encode()).decode()) \
            if user is not None and password is not None else None
        self.port = self.httpd.server_address[1]
        self.thread = threading.Thread(target=self.httpd.serve_forever, daemon=True)

    def start(self) -> "PieceHttpServer":
        self.thread.start()
        return self

    def stop(self):
        self.httpd.shutdown()
        self.httpd.server_close()


def from_env(env: dict | None = None) -> LocalFs | HttpTransport:
    """Worker transport from the environment: ``MIVC_TRANSPORT`` = localfs (default) | http."""
    env = os.environ if env is None else env
    kind = env.get("MIVC_TRANSPORT", "localfs")
    if kind == "localfs":
        return LocalFs(env.get("MIVC_SRC_ROOT", "."), env.get("MIVC_OUT_ROOT", "out"))
    if kind == "http":
        return HttpTransport(env["SERVER_IP"], int(env.get("MIVC_HTTP_PORT", "8056")),
                             env.get("FTP_USERNAME"), env.get("FTP_PASSWORD"))
    raise TransportError(f"unknown transport {kind}")
