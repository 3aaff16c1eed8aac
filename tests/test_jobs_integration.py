"""T3/T4: localhost coordinator + workers over the real TCP protocol, with fault injection.

Workers run in threads (CPU backend = the C++ reference encoder) except where a fault
kills the process, which uses a subprocess worker."""
import json
import os
import socket
import subprocess
import sys
import threading
import time

import numpy as np
import pytest

from govideocompressor_amd.jobs import transport as T
from govideocompressor_amd.jobs.coordinator import Coordinator
from govideocompressor_amd.jobs.worker import Worker
from govideocompressor_amd.segment.split import piece_files, split
from govideocompressor_amd.utils import yuv

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.timeout(120)


def _make_split(tmp_path, n_pieces=4, frames_per=3, w=48, h=32):
    c = yuv.synth_clip_cpu(n_pieces * frames_per, w, h, seed=11)
    src = tmp_path / "clip.y4m"
    yuv.write_y4m(str(src), c)
    d, n = split(str(src), frames=frames_per, out_root=str(tmp_path), log=lambda s: None)
    assert n == n_pieces
    return c, d


class _Run:
    def __init__(self, tmp_path, d, args="264", **kw):
        self.logs = []
        kw.setdefault("lease_timeout", 30)
        kw.setdefault("out_root", str(tmp_path / "out"))
        self.co = Coordinator(d, args, port=0, host="127.0.0.1", log=self.logs.append, src_root=str(tmp_path), **kw)
        self.ready = threading.Event()
        orig = self.co.listening
        self.co.listening = lambda: (orig(), self.ready.set())
        self.rc = None
        self.th = threading.Thread(target=self._run, daemon=True)
        self.th.start()
        assert self.ready.wait(20), self.logs

    def _run(self):
        self.rc = self.co.run()
        self.ready.set()

    @property
    def port(self):
        return self.co.port

    def join(self, t=60):
        self.th.join(t)
        assert not self.th.is_alive(), "coordinator did not finish:\n" + "\n".join(self.logs)
        return self.rc


def _worker(tmp_path, port, faults=None, backend="cpu", transport=None, leases=1, name=None):
    from govideocompressor_amd.backends import get_backend
    tr = transport or T.LocalFs(str(tmp_path), str(tmp_path / "out"))
    return Worker("127.0.0.1", port, get_backend(backend), tr, leases=leases, retry_s=0.1, heartbeat_s=0.2,
                  idle_exit_s=1.5, faults=faults or "", worker_id=name, batch_wait_s=0.05)


def _start(w):
    th = threading.Thread(target=w.run, daemon=True)
    th.start()
    return th


def _check_outputs(host, tmp_path, clip, n, per):
    out = tmp_path / "out" / "12clip.y4m"
    for i in range(n):
        es = host.mp4_demux((out / f"{i}.mp4").read_bytes())
        pics = host.decode(es)
        assert len(pics) == per
        st = json.loads((out / f"c{i}.mp4.log").read_text())
        assert st["frames"] == per and st["psnr_y"] > 30
    return out


def test_two_workers_complete_all(tmp_path, host):
    clip, d = _make_split(tmp_path)
    r = _Run(tmp_path, d, merge=True)
    ths = [_start(_worker(tmp_path, r.port, name=f"w{i}")) for i in range(2)]
    assert r.join() == 0
    for t in ths:
        t.join(10)
    logs = "\n".join(r.logs)
    assert "pieceNum[4]" in logs and "------Convert All Done-----" in logs
    assert "OnConnect send success[12clip.y4m;3]" in logs
    sends = [ln for ln in r.logs if "OnConnect send success" in ln]
    assert sends[0].endswith(";3]")                          # descending dispatch (server.go:170-185)
    assert "[3]remain job[map[0:0 1:1 2:2]]" in logs or "remain job" in logs
    assert piece_files(d) == {}                              # sources deleted on success (server.go:288)
    out = _check_outputs(host, tmp_path, clip, 4, 3)
    merged = host.decode(host.mp4_demux((out / "output.mp4").read_bytes()))
    assert len(merged) == 12
    st = json.load(open(os.path.join(d, ".mivc_state.json")))
    assert sorted(st["done"], key=int) == ["0", "1", "2", "3"]
    assert set(r.co.workers) == {"w0", "w1"}


def test_fail_is_requeued(tmp_path, host):
    clip, d = _make_split(tmp_path, 3)
    r = _Run(tmp_path, d)
    ths = [_start(_worker(tmp_path, r.port, faults="fail")), _start(_worker(tmp_path, r.port))]
    assert r.join() == 0
    logs = "\n".join(r.logs)
    assert "piece convert fail" in logs and "@@reason[injected failure]" in logs
    assert sorted(p.attempts for p in r.co.pieces.values()) == [1, 1, 2]
    _check_outputs(host, tmp_path, clip, 3, 3)
    for t in ths:
        t.join(10)


@pytest.mark.parametrize("fault", ["garbage", "short", "disconnect"])
def test_bad_replies_are_requeued(tmp_path, host, fault):
    clip, d = _make_split(tmp_path, 2)
    r = _Run(tmp_path, d)
    ths = [_start(_worker(tmp_path, r.port, faults=fault)), _start(_worker(tmp_path, r.port))]
    assert r.join() == 0
    assert max(p.attempts for p in r.co.pieces.values()) >= 2
    _check_outputs(host, tmp_path, clip, 2, 3)
    for t in ths:
        t.join(10)


def test_hung_worker_lease_times_out(tmp_path, host):
    clip, d = _make_split(tmp_path, 2)
    r = _Run(tmp_path, d, lease_timeout=1.0)
    ths = [_start(_worker(tmp_path, r.port, faults="hang")), _start(_worker(tmp_path, r.port))]
    assert r.join() == 0
    assert any("lease timed out" in ln for ln in r.logs)
    _check_outputs(host, tmp_path, clip, 2, 3)
    for t in ths:
        t.join(10)


def test_heartbeats_keep_slow_lease(tmp_path):
    """A busy v1 worker renews its lease: with a lease timeout shorter than the encode,
    heartbeats must prevent a spurious re-queue."""
    clip, d = _make_split(tmp_path, 1, frames_per=2)

    class SlowBackend:
        name = "slow"

        def run(self, jobs, args):
            from govideocompressor_amd.backends import get_backend
            time.sleep(1.5)
            b = get_backend("cpu")
            try:
                return b.run(jobs, args)
            finally:
                b.close()

        def close(self):
            pass

    r = _Run(tmp_path, d, lease_timeout=0.6)
    w = Worker("127.0.0.1", r.port, SlowBackend(), T.LocalFs(str(tmp_path), str(tmp_path / "out")),
               retry_s=0.1, heartbeat_s=0.1, idle_exit_s=1.0)
    th = _start(w)
    assert r.join() == 0
    assert r.co.pieces["0"].attempts == 1
    th.join(10)


def test_worker_crash_subprocess(tmp_path, host):
    clip, d = _make_split(tmp_path, 3)
    r = _Run(tmp_path, d)
    env = dict(os.environ, SERVER_IP="127.0.0.1", SERVER_PORT=str(r.port), MIVC_FAULT="crash_after_fetch",
               MIVC_SRC_ROOT=str(tmp_path), MIVC_OUT_ROOT=str(tmp_path / "out"), PYTHONPATH=ROOT)
    p = subprocess.Popen([sys.executable, "-m", "govideocompressor_amd.cli", "client", "--backend", "cpu",
                          "--retry", "0.1", "--idle-exit", "2"], env=env)
    assert p.wait(60) == 17           # died holding a lease
    th = _start(_worker(tmp_path, r.port))
    assert r.join() == 0
    assert any("disconnected" in ln for ln in r.logs)
    _check_outputs(host, tmp_path, clip, 3, 3)
    th.join(10)


def test_retries_exhausted_reports_failed(tmp_path):
    _, d = _make_split(tmp_path, 2)
    r = _Run(tmp_path, d, max_retries=1)
    r.co.args = ""   # every worker answers fail;idx;conversion arguments are empty (client.go:87-90)
    th = _start(_worker(tmp_path, r.port))
    assert r.join() == 1
    logs = "\n".join(r.logs)
    assert "@@reason[conversion arguments are empty]" in logs
    assert "piece(s) failed: 0;1" in logs
    assert len(piece_files(d)) == 2     # nothing deleted
    th.join(10)


def test_partial_pieces_and_restart(tmp_path, host):
    clip, d = _make_split(tmp_path, 4)
    r = _Run(tmp_path, d, pieces=["1", "3"])
    th = _start(_worker(tmp_path, r.port))
    assert r.join() == 0
    sends = [ln.rsplit(";", 1)[1] for ln in r.logs if "OnConnect send success" in ln]
    assert sends == ["3]", "1]"]                    # last -p token first
    assert not os.path.exists(tmp_path / "out" / "12clip.y4m" / "filelist.txt")   # partial: no list
    th.join(10)
    # restart without -p: only the remaining actual pieces are handed out (D8 fixed)
    r2 = _Run(tmp_path, d)
    assert sorted(r2.co.queue, key=int) == ["0", "2"]
    th = _start(_worker(tmp_path, r2.port))
    assert r2.join() == 0
    th.join(10)
    _check_outputs(host, tmp_path, clip, 4, 3)
    fl = (tmp_path / "out" / "12clip.y4m" / "filelist.txt").read_text()
    assert fl == "".join(f"file '{i}.mp4'\n" for i in range(4))


def test_v0_worker_interop(tmp_path):
    """A reference-style worker: no hello, reads <=100 bytes, replies unframed, closes."""
    _, d = _make_split(tmp_path, 1)
    r = _Run(tmp_path, d, hello_wait=0.05)
    s = socket.create_connection(("127.0.0.1", r.port), timeout=10)
    msg = s.recv(100)
    assert msg == b"12clip.y4m;0;-threads 4 -vcodec libx264"      # no '\n' for a v0 peer
    s.sendall(b"success;0")
    s.close()
    assert r.join() == 0


def test_http_transport(tmp_path, host):
    clip, d = _make_split(tmp_path, 2)
    r = _Run(tmp_path, d, http_port=0, http_auth=("vuser", "pw"))
    port = r.co.http_port
    good = T.HttpTransport("127.0.0.1", port, "vuser", "pw")
    bad = T.HttpTransport("127.0.0.1", port, "vuser", "nope")
    # wrong password: upload refused -> fail -> re-queued to the good worker
    w_bad = _worker(tmp_path, r.port, transport=bad)
    w_bad.max_jobs = 1
    th1 = _start(w_bad)
    time.sleep(0.5)
    th2 = _start(_worker(tmp_path, r.port, transport=good))
    assert r.join() == 0
    assert any("upload failed: HTTP 401" in ln for ln in r.logs)
    _check_outputs(host, tmp_path, clip, 2, 3)
    th1.join(10)
    th2.join(10)


def test_http_server_rejects_traversal(tmp_path):
    (tmp_path / "d").mkdir()
    (tmp_path / "d" / "0.y4m").write_bytes(b"x")
    srv = T.PieceHttpServer(str(tmp_path), str(tmp_path / "o"), "127.0.0.1", 0).start()
    try:
        tr = T.HttpTransport("127.0.0.1", srv.port, None, None)
        p, tmp = tr.fetch("d", "0", str(tmp_path / "scratch"))
        assert tmp and open(p, "rb").read() == b"x"
        with pytest.raises(T.TransportError):
            tr.fetch("../etc", "0", str(tmp_path / "scratch"))
        import urllib.request
        with pytest.raises(Exception):
            urllib.request.urlopen(f"http://127.0.0.1:{srv.port}/%2e%2e/x", timeout=5)
    finally:
        srv.stop()


def test_census(tmp_path):
    from govideocompressor_amd.jobs.census import census
    logs, port = [], []
    ev = threading.Event()
    out = {}

    def run():
        out["c"] = census(1.5, 0, "127.0.0.1", log=logs.append, on_listen=lambda p: (port.append(p), ev.set()))
    th = threading.Thread(target=run)
    th.start()
    assert ev.wait(10)
    a = socket.create_connection(("127.0.0.1", port[0]))
    a.sendall(b"hello;gpu-worker-0;3\n")
    b = socket.create_connection(("127.0.0.1", port[0]))
    th.join(10)
    assert len(out["c"]) == 2
    assert "####Online Client[2]####" in logs
    assert any("gpu-worker-0 gpu[3]" in ln for ln in logs)
    a.close()
    b.close()


def test_fake_ffmpeg_backend(tmp_path):
    """Config-1 plumbing: the reference's raw ffmpeg argv through a stub binary on PATH."""
    _, d = _make_split(tmp_path, 2)
    bindir = tmp_path / "bin"
    bindir.mkdir()
    stub = bindir / "ffmpeg"
    stub.write_text("#!/bin/sh\n# fake ffmpeg: copy -i input to the last argument\n"
                    "in=\"\"; prev=\"\"; for a in \"$@\"; do [ \"$prev\" = \"-i\" ] && in=\"$a\"; prev=\"$a\"; last=\"$a\"; done\n"
                    "echo \"fake ffmpeg $*\" >&2\ncp \"$in\" \"$last\"\n")
    stub.chmod(0o755)
    from govideocompressor_amd.backends import get_backend
    r = _Run(tmp_path, d)
    be = get_backend("ffmpeg", binary=str(stub))
    w = Worker("127.0.0.1", r.port, be, T.LocalFs(str(tmp_path), str(tmp_path / "out")), retry_s=0.1,
               idle_exit_s=1.5)
    th = _start(w)
    assert r.join() == 0
    th.join(10)
    out = tmp_path / "out" / "12clip.y4m"
    assert (out / "0.mp4").read_bytes().startswith(b"YUV4MPEG2")
    assert b"fake ffmpeg -y -i" in (out / "c0.mp4.log").read_bytes()
    assert b"-vcodec libx264" in (out / "c1.mp4.log").read_bytes()


def test_worker_env_contract(monkeypatch, capsys):
    from govideocompressor_amd.jobs.worker import env_config
    with pytest.raises(SystemExit):
        env_config({})
    assert "SERVER_IP NIL" in capsys.readouterr().err
    with pytest.raises(SystemExit):
        env_config({"SERVER_IP": "1.2.3.4", "MIVC_TRANSPORT": "http"})
    err = capsys.readouterr().err
    assert "FTP_USERNAME NIL" in err and "FTP_PASSWORD NIL" in err
    assert env_config({"SERVER_IP": "1.2.3.4"}) == {"server_ip": "1.2.3.4", "port": 8055}
    assert env_config({"SERVER_IP": "h", "SERVER_PORT": "9"})["port"] == 9


def test_batched_leases_cpu(tmp_path, host):
    """One worker holding 3 leases encodes the pieces that arrive together as one batch."""
    clip, d = _make_split(tmp_path, 3)
    r = _Run(tmp_path, d)
    w = _worker(tmp_path, r.port, leases=3)
    w.batch_wait_s = 0.5
    calls = []
    orig = w.backend.run
    w.backend.run = lambda jobs, args: (calls.append(len(jobs)), orig(jobs, args))[1]
    th = _start(w)
    assert r.join() == 0
    th.join(10)
    assert max(calls) >= 2
    _check_outputs(host, tmp_path, clip, 3, 3)
    assert np.isfinite(len(calls))
