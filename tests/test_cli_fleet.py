"""CLI surface (App. A.1 flags/defaults) and the local fleet launcher."""
import os
import socket
import subprocess
import sys
import time

import pytest

from govideocompressor_amd import cli, fleet

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.timeout(120)


def test_cli_reference_flags_and_defaults():
    p = cli.build_parser()
    a = p.parse_args(["server", "s", "movie.mp4"])
    assert a.size == 10
    a = p.parse_args(["server", "s", "movie.mp4", "-s", "25"])
    assert a.size == 25
    a = p.parse_args(["server", "c", "12movie.mp4"])
    assert (a.ff, a.piece, a.port) == ("", "", "8055")
    a = p.parse_args(["server", "c", "12movie.mp4", "-f", "264", "-p", "3;7", "--port", "9000"])
    assert (a.ff, a.piece, a.port) == ("264", "3;7", "9000")
    a = p.parse_args(["server", "t"])
    assert (a.duration, a.port) == ("11", "8055")
    a = p.parse_args(["server", "t", "5", "-p", "9001"])        # -p is --port under t
    assert (a.duration, a.port) == ("5", "9001")


def test_cli_bad_piece_list(capsys, tmp_path):
    rc = cli.main(["server", "c", str(tmp_path), "-f", "264", "-p", "x;1"])
    assert rc == 2
    assert "输入参数错误[x;1]" in capsys.readouterr().out


def _run(args, **kw):
    env = dict(os.environ, PYTHONPATH=ROOT)
    return subprocess.run([sys.executable, "-m", "govideocompressor_amd.cli"] + args, capture_output=True,
                          text=True, env=env, timeout=100, **kw)


def test_cli_synth_split_encode_merge(tmp_path):
    r = _run(["synth", "-o", "a.y4m", "--frames", "12", "--size", "64x48"], cwd=tmp_path)
    assert r.returncode == 0, r.stderr
    r = _run(["probe", "a.y4m"], cwd=tmp_path)
    assert '"frames": 12' in r.stdout
    r = _run(["server", "s", "a.y4m", "--frames", "6"], cwd=tmp_path)
    assert r.returncode == 0 and "[./12a.y4m] [2]" in r.stdout
    r = _run(["encode", "a.y4m", "-o", "enc.mp4", "--backend", "cpu", "--slots", "2"], cwd=tmp_path)
    assert r.returncode == 0, r.stderr
    r = _run(["decode", "enc.mp4", "-o", "dec.y4m"], cwd=tmp_path)
    assert r.returncode == 0 and "decoded [12] frames 64x48" in r.stdout
    r = _run(["merge", "enc.mp4", "enc.mp4", "-o", "twice.264"], cwd=tmp_path)
    assert r.returncode == 0 and "merged [2] pieces" in r.stdout


def test_fleet_create_ls_rm(tmp_path):
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]          # nothing listens: workers sit in their dial/backoff loop
    state = str(tmp_path / "fleet.json")
    env = {"SERVER_IP": "127.0.0.1", "SERVER_PORT": str(port), "PYTHONPATH": ROOT}
    ws = fleet.create(2, ["--backend", "cpu", "--retry", "0.2"], state=state, gpus=2, env_extra=env)
    assert [w["gpu"] for w in ws] == ["0", "1"]
    t_end = time.time() + 30
    while time.time() < t_end and not all(w["alive"] for w in fleet.ls(state)):
        time.sleep(0.1)
    assert all(w["alive"] for w in fleet.ls(state))
    assert len(fleet.addrs(state)) == 2
    assert fleet.rm_all(state) == 2
    assert fleet.ls(state) == []
    for w in ws:
        assert not fleet._alive(w["pid"])


def test_fleet_never_kills_foreign_pids(tmp_path):
    state = str(tmp_path / "fleet.json")
    p = subprocess.Popen([sys.executable, "-c", "import time; time.sleep(30)"])
    try:
        fleet._save(state, {"workers": [{"id": 0, "pid": p.pid, "gpu": "", "cmd": [], "started": 0}]})
        assert fleet.rm_all(state) == 0           # not our worker: left alone
        assert p.poll() is None
    finally:
        p.kill()
        p.wait()


def test_cli_config_overlay(tmp_path):
    """--config FILE: per-command option defaults (JSON/YAML); explicit flags win."""
    import json as _json

    from govideocompressor_amd import cli
    cfgp = tmp_path / "c.json"
    cfgp.write_text(_json.dumps({"server c": {"port": 9100, "ff": "265"}, "server t": {"port": 9200}}))
    ap = cli.build_parser()
    argv = ["server", "c", "x.mp4"]
    cli._apply_config(ap, cli._load_config(str(cfgp)), argv)
    a = ap.parse_args(argv)
    assert int(a.port) == 9100 and a.ff == "265"
    ap = cli.build_parser()
    argv = ["server", "c", "x.mp4", "--port", "9300"]
    cli._apply_config(ap, cli._load_config(str(cfgp)), argv)
    assert int(ap.parse_args(argv).port) == 9300
    y = tmp_path / "c.yaml"
    y.write_text("server t:\n  port: 9400\n")
    ap = cli.build_parser()
    argv = ["server", "t"]
    cli._apply_config(ap, cli._load_config(str(y)), argv)
    assert int(ap.parse_args(argv).port) == 9400
    bad = tmp_path / "b.json"
    bad.write_text(_json.dumps({"server c": {"nonsense": 1}}))
    ap = cli.build_parser()
    with pytest.raises(SystemExit):
        cli._apply_config(ap, cli._load_config(str(bad)), ["server", "c", "x.mp4"])
