"""Command line: ``python -m govideocompressor_amd.cli <command>`` (installed as ``mivc``).

Reference surface (server.go:17-36, client.go:14-36) with the
same command names, flags, shorts and defaults:

    server s <fileName> [-s/--size 10]                       split   (server.go:47-63)
    server c <fileName> [-f/--ff ""] [-p/--piece ""] [--port 8055]   coordinate (:65-121)
    server t [duration=11] [-p/--port 8055]                  census  (:123-156)
    client                                                   worker  (client.go; env SERVER_IP,
                                                             SERVER_PORT, FTP_USERNAME, FTP_PASSWORD)

Note ``-p`` is ``--piece`` under ``c`` but ``--port`` under ``t``, as in the reference.
New commands: ``encode`` (single-node multi-GPU file encode), ``fleet`` (local GPU
worker launcher replacing doOpt.go), ``probe``, ``decode``, ``synth``, ``merge``.
Every command takes ``--config FILE`` (or ``MIVC_CONFIG``): a JSON/YAML overlay of
option defaults per command; explicit flags win.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys


def _wh(s: str) -> tuple[int, int]:
    w, h = s.lower().split("x")
    return int(w), int(h)


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


# ---------------------------------------------------------------------------- server
def cmd_server_s(a) -> int:
    from .segment.split import split
    w, h = _wh(a.raw_size) if a.raw_size else (0, 0)
    split(a.fileName, size_mb=a.size, seconds=a.seconds, frames=a.frames, out_root=a.out_root, width=w, height=h,
          fps=a.fps, bit_depth=a.bit_depth)
    return 0


def cmd_server_c(a) -> int:
    from .jobs.coordinator import Coordinator
    from .jobs.ffargs import expand_preset
    from .segment.plan import parse_pieces
    pieces = None
    if a.piece:
        try:
            pieces = parse_pieces(a.piece)
        except ValueError:
            print(f"输入参数错误[{a.piece}]  (bad input argument)")
            return 2
    auth = None
    if os.environ.get("FTP_USERNAME") and os.environ.get("FTP_PASSWORD"):
        auth = (os.environ["FTP_USERNAME"], os.environ["FTP_PASSWORD"])
    co = Coordinator(a.fileName, expand_preset(a.ff), pieces=pieces, port=int(a.port), host=a.host,
                     out_root=a.out, lease_timeout=a.lease_timeout, max_retries=a.retries,
                     delete_source=not a.keep_source, merge=a.merge, http_port=a.http_port, http_auth=auth,
                     log=lambda s: print(s, flush=True), src_root=a.src_root)
    return co.run()


def cmd_server_t(a) -> int:
    from .jobs.census import census
    census(float(a.duration), int(a.port), a.host, log=lambda s: print(s, flush=True))
    return 0


# ---------------------------------------------------------------------------- worker
def cmd_client(a) -> int:
    from .backends import get_backend
    from .jobs import transport
    from .jobs.worker import Worker, env_config
    conf = env_config()
    gpu = os.environ.get("HIP_VISIBLE_DEVICES", "")
    be = get_backend(a.backend)
    w = Worker(conf["server_ip"], conf["port"], be, transport.from_env(), leases=a.leases,
               worker_id=os.environ.get("MIVC_WORKER_ID"), gpu=gpu, retry_s=a.retry, heartbeat_s=a.heartbeat,
               idle_exit_s=a.idle_exit, max_jobs=a.max_jobs, out_ext=a.out_ext,
               log=(lambda s: print(s, flush=True)) if a.verbose else None)
    return w.run()


# ---------------------------------------------------------------------------- encode
def cmd_encode(a) -> int:
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # one process per GPU; this parent never touches the GPU, it only waits
        argv = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
                "--master-addr=127.0.0.1", f"--master-port={_free_port()}", "-m", "govideocompressor_amd.cli"]
        argv += [x for x in sys.argv[1:]]
        return subprocess.call(argv)
    from .pipeline import encode_file
    encode_file(a.input, a.output, args=a.ff, backend=a.backend, slots=a.slots, seg_frames=a.seg_frames,
                schedule=a.schedule, raw_size=_wh(a.raw_size) if a.raw_size else None, fps=a.fps,
                resume=a.resume, work_dir=a.work_dir)
    return 0


# ---------------------------------------------------------------------------- fleet
def cmd_fleet(a) -> int:
    from . import fleet
    if a.verb == "create":
        ws = fleet.create(a.n, a.rest, state=a.state, gpus=a.gpus)
        for w in ws:
            print(f"worker{w['id']} pid[{w['pid']}] gpu[{w['gpu']}]")
    elif a.verb == "ls":
        for w in fleet.ls(a.state):
            print(f"worker{w['id']} pid[{w['pid']}] gpu[{w['gpu']}] {'alive' if w['alive'] else 'dead'}")
    elif a.verb == "rm":
        if not a.all:
            print("rm needs --all")
            return 2
        print(f"stopped [{fleet.rm_all(a.state)}] worker(s)")
    elif a.verb == "addrs":
        for s in fleet.addrs(a.state):
            print(s)
    elif a.verb == "exec":
        codes = fleet.exec_all(a.rest, gpus=a.gpus)
        return max(codes) if codes else 0
    return 0


# ---------------------------------------------------------------------------- tools
def cmd_probe(a) -> int:
    from .segment.probe import probe
    w, h = _wh(a.raw_size) if a.raw_size else (0, 0)
    print(json.dumps(probe(a.file, w, h, a.fps).as_dict()))
    return 0


def cmd_decode(a) -> int:
    from .backends import load_clip
    from .utils import yuv
    clip = load_clip(a.input)
    if a.output.endswith(".y4m"):
        yuv.write_y4m(a.output, clip)
    else:
        yuv.write_yuv(a.output, clip)
    print(f"decoded [{clip.frames}] frames {clip.width}x{clip.height} -> {a.output}")
    return 0


def cmd_synth(a) -> int:
    from .utils import yuv
    w, h = _wh(a.size)
    clip = yuv.synth_clip_cpu(a.frames, w, h, seed=a.seed, fps=a.fps)
    if a.output.endswith(".y4m"):
        yuv.write_y4m(a.output, clip)
    else:
        yuv.write_yuv(a.output, clip)
    return 0


def cmd_merge(a) -> int:
    from .segment import merge as M
    files = list(a.files)
    if a.list:
        files = M.read_filelist(a.list) + files
    if not files:
        print("nothing to merge")
        return 2
    n = M.merge_files(files, a.output)
    print(f"merged [{len(files)}] pieces -> {a.output} ({n} bytes)")
    return 0


def build_parser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(prog="mivc", description="MI355X distributed video compressor")
    sub = ap.add_subparsers(dest="cmd", required=True)

    srv = sub.add_parser("server", help="split / coordinate / census (the reference's server binary)")
    ss = srv.add_subparsers(dest="sub", required=True)
    s = ss.add_parser("s", help="Split video.")
    s.add_argument("fileName")
    s.add_argument("-s", "--size", type=int, default=10, help="segment size (MB) for compressed input")
    s.add_argument("--seconds", type=float, default=None, help="segment duration (overrides --size)")
    s.add_argument("--frames", type=int, default=None, help="segment length in frames")
    s.add_argument("--raw-size", default=None, help="WxH of a raw .yuv input")
    s.add_argument("--fps", type=float, default=30.0)
    s.add_argument("--bit-depth", type=int, default=8)
    s.add_argument("--out-root", default=".")
    s.set_defaults(fn=cmd_server_s)
    c = ss.add_parser("c", help="Convert video.")
    c.add_argument("fileName")
    c.add_argument("-f", "--ff", default="", help='ffmpeg-style args or the presets "264" / "265"')
    c.add_argument("-p", "--piece", default="", help='convert only some pieces, ";"-separated')
    c.add_argument("--port", default="8055")
    c.add_argument("--host", default="0.0.0.0")
    c.add_argument("--out", default="out", help="output root (the reference's /home/vuser)")
    c.add_argument("--lease-timeout", type=float, default=600.0)
    c.add_argument("--retries", type=int, default=3)
    c.add_argument("--keep-source", action="store_true", help="do not delete a source piece on success")
    c.add_argument("--merge", action="store_true", help="merge the outputs when every piece is done")
    c.add_argument("--http-port", type=int, default=None, help="serve pieces / accept outputs over HTTP")
    c.add_argument("--src-root", default=None, help="root the job's <dir> is relative to (default: CWD)")
    c.set_defaults(fn=cmd_server_c)
    t = ss.add_parser("t", help="Touch client")
    t.add_argument("duration", nargs="?", default="11")
    t.add_argument("-p", "--port", default="8055")
    t.add_argument("--host", default="0.0.0.0")
    t.set_defaults(fn=cmd_server_t)

    cl = sub.add_parser("client", help="pull-based worker (env: SERVER_IP, SERVER_PORT, FTP_USERNAME, FTP_PASSWORD)")
    cl.add_argument("--backend", default=os.environ.get("MIVC_BACKEND", "auto"), choices=["auto", "gpu", "cpu", "ffmpeg"])
    cl.add_argument("--leases", type=int, default=int(os.environ.get("MIVC_LEASES", "1")))
    cl.add_argument("--retry", type=float, default=float(os.environ.get("MIVC_RETRY_S", "10")))
    cl.add_argument("--heartbeat", type=float, default=5.0)
    cl.add_argument("--idle-exit", type=float, default=None)
    cl.add_argument("--max-jobs", type=int, default=None)
    cl.add_argument("--out-ext", default="mp4", choices=["mp4", "264"])
    cl.add_argument("-v", "--verbose", action="store_true")
    cl.set_defaults(fn=cmd_client)

    en = sub.add_parser("encode", help="encode one file on this node's GPUs")
    en.add_argument("input")
    en.add_argument("-o", "--output", required=True)
    en.add_argument("-f", "--ff", default="264")
    en.add_argument("--backend", default="auto", choices=["auto", "gpu", "cpu"])
    en.add_argument("--gpus", type=int, default=1)
    en.add_argument("--slots", type=int, default=16, help="segments encoded together per GPU")
    en.add_argument("--seg-frames", type=int, default=None)
    en.add_argument("--schedule", default="static", choices=["static", "dynamic"])
    en.add_argument("--raw-size", default=None)
    en.add_argument("--fps", type=float, default=30.0)
    en.add_argument("--resume", action="store_true", help="checkpoint every segment; skip finished ones on restart")
    en.add_argument("--work-dir", default=None, help="checkpoint directory (default <output>.parts)")
    en.set_defaults(fn=cmd_encode)

    fl = sub.add_parser("fleet", help="launch / list / stop local GPU workers")
    fl.add_argument("verb", choices=["create", "ls", "rm", "addrs", "exec"])
    fl.add_argument("n", nargs="?", type=int, default=1)
    fl.add_argument("--all", action="store_true")
    fl.add_argument("--gpus", type=int, default=None)
    fl.add_argument("--state", default=os.environ.get("MIVC_FLEET_STATE", ".mivc_fleet.json"))
    fl.add_argument("rest", nargs=argparse.REMAINDER, help="-- worker args (create) or command (exec)")
    fl.set_defaults(fn=cmd_fleet)

    pr = sub.add_parser("probe")
    pr.add_argument("file")
    pr.add_argument("--raw-size", default=None)
    pr.add_argument("--fps", type=float, default=30.0)
    pr.set_defaults(fn=cmd_probe)
    de = sub.add_parser("decode")
    de.add_argument("input")
    de.add_argument("-o", "--output", required=True)
    de.set_defaults(fn=cmd_decode)
    sy = sub.add_parser("synth")
    sy.add_argument("-o", "--output", required=True)
    sy.add_argument("--frames", type=int, default=60)
    sy.add_argument("--size", default="1920x1080")
    sy.add_argument("--fps", type=float, default=30.0)
    sy.add_argument("--seed", type=int, default=0)
    sy.set_defaults(fn=cmd_synth)
    me = sub.add_parser("merge")
    me.add_argument("files", nargs="*")
    me.add_argument("--list", default=None)
    me.add_argument("-o", "--output", required=True)
    me.set_defaults(fn=cmd_merge)
    return ap


# ---------------------------------------------------------------------------- config overlay
def _load_config(path: str) -> dict:
    """``--config FILE`` (JSON, or YAML by extension): option defaults per command, e.g.
    ``{"*": {...}, "encode": {"slots": 64, "args": "265"}, "server c": {"port": 9000}}``.
    Keys are argparse destinations; explicit command-line flags still win."""
    with open(path) as f:
        if path.endswith((".yaml", ".yml")):
            import yaml
            data = yaml.safe_load(f)
        else:
            data = json.load(f)
    if not isinstance(data, dict):
        raise SystemExit(f"{path}: config must be a mapping of command -> options")
    return data


def _subparser(ap: argparse.ArgumentParser, path: list[str]):
    for name in path:
        acts = [x for x in ap._actions if isinstance(x, argparse._SubParsersAction)]
        if not acts or name not in acts[0].choices:
            return None
        ap = acts[0].choices[name]
    return ap


def _apply_config(ap: argparse.ArgumentParser, cfg: dict, argv: list[str]) -> None:
    words = [w for w in argv if not w.startswith("-")]
    for section, opts in cfg.items():
        if not isinstance(opts, dict):
            raise SystemExit(f"config section {section!r} must be a mapping")
        path = section.replace(".", " ").split() if section != "*" else []
        if path and words[:len(path)] != path:
            continue  # a section for another command
        targets = [_subparser(ap, words[:k]) for k in range(len(words) + 1)] if not path else [_subparser(ap, path)]
        targets = [t for t in targets if t is not None]
        for t in targets:
            dests = {x.dest for x in t._actions}
            known = {k: v for k, v in opts.items() if k in dests}
            if path:
                unknown = set(opts) - dests
                if unknown:
                    raise SystemExit(f"config section {section!r}: unknown options {sorted(unknown)}")
            t.set_defaults(**known)


def main(argv: list[str] | None = None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    cfg_path = os.environ.get("MIVC_CONFIG")
    for i, w in enumerate(argv):
        if w == "--config" and i + 1 < len(argv):
            cfg_path = argv[i + 1]
            del argv[i:i + 2]
            break
        if w.startswith("--config="):
            cfg_path = w.split("=", 1)[1]
            del argv[i]
            break
    ap = build_parser()
    if cfg_path:
        _apply_config(ap, _load_config(cfg_path), argv)
    a = ap.parse_args(argv)
    if getattr(a, "rest", None) and a.rest[:1] == ["--"]:
        a.rest = a.rest[1:]
    return int(a.fn(a) or 0)


if __name__ == "__main__":
    sys.exit(main())
