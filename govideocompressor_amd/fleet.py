"""``mivc fleet``: launch and manage local GPU workers.

Reference: ``doOpt.go`` provisions DigitalOcean droplets (``CreateDocker``,
doOpt.go:52-78), lists them (``ListAllDroplet``, :80-90), deletes *every* droplet
with a given image slug account-wide (``DeleteAllDocker``, :92-101, defect D15),
collects their IPs (:103-111) and runs ``docker run hey678/myclient`` over SSH with
host-key checking disabled (:133-181, 186-190); ``startDocker.go`` lists Arukas
containers.

On an MI355X node a "droplet" is one worker process pinned to one GPU
(``HIP_VISIBLE_DEVICES``).  Verbs:

* ``create N``  -- spawn N workers (GPU i % n_gpus), record PIDs in a state file;
* ``ls``        -- the recorded workers and whether each is alive;
* ``rm --all``  -- terminate ONLY the recorded PIDs, and only after checking the PID
  still runs our worker (no pattern kills, no account-wide deletes -- fixes D15);
* ``addrs``     -- host:GPU addresses of the live workers;
* ``exec CMD``  -- run a command once per GPU with that GPU's environment.
"""
from __future__ import annotations

import json
import os
import signal
import subprocess
import sys
import time

DEFAULT_STATE = os.environ.get("MIVC_FLEET_STATE", os.path.join(os.getcwd(), ".mivc_fleet.json"))
_MARK = "govideocompressor_amd"


def _load(path: str) -> dict:
    if os.path.exists(path):
        with open(path) as f:
            return json.load(f)
    return {"workers": []}


def _save(path: str, st: dict) -> None:
    tmp = path + ".tmp"
    with open(tmp, "w") as f:
        json.dump(st, f, indent=1)
    os.replace(tmp, path)


def _alive(pid: int) -> bool:
    """True if ``pid`` exists and its command line is one of our workers."""
    try:
        with open(f"/proc/{pid}/cmdline", "rb") as f:
            cmd = f.read().replace(b"\0", b" ").decode(errors="replace")
    except OSError:
        return False
    return _MARK in cmd and " client" in cmd


def gpu_count() -> int:
    env = os.environ.get("MIVC_FLEET_GPUS")
    if env:
        return int(env)
    try:
        import torch
        return torch.cuda.device_count()  # does not initialise HIP on this image
    except Exception:  # noqa: BLE001
        return 0


def create(n: int, worker_args: list[str] | None = None, state: str = DEFAULT_STATE, gpus: int | None = None,
           log_dir: str | None = None, env_extra: dict | None = None) -> list[dict]:
    st = _load(state)
    ng = gpus if gpus is not None else gpu_count()
    log_dir = log_dir or os.path.join(os.path.dirname(os.path.abspath(state)), "fleet_logs")
    os.makedirs(log_dir, exist_ok=True)
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = []
    base = len(st["workers"])
    for i in range(n):
        wid = base + i
        env = dict(os.environ)
        env.update(env_extra or {})
        env["PYTHONPATH"] = root + (os.pathsep + env["PYTHONPATH"] if env.get("PYTHONPATH") else "")
        gpu = ""
        if ng > 0:
            gpu = str(wid % ng)
            env["HIP_VISIBLE_DEVICES"] = gpu
        env.setdefault("MIVC_WORKER_ID", f"fleet{wid}")
        lf = open(os.path.join(log_dir, f"worker{wid}.log"), "ab")
        cmd = [sys.executable, "-m", "govideocompressor_amd.cli", "client"] + list(worker_args or [])
        p = subprocess.Popen(cmd, env=env, stdout=lf, stderr=subprocess.STDOUT, start_new_session=True)
        lf.close()
        ent = {"id": wid, "pid": p.pid, "gpu": gpu, "cmd": cmd, "started": time.time(),
               "log": os.path.join(log_dir, f"worker{wid}.log")}
        st["workers"].append(ent)
        out.append(ent)
    _save(state, st)
    return out


def ls(state: str = DEFAULT_STATE) -> list[dict]:
    st = _load(state)
    return [dict(w, alive=_alive(w["pid"])) for w in st["workers"]]


def addrs(state: str = DEFAULT_STATE) -> list[str]:
    import socket
    host = socket.gethostname()
    return [f"{host}:gpu{w['gpu'] or '-'}:pid{w['pid']}" for w in ls(state) if w["alive"]]


def rm_all(state: str = DEFAULT_STATE, timeout: float = 10.0) -> int:
    st = _load(state)
    n = 0
    for w in st["workers"]:
        pid = w["pid"]
        if _alive(pid):
            try:
                os.kill(pid, signal.SIGTERM)
                n += 1
            except ProcessLookupError:
                pass
    t_end = time.time() + timeout
    for w in st["workers"]:
        while _alive(w["pid"]) and time.time() < t_end:
            time.sleep(0.05)
        if _alive(w["pid"]):
            try:
                os.kill(w["pid"], signal.SIGKILL)
            except ProcessLookupError:
                pass
        try:  # reap if it is our child
            os.waitpid(w["pid"], os.WNOHANG)
        except ChildProcessError:
            pass
    st["workers"] = []
    _save(state, st)
    return n


def exec_all(cmd: list[str], gpus: int | None = None, timeout: float | None = None) -> list[int]:
    ng = gpus if gpus is not None else gpu_count()
    codes = []
    for g in range(max(1, ng)):
        env = dict(os.environ)
        if ng > 0:
            env["HIP_VISIBLE_DEVICES"] = str(g)
        codes.append(subprocess.run(cmd, env=env, timeout=timeout).returncode)
    return codes
