"""Multi-GPU readiness on a one-GPU box.  No 8-GPU node is available to the
builder, so the scaling curve itself is the driver's; these tests run the distributed code
on the device:

* ``bench.py`` at world 2 (two processes sharing the GPU, host collectives through
  ``MIVC_DIST_BACKEND=gloo``, launched by ``torch.distributed.run``) merges a stream
  byte-identical to the world-1 run of the same global batch;
* an ``nccl`` (RCCL) process group at world 1 executes every collective on device tensors
  (tools/dist_smoke.py).

Both run as child processes, so the ranks own their GPU contexts."""
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(args: list[str], extra: dict, timeout: int = 300) -> subprocess.CompletedProcess:
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_PORT"):
        env.pop(k, None)
    env.update(extra)
    env["HSA_ENABLE_IPC_MODE_LEGACY"] = "0"
    r = subprocess.run(args, cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    return r


def test_bench_world2_merge_matches_world1(tmp_path, host):
    common = ["--steps", "1", "--warmup", "0", "--frames", "8", "--width", "320", "--height", "192", "--no-quality",
              "--bframes", "2"]
    w1, w2 = tmp_path / "w1.264", tmp_path / "w2.264"
    _run([sys.executable, "bench.py", "--gpus", "1", "--slots", "8", *common, "--merged-out", str(w1)], {})
    _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
          "127.0.0.1", "--master-port", str(_port()), "bench.py", "--gpus", "2", "--slots", "4", *common,
          "--merged-out", str(w2)], {"MIVC_DIST_BACKEND": "gloo"})
    a, b = w1.read_bytes(), w2.read_bytes()
    assert len(a) > 1000 and a == b
    assert len(host.decode(a)) == 8 * 8


def test_rccl_world1_collectives_on_device():
    r = _run([sys.executable, "tools/dist_smoke.py"],
             {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0", "MASTER_ADDR": "127.0.0.1",
              "MASTER_PORT": str(_port()), "MIVC_DIST_FORCE": "1"}, timeout=200)
    assert r.stdout.strip().endswith("OK")


def test_config3_transcode_world2_merge_matches_world1(tmp_path, host):
    """BASELINE config 3 as an 8-GPU-ready harness: bench/run.py --config 3 under
    torch.distributed.run shards the pieces over the ranks, each transcodes its share (GPU
    decode + re-encode) and rank 0 merges ONE stream in piece order.  At world 2 (two ranks on
    this GPU, host collectives) the merged stream is byte-identical to world 1's, and every
    picture of it decodes."""
    common = ["bench/run.py", "--config", "3", "--size3", "320x192", "--segments3", "8", "--slots3", "4",
              "--frames3", "8", "--codec3", "h264", "--warmup", "0", "--no-encode-only3"]
    w1, w2 = tmp_path / "w1", tmp_path / "w2"
    _run([sys.executable, *common, "--merged-out3", str(w1)], {})
    _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
          "127.0.0.1", "--master-port", str(_port()), *common, "--merged-out3", str(w2)], {"MIVC_DIST_BACKEND": "gloo"})
    a, b = (tmp_path / "w1.h264").read_bytes(), (tmp_path / "w2.h264").read_bytes()
    assert len(a) > 1000 and a == b
    assert len(host.decode(a)) == 8 * 8
