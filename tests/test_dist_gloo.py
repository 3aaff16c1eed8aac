"""T5: the distributed encode path with the gloo backend on CPU (world sizes 2 and 3).

Same code as the RCCL path: CC-1 stats all-reduce, CC-2/CC-3 bitstream all-gather,
CC-4 plan broadcast, TCPStore tickets.  The merged stream of a multi-rank encode must be
byte-identical to the single-process encode."""
import os
import socket

import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.timeout(300)


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _env(rank, world, port):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))


def _collectives(rank, world, port, q):
    _env(rank, world, port)
    import torch
    from govideocompressor_amd.parallel import dist as D
    from govideocompressor_amd.parallel.tickets import TicketDispenser
    env = D.init(prefer_gpu=False)
    try:
        # CC-1: each rank fills its rows
        st = torch.zeros(6, 4)
        st[rank::world] = rank + 1
        D.allreduce_stats(env, st)
        # CC-2/3: variable-size payloads, including an empty one
        pieces = [bytes([rank]) * (rank * 3 + 1), b"", bytes([7]) * rank] if rank else [b"zero"]
        got = D.BitstreamGather(env, pieces).start().wait()
        # CC-4
        obj = D.broadcast_object(env, {"plan": [1, 2, 3]} if rank == 0 else None)
        # tickets: every index handed out exactly once over all ranks
        td = TicketDispenser(23)
        mine = []
        while True:
            c = td.claim(4)
            if not c:
                break
            mine += c
        mx = D.max_over_ranks(env, float(rank))
        q.put((rank, st.tolist(), got, obj, mine, mx))
    finally:
        D.shutdown(env)


def test_collectives_gloo():
    world, port = 3, _port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_collectives, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted([q.get(timeout=240) for _ in range(world)])
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    tickets = []
    for rank, st, got, obj, mine, mx in res:
        assert [row[0] for row in st] == [1, 2, 3, 1, 2, 3]
        if rank == 0:  # the payloads are gathered to rank 0 only
            assert got[0] == [b"zero"]
            assert got[1] == [b"\x01" * 4, b"", b"\x07"]
            assert got[2] == [b"\x02" * 7, b"", b"\x07\x07"]
        else:
            assert got is None
        assert obj == {"plan": [1, 2, 3]}
        assert mx == world - 1
        tickets += mine
    assert sorted(tickets) == list(range(23))


def _merge(rank, world, port, q):
    _env(rank, world, port)
    from govideocompressor_amd.parallel import dist as D
    env = D.init(prefer_gpu=False)
    try:
        m = D.SegmentMerge(env)
        outs = []
        for it in range(2):  # buffers are reused across calls
            sc = b"\0\0\0\1"
            if rank == 1:
                pieces = []  # a rank with nothing to contribute
            else:
                pieces = [sc + bytes([rank, it]) * (5 + rank), [sc, bytes([9]) * (3 + it), bytes([rank])]]
            got = m.run(pieces)
            outs.append(None if got is None else bytes(got))
        # streaming merge: rank 0 writes every rank's bytes to a sink instead
        import io
        sink = io.BytesIO() if rank == 0 else None
        n = m.run([b"\0\0\0\1" + bytes([rank]) * (rank + 2)], sink=sink)
        outs.append((n, sink.getvalue()) if rank == 0 else n)
        bad = None
        try:
            m.run([b"\1\2\3\4\5"])
        except RuntimeError as e:
            bad = str(e)
        q.put((rank, outs, bad))
    finally:
        D.shutdown(env)


def test_segment_merge_gloo():
    world, port = 3, _port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_merge, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted([q.get(timeout=240) for _ in range(world)])
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    sc = b"\0\0\0\1"
    for it in range(2):
        want = b""
        for r in (0, 2):
            want += sc + bytes([r, it]) * (5 + r) + sc + bytes([9]) * (3 + it) + bytes([r])
        assert res[0][1][it] == want
        assert res[1][1][it] is None and res[2][1][it] is None
    want = b"".join(sc + bytes([r]) * (r + 2) for r in range(world))
    assert res[0][1][2] == (len(want), want)
    assert res[1][1][2] is None and res[2][1][2] is None
    assert all(bad and "start code" in bad for _, _, bad in res)


def _encode(rank, world, port, src, out, schedule):
    _env(rank, world, port)
    from govideocompressor_amd.pipeline import encode_file
    encode_file(src, out, args="-vcodec libx264 -crf 26", backend="cpu", slots=2, schedule=schedule,
                log=lambda s: None)


@pytest.mark.parametrize("schedule", ["static", "dynamic"])
def test_multi_rank_encode_matches_single(tmp_path, host, schedule):
    from govideocompressor_amd.pipeline import encode_file
    from govideocompressor_amd.utils import yuv
    src = tmp_path / "in.y4m"
    yuv.write_y4m(str(src), yuv.synth_clip_cpu(40, 64, 48, seed=21))
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        os.environ.pop(k, None)
    ref = tmp_path / "ref.264"
    # world=1 with the same plan granularity as world=2 (segment count depends on world*slots)
    os.environ["WORLD_SIZE"] = "1"
    r1 = encode_file(str(src), str(ref), args="-vcodec libx264 -crf 26", backend="cpu", slots=4,
                     log=lambda s: None)
    os.environ.pop("WORLD_SIZE")
    assert r1["segments"] == 4
    out = tmp_path / "out.264"
    world, port = 2, _port()
    ctx = mp.get_context("spawn")
    ps = [ctx.Process(target=_encode, args=(r, world, port, str(src), str(out), schedule)) for r in range(world)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(240)
        assert p.exitcode == 0
    assert out.read_bytes() == ref.read_bytes()
    assert len(host.decode(out.read_bytes())) == 40


def _bench_merge(rank, world, port, q, steps):
    """bench.py's merge flow on CPU: each step the rank's pieces go through SegmentMerge on
    a side thread (merge of step k overlaps step k + 1), rank-major order."""
    import concurrent.futures as cf

    _env(rank, world, port)
    from govideocompressor_amd.parallel import dist as D
    env = D.init(prefer_gpu=False)
    try:
        m = D.SegmentMerge(env)
        pool = cf.ThreadPoolExecutor(max_workers=1)
        fut, outs = None, []
        for k in range(steps):
            pieces = _bench_pieces(rank, k)
            if fut is not None:
                got = fut.result()
                outs.append(None if got is None else bytes(got))
            fut = pool.submit(m.run, pieces)
        got = fut.result()
        outs.append(None if got is None else bytes(got))
        pool.shutdown()
        D.barrier(env)
        q.put((rank, outs))
    finally:
        D.shutdown(env)


def _bench_pieces(rank, step, slots=3):
    import numpy as np
    rng = np.random.default_rng(1000 * step + rank)
    out = []
    for b in range(slots):
        n = int(rng.integers(0, 4000)) if (rank + b) % 5 else 0  # some ranks / slots tiny
        out.append([b"\0\0\0\1\x67" + bytes([rank, b, step]), rng.integers(0, 256, n, dtype=np.uint8).tobytes()])
    return out


@pytest.mark.parametrize("world", [4, 8])
def test_bench_merge_flow_world_4_8(world):
    """T5 at world 4 / 8: the merged stream on rank 0 is byte-identical to world = 1's
    concatenation of every rank's pieces (rank-major), for several pipelined steps."""
    steps, port = 3, _port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_bench_merge, args=(r, world, port, q, steps)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted([q.get(timeout=300) for _ in range(world)])
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    for k in range(steps):
        want = b"".join(b"".join(b"".join(parts) for parts in _bench_pieces(r, k)) for r in range(world))
        assert res[0][1][k] == want, k
        assert all(res[r][1][k] is None for r in range(1, world))


def test_encode_file_resume_skips_finished_segments(tmp_path, host):
    """Checkpoint/resume: an interrupted run leaves per-segment parts + a
    manifest; the restart encodes only the missing segments and the output is byte-identical
    to an uninterrupted run.  A corrupted part is re-encoded."""
    from govideocompressor_amd.pipeline import encode_file
    from govideocompressor_amd.utils import yuv
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        os.environ.pop(k, None)
    src = tmp_path / "in.y4m"
    yuv.write_y4m(str(src), yuv.synth_clip_cpu(32, 64, 48, seed=5))
    ref = tmp_path / "ref.264"
    r0 = encode_file(str(src), str(ref), args="-vcodec libx264 -crf 26", backend="cpu", slots=4, seg_frames=8,
                     log=lambda s: None)
    assert r0["segments"] == 4
    out = tmp_path / "out.264"
    wd = tmp_path / "parts"
    r1 = encode_file(str(src), str(out), args="-vcodec libx264 -crf 26", backend="cpu", slots=4, seg_frames=8,
                     log=lambda s: None, resume=True, work_dir=str(wd))
    assert r1["resumed_segments"] == 0 and out.read_bytes() == ref.read_bytes()
    # simulate an interruption: drop one part, corrupt another
    (wd / "3.seg").unlink()
    (wd / "1.seg").write_bytes(b"\x00\x00\x00\x01garbage")
    out.unlink()
    r2 = encode_file(str(src), str(out), args="-vcodec libx264 -crf 26", backend="cpu", slots=4, seg_frames=8,
                     log=lambda s: None, resume=True, work_dir=str(wd))
    assert r2["resumed_segments"] == 2
    assert out.read_bytes() == ref.read_bytes()
    # different arguments invalidate the checkpoint
    r3 = encode_file(str(src), str(tmp_path / "o3.264"), args="-vcodec libx264 -crf 30", backend="cpu", slots=4,
                     seg_frames=8, log=lambda s: None, resume=True, work_dir=str(wd))
    assert r3["resumed_segments"] == 0
    # the same path and byte size with different content invalidates the checkpoint too
    r4 = encode_file(str(src), str(tmp_path / "o4.264"), args="-vcodec libx264 -crf 30", backend="cpu", slots=4,
                     seg_frames=8, log=lambda s: None, resume=True, work_dir=str(wd))
    assert r4["resumed_segments"] == 4
    size = src.stat().st_size
    yuv.write_y4m(str(src), yuv.synth_clip_cpu(32, 64, 48, seed=6))
    assert src.stat().st_size == size
    os.utime(src, ns=(src.stat().st_atime_ns, (tmp_path / "o4.264").stat().st_mtime_ns))
    r5 = encode_file(str(src), str(tmp_path / "o5.264"), args="-vcodec libx264 -crf 30", backend="cpu", slots=4,
                     seg_frames=8, log=lambda s: None, resume=True, work_dir=str(wd))
    assert r5["resumed_segments"] == 0


def test_encode_file_json_segment_metrics(tmp_path, monkeypatch):
    """MIVC_LOG_JSON receives one JSON line per encoded segment (frames, bits,
    PSNR) and a closing line per rank."""
    import json as _json

    from govideocompressor_amd.pipeline import encode_file
    from govideocompressor_amd.utils import yuv
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        monkeypatch.delenv(k, raising=False)
    src = tmp_path / "in.y4m"
    yuv.write_y4m(str(src), yuv.synth_clip_cpu(16, 64, 48, seed=2))
    logp = tmp_path / "log.jsonl"
    monkeypatch.setenv("MIVC_LOG_JSON", str(logp))
    encode_file(str(src), str(tmp_path / "o.264"), args="-vcodec libx264 -crf 26", backend="cpu", slots=2,
                seg_frames=8, log=lambda s: None)
    recs = [_json.loads(x) for x in logp.read_text().splitlines()]
    segs = [r for r in recs if r["event"] == "segment"]
    assert sorted(r["segment"] for r in segs) == [0, 1]
    assert all(r["frames"] == 8 and r["bits"] > 0 and r["psnr_y"] > 20 and r["component"] == "encode" for r in segs)
    assert recs[-1]["event"] == "done"
