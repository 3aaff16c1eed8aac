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
        assert got[0] == [b"zero"]
        assert got[1] == [b"\x01" * 4, b"", b"\x07"]
        assert got[2] == [b"\x02" * 7, b"", b"\x07\x07"]
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
