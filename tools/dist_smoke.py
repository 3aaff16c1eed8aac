"""RCCL smoke of the distributed collectives at world 1 (one GPU): run with
``WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=<p> MIVC_DIST_FORCE=1``.

Initialises an ``nccl`` process group on the device and executes CC-1 (``allreduce_stats``),
CC-2/CC-3 (``BitstreamGather``, ``SegmentMerge``, also streaming into a sink) and CC-4/CC-5
on device tensors -- the code paths of an 8-GPU node, minus the peers.  Prints ``OK``."""
import io
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> None:
    import torch

    from govideocompressor_amd.parallel import dist as D
    env = D.init(prefer_gpu=True)
    assert env.initialized and env.backend == "nccl", (env.backend, env.initialized)
    try:
        st = torch.arange(12, dtype=torch.float64, device=env.device).view(3, 4)
        D.allreduce_stats(env, st)
        assert st.cpu().flatten().tolist() == list(range(12))
        pieces = [b"\0\0\0\1" + bytes([i]) * (i + 3) for i in range(4)]
        got = D.BitstreamGather(env, pieces).start().wait()
        assert got == [pieces], got
        m = D.SegmentMerge(env)
        with torch.cuda.stream(torch.cuda.Stream(env.device)):
            merged = m.run(pieces)
        assert bytes(merged) == b"".join(pieces)
        sink = io.BytesIO()
        n = m.run([[p[:2], p[2:]] for p in pieces], sink=sink)
        assert n == sum(map(len, pieces)) and sink.getvalue() == b"".join(pieces)
        assert D.broadcast_object(env, {"k": 1}) == {"k": 1}
        assert D.max_over_ranks(env, 2.5) == 2.5
        D.barrier(env)
        torch.cuda.synchronize()
    finally:
        D.shutdown(env)
    print("OK")


if __name__ == "__main__":
    main()
