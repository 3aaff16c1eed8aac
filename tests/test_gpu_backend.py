"""GPU worker backend + single-node pipeline on the MI355X (T1/T2 through the job API).

Pieces of unequal length and a keyint shorter than a piece exercise the batching
(padding, truncation, per-unit idr_pic_id); every output must decode with the
independent CPU decoder to the right number of frames at a sane PSNR."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _psnr(a, b):
    mse = np.mean((a.astype(np.float64) - b.astype(np.float64)) ** 2)
    return 100.0 if mse == 0 else 10 * np.log10(255 ** 2 / mse)


def test_gpu_backend_batch(tmp_path, host):
    from govideocompressor_amd.backends import PieceJob, get_backend
    from govideocompressor_amd.utils import yuv

    jobs, clips = [], {}
    for i, n in enumerate([10, 7, 12]):
        c = yuv.synth_clip_cpu(n, 176, 144, seed=i)
        p = tmp_path / f"{i}.y4m"
        yuv.write_y4m(str(p), c)
        clips[str(i)] = c
        jobs.append(PieceJob(str(i), str(p), str(tmp_path / f"o{i}.mp4"), str(tmp_path / f"c{i}.mp4.log")))
    be = get_backend("gpu")
    res = be.run(jobs, "-vcodec libx264 -crf 24 -g 5")
    be.close()
    for j, r in zip(jobs, res):
        assert r.ok, r.reason
        data = open(j.out_path, "rb").read()
        es = host.mp4_demux(data)
        pics = host.decode(es)
        c = clips[j.idx]
        assert len(pics) == c.frames
        assert sum(p["idr"] for p in pics) == (c.frames + 4) // 5
        y = np.stack([p["i420"][: 176 * 144].reshape(144, 176) for p in pics])
        assert _psnr(y, c.y) > 27  # CRF 23 with AQ + MB-tree (x264 defaults) on noise-textured content
        assert os.path.exists(j.log_path)


def test_gpu_backend_scaling(tmp_path, host):
    from govideocompressor_amd.backends import PieceJob, get_backend
    from govideocompressor_amd.utils import yuv

    c = yuv.synth_clip_cpu(4, 352, 288, seed=5)
    p = tmp_path / "0.y4m"
    yuv.write_y4m(str(p), c)
    be = get_backend("gpu")
    (r,) = be.run([PieceJob("0", str(p), str(tmp_path / "o.264"))], "-vcodec libx264 -s 176x144")
    be.close()
    assert r.ok, r.reason
    pics = host.decode(open(tmp_path / "o.264", "rb").read())
    assert len(pics) == 4 and pics[0]["width"] == 176 and pics[0]["height"] == 144


def test_pipeline_encode_file_gpu(tmp_path, host):
    from govideocompressor_amd.pipeline import encode_file
    from govideocompressor_amd.utils import yuv

    c = yuv.synth_clip_cpu(40, 320, 240, seed=9)
    src = tmp_path / "in.y4m"
    yuv.write_y4m(str(src), c)
    out = tmp_path / "out.264"
    r = encode_file(str(src), str(out), args="264", backend="gpu", slots=4, log=lambda s: None)
    assert r["segments"] >= 2
    pics = host.decode(open(out, "rb").read())
    assert len(pics) == 40
    y = np.stack([p["i420"][: 320 * 240].reshape(240, 320) for p in pics])
    assert _psnr(y, c.y) > 27  # CRF 23 with AQ + MB-tree (x264 defaults)


def test_gpu_backend_transcode_pipelined_groups(tmp_path, host, monkeypatch):
    """Compressed pieces go through the two-stage pipeline of GpuBackend.transcode (decode of
    group k+1 on its own stream while group k encodes): groups of 2 must give the same bytes
    as one group holding every piece."""
    from govideocompressor_amd.backends import PieceJob, get_backend
    from govideocompressor_amd.utils import yuv

    jobs = []
    for i in range(5):
        c = yuv.synth_clip_cpu(8, 176, 144, seed=20 + i)
        y = tmp_path / f"{i}.y4m"
        yuv.write_y4m(str(y), c)
        jobs.append(PieceJob(str(i), str(y), str(tmp_path / f"{i}.264")))
    be = get_backend("gpu")
    for r in be.run(jobs, "-vcodec libx264 -qp 22"):
        assert r.ok, r.reason
    outs = {}
    for g in ("2", "64"):
        monkeypatch.setenv("MIVC_TRANSCODE_GROUP", g)
        tj = [PieceJob(j.idx, j.out_path, str(tmp_path / f"t{g}_{j.idx}.264")) for j in jobs]
        for r in be.run(tj, "-vcodec libx264 -crf 23"):
            assert r.ok, r.reason
        outs[g] = [open(j.out_path, "rb").read() for j in tj]
    be.close()
    assert outs["2"] == outs["64"]
    for s in outs["2"]:
        assert len(host.decode(s)) == 8
