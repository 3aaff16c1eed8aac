"""T0/T2: raw video I/O, probe, split (raw + compressed), merge, filelist/concat.sh."""
import json
import os

import numpy as np
import pytest

from govideocompressor_amd.segment import merge as M
from govideocompressor_amd.segment.probe import probe, reference_seconds
from govideocompressor_amd.segment.split import file_count, piece_files, split, split_dir_name
from govideocompressor_amd.utils import yuv


def _encode(host, clip, qp=28, keyint=1 << 30, idr=0):
    enc = host.CpuEncoder(dict(width=clip.width, height=clip.height, fps=clip.fps, qp=qp, keyint=keyint))
    return enc.encode(clip.i420(), clip.frames, idr)


def test_y4m_roundtrip(tmp_path):
    c = yuv.synth_clip_cpu(5, 64, 48, seed=1, fps=25)
    p = tmp_path / "a.y4m"
    yuv.write_y4m(str(p), c)
    d = yuv.read_y4m(str(p))
    assert d.fps == 25 and d.frames == 5
    assert np.array_equal(d.y, c.y) and np.array_equal(d.u, c.u) and np.array_equal(d.v, c.v)
    part = yuv.read_y4m(str(p), 2, 2)
    assert np.array_equal(part.y, c.y[2:4])
    assert np.array_equal(yuv.read_y4m(p.read_bytes()).v, c.v)
    ntsc = yuv.Clip(c.y, c.u, c.v, 30000 / 1001)
    assert abs(yuv.read_y4m(yuv.y4m_bytes(ntsc)).fps - 29.97) < 0.01


def test_yuv_raw_and_probe(tmp_path):
    c = yuv.synth_clip_cpu(6, 32, 16, seed=2)
    p = tmp_path / "a.yuv"
    yuv.write_yuv(str(p), c)
    info = probe(str(p), 32, 16, 30)
    assert (info.kind, info.frames, info.width) == ("yuv", 6, 32)
    assert reference_seconds(info) == 1   # 0.2 s -> int + 1 (server.go:262)
    assert np.array_equal(yuv.read_yuv(str(p), 32, 16, start=3).y, c.y[3:])
    with pytest.raises(ValueError):
        probe(str(p))                    # raw needs geometry


def test_split_raw_y4m(tmp_path):
    c = yuv.synth_clip_cpu(20, 48, 32, seed=3)
    src = tmp_path / "clip.y4m"
    yuv.write_y4m(str(src), c)
    logs = []
    d, n = split(str(src), frames=6, out_root=str(tmp_path), log=logs.append)
    assert os.path.basename(d) == "12clip.y4m" and n == 4
    assert logs[1] == "split video....wait" and logs[-1] == f"[{d}] [4]"
    files = piece_files(d)
    assert sorted(files, key=int) == ["0", "1", "2", "3"]
    frames = [yuv.read_y4m(os.path.join(d, files[str(i)])) for i in range(4)]
    assert [f.frames for f in frames] == [6, 6, 6, 2]
    assert np.array_equal(np.concatenate([f.y for f in frames]), c.y)
    man = json.load(open(os.path.join(d, "plan.json")))
    assert man["segment_frames"] == 6 and len(man["pieces"]) == 4
    assert file_count(d) == 5      # pieces + plan.json (the reference's recursive count)


def test_split_dir_name():
    assert split_dir_name("movie.mp4") == "12movie.mp4"
    assert split_dir_name("/data/in/movie.mp4") == "12movie.mp4"     # D16 fixed
    assert split_dir_name("C:\\v\\m.mp4") == "12C:.v.m.mp4"


def test_split_and_merge_compressed(tmp_path, host):
    c = yuv.synth_clip_cpu(12, 64, 48, seed=4)
    es = _encode(host, c, keyint=3)
    src = tmp_path / "movie.264"
    src.write_bytes(es)
    info = probe(str(src))
    assert (info.kind, info.frames, info.idr_frames, info.entropy) == ("h264", 12, 4, "cavlc")
    d, n = split(str(src), frames=5, out_root=str(tmp_path), log=lambda s: None)
    assert n == 2   # cuts at the first IDR at/after 5 frames: [0..5], [6..11]
    files = piece_files(d)
    pieces = [open(os.path.join(d, files[str(i)]), "rb").read() for i in range(n)]
    assert [host.stream_info(p)["frames"] for p in pieces] == [6, 6]
    # every piece decodes on its own, and the merge is the original stream
    out = tmp_path / "merged.264"
    M.merge_files([os.path.join(d, files[str(i)]) for i in range(n)], str(out))
    dec_a = host.decode(out.read_bytes())
    dec_b = host.decode(es)
    assert len(dec_a) == 12
    for a, b in zip(dec_a, dec_b):
        assert np.array_equal(a["i420"], b["i420"])


def test_split_mp4_and_mp4_merge(tmp_path, host):
    c = yuv.synth_clip_cpu(8, 64, 48, seed=5)
    es = _encode(host, c, keyint=4)
    src = tmp_path / "m.mp4"
    src.write_bytes(host.mp4_mux(es, 30.0))
    assert probe(str(src)).frames == 8
    d, n = split(str(src), frames=4, out_root=str(tmp_path), log=lambda s: None)
    assert n == 2 and all(f.endswith(".mp4") for f in piece_files(d).values())
    M.make_filelist(n, d, "mp4")
    assert open(os.path.join(d, "filelist.txt")).read() == "file '0.mp4'\nfile '1.mp4'\n"
    out = M.merge_dir(d)
    info = probe(out)
    assert info.kind == "mp4" and info.frames == 8 and info.idr_frames == 2
    got = host.decode(host.mp4_demux(open(out, "rb").read()))
    ref = host.decode(es)
    assert all(np.array_equal(a["i420"], b["i420"]) for a, b in zip(got, ref))


def test_filelist_concat_only_if_absent(tmp_path):
    d = str(tmp_path)
    M.make_filelist(3, d)
    M.make_filelist(["0"], d)          # second call keeps the original list (server.go:333-335)
    assert M.read_filelist(os.path.join(d, "filelist.txt")) == [os.path.join(d, f"{i}.mp4") for i in range(3)]
    sh = M.make_concat_script(d)
    assert os.access(sh, os.X_OK)
    body = open(sh).read()
    assert body.startswith("#!/bin/sh") and "merge --list filelist.txt -o output.mp4" in body
    with pytest.raises(FileNotFoundError):
        M.merge_files(M.read_filelist(os.path.join(d, "filelist.txt")), os.path.join(d, "o.264"))
