"""T0: wire protocol codec, -p parsing, size->time heuristic, ffmpeg-arg interpreter."""
import pytest

from govideocompressor_amd.jobs import ffargs
from govideocompressor_amd.jobs import protocol as proto
from govideocompressor_amd.segment import plan as P


def test_job_roundtrip_v1_and_v0():
    j = proto.Job("12movie.mp4", "7", "-threads 4 -vcodec libx264")
    assert j.encode() == b"12movie.mp4;7;-threads 4 -vcodec libx264\n"
    assert j.encode(v1=False) == b"12movie.mp4;7;-threads 4 -vcodec libx264"
    assert proto.parse_job(j.encode()) == j
    assert proto.parse_job(j.encode(v1=False)) == j      # v0 peers send no terminator
    assert j.piece_path == "12movie.mp4/7"


def test_job_rejects_separators_and_v0_window():
    with pytest.raises(proto.ProtocolError):
        proto.Job("d", "1", "-vf a;b").encode()
    with pytest.raises(proto.ProtocolError):
        proto.Job("d;x", "1", "").encode()
    long_args = "-vcodec libx264 " + "-preset medium " * 10
    assert len(proto.Job("d", "1", long_args).encode()) > proto.V0_READ   # v1 has no 100-byte limit
    with pytest.raises(proto.ProtocolError):
        proto.Job("d", "1", long_args).encode(v1=False)


def test_job_args_with_extra_fields_and_malformed():
    # a 2-field message is a valid job with empty args (the reference crashed, D10)
    assert proto.parse_job(b"dir;3") == proto.Job("dir", "3", "")
    for bad in (b"", b"dironly", b";3;x", b"dir;;x"):
        with pytest.raises(proto.ProtocolError):
            proto.parse_job(bad)


def test_reply_codec():
    assert proto.Reply(True, "3").encode() == b"success;3\n"
    assert proto.Reply(False, "3").encode() == b"fail;3\n"
    assert proto.Reply(False, "3", "a;b\nc").encode() == b"fail;3;a,b c\n"
    assert proto.parse_reply(b"success;12") == proto.Reply(True, "12")
    assert proto.parse_reply(b"fail;4;\xe8\xbd\xac\xe6\x8d\xa2\xe5\x8f\x82\xe6\x95\xb0\xe4\xb8\xba\xe7\xa9\xba") \
        == proto.Reply(False, "4", "转换参数为空")
    for bad in (b"su", b"success", b"fail", b"heart", b"garbage;1"):
        with pytest.raises(proto.ProtocolError):
            proto.parse_reply(bad)
    assert proto.is_heartbeat(b"heart;3\n") and proto.is_heartbeat("heart")


def test_line_socket_keeps_remainder():
    import socket
    a, b = socket.socketpair()
    try:
        a.sendall(b"hello;w;0\nheart;1\nsucc")
        a.sendall(b"ess;1")
        a.shutdown(socket.SHUT_WR)
        ls = proto.LineSocket(b)
        assert ls.recv_message(1) == b"hello;w;0\n"
        assert ls.recv_message(1) == b"heart;1\n"
        assert ls.recv_message(1) == b"success;1"      # unterminated v0 tail at EOF
        assert ls.recv_message(1) == b""
    finally:
        a.close()
        b.close()


def test_parse_pieces():
    assert P.parse_pieces("3;7") == ["3", "7"]
    assert P.parse_pieces("03;3;7;7") == ["03", "7"]          # verbatim tokens, dedup by value
    assert P.parse_pieces("5") == ["5"]
    for bad in ("3;", "a;1", " 3", "3.5", ""):
        with pytest.raises(ValueError):
            P.parse_pieces(bad)


def test_reference_segment_seconds():
    # server.go:54-58: size * (dur+1) / fileMiB in integers
    assert P.reference_segment_seconds(10, 601, 200 * 1024 * 1024) == 30
    assert P.reference_segment_seconds(10, 61, 1024 * 1024 * 7 + 5) == 87
    assert P.reference_segment_seconds(10, 11, 100) >= 1          # D1: no division by zero
    assert P.reference_segment_seconds(1, 2, 500 * 1024 * 1024) == 1


def test_plans():
    fp = P.fixed_plan(25, 8)
    assert fp[:, 0].tolist() == [0, 8, 16, 24] and fp[:, 1].tolist() == [8, 8, 8, 1]
    bp = P.balanced_plan(600, world=4, per_rank=4)
    assert len(bp) == 16 and bp[:, 1].sum() == 600 and bp[:, 1].max() - bp[:, 1].min() <= 1
    gp = P.balanced_plan(100, world=2, per_rank=2, gop=12)
    assert gp[:, 1].sum() == 100 and all(s % 12 == 0 for s in gp[:, 0])
    assert len(P.balanced_plan(10, world=8, per_rank=4, min_frames=5)) == 2
    # cost-balanced sharding
    pl = P.weight_plan(P.fixed_plan(8, 1), [10, 1, 1, 1, 1, 1, 1, 10])
    s0, s1 = P.shard(pl, 0, 2, by_cost=True), P.shard(pl, 1, 2, by_cost=True)
    assert sorted(s0 + s1) == list(range(8))
    assert abs(sum(pl[s0, 2]) - sum(pl[s1, 2])) <= 2
    assert P.shard(pl, 1, 3) == [1, 4, 7]


def test_ffargs_presets_and_defaults():
    c = ffargs.parse("264")
    assert c.codec == "h264" and c.crf == 23.0 and "-threads 4" in c.ignored
    c = ffargs.parse("265")
    assert c.codec == "hevc" and c.crf == 26.0
    c = ffargs.parse("-vcodec libx265")
    assert c.crf == 28.0
    c = ffargs.parse("-c:v h264 -qp 30 -s 1280x720 -r 25 -g 48 -preset fast -y -an")
    assert (c.qp, c.crf, c.size, c.fps, c.keyint, c.preset) == (30, None, (1280, 720), 25.0, 48, "fast")
    c = ffargs.parse("-vcodec libx264 -b:v 2500k -pass 2")
    assert c.bitrate == 2_500_000 and c.crf is None and c.two_pass == 2
    c = ffargs.parse("-vcodec libx265 -pix_fmt yuv420p10le -crf 20")
    assert c.bit_depth == 10 and c.crf == 20


def test_ffargs_errors():
    for bad in ("", "   ", "-vcodec vp9", "-vf scale=1:1", "-s 1281x720", "-s big", "-crf", "-pass 3",
                "-pix_fmt rgb24", "-crf abc", "-g x", "-vcodec \"libx264"):
        with pytest.raises(ffargs.FfArgsError):
            ffargs.parse(bad)


def test_ffargs_rate_vbv_audio_options():
    c = ffargs.parse("-vcodec libx264 -b:v 2M -maxrate 3M -bufsize 4M -pass 1 -passlogfile /tmp/x -preset SLOW")
    assert (c.bitrate, c.maxrate, c.bufsize, c.two_pass, c.passlogfile, c.preset) == (
        2_000_000, 3_000_000, 4_000_000, 1, "/tmp/x", "slow")
    assert ffargs.parse("264 -an".replace("264", "-vcodec libx264")).audio == "none"
    assert ffargs.parse("-vcodec libx264 -acodec copy").audio == "copy"
    for bad in ("-vcodec libx264 -pass 2", "-vcodec libx264 -b:v 1M -maxrate 2M", "-vcodec libx264 -preset warp9",
                "-vcodec libx264 -acodec aac", "-vcodec libx264 -b:v 0"):
        with pytest.raises(ffargs.FfArgsError):
            ffargs.parse(bad)


def test_ffargs_profile_tune_level_params():
    """-profile:v / -tune / -level / -x26x-params map onto encoder knobs."""
    from govideocompressor_amd.models.h264_gpu import H264Params
    from govideocompressor_amd.models.hevc_gpu import HevcParams
    from govideocompressor_amd.ops import native
    host = native.host()
    c = ffargs.parse("-vcodec libx264 -profile:v baseline")
    p = c.apply_opts(H264Params(width=640, height=360))
    assert p.cabac is False and p.eff_bframes() == 0 and not p.eff_t8x8()
    sps = host.stream_info(host.parameter_sets(p.host_cfg()))
    assert sps["profile_idc"] == 66                                   # Constrained Baseline
    p = ffargs.parse("-vcodec libx264 -profile:v main").apply_opts(H264Params(width=640, height=360))
    assert p.cabac and not p.eff_t8x8() and host.stream_info(host.parameter_sets(p.host_cfg()))["profile_idc"] == 77
    c = ffargs.parse("-vcodec libx264 -level 4.1 -tune zerolatency -x264-params bframes=0:aq-mode=0:keyint=48:crf=20")
    assert (c.level, c.keyint, c.crf, c.tune) == (41, 48, 20.0, "zerolatency")
    p = c.apply_opts(H264Params(width=1920, height=1080))
    assert (p.bframes, p.lookahead, p.mbtree, p.aq_strength, p.level_idc) == (0, False, False, 0.0, 41)
    assert host.stream_info(host.parameter_sets(p.host_cfg()))["level_idc"] == 41
    with pytest.raises(RuntimeError):                                 # 1080p30 does not fit level 3
        host.parameter_sets(ffargs.parse("-vcodec libx264 -level 3").apply_opts(H264Params(1920, 1080)).host_cfg())
    c = ffargs.parse("-vcodec libx265 -profile:v main10 -level 5.1 -x265-params sao=0:max-merge=5:no-cutree=1")
    assert c.bit_depth == 10 and c.level == 153 and c.crf == 28.0
    p = c.apply_opts(HevcParams(width=1920, height=1080, bit_depth=10))
    assert (p.sao, p.max_merge, p.cutree, p.level_idc) == (False, 5, False, 153)
    assert ffargs.parse("-vcodec libx265 -x265-params crf=22").crf == 22.0
    assert ffargs.parse("-vcodec libx265 -profile:v mainstillpicture").opts == {"intra_only": True}
    assert ffargs.parse("-vcodec libx265 -tune fastdecode").opts == {"deblock": False, "sao": False}
    # x265's own B-picture structure on request (bframes 4 with a reference-B pyramid, TMVP)
    p = ffargs.parse("-vcodec libx265 -x265-params bframes=4:b-pyramid=1:tmvp=1").apply_opts(HevcParams(64, 64))
    assert (p.bframes, p.pyramid, p.tmvp, p.eff_bframes()) == (4, True, True, 4)
    assert ffargs.parse("-vcodec libx265 -tune zerolatency").apply_opts(HevcParams(64, 64)).eff_bframes() == 0


def test_ffargs_strict_rejections():
    """Options the native encoders cannot honour are errors, never silently dropped."""
    for bad in ("-vcodec libx264 -tune film", "-vcodec libx264 -tune ssim", "-vcodec libx264 -profile:v high10",
                "-vcodec libx264 -profile:v high444", "-vcodec libx265 -profile:v main12",
                "-vcodec libx264 -x264-params ref=5", "-vcodec libx264 -x264-params direct=auto",
                "-vcodec libx264 -x264-params b-adapt=2", "-vcodec libx264 -x264-params b-pyramid=strict",
                "-vcodec libx264 -x264-params foo=1", "-vcodec libx264 -x265-params sao=0",
                "-vcodec libx265 -x265-params bframes=9", "-vcodec libx265 -x265-params ctu=16",
                "-vcodec libx264 -x264-params aq-mode=2", "-vcodec libx264 -x264-params deblock=1,1",
                "-vcodec libx264 -profile:v baseline -x264-params bframes=3", "-vcodec libx264 -level 9",
                "-vcodec libx265 -profile:v main -pix_fmt yuv420p10le", "-vcodec copy -tune psnr"):
        with pytest.raises(ffargs.FfArgsError):
            ffargs.parse(bad)


def test_ffargs_reference_and_weighting_knobs():
    """-x264-params ref / weightp / weightb / trellis and -x265-params ctu reach the encoders;
    the speed presets carry x264's / x265's values for them."""
    from govideocompressor_amd.models.h264_gpu import H264Params
    from govideocompressor_amd.models.hevc_gpu import HevcParams
    from govideocompressor_amd.rc import presets
    p = ffargs.parse("-vcodec libx264 -x264-params ref=1:weightp=0:trellis=0:no-weightb=1").apply_opts(H264Params(64, 64))
    assert (p.refs, p.weightp, p.trellis, p.weightb) == (1, False, 0, False)
    p = ffargs.parse("-vcodec libx264 -x264-params ref=4:weightp=2:trellis=2:direct=temporal").apply_opts(H264Params(64, 64))
    assert (p.refs, p.weightp, p.trellis, p.eff_refs(), p.direct) == (4, True, 2, 4, "temporal")
    p = ffargs.parse("-vcodec libx264 -x264-params direct=spatial").apply_opts(H264Params(64, 64))
    assert p.direct == "spatial"
    assert presets.apply(H264Params(64, 64), "slower").direct == "spatial"
    # x264 --b-pyramid normal: slower and up, or asked for (implies spatial direct here)
    sl = presets.apply(H264Params(64, 64), "slower")
    assert sl.pyramid and sl.spatial_wavefront and not presets.apply(H264Params(64, 64), "medium").pyramid
    p = ffargs.parse("-vcodec libx264 -x264-params b-pyramid=normal").apply_opts(H264Params(64, 64))
    assert (p.pyramid, p.direct, p.spatial_wavefront) == (True, "spatial", True)
    p = ffargs.parse("-vcodec libx264 -x264-params direct=temporal").apply_opts(sl)
    assert (p.pyramid, p.direct) == (False, "temporal")
    with pytest.raises(ffargs.FfArgsError):
        ffargs.parse("-vcodec libx264 -x264-params b-pyramid=normal:direct=temporal").apply_opts(H264Params(64, 64))
    assert presets.apply(H264Params(64, 64), "medium").direct == "temporal"
    assert H264Params(64, 64, cabac=False, refs=3).eff_refs() == 1     # Constrained Baseline: one reference
    assert presets.apply(H264Params(64, 64), "ultrafast").refs == 1
    assert presets.apply(H264Params(64, 64), "fast").refs == 2
    assert presets.apply(H264Params(64, 64), "slow").refs == 4
    p = ffargs.parse("-vcodec libx265 -x265-params ctu=32").apply_opts(HevcParams(64, 64))
    assert p.ctu64 is False and HevcParams(64, 64).ctu64 is True
    assert presets.apply(HevcParams(64, 64), "ultrafast").ctu64 is False
