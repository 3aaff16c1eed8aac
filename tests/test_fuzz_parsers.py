"""Fuzzing the parsers that see network-fetched pieces (a worker decodes whatever the
coordinator serves it: client.go:92-96 in the reference).  Truncated, bit-flipped and
spliced H.264 / HEVC Annex-B and MP4 data must end in a Python exception (ValueError /
RuntimeError from the C++ layer), never a crash or a hang.  Run under the ASan+UBSan
build of ``_host`` by tools/asan_tests.sh."""
import numpy as np
import pytest
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from govideocompressor_amd.segment import mp4
from govideocompressor_amd.utils import yuv

_SETTINGS = settings(max_examples=60, deadline=None, suppress_health_check=list(HealthCheck), derandomize=True)
_OK = (ValueError, RuntimeError, IndexError, OverflowError, MemoryError)


@pytest.fixture(scope="module")
def seeds(host):
    c = yuv.synth_clip_cpu(6, 48, 32, seed=2)
    cavlc = host.CpuEncoder(dict(width=48, height=32, qp=30, keyint=3)).encode(c.i420(), 6, 0)
    from govideocompressor_amd.utils.h264_synth import random_stream
    cabac = random_stream(host, 48, 32, 4, seed=3, cabac=True, t8x8=True)
    from govideocompressor_amd.utils import hevc_synth
    hevc, _ = hevc_synth.random_stream(host, 64, 64, 2, seed=4)
    box = mp4.write([mp4.h264_track(cavlc, 30.0)])
    from govideocompressor_amd.utils import container_synth as CS
    aac = [bytes([k]) * (40 + k) for k in range(12)]
    return dict(cavlc=cavlc, cabac=cabac, hevc=hevc, mp4=box, ts=CS.write_ts(cabac, 30.0, aac),
                mkv=CS.write_mkv(hevc, 30.0, aac))


def _mutate(data: bytes, ops) -> bytes:
    b = bytearray(data)
    for kind, pos, val in ops:
        if not b:
            break
        p = pos % len(b)
        if kind == 0:
            b[p] ^= 1 << (val % 8)
        elif kind == 1:
            del b[p:]
        elif kind == 2:
            b[p:p] = bytes([val & 255]) * (1 + val % 7)
        else:
            b[p] = val & 255
    return bytes(b)


_ops = st.lists(st.tuples(st.integers(0, 3), st.integers(0, 1 << 20), st.integers(0, 1 << 12)), min_size=1,
                max_size=6)


def _try(fn, *a):
    try:
        fn(*a)
    except _OK:
        pass


@_SETTINGS
@given(ops=_ops, which=st.sampled_from(["cavlc", "cabac"]))
def test_fuzz_h264_decode_and_parse(host, seeds, ops, which):
    data = _mutate(seeds[which], ops)
    _try(host.decode, data)
    _try(lambda d: host.parse([d], 1), data)
    _try(host.stream_info, data)
    _try(host.h264_samples, data)
    _try(lambda d: host.split_pieces(d, 2), data)


@_SETTINGS
@given(ops=_ops)
def test_fuzz_hevc_decode(host, seeds, ops):
    _try(host.hevc_decode, _mutate(seeds["hevc"], ops))


@_SETTINGS
@given(ops=_ops)
def test_fuzz_mp4_demux(host, seeds, ops):
    data = _mutate(seeds["mp4"], ops)
    _try(mp4.read, data)
    _try(mp4.annexb_from_mp4, data)
    _try(host.mp4_demux, data)


@_SETTINGS
@given(data=st.binary(min_size=0, max_size=600))
def test_fuzz_random_bytes(host, data):
    for fn in (host.decode, host.hevc_decode, host.stream_info, host.mp4_demux, host.h264_samples, mp4.read):
        _try(fn, data)
    _try(host.decode, b"\x00\x00\x00\x01\x67" + data)
    _try(host.decode, b"\x00\x00\x00\x01\x65" + data)


@_SETTINGS
@given(ops=_ops, which=st.sampled_from(["ts", "mkv"]))
def test_fuzz_ts_mkv_demux(host, seeds, ops, which):
    from govideocompressor_amd.segment import containers
    data = _mutate(seeds[which], ops)
    _try(containers.ts_demux if which == "ts" else containers.mkv_demux, data)
