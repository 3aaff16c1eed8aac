"""H264Params / GpuH264Encoder host-side rules that need no GPU."""
import pytest
from govideocompressor_amd.models.h264_gpu import GpuH264Encoder, H264Params


def test_auto_slice_count_by_height():
    """slices = 0 (auto): one slice up to 68 MB rows (1080p), one per 34 rows above."""
    for (w, h), n in (((1280, 720), 1), ((1920, 1080), 1), ((3840, 2160), 4), ((7680, 4320), 8)):
        p = H264Params(width=w, height=h, slices=0)
        assert p.eff_slices() == n, (w, h)
        if n > 1:
            assert p.slice_rows() * (n - 1) < (h + 15) // 16 <= p.slice_rows() * n
    # an explicit count wins; CAVLC has no slices here
    assert H264Params(width=1920, height=1080, slices=4).eff_slices() == 4
    assert H264Params(width=3840, height=2160, slices=1).eff_slices() == 1
    assert H264Params(width=3840, height=2160, slices=0, cabac=False).eff_slices() == 1
    # the wavefront spatial-direct decision works on one slice only
    p = H264Params(width=3840, height=2160, slices=0, direct="spatial", spatial_wavefront=True)
    assert p.eff_slices() == 1


def test_cabac_groups_isolate_the_idr_step():
    """The IDR step (every slot's step 0) gets its own arithmetic-coder group; the rest are
    G-step groups with the last full one split in two; every step is covered once."""
    for F, G in ((60, 20), (4, 20), (9, 3), (61, 20), (2, 20), (1, 20)):
        groups = GpuH264Encoder._cabac_groups(F, G)
        steps = [t for t0, n in groups for t in range(t0, t0 + n)]
        assert steps == list(range(F)), (F, G, groups)
        if F > 2 and G > 1:
            assert groups[0] == (0, 1)
            assert all(n <= G for _, n in groups)
    assert GpuH264Encoder._cabac_groups(60, 20) == [(0, 1), (1, 20), (21, 20), (41, 10), (51, 9)]


def test_pending_encode_redoes_a_pool_overflow(monkeypatch):
    """PendingEncode.result(): a symbol-pool overflow in a deferred batch drains the other
    batch in flight, grows the pool and re-encodes synchronously; other errors propagate."""
    import pytest
    import torch
    from govideocompressor_amd.models.h264_gpu import CabacPoolExhausted, PendingEncode

    monkeypatch.setattr(torch.cuda, "synchronize", lambda *a, **k: None)
    calls = []

    class FakeEnc:
        dev = "cpu"
        cab_G, cab_grow = 20, 1
        stats: dict = {}

        def __init__(self):
            self._inflight = []

        def _alloc_cabac(self, g, grow):
            calls.append(("grow", grow))
            self.cab_grow = grow

        def encode(self, *planes, **kw):
            calls.append(("encode", planes, kw))
            return ["redone"]

    enc = FakeEnc()

    def overflow():
        raise CabacPoolExhausted("pool")

    other = PendingEncode(enc, lambda: ["other"], ("y2",), {})
    bad = PendingEncode(enc, overflow, ("y", "u", "v"), {"analysis": None})
    enc._inflight += [bad, other]
    assert bad.result() == ["redone"]
    assert other.done() and other.result() == ["other"]     # drained before the pool grew
    assert calls[0] == ("grow", 4) and calls[1][0] == "encode" and calls[1][1] == ("y", "u", "v")
    assert enc._inflight == []

    def boom():
        raise RuntimeError("coder error")
    p = PendingEncode(enc, boom, ("y",), {})
    with pytest.raises(RuntimeError, match="coder error"):
        p.result()


def test_env_knobs_are_explicit(monkeypatch):
    """MIVC_* encoder knobs no longer change H264Params defaults behind the caller's back:
    they apply only through models/knobs.py encoder_overrides (bench.py --allow-knobs), and
    check_environment refuses unknown names and unrequested encoder knobs (round-4 review)."""
    import dataclasses

    from govideocompressor_amd.models import knobs as K
    from govideocompressor_amd.models.h264_gpu import H264Params
    from govideocompressor_amd.models.hevc_gpu import HevcParams
    monkeypatch.setenv("MIVC_TRELLIS", "1")
    monkeypatch.setenv("MIVC_DIRECT", "spatial")
    monkeypatch.setenv("MIVC_LA_SEED", "0")
    monkeypatch.setenv("MIVC_TRELLIS_LAMBDA", "0.75")
    monkeypatch.setenv("MIVC_ENTROPY_THREADS", "4")
    p = H264Params(width=64, height=64)
    assert p.trellis == 2 and p.direct == "temporal" and p.lowres_seed
    assert K.encoder_overrides(H264Params) == dict(trellis=1, direct="spatial", lowres_seed=False, trellis_lambda=0.75)
    assert K.encoder_overrides(HevcParams) == {}
    with pytest.raises(SystemExit, match="allow-knobs"):
        K.check_environment(False)
    s = K.check_environment(True)
    assert s["runtime"] == {"MIVC_ENTROPY_THREADS": "4"} and "MIVC_TRELLIS" in s["encoder"]
    monkeypatch.setenv("MIVC_TRELIS", "1")  # typo
    with pytest.raises(SystemExit, match="unknown"):
        K.check_environment(True)
    # every knob names a real field
    for table, cls in ((K.H264, H264Params), (K.HEVC, HevcParams)):
        names = {f.name for f in dataclasses.fields(cls)}
        assert set(table.values()) <= names
