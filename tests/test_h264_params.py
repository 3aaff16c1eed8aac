"""H264Params / GpuH264Encoder host-side rules that need no GPU."""
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
