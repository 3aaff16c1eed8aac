"""Bicubic resampling kernel (scale.hip) against its numpy model, bit-exact, plus the RGB
-> I420 conversion; 8-bit and 10-bit, up / down / anisotropic, with coded-size padding."""
import numpy as np
import pytest

from govideocompressor_amd.ops import scale

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("w,h,ow,oh,bd", [(96, 64, 64, 36, 8), (64, 48, 100, 76, 8), (320, 180, 80, 46, 8),
                                          (176, 144, 176, 72, 10), (50, 34, 128, 96, 10), (640, 360, 1280, 720, 8)])
def test_scale_matches_numpy(w, h, ow, oh, bd):
    import torch
    rng = np.random.default_rng(w * 7 + ow)
    dt = np.uint8 if bd == 8 else np.uint16
    src = (rng.random((3, h, w)) * ((1 << bd) - 1)).astype(dt)
    # smooth structure as well as noise: ramps + a disc
    yy, xx = np.mgrid[0:h, 0:w]
    src[1] = (((xx * 3 + yy * 5) % (1 << bd))).astype(dt)
    src[2] = np.where((xx - w / 2) ** 2 + (yy - h / 2) ** 2 < (min(w, h) / 3) ** 2, (1 << bd) - 1, 0).astype(dt)
    want = scale.scale_plane_ref(src, ow, oh, bd)
    t = torch.from_numpy(src.astype(np.int16) if bd == 10 else src).cuda()
    sc = scale.GpuScaler("cuda")
    got = sc.plane(t, ow, oh, bd).cpu().numpy()
    if bd == 10:
        got = got.astype(np.uint16)
    assert np.array_equal(got, want), np.argwhere(got != want)[:5]
    # coded-size padding replicates the last display column / row
    W, H = (ow + 15) // 16 * 16, (oh + 15) // 16 * 16
    padded = sc.plane(t, ow, oh, bd, W=W, H=H).cpu().numpy()
    if bd == 10:
        padded = padded.astype(np.uint16)
    assert np.array_equal(padded[:, :oh, :ow], want)
    assert np.array_equal(padded[:, :oh, ow:], np.repeat(want[:, :, -1:], W - ow, axis=2))


def test_scale_clip_and_backend_resize(tmp_path, host):
    """-s through the GPU backend equals the numpy model's scaled input fed to the encoder
    (checked on the decoded size and PSNR against the model-scaled source)."""
    from govideocompressor_amd.backends import PieceJob, get_backend
    from govideocompressor_amd.utils import yuv
    c = yuv.synth_clip_cpu(4, 352, 288, seed=9)
    p = tmp_path / "0.y4m"
    yuv.write_y4m(str(p), c)
    be = get_backend("gpu")
    (r,) = be.run([PieceJob("0", str(p), str(tmp_path / "o.264"))], "-vcodec libx265 -s 176x144 -crf 20")
    be.close()
    assert r.ok, r.reason
    pics = host.hevc_decode(open(tmp_path / "o.264", "rb").read())
    assert len(pics) == 4
    ref = scale.scale_plane_ref(c.y, 176, 144)
    y = np.stack([np.asarray(pp["y"])[:144, :176] for pp in pics]).astype(np.float64)
    mse = np.mean((y - ref) ** 2)
    # a wrong scaler lands far below this; x265-style variance AQ (default on) costs ~0.6 dB
    # of PSNR on this 176x144 clip
    assert 10 * np.log10(255 ** 2 / mse) > 28


def test_rgb_to_i420_matches_numpy():
    import torch
    rgb = (np.random.default_rng(3).random((2, 32, 48, 3)) * 255).astype(np.uint8)
    y, u, v = scale.rgb_to_i420(torch.from_numpy(rgb).cuda())
    wy, wu, wv = scale.rgb_to_i420_ref(rgb)
    for a, b in ((y, wy), (u, wu), (v, wv)):
        assert np.abs(a.cpu().numpy().astype(int) - b.astype(int)).max() <= 1
