"""CPU reference encoder edge cases (host library, no GPU)."""
import numpy as np


def test_cpu_encoder_keyint_zero_is_one_idr(host):
    """keyint <= 0 means "the first picture is the only IDR" (the GPU encoders' convention);
    it used to divide by zero."""
    from govideocompressor_amd.utils import yuv
    c = yuv.synth_clip_cpu(4, 64, 48, seed=2)
    st = host.CpuEncoder(dict(width=64, height=48, qp=28, keyint=0)).encode(c.i420(), 4, 0)
    pics = host.decode(st)
    assert len(pics) == 4
    assert [bool(p["idr"]) for p in pics] == [True, False, False, False]
    assert (pics[0]["width"], pics[0]["height"]) == (64, 48)
