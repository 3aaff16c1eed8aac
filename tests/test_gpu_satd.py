"""The 4x4 SATD primitives of the decision kernels (csrc/kernels/kcommon.h) against a numpy
fp32 model of x264's satd (sum of |4x4 Hadamard of the residual| / 2), bit-exact: the
packed 16-bit form (satd4x4_u8) is what b_decide, p_mv_refine, p_part8x8 and encode_inter
price candidates with, so any difference would change decisions and bytes."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

H4 = np.array([[1, 1, 1, 1], [1, 1, -1, -1], [1, -1, -1, 1], [1, -1, 1, -1]], np.float32)


def _satd_ref(s, p):
    r = s.astype(np.float32).reshape(-1, 4, 4) - p.astype(np.float32).reshape(-1, 4, 4)
    t = np.einsum("ij,njk,lk->nil", H4, r, H4)
    return (np.abs(t).sum(axis=(1, 2)) / 2).astype(np.int64)


@pytest.mark.parametrize("mode", [0, 1])
def test_satd_primitives_match_numpy(mode):
    from govideocompressor_amd.ops import native
    hip = native.hip()
    rng = np.random.default_rng(3)
    n = 64 * 97
    s = rng.integers(0, 256, (n, 16), dtype=np.uint8)
    p = rng.integers(0, 256, (n, 16), dtype=np.uint8)
    # extremes: full-scale residuals of both signs, flat blocks, one-sample spikes
    s[:64], p[:64] = 255, 0
    s[64:128], p[64:128] = 0, 255
    s[128:192] = p[128:192]
    s[192:256], p[192:256] = 0, 0
    s[192:256, 5] = 255
    s[256:320] = np.where(np.arange(16) % 2, 255, 0)
    p[256:320] = np.where(np.arange(16) % 3, 0, 255)
    dev = torch.device("cuda")
    ts, tp = torch.from_numpy(s).to(dev), torch.from_numpy(p).to(dev)
    out = torch.empty(n, dtype=torch.int32, device=dev)
    hip.satd_blocks(ts.data_ptr(), tp.data_ptr(), out.data_ptr(), n, mode, torch.cuda.current_stream().cuda_stream)
    got = out.cpu().numpy().astype(np.int64)
    want = _satd_ref(s, p)
    assert np.array_equal(got, want), np.argwhere(got != want)[:5]
