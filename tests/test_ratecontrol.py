"""Rate control math (CRF mapping, two-pass ABR solve) and the CC-1 statistics table."""
import numpy as np

from govideocompressor_amd.rc import ratecontrol as rc


def test_qscale_roundtrip():
    for qp in (0, 12, 23, 36, 51):
        assert abs(rc.qscale2qp(rc.qp2qscale(qp)) - qp) < 1e-9


def test_crf_qps_monotonic_in_crf_and_complexity():
    intra = np.full(10, 8000.0 * 80)
    inter = np.full(10, 3000.0 * 80)
    q23 = rc.crf_qps(intra, inter, 23, mb_count=8160)
    q30 = rc.crf_qps(intra, inter, 30, mb_count=8160)
    assert (q30 >= q23).all() and (q30 > q23).any()
    assert q23[0] == q23[1] - rc.IP_OFFSET or q23[0] < q23[1]        # key frame gets a lower QP
    hard = rc.crf_qps(intra * 4, inter * 4, 23, mb_count=8160)
    assert (hard >= q23).all() and hard[5] > q23[5]                   # qcomp: complex frames get higher QP
    gop = rc.crf_qps(intra, inter, 23, mb_count=8160, keyint=5)
    assert gop[5] < gop[4]


def test_abr_solve_hits_target():
    rng = np.random.default_rng(0)
    stats = np.zeros((50, 4))
    stats[:, 2] = rng.uniform(1e5, 3e5, 50)   # pass-1 bits
    stats[:, 3] = 26
    tot = stats[:, 2].sum()
    d = rc.abr_solve(stats, tot / 2)
    assert abs(d - 6.0) < 1e-9                 # half the bits = +6 QP at exponent 1
    q = rc.abr_qps(stats, tot / 2)
    assert (q == 32).all()
    assert abs(rc.estimate_exponent(1000, 20, 500, 26) - 1.0) < 1e-9


def test_global_stats_single_process():
    g = rc.GlobalStats(6)
    g.put(0, np.ones((3, 4)))
    g.put(3, 2 * np.ones((3, 4)))
    t = g.reduce()
    assert t[:, 0].tolist() == [1, 1, 1, 2, 2, 2]


def test_scenecut_flags_and_keyframe_qps():
    B, F = 2, 6
    costs = np.zeros((B, F, 2))
    costs[:, :, 0] = 1000.0          # intra cost
    costs[:, :, 1] = 200.0           # inter predicts well ...
    costs[0, 3, 1] = 990.0           # ... except at a cut in slot 0, frame 3
    costs[1, 3, 1] = 950.0           # saving 5 % right after a key frame is no cut (x264 bias 0.025)
    costs[1, 0, 1] = 1000.0          # frame 0 is a key frame anyway: never flagged
    f = rc.scenecut_flags(costs, 40.0)
    assert f.tolist() == [[False, False, False, True, False, False], [False] * 6]
    assert not rc.scenecut_flags(costs, 0.0).any()
    q = rc.crf_qps_batch(costs, 23.0, 100, scenecuts=f)
    q0 = rc.crf_qps_batch(costs, 23.0, 100)
    assert q[0, 3] < q0[0, 3]        # intra complexity and the I-frame offset at the cut
    assert (q[1] == q0[1]).all()


def test_scenecut_bias_grows_with_the_distance_from_the_key_frame():
    """x264 scenecut_internal: 50 frames after the key frame (past keyint_min 25) the bias is
    0.1 + 0.3 * 25 / 225 = 0.133: a frame whose inter prediction saves 10 % is a cut there,
    one saving 15 % is not; 5 frames in, neither is."""
    costs = np.zeros((1, 60, 2))
    costs[..., 0] = 1000.0
    costs[..., 1] = 300.0
    costs[0, 50, 1] = 900.0
    costs[0, 55, 1] = 850.0
    costs[0, 5, 1] = 900.0
    f = rc.scenecut_flags(costs, 40.0)
    assert f[0, 50] and not f[0, 55] and not f[0, 5]
