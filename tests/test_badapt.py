"""x264 --b-adapt 1 decisions (rc/badapt.py) on synthetic lowres costs, and the anchor CRF
curve (rc/ratecontrol.crf_qps_anchors).  The reference's ``264`` preset is bare
``-vcodec libx264`` (server.go:69-70), whose default is --b-adapt 1; x264's own decisions on
real content are not reproducible here (no x264 in the image): parity unpinned, these pin
the rule itself."""
import numpy as np

from govideocompressor_amd.rc import ratecontrol as rc
from govideocompressor_amd.rc.badapt import anchor_complexity, b_adapt_types


def _costs(F, p_at_distance, b_cost, mb=100):
    p1 = np.array([0.0] + [p_at_distance(1)] * (F - 1)) * mb
    pd = np.zeros((F, 8))
    for d in range(2, 8):
        pd[:, d] = p_at_distance(d) * mb
    bc = np.full(F, b_cost * mb)
    return p1, pd, bc


def test_static_content_takes_full_b_runs():
    p1, pd, bc = _costs(13, lambda d: 20.0 + 2 * d, b_cost=8.0)
    assert b_adapt_types(p1, pd, bc, 3, 100) == "IBBBPBBBPBBBP"


def test_fast_motion_keeps_p_pictures():
    # the cost of predicting across two pictures grows much faster than a B saves
    p1, pd, bc = _costs(9, lambda d: 100.0 * d * d, b_cost=90.0)
    assert b_adapt_types(p1, pd, bc, 3, 100) == "IPPPPPPPP"


def test_runs_end_where_distant_p_gets_expensive():
    # B pays off, but a P four pictures away costs more than 200 per MB: runs of 2
    p1, pd, bc = _costs(10, lambda d: {1: 60.0, 2: 80.0, 3: 180.0, 4: 400.0}.get(d, 800.0), b_cost=10.0)
    t = b_adapt_types(p1, pd, bc, 3, 100)
    assert t.startswith("IBBP") and "BBB" not in t


def test_forced_anchors_end_runs_and_are_never_b():
    p1, pd, bc = _costs(13, lambda d: 20.0 + 2 * d, b_cost=8.0)
    t = b_adapt_types(p1, pd, bc, 3, 100, forced=[2, 7])
    assert t[2] == "P" and t[7] == "P" and t[-1] == "P" and t[0] == "I"
    assert all(len(run) <= 3 for run in t[1:].replace("P", " ").split())


def test_anchor_complexity_uses_the_real_distance():
    costs = np.array([[1000, 1000], [900, 100], [900, 110], [900, 120], [900, 130]], dtype=float)
    multi = np.zeros((5, 8))
    multi[4, 4] = 333
    multi[2, 2] = 222
    c = anchor_complexity("IBBBP", costs, multi)
    assert c[0] == 1000 and c[4] == 333 and np.isnan(c[1:4]).all()
    c = anchor_complexity("IBPPP", costs, multi)
    assert c[2] == 222 and c[3] == 120 and c[4] == 130


def test_crf_anchor_curve_ignores_b_pictures_and_uses_the_b_constant():
    B, F = 2, 5
    cplx = np.array([[np.nan, np.nan, np.nan, np.nan, 5000.0]] * B)
    intra = np.full((B, F), 20000.0)
    keys = np.zeros((B, F), bool)
    keys[:, 0] = True
    q3 = rc.crf_qps_anchors(cplx, intra, 23.0, 100, keys, bframes=3)
    q0 = rc.crf_qps_anchors(cplx, intra, 23.0, 100, keys, bframes=0)
    # base complexity 120 (B pictures on) vs 80: the same anchor is coded finer
    assert q3[0, 4] < q0[0, 4]
    assert q3[0, 0] == q3[1, 0]


def test_b_costs_are_scaled_like_x264():
    """x264 prices a lowres B frame at 100 / 120 of its SATD sum (slicetype frame cost with
    --b-bias 0): a B that costs 125 against a 120 P pair still wins (0.833 * 45 + 80 < 120)."""
    p1, pd, bc = _costs(4, lambda d: {1: 60.0, 2: 80.0}.get(d, 900.0), b_cost=45.0)
    assert b_adapt_types(p1, pd, bc, 3, 100)[:3] == "IBP"


def test_intra_guards_force_p_like_x264():
    """x264's i_intra_mbs checks: a P two pictures away that is mostly intra (> mb / 2) keeps
    both pictures P; a closing P more than a third intra ends a B run early."""
    p1, pd, bc = _costs(13, lambda d: 20.0 + 2 * d, b_cost=8.0)
    assert b_adapt_types(p1, pd, bc, 3, 100) == "IBBBPBBBPBBBP"
    intra = np.zeros((13, 8), np.int64)
    intra[2, 2] = 51  # P(2 | 0) mostly intra: 1 and 2 stay P
    t = b_adapt_types(p1, pd, bc, 3, 100, pd_intra=intra)
    assert t.startswith("IPP"), t
    intra[:] = 0
    intra[4, 4] = 34  # closing the run at 4 from 0 is a third intra: the run stops at 2 B
    t = b_adapt_types(p1, pd, bc, 3, 100, pd_intra=intra)
    assert t.startswith("IBBP"), t
    intra[4, 4] = 33  # not more than a third: unchanged
    assert b_adapt_types(p1, pd, bc, 3, 100, pd_intra=intra) == "IBBBPBBBPBBBP"


def test_with_anchors_splits_b_runs_only():
    from govideocompressor_amd.rc.badapt import with_anchors
    assert with_anchors("IBBBPBBBP", {2, 6}) == "IBPBPBPBP"
    assert with_anchors("IBBBPBBBP", {0, 4, 8}) == "IBBBPBBBP"
