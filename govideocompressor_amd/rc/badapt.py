"""Adaptive B-picture placement (x264 ``--b-adapt 1``) from the GPU lookahead's costs.

The reference's ``264`` preset is bare ``-vcodec libx264`` (server.go:69-70), whose default
``--b-adapt 1`` ("fast") decides per run of pictures whether the next ones are B or P from
the half-resolution costs of coding them either way.  Here the costs come from
``csrc/kernels/lookahead.hip`` (la_cost: P at distance 1 and intra; la_multi: P at distances
2..bframes+1, B between the two neighbours), computed for every frame of every slot in one
launch, and the decision runs per slot on the host (a few integer comparisons per picture):

* picture i is the last anchor.  Coding i+1 as P then i+2 as P costs
  ``P(i+1 | i) + P(i+2 | i+1)``; coding i+1 as B between i and i+2 costs
  ``B(i+1 | i, i+2) + P(i+2 | i)``.  The cheaper wins;
* B costs enter every comparison scaled by 100 / (120 + bframe_bias) (x264 prices a lowres B
  frame that much cheaper than its raw SATD sum: B pictures are coded at a higher QP);
* a B run then grows picture by picture while the P that would close it, predicted from i
  across the whole run, stays below ``INTER_THRESH - P_SENS_BIAS * (run - 1)`` per macroblock
  (x264's thresholds, 300 and 50: fast motion or a change of content ends the run early);
* forced anchors (scene cuts, segment ends the caller needs) are never B and end any run;
* intra guards (x264's ``i_intra_mbs`` checks, with the lookahead's intra block counts): when
  more than half the blocks of P(i+2 | i) would be intra, the two pictures cannot share
  references usefully -- both become P; a run stops growing when more than a third of the
  blocks of the P that would close it would be intra (a change of content inside the run).

Costs are the lookahead's per-frame sums of ``min(intra, candidate)`` over the lowres 8x8
blocks (one per macroblock), the unit x264's thresholds are written in.
"""
from __future__ import annotations

import numpy as np

INTER_THRESH = 300
P_SENS_BIAS = 50
B_COST_SCALE = 100.0 / 120.0  # x264 slicetype frame cost of a B frame, --b-bias 0


def b_adapt_types(p1: np.ndarray, pd: np.ndarray, bcost: np.ndarray, bframes: int, mb_count: int,
                  forced=(), b_bias: int = 0, pd_intra: np.ndarray | None = None) -> str:
    """Display-order picture types of one segment (``"IPBBP..."``).

    p1[f]: P cost of f from f - 1; pd[f, d]: P cost of f from f - d (d = 2..bframes + 1,
    columns of la_multi); bcost[f]: B cost of f between f - 1 and f + 1.  ``b_bias``: x264
    --b-bias (B costs scaled by 100 / (120 + b_bias), run threshold slope 50 - b_bias).
    pd_intra[f, d]: intra block counts of the pd candidates (la_multi); None = no guards."""
    b_scale = 100.0 / (120.0 + b_bias)
    sens = P_SENS_BIAS - b_bias
    F = len(p1)
    if F == 0:
        return ""
    types = ["I"] + ["P"] * (F - 1)
    if bframes <= 0 or F < 3:
        return "".join(types)
    forced = {int(d) for d in forced if 0 < int(d) < F}
    forced.add(F - 1)

    def pcost(f: int, d: int) -> float:
        return float(p1[f]) if d == 1 else float(pd[f, d])

    def intra_blocks(f: int, d: int) -> int:
        return 0 if pd_intra is None or d < 2 else int(pd_intra[f, d])

    i = 0
    while i < F - 1:
        if i + 1 in forced or i + 2 >= F:
            i += 1  # i + 1 is an anchor (forced, or the last picture)
            continue
        if intra_blocks(i + 2, 2) > mb_count // 2:
            i += 2  # i + 1 and i + 2 stay P
            continue
        keep_p = pcost(i + 1, 1) + pcost(i + 2, 1)
        as_b = b_scale * float(bcost[i + 1]) + pcost(i + 2, 2)
        if keep_p < as_b:
            i += 1
            continue
        types[i + 1] = "B"
        j = i + 2
        while j <= min(i + bframes, F - 2) and j not in forced:
            pthresh = max(INTER_THRESH - sens * (j - i - 1), INTER_THRESH / 10)
            if j + 1 - i > bframes + 1 or pcost(j + 1, j + 1 - i) > pthresh * mb_count:
                break
            if intra_blocks(j + 1, j + 1 - i) > mb_count // 3:
                break
            types[j] = "B"
            j += 1
        i = j  # picture j closes the run as an anchor
    return "".join(types)


def with_anchors(types: str, anchors) -> str:
    """``types`` with the pictures at ``anchors`` turned into P anchors (B runs only split, so
    they stay within the pattern's run length); picture 0 keeps its type."""
    t = list(types)
    for d in anchors:
        d = int(d)
        if 0 < d < len(t) and t[d] == "B":
            t[d] = "P"
    return "".join(t)


def b_adapt_batch(costs: np.ndarray, multi: np.ndarray, bframes: int, mb_count: int, forced_per_slot,
                  b_bias: int = 0, multi_intra: np.ndarray | None = None) -> list[str]:
    """Per-slot types of a batch: costs [B, F, 2] (la_cost frame sums: intra, min(intra,
    inter at distance 1)), multi [B, F, 8] (la_multi), forced_per_slot: one iterable per slot."""
    B = costs.shape[0]
    out = []
    for b in range(B):
        out.append(b_adapt_types(costs[b, :, 1], multi[b], multi[b, :, 0], bframes, mb_count, forced_per_slot[b],
                                 b_bias, None if multi_intra is None else multi_intra[b]))
    return out


def anchor_complexity(types: str, costs: np.ndarray, multi: np.ndarray | None) -> np.ndarray:
    """Per display picture, the complexity the CRF curve sees: intra cost for I, the P cost
    from the previous anchor (at its real distance) for P, NaN for B pictures (they take
    their references' QP, rc/ratecontrol.b_qps_from_refs)."""
    F = len(types)
    c = np.full(F, np.nan)
    last = 0
    for f, t in enumerate(types):
        if t == "I":
            c[f] = costs[f, 0]
            last = f
        elif t == "P":
            d = f - last
            c[f] = costs[f, 1] if (d == 1 or multi is None) else multi[f, min(d, multi.shape[1] - 1)]
            last = f
    return c
