"""Rate control: CRF from lowres complexity, two-pass ABR with a
global statistics all-reduce (CC-1)."""
from .ratecontrol import (GlobalStats, TwoPassFeedback, abr_qps, abr_solve, crf_qps, crf_qps_batch, estimate_exponent,
                          frame_complexity, qp2qscale, qscale2qp)

__all__ = ["GlobalStats", "TwoPassFeedback", "abr_qps", "abr_solve", "crf_qps", "crf_qps_batch", "estimate_exponent", "frame_complexity",
           "qp2qscale", "qscale2qp"]
