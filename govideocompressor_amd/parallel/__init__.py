"""Distributed execution: process group (RCCL/gloo), collectives, tickets, launcher."""
from .dist import BitstreamGather, DistEnv, allreduce_stats, barrier, init, max_over_ranks  # noqa: F401
