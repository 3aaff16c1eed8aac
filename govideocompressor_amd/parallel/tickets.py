"""Dynamic segment scheduling without a coordinator thread.

The reference's load balancing is pull-based: whichever worker connects next gets
the next piece (server.go:175-189).  Inside one node that maps to an atomic
counter on the ``torch.distributed`` TCPStore: ``store.add(key, k)`` returns the
post-increment value, so a rank claims tickets ``[v-k, v)`` with one round trip
and no central loop.  Segments are claimed in chunks of ``k`` =
the GPU batch width so that each claim becomes one batched encode.
"""
from __future__ import annotations

import torch.distributed as dist


class TicketDispenser:
    def __init__(self, n_items: int, key: str = "mivc_next_seg", store=None):
        self.n = int(n_items)
        self.key = key
        self.store = store
        if self.store is None and dist.is_initialized():
            from torch.distributed.distributed_c10d import _get_default_store
            self.store = _get_default_store()
        self._local = 0  # world == 1 fallback

    def claim(self, k: int = 1) -> list[int]:
        """Claim up to ``k`` consecutive items; [] when everything has been handed out."""
        if self.store is None:
            start = self._local
            self._local += k
        else:
            end = int(self.store.add(self.key, k))
            start = end - k
        return [i for i in range(start, min(start + k, self.n))]

    def __iter__(self):
        while True:
            got = self.claim(1)
            if not got:
                return
            yield got[0]
