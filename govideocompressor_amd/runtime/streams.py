"""HIP streams per pipeline stage.

The encode loop runs kernels on the compute stream; device->host copies of the
entropy-coded bytes and host->device uploads of the next batch run on their own
streams, ordered by events (the encoder's ``copy_stream``/``copy_done`` pattern),
and RCCL collectives use the process group's internal stream (``async_op=True``).
"""
from __future__ import annotations


class StageStreams:
    def __init__(self, device=None):
        import torch
        self.enabled = torch.cuda.is_available()
        if not self.enabled:
            self.compute = self.h2d = self.d2h = None
            return
        dev = device if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.compute = torch.cuda.current_stream(dev)
        self.h2d = torch.cuda.Stream(device=dev)
        self.d2h = torch.cuda.Stream(device=dev)

    def upload(self, host_tensors, device):
        """Start H2D copies of pinned tensors on the upload stream; returns (device tensors, event)."""
        import torch
        if not self.enabled:
            return [t for t in host_tensors], None
        with torch.cuda.stream(self.h2d):
            out = [t.to(device, non_blocking=True) for t in host_tensors]
            ev = torch.cuda.Event()
            ev.record(self.h2d)
        for t in out:  # the consumer is the compute stream: keep the blocks alive for it
            t.record_stream(self.compute)
        return out, ev

    def wait(self, ev) -> None:
        if ev is not None and self.enabled:
            self.compute.wait_event(ev)
