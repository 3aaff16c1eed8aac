"""Device runtime (SURVEY.md 2.6 "runtime/{device,pool,streams}"): device selection,
preallocated HBM encoder pools, pinned host staging, and per-stage HIP streams."""
from .device import DeviceInfo, device_info, local_device
from .pool import EncoderPool, PinnedPool
from .streams import StageStreams

__all__ = ["DeviceInfo", "device_info", "local_device", "EncoderPool", "PinnedPool", "StageStreams"]
