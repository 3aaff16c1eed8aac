"""Device discovery and selection: one process per GPU (LOCAL_RANK -> device)."""
from __future__ import annotations

import os
from dataclasses import dataclass


@dataclass
class DeviceInfo:
    index: int
    name: str
    arch: str
    cus: int
    hbm_bytes: int

    def fits(self, nbytes: int, reserve: float = 0.1) -> bool:
        return nbytes <= self.hbm_bytes * (1.0 - reserve)


def local_device():
    """The torch device this process owns: ``cuda:LOCAL_RANK`` (modulo visible GPUs) or cpu."""
    import torch
    if not torch.cuda.is_available():
        return torch.device("cpu")
    n = torch.cuda.device_count()
    idx = int(os.environ.get("LOCAL_RANK", "0")) % max(1, n)
    return torch.device("cuda", idx)


def device_info(index: int = 0) -> DeviceInfo | None:
    import torch
    if not torch.cuda.is_available():
        return None
    p = torch.cuda.get_device_properties(index)
    arch = getattr(p, "gcnArchName", "") or ""
    return DeviceInfo(index, p.name, arch.split(":")[0], p.multi_processor_count, p.total_memory)


def slots_for(width: int, height: int, frames: int, info: DeviceInfo | None, cap: int = 512) -> int:
    """Segments to encode concurrently on one GPU: enough to put >= 1 frame wavefront on
    every CU, bounded by HBM (input clip + encoder state per slot)."""
    if info is None:
        return 1
    coded = ((width + 15) // 16 * 16) * ((height + 15) // 16 * 16)
    per_slot = coded * 3 // 2 * (frames + 4) + coded // 256 * (64 + 816 + 400)
    by_mem = max(1, int(info.hbm_bytes * 0.6) // max(1, per_slot))
    return max(1, min(cap, by_mem, max(info.cus, 1)))


def cgroup_mem_limit() -> int | None:
    """The memory limit of this process's cgroup in bytes (v2 ``memory.max``, v1
    ``memory.limit_in_bytes``), or None when unlimited / unreadable."""
    paths = ["/sys/fs/cgroup/memory.max", "/sys/fs/cgroup/memory/memory.limit_in_bytes"]
    try:  # the process's own cgroup v2 directory, when it is not the root
        with open("/proc/self/cgroup") as f:
            for line in f:
                parts = line.strip().split(":", 2)
                if len(parts) == 3 and parts[0] == "0" and parts[2] not in ("", "/"):
                    paths.insert(0, "/sys/fs/cgroup" + parts[2] + "/memory.max")
    except OSError:
        pass
    for p in paths:
        try:
            with open(p) as f:
                v = f.read().strip()
        except OSError:
            continue
        if v and v != "max" and v.isdigit() and int(v) < (1 << 60):
            return int(v)
    return None


def host_mem_total() -> int:
    """Host RAM this process may use in bytes: ``/proc/meminfo`` MemTotal capped by the
    cgroup memory limit (a container or a batch slot sees the machine's MemTotal but may
    only hold its limit); 64 GiB if unreadable."""
    total = 64 << 30
    try:
        with open("/proc/meminfo") as f:
            for line in f:
                if line.startswith("MemTotal:"):
                    total = int(line.split()[1]) * 1024
                    break
    except OSError:
        pass
    lim = cgroup_mem_limit()
    return min(total, lim) if lim else total


def pinned_budget(local_world: int | None = None) -> int:
    """Page-locked host bytes one rank may hold.

    ``MIVC_PINNED_BUDGET_MB`` if set, else a quarter of host RAM shared by the ranks on this
    host (``LOCAL_WORLD_SIZE``, torchrun's count): 8 ranks on a 2 TB MI355X node get 64 GB
    each, one rank on a 3 GB lease box 768 MB.  Encoders size their pinned rings from it and
    the merge falls back to pageable buffers beyond it."""
    env = os.environ.get("MIVC_PINNED_BUDGET_MB")
    if env:
        return int(float(env) * (1 << 20))
    n = local_world or int(os.environ.get("LOCAL_WORLD_SIZE", os.environ.get("WORLD_SIZE", "1")))
    return max(64 << 20, host_mem_total() // 4 // max(1, n))
