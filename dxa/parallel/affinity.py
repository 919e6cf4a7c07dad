"""Host-side NUMA placement for one-process-per-GPU jobs.

On a multi-socket MI355X node each GPU hangs off one socket's PCIe root.  Pinned host buffers (ingest frames, output
staging) are allocated by first touch, so a rank whose threads run on the far socket stages every H2D/D2H byte
across the inter-socket fabric — with eight ranks streaming ~50 GB/s each that link, not PCIe, becomes the limit.
``bind_to_device`` restricts the calling process to the CPUs local to its GPU (sysfs ``local_cpulist`` of the GPU's
PCI function) before any pinned buffer exists.  Everything here is best effort: missing sysfs entries, containers
without the right to change affinity, or CPU-only runs leave the process untouched.
"""
from __future__ import annotations

import os
from typing import Optional, Set


def parse_cpulist(text: str) -> Set[int]:
    """``"0-3,8,10-11"`` → {0, 1, 2, 3, 8, 10, 11}."""
    cpus: Set[int] = set()
    for part in text.strip().split(","):
        part = part.strip()
        if not part:
            continue
        if "-" in part:
            lo, hi = part.split("-", 1)
            cpus.update(range(int(lo), int(hi) + 1))
        else:
            cpus.add(int(part))
    return cpus


def device_pci_path(index: int) -> Optional[str]:
    import torch
    try:
        p = torch.cuda.get_device_properties(index)
        bdf = f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}.0"
    except Exception:
        return None
    path = f"/sys/bus/pci/devices/{bdf}"
    return path if os.path.isdir(path) else None


def local_cpus(index: int) -> Optional[Set[int]]:
    path = device_pci_path(index)
    if path is None:
        return None
    try:
        with open(os.path.join(path, "local_cpulist")) as f:
            cpus = parse_cpulist(f.read())
    except (OSError, ValueError):
        return None
    return cpus or None


def bind_to_device(index: int) -> Optional[Set[int]]:
    """Pin this process to the CPUs local to GPU ``index`` (intersected with the CPUs it may use now).  Returns the
    new CPU set, or None when nothing was changed."""
    if os.environ.get("DXA_NUMA_BIND", "1") == "0" or not hasattr(os, "sched_setaffinity"):
        return None
    cpus = local_cpus(index)
    if not cpus:
        return None
    allowed = os.sched_getaffinity(0)
    want = cpus & allowed
    if not want or want == allowed:
        return None
    try:
        os.sched_setaffinity(0, want)
    except OSError:
        return None
    return want
